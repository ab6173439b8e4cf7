"""Regenerate tests/golden/config_digests.json: per-level SHA-256 digests of
every BASELINE config x method, from the oracle (oracle/ds_oracle.c) on the
splitmix64 inputs of tests/digest_util.py.

    python tests/golden/make_digests.py

Needs only the built oracle (make -C oracle); never the reference.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import digest_util as du  # noqa: E402
import oracle  # noqa: E402


def make_oracle(dims, dtype, method):
    geo = oracle.level_geometry(oracle.plan_levels(dims))
    return oracle.OracleDownsampler(geo, dtype, method), geo


def main():
    out = {"generator": "tests/digest_util.py (splitmix64, seed 0xA0C2A11 + sorted config index)",
           "digest": "sha256 of each level's taken frames, concatenated in order",
           "made_by": "oracle/ds_oracle.c via tests/golden/make_digests.py",
           "configs": {}}
    for name in du.CONFIGS:
        dims, dtype, frames = du.CONFIGS[name]
        entry = {"dims": dims, "dtype": str(__import__("numpy").dtype(dtype)),
                 "frames": frames, "methods": {}}
        for m, mname in enumerate(du.METHOD_NAMES):
            entry["methods"][mname] = du.run_stream(make_oracle, name, m)
            print(name, mname, entry["methods"][mname], flush=True)
        out["configs"][name] = entry
    with open(du.ORACLE_DIGESTS, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
