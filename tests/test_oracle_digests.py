"""The oracle reproduces the committed per-level digests of every BASELINE
config x method at full size — tests/golden/reference_digests.json, made by
the REFERENCE ITSELF (oracle/_ref, tests/golden/make_reference_vectors.py
--digests).  The GPU path is held to the same digests in
tests/test_gpu_digests.py; the oracle's own copy (config_digests.json,
make_digests.py) equals them (tests/test_reference_pin.py)."""
import json

import pytest

import digest_util as du

with open(du.GOLDEN) as f:
    GOLD = json.load(f)["configs"]

CASES = [(c, m) for c in du.CONFIGS for m in range(len(du.METHOD_NAMES))]


def test_generator_known_values():
    # splitmix64 reference outputs for seed 0 (the published algorithm's
    # first outputs from state 0: 0xE220A8397B1DCDAF, 0x6E789E6AA1B965F4)
    import numpy as np
    z = du.splitmix64(np.arange(2, dtype=np.uint64), 0)
    assert [int(v) for v in z] == [0xE220A8397B1DCDAF, 0x6E789E6AA1B965F4]


@pytest.mark.parametrize("name,method", CASES,
                         ids=[f"{c}-{du.METHOD_NAMES[m]}" for c, m in CASES])
def test_oracle_matches_digests(oracle, name, method):
    def make(dims, dtype, m):
        geo = oracle.level_geometry(oracle.plan_levels(dims))
        return oracle.OracleDownsampler(geo, dtype, m), geo
    got = du.run_stream(make, name, method)
    assert got == GOLD[name]["methods"][du.METHOD_NAMES[method]]
