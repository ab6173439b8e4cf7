"""Generate tests/golden/blosc_frames.npz: c-blosc frames as fixtures.

Each case is one chunk buffer compressed the way compress_in_place does it
(zarr.common.cpp:106-137): blosc_compress_ctx(clevel, shuffle, typesize,
nbytes, src, dest, nbytes + 16, cname, 0, 1).  The frames come from the
image's c-blosc 1.21.0 (/opt/conda/lib/libblosc.so.1, oracle/blosc_ref.py),
the inputs are stored next to them, so tests/test_blosc_frames.py can check
the product's frame writer against them even where libblosc is absent.

Run: python tests/golden/make_blosc_frames.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import blosc_ref  # noqa: E402


def inputs():
    rng = np.random.default_rng(20261017)
    yy, xx = np.mgrid[0:128, 0:128]
    smooth16 = (1000 + 30 * np.sin(xx / 9.0) * np.cos(yy / 7.0) * 40
                + rng.normal(0, 3, (128, 128))).astype(np.uint16)          # 32 KiB
    yield "smooth_u16_128x128", smooth16, 2
    yield "random_u8_4099", rng.integers(0, 256, 4099, dtype=np.uint8), 1
    mixed = np.zeros(40000, np.uint8)
    mixed[14000:26000] = rng.integers(0, 256, 12000, dtype=np.uint8)
    yield "mixed_u8_40000", mixed, 1
    f32 = (np.cumsum(rng.normal(0, 1, 9000)) * 10).astype(np.float32)  # 36000 B
    yield "walk_f32_9000", f32, 4
    yield "small_u16_50", np.arange(50, dtype=np.uint16), 2
    yield "ramp_u64_5000", (np.arange(5000, dtype=np.uint64) * 977) % 65536, 8
    yield "odd_ts3_30001", rng.integers(0, 4, 30001, dtype=np.uint8), 3


CASES = [
    ("lz4", 1, 1), ("lz4", 5, 1), ("lz4", 9, 2), ("lz4", 3, 0),
    ("zstd", 1, 1), ("zstd", 5, 2), ("zstd", 9, 1), ("zstd", 0, 1),
]


def main():
    out = {}
    names = []
    for name, arr, ts in inputs():
        raw = np.ascontiguousarray(arr).view(np.uint8).reshape(-1)
        out[f"in__{name}"] = raw
        for cname, clevel, shuffle in CASES:
            fr = blosc_ref.compress(raw, clevel, shuffle, ts, cname)
            assert not isinstance(fr, int), (name, cname, clevel, shuffle, fr)
            key = f"{name}__{cname}__{clevel}__{shuffle}__{ts}"
            out[f"frame__{key}"] = np.frombuffer(fr, np.uint8)
            names.append(key)
    out["version"] = np.frombuffer(blosc_ref.version().encode(), np.uint8)
    path = os.path.join(HERE, "blosc_frames.npz")
    np.savez_compressed(path, **out)
    print(path, len(names), "frames", os.path.getsize(path), "bytes, c-blosc",
          blosc_ref.version())


if __name__ == "__main__":
    main()
