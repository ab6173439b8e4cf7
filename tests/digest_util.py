"""Deterministic full-size inputs and per-level digests for the BASELINE
configs (SURVEY §8(c) "golden plan", §8(d) input definition).

Pixels come from a counter-based splitmix64: value i of frame k of a config
is mix(seed + (k * N + i + 1) * 0x9E3779B97F4A7C15), N = pixels per frame.
Integers take the low bits; float32 takes the top 24 bits scaled to
[-1000, 1000).  Both the oracle (CPU tests) and the
HIP path (GPU tests) are checked against the SHA-256 of every level's frames,
concatenated in emit order.  GOLDEN, tests/golden/reference_digests.json, was
made by the REFERENCE ITSELF (oracle/_ref: downsampler.cpp compiled
unmodified; tests/golden/make_reference_vectors.py --digests).  The oracle's
own digests (tests/golden/config_digests.json, tests/golden/make_digests.py)
must equal them (tests/test_reference_pin.py).
"""
import hashlib
import os

import numpy as np

_GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
GOLDEN = os.path.join(_GOLDEN_DIR, "reference_digests.json")      # made by the reference
ORACLE_DIGESTS = os.path.join(_GOLDEN_DIR, "config_digests.json")  # made by the oracle
SEED = 0xA0C2A11
SPACE, TIME = 0, 2

# name: (dims in storage order (type, size, chunk, shard), dtype, frames)
CONFIGS = {
    "C1b_512x512_u8": ([(TIME, 0, 1, 1), (SPACE, 512, 128, 1), (SPACE, 512, 128, 1)],
                       np.uint8, 4),
    "C2_2048x2048_u16": ([(TIME, 0, 1, 1), (SPACE, 2048, 256, 1), (SPACE, 2048, 256, 1)],
                         np.uint16, 2),
    "H_4096x4096_u16": ([(TIME, 0, 1, 1), (SPACE, 4096, 256, 1), (SPACE, 4096, 256, 1)],
                        np.uint16, 2),
    "F_4096x4096_f32": ([(TIME, 0, 1, 1), (SPACE, 4096, 256, 1), (SPACE, 4096, 256, 1)],
                        np.float32, 1),
    "V_1024x1024x256_u16": ([(TIME, 0, 1, 1), (SPACE, 256, 64, 1), (SPACE, 1024, 256, 1),
                             (SPACE, 1024, 256, 1)], np.uint16, 256),
}
METHOD_NAMES = ["decimate", "mean", "min", "max"]

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(counter: np.ndarray, seed: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (counter + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def config_seed(name: str) -> int:
    return SEED + sorted(CONFIGS).index(name)


def frame(name: str, k: int, width: int, height: int, dtype) -> np.ndarray:
    """Frame (or plane) k of config `name`."""
    n = width * height
    ctr = np.arange(k * n, (k + 1) * n, dtype=np.uint64)
    z = splitmix64(ctr, config_seed(name))
    dt = np.dtype(dtype)
    if dt.kind == "f":
        u = (z >> np.uint64(40)).astype(np.float64)
        x = (u / 16777216.0 * 2000.0 - 1000.0).astype(dt)
    else:
        x = (z & np.uint64((1 << (8 * dt.itemsize)) - 1)).astype(dt)
    return x.reshape(height, width)


class LevelHashes:
    """SHA-256 per level over the frames taken there, in order."""

    def __init__(self, n_levels):
        self.h = {L: hashlib.sha256() for L in range(1, n_levels)}
        self.count = {L: 0 for L in range(1, n_levels)}

    def add(self, level, arr):
        self.h[level].update(np.ascontiguousarray(arr).tobytes())
        self.count[level] += 1

    def result(self):
        return {str(L): {"frames": self.count[L], "sha256": self.h[L].hexdigest()}
                for L in self.h}


def run_stream(make_downsampler, name, method):
    """Feed config `name` through a Downsampler-like object (add_frame /
    take_frame(L) -> array or None), taking every level after every frame."""
    dims, dtype, frames = CONFIGS[name]
    ds, geo = make_downsampler(dims, dtype, method)
    W, H, _ = geo[0]
    hs = LevelHashes(len(geo))
    for k in range(frames):
        ds.add_frame(frame(name, k, W, H, dtype))
        for L in range(1, len(geo)):
            out = ds.take_frame(L)
            if out is not None:
                hs.add(L, out)
    return hs.result()
