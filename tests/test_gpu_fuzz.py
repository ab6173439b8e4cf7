"""Seeded random geometries through the fused batch path and the streaming
path, against the oracle.

The batch launcher picks among several store schemes by frame width, dtype
and the alignment of every level's rows and buffers: direct stores, band
workgroups, aligned bands behind a barrier (whole or in 4- or 8-tile
segments), misaligned bands stored by their last wave (whole, or in segments
with one LDS slot per level row).  The fixed geometries in test_gpu_parity.py
pin each scheme once; these cases sweep widths from 1 to 9000 px, heights
(1-160) with partial bottom bands, 2-6 levels, all ten dtypes and four methods, and
input and output buffers at element-aligned but otherwise arbitrary byte
offsets (which turns aligned rows into misaligned ones).  Integers bit-exact,
floats within 1 ulp (assert_parity).  Also: chunk-tiled batches with random
tile shapes, and Z stacks (fused 2x2x2 or the Z state machine)."""
import os
import re
import zlib

import numpy as np
import pytest

from gpu_util import (assert_parity, empty_device, from_device, launch_stream,
                      random_frames, to_device, torch_cuda)

pytestmark = pytest.mark.gpu

DTYPES = [np.uint8, np.uint16, np.uint32, np.uint64, np.int8, np.int16,
          np.int32, np.int64, np.float32, np.float64]
# $AQZ_FUZZ_CASES widens the sweep for one-off runs (scripts/r06_fuzzwide.sh)
N_CASES = int(os.environ.get("AQZ_FUZZ_CASES", "256"))


def case_params(i):
    rng = np.random.default_rng(zlib.crc32(f"fuzz{i}".encode()))
    # the camera types most often, every type some of the time
    weights = np.array([3, 6, 1, 1, 1, 1, 1, 1, 4, 1], dtype=float)
    dtype = DTYPES[int(rng.choice(len(DTYPES), p=weights / weights.sum()))]
    method = int(rng.integers(4))
    # widths: tile-multiple neighbourhoods, the wide band regime (2000-9000
    # px, where the misaligned schemes live), or log-uniform over [1, 9000]
    u = rng.random()
    if u < 0.25:
        w = int(rng.choice([256, 512, 1024, 2048, 4096])) * int(rng.integers(1, 3))
        w = max(1, w + int(rng.integers(-3, 4)))
    elif u < 0.6:
        w = int(rng.integers(2000, 9001))
    else:
        w = int(np.exp(rng.uniform(0, np.log(9000))))
    h = int(rng.integers(1, 161))
    n_levels = int(rng.integers(2, 7))
    frames = int(rng.integers(1, 4))
    in_off = int(rng.integers(0, 8))
    out_off = [int(rng.integers(0, 8)) for _ in range(n_levels)]
    return dtype, method, w, h, n_levels, frames, in_off, out_off, rng


def geometry(w, h, n_levels):
    geo = [(w, h, 1)]
    for _ in range(1, n_levels):
        w, h = (w + 1) // 2, (h + 1) // 2
        geo.append((w, h, 1))
    return geo


def oracle_stream(oracle, geo, dtype, method, frames):
    ref = oracle.OracleDownsampler(geo, dtype, method)
    expected = {L: [] for L in range(1, len(geo))}
    for f in frames:
        ref.add_frame(f)
        for L in expected:
            r = ref.take_frame(L)
            if r is not None:
                expected[L].append(r)
    return expected


@pytest.mark.parametrize("case", range(N_CASES))
def test_fuzz_device_batch(aqz, oracle, case):
    torch_cuda()
    dtype, method, w, h, n_levels, n, in_off, out_off, rng = case_params(case)
    geo = geometry(w, h, n_levels)
    bpp = np.dtype(dtype).itemsize
    frames = random_frames(rng, dtype, (n, h, w))
    expected = oracle_stream(oracle, geo, dtype, method, frames)
    # input and every level at a random element offset into its buffer
    raw = np.zeros(in_off * bpp + frames.nbytes, dtype=np.uint8)
    raw[in_off * bpp:] = frames.view(np.uint8).reshape(-1)
    d_in = to_device(raw)
    outs = [None] + [empty_device((out_off[L] + n * gw * gh) * bpp)
                     for L, (gw, gh, _) in enumerate(geo) if L > 0]
    ptrs = [0] + [outs[L].data_ptr() + out_off[L] * bpp for L in range(1, n_levels)]
    ds = aqz.Downsampler(geo, dtype, method)
    counts = ds.run_device_batch(d_in.data_ptr() + in_off * bpp, n, ptrs, launch_stream())
    ctx = f"case {case}: {np.dtype(dtype).name} m{method} {w}x{h} L{n_levels} n{n}"
    for L in range(1, n_levels):
        gw, gh, _ = geo[L]
        assert counts[L] == len(expected[L]), ctx
        got = from_device(outs[L], np.uint8, (-1,))[out_off[L] * bpp:]
        got = got.view(dtype).reshape(n, gh, gw)
        for k, e in enumerate(expected[L]):
            assert_parity(got[k], e, f"{ctx} level {L} frame {k}")
    ds.close()


@pytest.mark.parametrize("case", range(0, N_CASES, 4))
def test_fuzz_stream(aqz, oracle, case):
    """The same geometries through add_frame / take_frame (one fused launch
    per frame, or the per-level state machine), frame by frame."""
    torch_cuda()
    dtype, method, w, h, n_levels, n, _, _, rng = case_params(case)
    geo = geometry(w, h, n_levels)
    frames = random_frames(rng, dtype, (n, h, w))
    ds = aqz.Downsampler(geo, dtype, method)
    ref = oracle.OracleDownsampler(geo, dtype, method)
    for i, f in enumerate(frames):
        ds.add_frame(f)
        ref.add_frame(f)
        for L in range(1, n_levels):
            a, b = ds.take_frame(L), ref.take_frame(L)
            assert (a is None) == (b is None), f"case {case} frame {i} level {L}"
            if a is not None:
                assert_parity(a, b, f"case {case} frame {i} level {L}")
    ds.close()


def tiled_case_params(i):
    rng = np.random.default_rng(zlib.crc32(f"fuzz-tiled{i}".encode()))
    weights = np.array([3, 6, 1, 1, 1, 1, 1, 1, 4, 1], dtype=float)
    dtype = DTYPES[int(rng.choice(len(DTYPES), p=weights / weights.sum()))]
    method = int(rng.integers(4))
    w = int(np.exp(rng.uniform(0, np.log(6000))))
    h = int(np.exp(rng.uniform(0, np.log(400))))
    n_levels = int(rng.integers(2, 7))

    def side():
        if rng.random() < 0.4:
            return int(rng.choice([16, 32, 64, 128, 256, 512]))
        return int(np.exp(rng.uniform(0, np.log(300))))

    return dtype, method, w, h, n_levels, side(), side(), int(rng.integers(1, 3)), rng


@pytest.mark.parametrize("case", range(96))
def test_fuzz_tiled_batch(aqz, oracle, case):
    """Chunk-tiled levels straight from the pyramid kernel
    (aqz_ds_run_device_batch_tiled): random frame and tile shapes, poisoned
    outputs, tile bytes and the zero scan against oracle_tile_frame."""
    from test_gpu_tiled import run_tiled

    dtype, method, w, h, n_levels, tr, tc, n, rng = tiled_case_params(case)
    geo = geometry(w, h, n_levels)
    frames = [random_frames(rng, dtype, (h, w)) for _ in range(n)]
    frames[0][: h // 2, : w // 3] = 0  # all-zero tiles at some levels
    ctx = f"case {case}: {np.dtype(dtype).name} m{method} {w}x{h} L{n_levels} tile {tr}x{tc}"
    try:
        got, _ = run_tiled(aqz, geo, dtype, method, frames, tr, tc)
    except aqz.AqzError as e:
        # documented refusals (aqz_downsampler.h): a fused run's first level
        # (level 0, 4, 8, ...) narrower than one 16-byte load, or a level
        # that does not halve (1 x 1 onwards: a copy, not a pure-XY pyramid)
        m = re.search(r"level (\d+) is narrower than one vector load", str(e))
        c = re.search(r"level (\d+) does not halve XY alone", str(e))
        assert m or c, f"{ctx}: {e}"
        if m:
            L0 = int(m.group(1))
            assert L0 % 4 == 0 and geo[L0][0] * np.dtype(dtype).itemsize < 16, f"{ctx}: {e}"
        else:
            L = int(c.group(1))
            assert geo[L][:2] == geo[L - 1][:2], f"{ctx}: {e}"
        return
    for k, fr in enumerate(frames):
        ref = oracle.cascade_2d(fr, n_levels, method)
        for L in range(1, n_levels):
            want_t, want_nz = oracle.tile_frame(ref[L - 1], tr, tc)
            t, f = got[L - 1]
            assert_parity(t[k], want_t, f"{ctx} frame {k} L{L} tiles")
            assert np.array_equal(f[k], want_nz), f"{ctx} frame {k} L{L} zero scan"


def volume_case_params(i):
    rng = np.random.default_rng(zlib.crc32(f"fuzz-volume{i}".encode()))
    weights = np.array([3, 6, 1, 1, 1, 1, 1, 1, 4, 1], dtype=float)
    dtype = DTYPES[int(rng.choice(len(DTYPES), p=weights / weights.sum()))]
    method = int(rng.integers(4))
    w = int(np.exp(rng.uniform(0, np.log(2500))))
    h = int(rng.integers(1, 48))
    planes = int(rng.integers(1, 20))
    n_levels = int(rng.integers(2, 5))
    # Z halves at a level with probability 3/4 while there is more than one
    # plane (pure 2x2x2 pyramids take the fused volume kernel, the rest the
    # per-level state machine)
    geo = [(w, h, planes)]
    for _ in range(1, n_levels):
        w, h = (w + 1) // 2, (h + 1) // 2
        if planes > 1 and rng.random() < 0.75:
            planes = (planes + 1) // 2
        geo.append((w, h, planes))
    frames = int(rng.integers(1, 3)) * geo[0][2]  # whole stacks, or more
    return dtype, method, geo, frames, rng


@pytest.mark.parametrize("case", range(64))
def test_fuzz_volume_batch(aqz, oracle, case):
    """Z stacks: the fused 2x2x2 kernel or the per-level Z state machine,
    frames streamed plane by plane in a device batch, against the oracle's
    add_frame / take_frame sequence."""
    torch_cuda()
    dtype, method, geo, n, rng = volume_case_params(case)
    w, h, _ = geo[0]
    bpp = np.dtype(dtype).itemsize
    frames = random_frames(rng, dtype, (n, h, w))
    expected = oracle_stream(oracle, geo, dtype, method, frames)
    d_in = to_device(frames)
    outs = [None] + [empty_device(n * gw * gh * bpp) for gw, gh, _ in geo[1:]]
    ds = aqz.Downsampler(geo, dtype, method)
    counts = ds.run_device_batch(d_in.data_ptr(), n, [0] + [o.data_ptr() for o in outs[1:]],
                                 launch_stream())
    ctx = f"case {case}: {np.dtype(dtype).name} m{method} {geo} n{n}"
    for L in range(1, len(geo)):
        gw, gh, _ = geo[L]
        assert counts[L] == len(expected[L]), ctx
        got = from_device(outs[L], dtype, (n, gh, gw))
        for k, e in enumerate(expected[L]):
            assert_parity(got[k], e, f"{ctx} level {L} frame {k}")
    ds.close()
