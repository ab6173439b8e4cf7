"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on the
same seeded inputs, plus the reference's known answers and full-size
properties.  Integers must be bit-exact; floats within 1 ulp (NaN positions
equal) — and are additionally checked bit-exact where stated."""
import os
import subprocess
import zlib

import numpy as np
import pytest

import kat_runner
from gpu_util import (assert_parity, empty_device, from_device, launch_stream,
                      random_frames, to_device, torch_cuda)

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DTYPES = [np.uint8, np.uint16, np.uint32, np.uint64, np.int8, np.int16,
          np.int32, np.int64, np.float32, np.float64]
METHODS = [0, 1, 2, 3]


def seed_of(*parts):
    return zlib.crc32(repr(parts).encode())


def halving_geometry(w, h, n_levels, planes=1):
    geo = [(w, h, planes)]
    for _ in range(1, n_levels):
        w, h = (w + 1) // 2, (h + 1) // 2
        geo.append((w, h, planes))
    return geo


def run_both(aqz, oracle, geo, dtype, method, frames, levels=None):
    """Feed `frames` through both implementations, taking every level after
    each frame; returns the two lists of (frame_idx, level, array)."""
    ds = aqz.Downsampler(geo, dtype, method)
    ref = oracle.OracleDownsampler(geo, dtype, method)
    got, want = [], []
    levels = levels or range(1, len(geo))
    for i, f in enumerate(frames):
        ds.add_frame(f)
        ref.add_frame(f)
        for L in levels:
            a = ds.take_frame(L)
            b = ref.take_frame(L)
            assert (a is None) == (b is None), f"frame {i} level {L} readiness"
            if a is not None:
                got.append((i, L, a))
                want.append((i, L, b))
    ds.close()
    return got, want


# ---- reference C++ unit tests, restated against aqz::Downsampler ----------

@pytest.mark.parametrize("name", ["test_downsampler", "test_downsampler_odd_z"])
def test_cpp_reference_unit_tests(name):
    exe = os.path.join(ROOT, "tests", "cpp", "bin", name)
    assert os.path.exists(exe), f"{exe} not built (run __graft_entry__.build())"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


# ---- golden KATs through the Python binding --------------------------------

KATS = kat_runner.load()


@pytest.mark.parametrize("case", KATS["stream"], ids=lambda c: c["name"])
def test_stream_kats_gpu(aqz, case):
    def make(case, dtype, method):
        levels = aqz.plan_levels(kat_runner.full_dims(case))
        return aqz.Downsampler(aqz.level_geometry(levels), dtype, method)
    kat_runner.run_stream_case(case, make)


# ---- randomized parity, all dtypes x methods -------------------------------

SIZES_2D = [
    (64, 48, 3),      # reference odd-z frame size, fused cascade
    (11, 11, 3),      # odd edges, generic path
    (1000, 600, 5),   # non-power-of-two, boundary tiles in the cascade
    (2048, 40, 4),    # wide and short: row-edge tiles at every level
    (37, 1023, 4),    # odd width (generic) and odd heights
    (520, 520, 6),    # two fused runs (4 + 1 levels)
]


@pytest.mark.parametrize("dtype", DTYPES, ids=lambda d: np.dtype(d).name)
@pytest.mark.parametrize("method", METHODS)
def test_random_2d_parity(aqz, oracle, dtype, method):
    rng = np.random.default_rng(seed_of(np.dtype(dtype).name, method))
    for (w, h, nl) in SIZES_2D:
        geo = halving_geometry(w, h, nl)
        frames = [random_frames(rng, dtype, (h, w)) for _ in range(2)]
        got, want = run_both(aqz, oracle, geo, dtype, method, frames)
        assert len(got) == 2 * (nl - 1)
        for (i, L, a), (_, _, b) in zip(got, want):
            assert_parity(a, b, f"{np.dtype(dtype).name} m{method} {w}x{h} f{i} L{L}")


@pytest.mark.parametrize("dtype", [np.float32, np.float64], ids=["f32", "f64"])
@pytest.mark.parametrize("method", METHODS)
def test_float_bit_exact(aqz, oracle, dtype, method):
    """The float path follows the reference's operation order exactly, so it
    is bit-exact (not merely within 1 ulp), NaN payloads included."""
    rng = np.random.default_rng(5 + method)
    geo = halving_geometry(512, 384, 5)
    frame = random_frames(rng, dtype, (384, 512))
    got, want = run_both(aqz, oracle, geo, dtype, method, [frame])
    ib = np.uint32 if dtype == np.float32 else np.uint64
    for (_, L, a), (_, _, b) in zip(got, want):
        assert np.array_equal(a.view(ib), b.view(ib)), f"level {L}"


# ---- Z pairing (3-D) --------------------------------------------------------

VOLUMES = [
    # (w, h, planes per stack, stacks, level geometry (w,h,planes) list)
    ("even_z", [(64, 64, 8), (32, 32, 4), (16, 16, 2)], 2),
    ("odd_z", [(64, 48, 15), (32, 24, 8), (16, 12, 4), (16, 12, 2)], 2),
    ("z_only", [(40, 30, 6), (40, 30, 3), (40, 30, 2)], 3),
    ("odd_xy_z", [(33, 17, 5), (17, 9, 3), (9, 5, 2)], 3),
]


@pytest.mark.parametrize("dtype", DTYPES, ids=lambda d: np.dtype(d).name)
@pytest.mark.parametrize("method", METHODS)
@pytest.mark.parametrize("vol", VOLUMES, ids=lambda v: v[0])
def test_random_3d_parity(aqz, oracle, dtype, method, vol):
    name, geo, stacks = vol
    rng = np.random.default_rng(seed_of(name, np.dtype(dtype).name, method))
    w, h, z = geo[0]
    frames = [random_frames(rng, dtype, (h, w)) for _ in range(z * stacks)]
    got, want = run_both(aqz, oracle, geo, dtype, method, frames)
    assert len(got) == len(want) and len(got) > 0
    for (i, L, a), (_, _, b) in zip(got, want):
        assert_parity(a, b, f"{name} {np.dtype(dtype).name} m{method} f{i} L{L}")


def test_untaken_frame_is_not_overwritten(aqz, oracle):
    """emplace_downsampled_frame_ keeps the first untaken frame
    (downsampler.cpp:599-605)."""
    geo = halving_geometry(64, 64, 3)
    ds = aqz.Downsampler(geo, np.uint16, 1)
    ds.add_frame(np.full((64, 64), 10, np.uint16))
    ds.add_frame(np.full((64, 64), 20, np.uint16))
    assert np.all(ds.take_frame(1) == 10)
    assert ds.take_frame(1) is None
    ds.add_frame(np.full((64, 64), 30, np.uint16))
    assert np.all(ds.take_frame(2) == 10)  # level 2 also kept the first
    assert np.all(ds.take_frame(1) == 30)


# ---- device-resident batch API --------------------------------------------

BATCH_GEOMETRIES = {
    # name: (geometry, frames in the batch, expected batch path)
    "2d": (halving_geometry(1024, 512, 5), 7, 1),
    "2d_odd": (halving_geometry(1000, 333, 4), 7, 1),
    "2d_generic": (halving_geometry(1001, 333, 3), 5, 1),               # odd width
    "3d_odd_stack": ([(256, 128, 6), (128, 64, 3), (64, 32, 2)], 7, 0),  # per-frame
    "3d_fused": ([(256, 128, 8), (128, 64, 4), (64, 32, 2)], 8, 2),      # volume
    "3d_fused_deep": ([(512, 256, 16), (256, 128, 8), (128, 64, 4), (64, 32, 2)], 16, 2),
    "3d_fused_edge": ([(200, 61, 8), (100, 31, 4), (50, 16, 2)], 8, 2),  # odd rows
    # narrow tiles (half the columns per lane): u8 512 wide (a wide wave
    # would span 1024 px), 520 wide (only the narrow tile divides u8 rows)
    "2d_narrow": (halving_geometry(512, 512, 3), 9, 1),
    "2d_narrow_odd": (halving_geometry(520, 301, 3), 5, 1),
    # six levels: a second fused run from a 63 x 38 level
    "2d_six": (halving_geometry(1000, 600, 6), 3, 1),
    # odd widths at every level, frames at odd byte offsets in the batch
    "2d_oddw_deep": (halving_geometry(1031, 517, 5), 3, 1),
    "3d_fused_oddw": ([(201, 61, 8), (101, 31, 4), (51, 16, 2)], 8, 2),
    # Decimate takes 4 row units per wave when H % 2^NL == 0 and the row
    # units divide by 4: with column edges, and with one fused level (NL = 1)
    "3d_fused_oddw_even_h": ([(201, 64, 8), (101, 32, 4), (51, 16, 2)], 8, 2),
    "3d_fused_one_level": ([(256, 64, 4), (128, 32, 2)], 4, 2),
    # 128 plane groups and more: Decimate takes the plane groups fastest in
    # the unit order (round 5); column edges in the second
    "3d_fused_many_groups": ([(64, 32, 8), (32, 16, 4), (16, 8, 2)], 512, 2),
    "3d_fused_many_groups_edge": ([(72, 40, 8), (36, 20, 4), (18, 10, 2)], 520, 2),
    # level rows that split 64-B bursts: band-staged stores when a row band
    # is <= 4 tiles (1500 px u16), direct stores from band-aligned
    # workgroups for wider bands (2600 px u16 / f32, i64)
    "2d_wide_misaligned": (halving_geometry(2600, 70, 4), 3, 1),
    "2d_band_staged": (halving_geometry(1500, 90, 4), 3, 1),
    # aligned row bands of 5-8 tiles: every level staged by 8-wave (u16, f32
    # with 85 KiB of LDS) or 6-wave workgroups; u8 / i64 keep direct stores
    "2d_band8_aligned": (halving_geometry(4096, 48, 4), 3, 1),
    "2d_band6_edge_rows": (halving_geometry(3072, 37, 4), 3, 1),
    # aligned bands wider than 8 tiles: 8-tile segments (u8 9 tiles, u16 /
    # f32 17, i64 34), a last segment of one or two tiles, odd band rows
    "2d_band_segments": (halving_geometry(8704, 40, 4), 2, 1),
    # misaligned bands of up to 8 tiles in band-aligned workgroups (round
    # 3): 8 tiles (u16 / f32) with an odd band at the bottom; a last tile of
    # 10 px, so deep levels hold bursts shared by three waves
    "2d_complete_8tile": (halving_geometry(3900, 37, 4), 2, 1),
    "2d_complete_short_last": (halving_geometry(2570, 50, 4), 3, 1),
    # misaligned bands of more than 8 tiles (u16 / f32: 10): balanced 4-tile
    # segments, every level row its own LDS piece, stored by the segment's
    # last wave; odd band at the bottom
    "2d_mis_segments": (halving_geometry(4700, 41, 4), 2, 1),
}


@pytest.mark.parametrize("dtype", [np.uint8, np.uint16, np.float32, np.int64],
                         ids=lambda d: np.dtype(d).name)
@pytest.mark.parametrize("method", [0, 1, 2, 3])
@pytest.mark.parametrize("geo_kind", sorted(BATCH_GEOMETRIES))
def test_device_batch_matches_stream(aqz, oracle, dtype, method, geo_kind):
    torch = torch_cuda()
    rng = np.random.default_rng(seed_of(geo_kind, np.dtype(dtype).name, method))
    geo, n, kind = BATCH_GEOMETRIES[geo_kind]
    w, h, _ = geo[0]
    frames = random_frames(rng, dtype, (n, h, w))
    bpp = np.dtype(dtype).itemsize
    d_in = to_device(frames)
    # oracle stream: every emitted frame per level in order
    ref = oracle.OracleDownsampler(geo, dtype, method)
    expected = {L: [] for L in range(1, len(geo))}
    for f in frames:
        ref.add_frame(f)
        for L in expected:
            r = ref.take_frame(L)
            if r is not None:
                expected[L].append(r)
    outs = [None] + [empty_device(n * gw * gh * bpp) for gw, gh, _ in geo[1:]]
    ds = aqz.Downsampler(geo, dtype, method)
    counts = ds.run_device_batch(d_in.data_ptr(), n,
                                 [0] + [o.data_ptr() for o in outs[1:]],
                                 launch_stream())
    torch.cuda.synchronize()
    # the fused kernels take frames of any width and byte offset, so every
    # 2-D batch is one fused path (kind 1), pure 2x2x2 stacks the volume
    # kernel (kind 2), anything else the per-frame state machine (kind 0)
    assert ds.last_batch_kind() == kind
    for L in expected:
        gw, gh, _ = geo[L]
        assert counts[L] == len(expected[L])
        got = from_device(outs[L], dtype, (n, gh, gw))
        for k, e in enumerate(expected[L]):
            assert_parity(got[k], e, f"batch {geo_kind} L{L} frame {k}")


# ---- headline geometry: full size -----------------------------------------

def test_headline_4096_u16_parity(aqz, oracle):
    """4096^2 uint16, 5 levels, Mean (BASELINE configs[2]): device batch of 4
    frames bit-exact against the oracle."""
    torch = torch_cuda()
    rng = np.random.default_rng(2024)
    geo = halving_geometry(4096, 4096, 5)
    n = 4
    frames = rng.integers(0, 65536, (n, 4096, 4096), dtype=np.uint16)
    d_in = to_device(frames)
    outs = [None] + [empty_device(n * w * h * 2) for w, h, _ in geo[1:]]
    ds = aqz.Downsampler(geo, np.uint16, 1)
    ds.run_device_batch(d_in.data_ptr(), n, [0] + [o.data_ptr() for o in outs[1:]],
                        launch_stream())
    torch.cuda.synchronize()
    for k in range(n):
        ref = oracle.cascade_2d(frames[k], 5, 1)
        for L in range(1, 5):
            w, h, _ = geo[L]
            got = from_device(outs[L], np.uint16, (n, h, w))[k]
            assert_parity(got, ref[L - 1], f"4096 frame {k} L{L}")


def test_full_size_properties(aqz):
    """At the bench size (64 frames of 4096^2 u16) check size-independent
    properties instead of a full oracle run: Decimate level L is exactly the
    stride-2^L subsample of the base; Min <= Mean <= Max elementwise at every
    level (truncating means stay inside the block's range through the
    cascade)."""
    torch = torch_cuda()
    geo = halving_geometry(4096, 4096, 5)
    n = 64
    g = torch.Generator(device="cuda").manual_seed(7)
    d_in = torch.randint(0, 256, (n * 4096 * 4096 * 2,), dtype=torch.uint8,
                         device="cuda", generator=g)
    s = launch_stream()
    res = {}
    for m in METHODS:
        outs = [None] + [empty_device(n * w * h * 2) for w, h, _ in geo[1:]]
        ds = aqz.Downsampler(geo, np.uint16, m)
        ds.run_device_batch(d_in.data_ptr(), n, [0] + [o.data_ptr() for o in outs[1:]], s)
        res[m] = outs
    torch.cuda.synchronize()
    base = d_in.view(torch.int16).view(n, 4096, 4096)
    for L in range(1, 5):
        w, h, _ = geo[L]
        dec = res[0][L].view(torch.int16).view(n, h, w)
        assert torch.equal(dec, base[:, ::2 ** L, ::2 ** L])
        lo = res[2][L].view(torch.int16).view(n, h, w).to(torch.int32) & 0xFFFF
        mid = res[1][L].view(torch.int16).view(n, h, w).to(torch.int32) & 0xFFFF
        hi = res[3][L].view(torch.int16).view(n, h, w).to(torch.int32) & 0xFFFF
        assert bool((lo <= mid).all()) and bool((mid <= hi).all())


@pytest.mark.parametrize("staged", ["0", "1"])
def test_host_staging_modes(aqz, oracle, monkeypatch, staged):
    """add_frame uploads straight from the caller's pageable frame by default;
    $AQZ_PINNED_STAGING=1 stages through pinned memory instead.  Both must
    give the oracle's frames, including when the caller overwrites its buffer
    right after add_frame returns and when levels are left untaken."""
    monkeypatch.setenv("AQZ_PINNED_STAGING", staged)
    rng = np.random.default_rng(77)
    geo = [(96, 64, 6), (48, 32, 3), (24, 16, 2)]
    ds = aqz.Downsampler(geo, np.uint16, 1)
    ref = oracle.OracleDownsampler(geo, np.uint16, 1)
    buf = np.empty((64, 96), np.uint16)
    for i in range(12):
        buf[:] = rng.integers(0, 65536, (64, 96), dtype=np.uint16)
        ds.add_frame(buf)
        ref.add_frame(buf.copy())
        buf[:] = 0  # the caller reuses its frame immediately
        levels = [1, 2] if i % 3 else [1]  # leave level 2 untaken sometimes
        for L in levels:
            a, b = ds.take_frame(L), ref.take_frame(L)
            assert (a is None) == (b is None)
            if a is not None:
                assert_parity(a, b, f"staged={staged} frame {i} L{L}")


def test_reference_example_stream(aqz, oracle):
    """BASELINE configs[0] as the reference ships it:
    examples/stream-raw-multiscale-to-filesystem.c — 5-D t10 c8 z6/2 y48/16
    x64/16 uint16, `downsampling_method` left zero-initialised (Decimate,
    zarr.types.h:92), 10 frames of `i*1000 + j` (wrapping uint16).  Levels
    z/y/x 6/48/64 -> 3/24/32 -> 2/12/16.  The GPU path
    must reproduce the oracle frame for frame, readiness included."""
    dims = [(aqz.TIME, 10, 5, 2), (aqz.CHANNEL, 8, 4, 2), (aqz.SPACE, 6, 2, 1),
            (aqz.SPACE, 48, 16, 1), (aqz.SPACE, 64, 16, 2)]
    levels = aqz.plan_levels(dims)
    geo = aqz.level_geometry(levels)
    assert geo == [(64, 48, 6), (32, 24, 3), (16, 12, 2)]
    assert levels == oracle.plan_levels(dims)
    for method in METHODS:  # the example's Decimate first, then the others
        ds = aqz.Downsampler(geo, np.uint16, method)
        ref = oracle.OracleDownsampler(geo, np.uint16, method)
        j = np.arange(48 * 64, dtype=np.uint32)
        for i in range(10):
            frame = ((i * 1000 + j) & 0xFFFF).astype(np.uint16).reshape(48, 64)
            ds.add_frame(frame)
            ref.add_frame(frame)
            for L in (1, 2):
                a, b = ds.take_frame(L), ref.take_frame(L)
                assert (a is None) == (b is None), f"m{method} frame {i} L{L}"
                if a is not None:
                    assert_parity(a, b, f"example m{method} frame {i} L{L}")
        assert ds.take_frame(1) is None and ref.take_frame(1) is None


@pytest.mark.parametrize("geo_kind", ["2d", "3d_odd_stack", "3d_fused", "2d_generic",
                                      "2d_six", "2d_narrow_odd"])
@pytest.mark.parametrize("pinned", [False, True])
def test_host_batch_pipeline(aqz, oracle, geo_kind, pinned):
    """aqz_ds_run_host_batch: double-buffered groups over three streams must
    equal add_frame + take_frame on every frame (oracle stream), with group
    boundaries landing mid-stack and a ragged last group."""
    torch = torch_cuda()
    geo, _, _ = BATCH_GEOMETRIES[geo_kind]
    w, h, _ = geo[0]
    n = 37 if geo_kind != "3d_fused" else 40
    rng = np.random.default_rng(seed_of("host_batch", geo_kind))
    frames = random_frames(rng, np.uint16, (n, h, w))
    ref = oracle.OracleDownsampler(geo, np.uint16, 1)
    expected = {L: [] for L in range(1, len(geo))}
    for f in frames:
        ref.add_frame(f)
        for L in expected:
            r = ref.take_frame(L)
            if r is not None:
                expected[L].append(r)
    if pinned:
        src = torch.from_numpy(frames.view(np.uint8).reshape(-1).copy()).pin_memory()
        outs = [None] + [torch.empty(n * gw * gh * 2, dtype=torch.uint8).pin_memory()
                         for gw, gh, _ in geo[1:]]
        src_ptr = src.data_ptr()
        out_ptrs = [0] + [o.data_ptr() for o in outs[1:]]
        views = [None] + [o.numpy() for o in outs[1:]]
    else:
        src_ptr = frames.ctypes.data
        views = [None] + [np.empty(n * gw * gh * 2, np.uint8) for gw, gh, _ in geo[1:]]
        out_ptrs = [0] + [v.ctypes.data for v in views[1:]]
    ds = aqz.Downsampler(geo, np.uint16, 1)
    counts = ds.run_host_batch(src_ptr, n, out_ptrs)
    for L in expected:
        gw, gh, _ = geo[L]
        assert counts[L] == len(expected[L])
        got = views[L].view(np.uint16).reshape(n, gh, gw)
        for k, e in enumerate(expected[L]):
            assert_parity(got[k], e, f"host batch {geo_kind} L{L} frame {k}")


FULL_CONFIGS = {
    # BASELINE.json configs at full size: (geometry, dtype, frames)
    "c1_512_u8": (halving_geometry(512, 512, 3), np.uint8, 4),
    "c2_2048_u16": (halving_geometry(2048, 2048, 4), np.uint16, 4),
    "c3_4096_f32": (halving_geometry(4096, 4096, 5), np.float32, 2),
    "c4_volume_1024x256_u16": ([(1024, 1024, 256), (512, 512, 128), (256, 256, 64)],
                               np.uint16, 256),
}


@pytest.mark.parametrize("name", sorted(FULL_CONFIGS))
@pytest.mark.parametrize("method", METHODS)
def test_full_size_configs_vs_oracle(aqz, oracle, name, method):
    """Every BASELINE config at its full size through the device batch path
    (the benchmarked kernels), checked frame by frame against the oracle;
    the volume is one whole 1024x1024x256 stack."""
    torch = torch_cuda()
    geo, dtype, n = FULL_CONFIGS[name]
    w, h, _ = geo[0]
    rng = np.random.default_rng(seed_of("full", name, method))
    if np.dtype(dtype).kind == "f":
        frames = rng.uniform(-1e3, 1e3, (n, h, w)).astype(dtype)
    else:
        frames = rng.integers(0, np.iinfo(dtype).max, (n, h, w), dtype=dtype,
                              endpoint=True)
    bpp = np.dtype(dtype).itemsize
    d_in = to_device(frames)
    outs = [None] + [empty_device(n * gw * gh * bpp) for gw, gh, _ in geo[1:]]
    ds = aqz.Downsampler(geo, dtype, method)
    counts = ds.run_device_batch(d_in.data_ptr(), n, [0] + [o.data_ptr() for o in outs[1:]],
                                 launch_stream())
    torch.cuda.synchronize()
    assert ds.last_batch_kind() in (1, 2)
    ref = oracle.OracleDownsampler(geo, dtype, method)
    got = {L: from_device(outs[L], dtype, (n, geo[L][1], geo[L][0]))
           for L in range(1, len(geo))}
    k = {L: 0 for L in got}
    for i in range(n):
        ref.add_frame(frames[i])
        for L in got:
            r = ref.take_frame(L)
            if r is not None:
                assert_parity(got[L][k[L]], r, f"{name} m{method} L{L} #{k[L]}")
                k[L] += 1
    assert [k[L] for L in got] == [counts[L] for L in got]


TILE_CASES = [
    # (level-0 w, h, levels, dtype, tile_rows, tile_cols)
    (64, 48, 3, np.uint16, 16, 16),      # reference array tests' 16x16 chunks
    (1000, 600, 4, np.float32, 64, 128),  # ragged tiles at every level
    (300, 7, 2, np.uint8, 4, 128),
    (4096, 4096, 5, np.uint16, 256, 256),  # headline chunking
    (257, 129, 3, np.int64, 32, 32),
]


@pytest.mark.parametrize("eager", ["on_demand", "eager", "eager_tile_pass"])
@pytest.mark.parametrize("case", TILE_CASES, ids=lambda c: f"{c[0]}x{c[1]}_{np.dtype(c[3]).name}")
def test_take_frame_tiled(aqz, oracle, case, eager, monkeypatch):
    """Chunk-tiled take (§8(f) row 2) equals the oracle's restatement of
    write_frame_to_chunks_ + write_tile_rows, zero scan included; some tiles
    are forced all-zero.  `eager`: levels tiled in the cascade launch itself
    (one pass), or by a tile pass behind it ($AQZ_STREAM_TILE_PASS=1)."""
    w, h, nl, dt, tr, tc = case
    geo = halving_geometry(w, h, nl)
    rng = np.random.default_rng(seed_of("tiled", w, h))
    frame = random_frames(rng, dt, (h, w), specials=False)
    frame[: h // 2, : w // 2] = 0  # zero tiles at every level
    monkeypatch.setenv("AQZ_STREAM_TILE_PASS", "1" if eager == "eager_tile_pass" else "0")
    ds = aqz.Downsampler(geo, dt, 1)
    if eager != "on_demand":  # tiles computed behind the pyramid (aqz_ds_set_level_tiling)
        for L in range(1, nl):
            ds.set_level_tiling(L, tr, tc)
    ref = oracle.OracleDownsampler(geo, dt, 1)
    ds.add_frame(frame)
    ref.add_frame(frame)
    for L in range(1, nl):
        got = ds.take_frame_tiled(L, tr, tc)
        want_frame = ref.take_frame(L)
        tiles, nz = oracle.tile_frame(want_frame, tr, tc)
        assert got is not None
        assert_parity(got[0], tiles, f"tiles L{L}")
        assert np.array_equal(got[1], nz), f"zero scan L{L}"
        assert ds.take_frame(L) is None  # the tiled take consumed the frame
    if eager == "eager":
        # every case here is one run of pure-XY levels: one tiled launch
        assert ds.stream_tiled_runs() == 1
    else:
        assert ds.stream_tiled_runs() == 0


def test_tile_frame_device_full_resolution(aqz, oracle):
    """aqz_tile_frame_device on a full-resolution 4096^2 u16 frame with the
    headline's 256x256 chunks (the tiling the reference does with OpenMP on the
    host, array.cpp:575)."""
    torch = torch_cuda()
    rng = np.random.default_rng(11)
    frame = rng.integers(0, 65536, (4096, 4096), dtype=np.uint16)
    frame[:256, :512] = 0
    d_in = to_device(frame)
    nt = 16 * 16
    d_tiles = empty_device(nt * 256 * 256 * 2)
    d_nz = torch.zeros(nt, dtype=torch.int32, device="cuda")
    s = launch_stream()
    aqz.tile_frame_device(np.uint16, d_in.data_ptr(), 4096, 4096, 256, 256,
                          d_tiles.data_ptr(), d_nz.data_ptr(), s)
    torch.cuda.synchronize()
    tiles, nz = oracle.tile_frame(frame, 256, 256)
    assert_parity(from_device(d_tiles, np.uint16, (nt, 256, 256)), tiles, "L0 tiles")
    assert np.array_equal(d_nz.cpu().numpy() != 0, nz)
    assert not nz[0] and not nz[1] and nz[2:].all()
    # the sliced-flag form (one launch, no pre-clear)
    sl = aqz.tile_slices(256, 256)
    d_sl = torch.full((nt * sl,), 7, dtype=torch.uint8, device="cuda")
    d_tiles.zero_()
    aqz.tile_frame_device_sliced(np.uint16, d_in.data_ptr(), 4096, 4096, 256, 256,
                                 d_tiles.data_ptr(), d_sl.data_ptr(), s)
    torch.cuda.synchronize()
    assert_parity(from_device(d_tiles, np.uint16, (nt, 256, 256)), tiles, "L0 tiles sliced")
    flags = d_sl.cpu().numpy().reshape(nt, sl)
    assert set(np.unique(flags)) <= {0, 1}
    assert np.array_equal(flags.any(axis=1), nz)


@pytest.mark.parametrize("dtype", [np.uint8, np.uint16, np.float32, np.float64],
                         ids=lambda d: np.dtype(d).name)
@pytest.mark.parametrize("method", METHODS)
def test_degenerate_frames(aqz, oracle, dtype, method):
    """Edge geometries: 1-pixel-wide and 1-pixel-tall frames (the right or
    bottom neighbour is always the replicated edge), 1x1 levels, 2x2 -> 1x1."""
    rng = np.random.default_rng(seed_of("degenerate", np.dtype(dtype).name, method))
    for geo in ([(1, 100, 1), (1, 50, 1), (1, 25, 1)],
                [(100, 1, 1), (50, 1, 1), (25, 1, 1)],
                [(2, 2, 1), (1, 1, 1)],
                [(3, 3, 1), (2, 2, 1), (1, 1, 1)],
                [(1, 1, 4), (1, 1, 2)]):
        w, h, z = geo[0]
        frames = [random_frames(rng, dtype, (h, w)) for _ in range(max(2, z))]
        got, want = run_both(aqz, oracle, geo, dtype, method, frames)
        assert len(got) == len(want)
        for (i, L, a), (_, _, b) in zip(got, want):
            assert_parity(a, b, f"{geo} f{i} L{L}")


def test_single_level_and_errors(aqz):
    """A one-level handle (no pyramid) emits nothing; wrong frame sizes and
    levels are rejected the way the reference's EXPECTs reject them."""
    ds = aqz.Downsampler([(64, 64, 1)], np.uint16, 1)
    ds.add_frame(np.zeros((64, 64), np.uint16))
    assert ds.take_frame(1) is None and ds.take_frame(0) is None
    ds = aqz.Downsampler(halving_geometry(64, 64, 3), np.uint16, 1)
    with pytest.raises(aqz.AqzError) as e:
        ds.add_frame(np.zeros((64, 63), np.uint16))
    assert e.value.status == 1
    with pytest.raises(TypeError):
        ds.add_frame(np.zeros((64, 64), np.uint8))
    assert ds.take_frame(7) is None and ds.take_frame(-1) is None
    ds.add_frame(np.ones((64, 64), np.uint16))
    assert np.all(ds.take_frame(2) == 1)


def test_max_size_frame_two_fused_runs(aqz, oracle):
    """16384^2 u16 with 64-px chunks: the planner gives 9 levels, i.e. one
    4-level cascade launch chained into a second 4-level launch from level 4
    (512 MiB frame), bit-exact against the oracle."""
    torch = torch_cuda()
    dims = [(aqz.TIME, 0, 1, 1), (aqz.SPACE, 16384, 64, 1), (aqz.SPACE, 16384, 64, 1)]
    geo = aqz.level_geometry(aqz.plan_levels(dims))
    assert len(geo) == 9 and geo[-1][:2] == (64, 64)
    rng = np.random.default_rng(16384)
    frame = rng.integers(0, 65536, (16384, 16384), dtype=np.uint16)
    d_in = to_device(frame)
    outs = [None] + [empty_device(w * h * 2) for w, h, _ in geo[1:]]
    ds = aqz.Downsampler(geo, np.uint16, 1)
    ds.run_device_batch(d_in.data_ptr(), 1, [0] + [o.data_ptr() for o in outs[1:]],
                        launch_stream())
    torch.cuda.synchronize()
    assert ds.last_batch_kind() == 1
    ref = oracle.cascade_2d(frame, 9, 1)
    for L in range(1, 9):
        w, h, _ = geo[L]
        assert_parity(from_device(outs[L], np.uint16, (h, w)), ref[L - 1], f"L{L}")


@pytest.mark.parametrize("tile_pass", ["0", "1"], ids=["one_pass", "tile_pass"])
def test_eager_tiling_follows_the_cached_frame(aqz, oracle, tile_pass, monkeypatch):
    """With eager tiling on, the tiles always belong to the cached frame: an
    untaken frame keeps its tiles while newer frames are dropped, a plain
    take_frame consumes the frame, and a different tile shape falls back to
    on-demand tiling."""
    monkeypatch.setenv("AQZ_STREAM_TILE_PASS", tile_pass)
    geo = halving_geometry(128, 96, 3)
    ds = aqz.Downsampler(geo, np.uint16, 1)
    ds.set_level_tiling(1, 16, 32)
    ds.set_level_tiling(2, 16, 16)
    rng = np.random.default_rng(8)
    f0, f1, f2 = (rng.integers(0, 65536, (96, 128), dtype=np.uint16) for _ in range(3))
    ds.add_frame(f0)
    ds.add_frame(f1)  # dropped at both levels: f0 still cached
    want1 = oracle.cascade_2d(f0, 3, 1)
    got = ds.take_frame_tiled(1, 16, 32)
    assert_parity(got[0], oracle.tile_frame(want1[0], 16, 32)[0], "L1 keeps f0")
    ds.add_frame(f2)  # level 1 now caches f2; level 2 still holds f0
    want2 = oracle.cascade_2d(f2, 3, 1)
    got = ds.take_frame_tiled(1, 8, 8)  # other shape: on-demand path
    assert_parity(got[0], oracle.tile_frame(want2[0], 8, 8)[0], "L1 f2 on demand")
    assert np.array_equal(ds.take_frame(2), want1[1])  # plain take of f0
    assert ds.take_frame_tiled(2, 16, 16) is None
    assert ds.stream_tiled_runs() == (3 if tile_pass == "0" else 0)
    ds.set_level_tiling(1, 0, 0)


# ---- §8(f) row 1: aqz_ds_add_frame_async -----------------------------------

@pytest.mark.parametrize("geo_kind", ["2d", "3d"])
def test_add_frame_async_matches_oracle(aqz, oracle, geo_kind):
    """add_frame_async + take_frame equals the oracle frame by frame, with
    the pending add settled by wait() on even frames and implicitly by the
    next take/add on odd ones."""
    if geo_kind == "2d":
        geo = halving_geometry(1000, 601, 4)
        shape, n = (601, 1000), 6
    else:
        geo = [(256, 128, 9), (128, 64, 5), (64, 32, 3), (32, 16, 2)]
        shape, n = (128, 256), 9
    ds = aqz.Downsampler(geo, np.uint16, 1)
    ref = oracle.OracleDownsampler(geo, np.uint16, 1)
    rng = np.random.default_rng(seed_of("async", geo_kind))
    for i in range(n):
        f = rng.integers(0, 65536, shape, dtype=np.uint16)
        ds.add_frame_async(f)
        if i % 2 == 0:
            ds.wait()
        ref.add_frame(f)
        for L in range(1, len(geo)):
            a, b = ds.take_frame(L), ref.take_frame(L)
            assert (a is None) == (b is None), f"frame {i} L{L} readiness"
            if a is not None:
                assert_parity(a, b, f"async frame {i} L{L}")
    # back-to-back asyncs: the second waits for the first
    f1 = rng.integers(0, 65536, shape, dtype=np.uint16)
    f2 = rng.integers(0, 65536, shape, dtype=np.uint16)
    ds.add_frame_async(f1)
    ds.add_frame_async(f2)
    ds.wait()
    ref.add_frame(f1)
    ref.add_frame(f2)
    for L in range(1, len(geo)):
        a, b = ds.take_frame(L), ref.take_frame(L)
        assert (a is None) == (b is None)
        if a is not None:
            assert_parity(a, b, f"back-to-back L{L}")
    ds.close()


@pytest.mark.parametrize("shape,tile", [((601, 1000), (64, 128)), ((4096, 4096), (256, 256)),
                                        ((3000, 3000), (256, 256))],
                         ids=["1000x601", "4096x4096", "3000x3000"])
def test_add_frame_async_tiled_takes(aqz, oracle, shape, tile):
    """The drop-in's streaming path as the patched MultiscaleArray::write_frame
    runs it: every level tiled behind the pyramid (one tiled-cascade launch),
    add_frame_async, then take_frame_tiled of every level — tiles and zero
    scan equal to the oracle's, frame by frame, with untaken frames kept."""
    H, W = shape
    dims = [(aqz.TIME, 0, 1, 1), (aqz.SPACE, H, tile[0], 1), (aqz.SPACE, W, tile[1], 1)]
    geo = aqz.level_geometry(aqz.plan_levels(dims))
    assert len(geo) >= 3
    ds = aqz.Downsampler(geo, np.uint16, 1)
    for L in range(1, len(geo)):
        ds.set_level_tiling(L, *tile)
    ref = oracle.OracleDownsampler(geo, np.uint16, 1)
    rng = np.random.default_rng(seed_of("async_tiled", H, W))
    for i in range(3):
        f = rng.integers(0, 65536, shape, dtype=np.uint16)
        f[: H // 3, : W // 3] = 0  # zero tiles at every level
        ds.add_frame_async(f)
        ref.add_frame(f)
        ds.wait()
        for L in range(1, len(geo)):
            if i == 1 and L == 2:
                continue  # left untaken: frame 2 must not replace it
            got = ds.take_frame_tiled(L, *tile)
            want = ref.take_frame(L)
            t, nz = oracle.tile_frame(want, *tile)
            assert_parity(got[0], t, f"frame {i} L{L} tiles")
            assert np.array_equal(got[1], nz), f"frame {i} L{L} zero scan"
    assert ds.stream_tiled_runs() == 3 * -(-(len(geo) - 1) // 4)
    ds.close()


@pytest.mark.parametrize("geo_kind", ["2d_tiled", "2d_plain", "3d_plain", "3d_tiled"])
def test_add_frame_async_take(aqz, oracle, geo_kind):
    """aqz_ds_add_frame_async_take: every level taken in the background job
    right behind the add, equal to add_frame + take_frame(_tiled) of the
    oracle frame by frame, readiness included.  Frame 1's level 2 is kept by
    the caller unconsumed across frame 2, whose add holds level 2
    (AQZ_TAKE_HOLD): frame 2's level-2 frame must be dropped, as the
    reference's emplace drops a frame while one is cached."""
    if geo_kind.startswith("2d"):
        geo = halving_geometry(1000, 601, 4)
        shape = (601, 1000)
    else:
        geo = [(256, 128, 9), (128, 64, 5), (64, 32, 3), (32, 16, 2)]
        shape = (128, 256)
    tiled = geo_kind.endswith("tiled")
    tile = (16, 32)
    tiles = [None] + [tile] * (len(geo) - 1) if tiled else None
    ds = aqz.Downsampler(geo, np.uint16, 1)
    if tiled:
        for L in range(1, len(geo)):
            ds.set_level_tiling(L, *tile)
    ref = oracle.OracleDownsampler(geo, np.uint16, 1)
    rng = np.random.default_rng(seed_of("async_take", geo_kind))

    def check(got, want, ctx):
        assert (got is None) == (want is None), ctx
        if want is None:
            return
        if tiled:
            t, nz = oracle.tile_frame(want, *tile)
            assert_parity(got[0], t, ctx)
            assert np.array_equal(got[1], nz), ctx
        else:
            assert_parity(got, want, ctx)

    kept = None
    for i in range(7):
        f = rng.integers(0, 65536, shape, dtype=np.uint16)
        f[: shape[0] // 3, : shape[1] // 3] = 0
        hold = (2,) if (i == 2 and kept is not None) else ()
        ds.add_frame_async_take(f, tiles, hold)
        ref.add_frame(f)
        res = ds.wait_takes()
        for L in range(1, len(geo)):
            if L in hold:
                assert res[L] is None
                continue
            if i == 1 and L == 2 and res[L] is not None:
                kept = res[L]  # the caller keeps it unconsumed for a frame
                continue
            check(res[L], ref.take_frame(L), f"frame {i} L{L}")
        if i == 2 and kept is not None:
            check(kept, ref.take_frame(2), "held level-2 frame")
    ds.close()


def test_add_frame_async_temporaries(aqz, oracle):
    """Frames passed as temporaries: the binding must keep each one alive
    until the next call has settled its upload.  Each temporary
    is dropped right after the call and new arrays of the same size are
    allocated and scribbled over, so a freed buffer would be reused."""
    geo = halving_geometry(2048, 1024, 4)
    ds = aqz.Downsampler(geo, np.uint16, 1)
    ref = oracle.OracleDownsampler(geo, np.uint16, 1)
    rng = np.random.default_rng(seed_of("async-temp"))
    base = rng.integers(0, 65536, (6, 1024, 2048), dtype=np.uint16)
    for i in range(6):
        ds.add_frame_async(np.ascontiguousarray(base[i][:, ::1].copy()))
        junk = [np.full((1024, 2048), 0xA5A5, np.uint16) for _ in range(3)]
        del junk
        ref.add_frame(base[i])
        if i % 3 == 2:  # two back-to-back temporaries, then takes
            continue
        for L in range(1, len(geo)):
            a, b = ds.take_frame(L), ref.take_frame(L)
            assert (a is None) == (b is None), f"frame {i} L{L} readiness"
            if a is not None:
                assert_parity(a, b, f"temporary frame {i} L{L}")
    ds.wait()
    ds.close()


def test_stream_batch_stream_interleave(aqz, oracle):
    """add_frame, then run_device_batch on a caller stream, then add_frame
    again on a Z-halving pyramid: the batch's per-frame fallback consumes the
    earlier plane the first add_frame stored on the handle's stream, and the
    later add_frame consumes the plane the batch stored (the two
    streams are joined both ways)."""
    torch = torch_cuda()
    geo = [(2048, 1024, 8), (1024, 512, 4), (512, 256, 2)]
    rng = np.random.default_rng(seed_of("interleave"))
    frames = rng.integers(0, 65536, (8, 1024, 2048), dtype=np.uint16)
    ds = aqz.Downsampler(geo, np.uint16, 1)
    ref = oracle.OracleDownsampler(geo, np.uint16, 1)

    def stream_one(i):
        ds.add_frame(frames[i])
        ref.add_frame(frames[i])
        for L in range(1, len(geo)):
            a, b = ds.take_frame(L), ref.take_frame(L)
            assert (a is None) == (b is None), f"frame {i} L{L} readiness"
            if a is not None:
                assert_parity(a, b, f"streamed frame {i} L{L}")

    stream_one(0)  # stores the earlier plane of level 1
    nb = 4  # frames 1..4: frame 4 is stored as the next earlier plane
    d_in = to_device(frames[1:1 + nb])
    outs = [None] + [empty_device(nb * w * h * 2) for w, h, _ in geo[1:]]
    counts = ds.run_device_batch(d_in.data_ptr(), nb, [0] + [o.data_ptr() for o in outs[1:]],
                                 launch_stream())
    assert ds.last_batch_kind() == 0  # a stored plane forces the per-frame path
    want = {L: [] for L in range(1, len(geo))}
    for i in range(1, 1 + nb):
        ref.add_frame(frames[i])
        for L in want:
            r = ref.take_frame(L)
            if r is not None:
                want[L].append(r)
    for L in want:
        w, h, _ = geo[L]
        assert counts[L] == len(want[L]), f"L{L} count"
        got = from_device(outs[L], np.uint16, (nb, h, w))
        for k, r in enumerate(want[L]):
            assert_parity(got[k], r, f"batch L{L} #{k}")
    torch.cuda.synchronize()
    for i in range(1 + nb, 8):  # frame 5 pairs with the plane the batch stored
        stream_one(i)
    ds.close()


def test_add_frame_async_errors(aqz):
    geo = halving_geometry(64, 64, 2)
    ds = aqz.Downsampler(geo, np.uint16, 1)
    with pytest.raises(aqz.AqzError):
        ds.add_frame_async(np.zeros((64, 63), np.uint16))  # size checked up front
    ds.wait()  # nothing pending: OK
    ds.add_frame_async(np.ones((64, 64), np.uint16))
    ds.close()  # destroy settles the pending add


def test_add_frame_async_take_checks_buffers_first(aqz, oracle):
    """every take buffer is checked before the background job is
    queued — a level-2 buffer too small fails the call with nothing queued,
    so level 1 is not taken (and lost) either; the same frame then goes
    through with proper buffers and matches the oracle."""
    import ctypes
    geo = halving_geometry(128, 96, 3)
    ds = aqz.Downsampler(geo, np.uint16, aqz.MEAN)
    frame = np.arange(128 * 96, dtype=np.uint16).reshape(96, 128)
    L = aqz.lib()
    takes = (aqz.LevelTake * 3)()
    b1 = np.empty((48, 64), np.uint16)
    b2 = np.empty(10, np.uint16)                     # level 2 needs 24 x 32
    takes[1] = aqz.LevelTake(aqz.TAKE_INTO, 0, 0, b1.ctypes.data, b1.nbytes, None, 0, 0)
    takes[2] = aqz.LevelTake(aqz.TAKE_INTO, 0, 0, b2.ctypes.data, b2.nbytes, None, 0, 0)
    rc = L.aqz_ds_add_frame_async_take(ds._h, frame.ctypes.data, frame.nbytes, takes)
    assert rc == 1 and b"take buffer" in L.aqz_ds_last_error(ds._h)
    assert L.aqz_ds_wait(ds._h) == 0                 # nothing was queued
    assert ds.take_frame(1) is None                  # and nothing was added
    ds.add_frame_async_take(frame, None)
    got = ds.wait_takes()
    ref = oracle.cascade_2d(frame, 3, aqz.MEAN)
    for lv in (1, 2):
        np.testing.assert_array_equal(got[lv], ref[lv - 1])
    ds.close()


# ---- §8(f) row 2: transposed storage order and level-0 take -----------------

TRANSPOSE_SHAPES = [(64, 64), (4096, 4096), (1000, 777), (129, 4100), (1, 5), (5, 1),
                    (512, 256), (3, 200), (192, 256), (96, 640), (384, 512)]


@pytest.mark.parametrize("dtype", DTYPES, ids=lambda d: np.dtype(d).name)
def test_transpose_frame_device(aqz, oracle, dtype):
    """aqz_transpose_frame_device equals the transpose_frame restatement
    (array.cpp:488-504) bit for bit, vector and element paths."""
    rng = np.random.default_rng(seed_of("transpose", np.dtype(dtype).name))
    for rows, cols in TRANSPOSE_SHAPES:
        if np.dtype(dtype).itemsize == 8 and rows * cols > 1 << 22:
            continue
        frame = random_frames(rng, dtype, (rows, cols), specials=False)
        d_src = to_device(frame)
        d_dst = empty_device(frame.nbytes)
        aqz.transpose_frame_device(dtype, d_src.data_ptr(), rows, cols, d_dst.data_ptr(),
                                   launch_stream())
        got = from_device(d_dst, dtype, (cols, rows))
        assert_parity(got, oracle.transpose_frame(frame), f"{rows}x{cols}")


@pytest.mark.parametrize("case", [
    # (storage w, h, levels, dtype, tile_rows, tile_cols)
    (30, 20, 2, np.int32, 15, 10),          # python test_write_transposed_array
    (1024, 768, 4, np.uint16, 256, 128),
    (600, 1000, 3, np.float32, 64, 64),
    (257, 129, 3, np.uint8, 32, 48),
], ids=lambda c: f"{c[0]}x{c[1]}_{np.dtype(c[3]).name}")
def test_input_transpose_pyramid_and_level0(aqz, oracle, case):
    """With input transposition the handle takes acquisition-order frames,
    transposes them on the GPU, and both the pyramid and the level-0 frame it
    hands back (raw and chunk-tiled) equal the reference flow: transpose_frame,
    then the downsampler and write_frame_to_chunks_ on the transposed frame."""
    w, h, nl, dt, tr, tc = case
    geo = halving_geometry(w, h, nl)
    ds = aqz.Downsampler(geo, dt, 1)
    ds.set_input_transpose(True)
    ref = oracle.OracleDownsampler(geo, dt, 1)
    rng = np.random.default_rng(seed_of("tin", w, h))
    for i in range(3):
        acq = random_frames(rng, dt, (w, h), specials=False)  # acquisition: w rows
        acq[: w // 3] = 0
        stored = oracle.transpose_frame(acq)                 # (h, w) storage order
        if i == 1:
            ds.add_frame_async(acq)
        else:
            ds.add_frame(acq)
        ref.add_frame(stored)
        if i == 0:
            assert_parity(ds.take_input_frame(), stored, "level 0 raw")
        else:
            tiles, nz = ds.take_input_frame(tr, tc)
            want_t, want_nz = oracle.tile_frame(stored, tr, tc)
            assert_parity(tiles, want_t, f"level 0 tiles #{i}")
            assert np.array_equal(nz, want_nz), f"level 0 zero scan #{i}"
        assert ds.take_input_frame() is None  # one-shot
        for L in range(1, nl):
            a, b = ds.take_frame(L), ref.take_frame(L)
            assert (a is None) == (b is None)
            if a is not None:
                assert_parity(a, b, f"transposed #{i} L{L}")
    ds.close()


def test_input_frame_take_and_batch_rules(aqz, oracle):
    """take_input_frame without transposition returns the frame as added;
    batches clear it, and are refused while transposition is on."""
    torch = torch_cuda()
    geo = halving_geometry(256, 128, 3)
    ds = aqz.Downsampler(geo, np.uint16, 1)
    rng = np.random.default_rng(5)
    f = rng.integers(0, 65536, (128, 256), dtype=np.uint16)
    assert ds.take_input_frame() is None
    ds.add_frame(f)
    assert np.array_equal(ds.take_input_frame(), f)
    d_f = to_device(f)
    ds.add_device_frame(d_f.data_ptr(), f.nbytes)
    tiles, nz = ds.take_input_frame(64, 64)
    assert_parity(tiles, oracle.tile_frame(f, 64, 64)[0], "device input tiles")
    ds.add_frame(f)
    bufs = [empty_device(ds.level_bytes(L) * 2) for L in (1, 2)]
    outs = [0] + [b.data_ptr() for b in bufs]
    ds.run_device_batch(d_f.data_ptr(), 1, outs)
    torch.cuda.synchronize()
    assert ds.take_input_frame() is None
    ds.set_input_transpose(True)
    with pytest.raises(aqz.AqzError):
        ds.run_device_batch(d_f.data_ptr(), 1, outs)
    with pytest.raises(aqz.AqzError):
        ds.take_input_frame(16, 0)
    ds.set_input_transpose(False)
    ds.close()


# ---- device placement ------------------------------------------------------

def test_spread_device_policy(aqz, oracle, monkeypatch):
    """$AQZ_GPU_DEVICE=spread: handles take the visible GPUs in turn (all 0
    on a one-GPU box) and each computes the right pyramid there."""
    torch = torch_cuda()
    n_dev = torch.cuda.device_count()
    monkeypatch.setenv("AQZ_GPU_DEVICE", "spread")
    geo = halving_geometry(96, 64, 3)
    rng = np.random.default_rng(seed_of("spread"))
    handles = [aqz.Downsampler(geo, np.uint16, aqz.MEAN) for _ in range(3)]
    devices = [h.device() for h in handles]
    assert all(0 <= d < n_dev for d in devices)
    if n_dev > 1:
        assert len(set(devices)) > 1
    for h in handles:
        frame = random_frames(rng, np.uint16, (64, 96))
        h.add_frame(frame)
        ref = oracle.cascade_2d(frame, len(geo), aqz.MEAN)
        for L in range(1, len(geo)):
            assert np.array_equal(h.take_frame(L), ref[L - 1])
        h.close()


def test_bad_device_ordinal_is_invalid_argument(aqz):
    n_dev = torch_cuda().cuda.device_count()
    with pytest.raises(aqz.AqzError) as e:
        aqz.Downsampler(halving_geometry(64, 64, 2), np.uint8, aqz.MEAN, device=n_dev + 7)
    assert e.value.status == 1  # AQZ_INVALID_ARGUMENT


# the oracle's NaN-rule KATs (tests/test_oracle_kats.py::test_mean_nan_payload_rule)
# through the GPU: one 2x2 frame -> mean4, two 1x1 planes -> mean2
_INF, _NINF, _ONE = 0x7F800000, 0xFF800000, 0x3F800000
_QA, _QB, _SA = 0x7FC01234, 0xFFC0ABCD, 0x7F800F00
NAN_KATS_4 = [
    ([_QA, _QB, _ONE, _ONE], _QA),
    ([_ONE, _QB, _QA, _ONE], _QB),
    ([_SA, _ONE, _ONE, _ONE], _SA | 0x00400000),
    ([_ONE, _SA, _QA, _ONE], _SA | 0x00400000),
    ([_INF, _NINF, _ONE, _ONE], 0xFFC00000),
    ([_INF, _NINF, _QA, _ONE], 0xFFC00000),
    ([_ONE, _INF, _ONE, _NINF], 0xFFC00000),
    ([_QB, _INF, _NINF, _ONE], _QB),
]
NAN_KATS_2 = [([_QA, _QB], _QA), ([_INF, _NINF], 0xFFC00000), ([_ONE, _SA], _SA | 0x00400000)]


@pytest.mark.parametrize("bits,want", NAN_KATS_4)
def test_mean4_nan_kats_gpu(aqz, bits, want):
    frame = np.array(bits, dtype=np.uint32).view(np.float32).reshape(2, 2)
    ds = aqz.Downsampler([(2, 2, 1), (1, 1, 1)], np.float32, aqz.MEAN)
    try:
        ds.add_frame(frame)
        got = ds.take_frame(1)
    finally:
        ds.close()
    assert int(got.view(np.uint32).reshape(-1)[0]) == want, hex(int(got.view(np.uint32)[0, 0]))


@pytest.mark.parametrize("bits,want", NAN_KATS_2)
def test_mean2_nan_kats_gpu(aqz, bits, want):
    planes = np.array(bits, dtype=np.uint32).view(np.float32).reshape(2, 1, 1)
    ds = aqz.Downsampler([(1, 1, 2), (1, 1, 1)], np.float32, aqz.MEAN)
    try:
        ds.add_frame(planes[0])
        assert ds.take_frame(1) is None      # the earlier plane waits for its pair
        ds.add_frame(planes[1])
        got = ds.take_frame(1)
    finally:
        ds.close()
    assert int(got.view(np.uint32).reshape(-1)[0]) == want, hex(int(got.view(np.uint32).reshape(-1)[0]))
