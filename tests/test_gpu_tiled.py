"""GPU parity of aqz_ds_run_device_batch_tiled: the pyramid kernel writes
every level straight into chunk-tile order (SURVEY §8(f) row 2,
array.cpp:507-622 + chunk.cpp:17-58).  Each level of each frame must equal
the oracle's scale_image cascade tiled by oracle_tile_frame — bytes and zero
scan — bit-exactly."""
import zlib

import numpy as np
import pytest

from gpu_util import (assert_parity, empty_device, from_device, launch_stream,
                      random_frames, to_device, torch_cuda)

pytestmark = pytest.mark.gpu

TILED_CASES = [
    # (w, h, levels, dtype, tile_rows, tile_cols, frames)
    (64, 48, 3, np.uint16, 16, 16, 3),       # the reference array tests' chunks
    (1000, 600, 4, np.float32, 64, 128, 2),  # ragged tiles at every level
    (300, 7, 2, np.uint8, 4, 128, 3),        # one short row band
    (4096, 4096, 5, np.uint16, 256, 256, 2),  # headline chunking
    (257, 129, 3, np.int64, 32, 32, 3),
    (5472, 3648, 5, np.uint16, 256, 256, 1),  # 20 MP sensor
    (3000, 3000, 5, np.uint16, 256, 256, 1),
    (1031, 517, 5, np.int16, 64, 64, 3),     # odd widths: frames at odd offsets
    (2100, 700, 7, np.uint8, 8, 16, 2),      # two fused runs, tiny tiles
    (4100, 600, 10, np.uint8, 8, 8, 2),      # three runs (chain ping-pong)
    (640, 480, 4, np.uint16, 100, 60, 2),    # tile widths not multiples of a lane's columns
    (512, 512, 4, np.float64, 3, 5, 2),      # blocks spanning several tiles
]


def _ids(c):
    return f"{c[0]}x{c[1]}_{np.dtype(c[3]).name}_{c[4]}x{c[5]}"


def halving(w, h, n):
    geo = [(w, h, 1)]
    for _ in range(1, n):
        w, h = (w + 1) // 2, (h + 1) // 2
        geo.append((w, h, 1))
    return geo


def run_tiled(aqz, geo, dtype, method, frames, tr, tc, with_flags=True):
    torch = torch_cuda()
    n = len(frames)
    bpp = np.dtype(dtype).itemsize
    d_in = to_device(np.stack(frames))
    tiles = [None] + [(tr, tc)] * (len(geo) - 1)
    ds = aqz.Downsampler(geo, dtype, method)
    outs, flags, shapes, slots = [None], [None], [None], [None]
    for L, (w, h, _) in enumerate(geo[1:], 1):
        nt = (-(-h // tr)) * (-(-w // tc))
        S = ds.tiled_flag_slots(L, tr, tc)
        assert S >= 1
        outs.append(empty_device(n * nt * tr * tc * bpp))
        flags.append(empty_device(n * nt * S) if with_flags else None)
        shapes.append(nt)
        slots.append(S)
    # poison the outputs: every byte (overhang and flag slots included) must
    # be written
    for o in outs[1:] + (flags[1:] if with_flags else []):
        o.fill_(0xA5)
    counts = ds.run_device_batch_tiled(
        d_in.data_ptr(), n, tiles, [0] + [o.data_ptr() for o in outs[1:]],
        [0] + [f.data_ptr() for f in flags[1:]] if with_flags else None, launch_stream())
    torch.cuda.synchronize()
    assert ds.last_batch_kind() == 4
    assert counts == [n] * len(geo)
    got = []
    for L in range(1, len(geo)):
        t = from_device(outs[L], dtype, (n, shapes[L], tr, tc))
        f = None
        if with_flags:
            raw = from_device(flags[L], np.uint8, (n, shapes[L], slots[L]))
            assert np.isin(raw, (0, 1)).all(), f"L{L}: flag slot left unwritten"
            f = raw.any(axis=-1)
        got.append((t, f))
    ds.close()
    return got, slots[1:]


@pytest.mark.parametrize("case", TILED_CASES, ids=_ids)
def test_tiled_batch_matches_oracle(aqz, oracle, case):
    w, h, nl, dt, tr, tc, n = case
    geo = halving(w, h, nl)
    rng = np.random.default_rng(w * 7919 + h)
    frames = [random_frames(rng, dt, (h, w), specials=False) for _ in range(n)]
    frames[0][: h // 2, : w // 2] = 0  # zero tiles at every level
    method = 1
    got, _ = run_tiled(aqz, geo, dt, method, frames, tr, tc)
    for k, fr in enumerate(frames):
        ref = oracle.cascade_2d(fr, nl, method)
        for L in range(1, nl):
            want_t, want_nz = oracle.tile_frame(ref[L - 1], tr, tc)
            t, f = got[L - 1]
            assert_parity(t[k], want_t, f"frame {k} L{L} tiles")
            assert np.array_equal(f[k], want_nz), f"frame {k} L{L} zero scan"


@pytest.mark.parametrize("dtype", [np.uint8, np.int16, np.uint32, np.int64, np.float32,
                                   np.float64], ids=lambda d: np.dtype(d).name)
@pytest.mark.parametrize("method", [0, 1, 2, 3])
def test_tiled_batch_dtypes_methods(aqz, oracle, dtype, method):
    """Every method over the signed/float edge cases (NaN, inf, -0.0:
    -0.0 is a nonzero byte for the scan), ragged tiles."""
    w, h, nl, tr, tc = 520, 301, 4, 64, 96
    geo = halving(w, h, nl)
    rng = np.random.default_rng(zlib.crc32(f"{np.dtype(dtype).name}/{method}".encode()))
    frames = [random_frames(rng, dtype, (h, w)) for _ in range(2)]
    frames[1][:] = 0
    if np.dtype(dtype).kind == "f":
        frames[1][-40:, -40:] = -0.0  # nonzero bytes, zero value
    got, _ = run_tiled(aqz, geo, dtype, method, frames, tr, tc)
    for k, fr in enumerate(frames):
        ref = oracle.cascade_2d(fr, nl, method)
        for L in range(1, nl):
            want_t, want_nz = oracle.tile_frame(ref[L - 1], tr, tc)
            t, f = got[L - 1]
            assert_parity(t[k], want_t, f"{np.dtype(dtype).name} m{method} f{k} L{L}")
            if np.dtype(dtype).kind == "f":  # bit-exact, NaN payloads included
                ib = np.uint32 if dtype == np.float32 else np.uint64
                assert np.array_equal(t[k].view(ib), want_t.view(ib))
            assert np.array_equal(f[k], want_nz), f"f{k} L{L} zero scan"


def test_tiled_batch_without_flags_and_errors(aqz, oracle):
    geo = halving(256, 128, 3)
    rng = np.random.default_rng(3)
    frames = [rng.integers(0, 65536, (128, 256), dtype=np.uint16) for _ in range(2)]
    got, _ = run_tiled(aqz, geo, np.uint16, 1, frames, 32, 32, with_flags=False)
    ref = oracle.cascade_2d(frames[1], 3, 1)
    assert_parity(got[1][0][1], oracle.tile_frame(ref[1], 32, 32)[0], "no flags")
    # a volume pyramid is not pure XY; a zero tile shape is rejected
    ds = aqz.Downsampler([(64, 64, 4), (32, 32, 2)], np.uint16, 1)
    d = empty_device(64 * 64 * 2 * 4)
    o = empty_device(32 * 32 * 2 * 2)
    with pytest.raises(aqz.AqzError):
        ds.run_device_batch_tiled(d.data_ptr(), 4, [None, (32, 32)], [0, o.data_ptr()])
    ds.close()
    ds = aqz.Downsampler(geo, np.uint16, 1)
    with pytest.raises(aqz.AqzError):
        ds.run_device_batch_tiled(d.data_ptr(), 1, [None, (0, 32), (32, 32)],
                                  [0, o.data_ptr(), o.data_ptr()])
    ds.close()


def test_tiled_batch_full_size_property(aqz):
    """64 headline frames (the bench batch), checked through a size-
    independent property: Decimate's tiles hold the stride-2^L subsample of
    the base frame in tile order."""
    torch = torch_cuda()
    geo = halving(4096, 4096, 5)
    n = 64
    g = torch.Generator(device="cuda").manual_seed(11)
    d_in = torch.randint(0, 256, (n * 4096 * 4096 * 2,), dtype=torch.uint8, device="cuda",
                         generator=g)
    outs = [None] + [empty_device(n * w * h * 2) for w, h, _ in geo[1:]]
    ds = aqz.Downsampler(geo, np.uint16, 0)
    ds.run_device_batch_tiled(d_in.data_ptr(), n, [None] + [(256, 256)] * 4,
                              [0] + [o.data_ptr() for o in outs[1:]], None, launch_stream())
    torch.cuda.synchronize()
    base = d_in.view(torch.int16).view(n, 4096, 4096)
    for L in range(1, 5):
        w = 4096 >> L
        nt = w // 256
        sub = base[:, :: 1 << L, :: 1 << L]  # (n, w, w)
        want = sub.reshape(n, nt, 256, nt, 256).permute(0, 1, 3, 2, 4).reshape(-1)
        got = outs[L].view(torch.int16)
        assert torch.equal(got, want), f"L{L}"
    ds.close()


def test_tiled_flag_slots_layout(aqz):
    """The headline's 256x256 chunks hold whole wave blocks at every level,
    so the zero scan needs no clear (one byte per block); tiles that split
    blocks fall back to one cleared byte per tile."""
    ds = aqz.Downsampler(halving(4096, 4096, 5), np.uint16, 1)
    # u16 blocks: 512 columns x 16 rows at level 0 -> 256x8, 128x4, 64x2, 32x1
    assert [ds.tiled_flag_slots(L, 256, 256) for L in range(1, 5)] == \
        [32 * 1, 64 * 2, 128 * 4, 256 * 8]
    assert ds.tiled_flag_slots(1, 100, 60) == 1
    assert ds.tiled_flag_slots(0, 256, 256) == 0
    ds.close()


def test_tiled_batch_chain_survives_on_demand_takes(aqz, oracle):
    """A deep tiled batch (its chain scratch allocated), on-demand tiled
    takes of a streamed frame (which grow the tiling scratch), then the deep
    batch again: both batches and the takes match the oracle."""
    geo = halving(2100, 700, 7)
    rng = np.random.default_rng(29)
    frames = [rng.integers(0, 256, (700, 2100), dtype=np.uint8) for _ in range(2)]
    ds = aqz.Downsampler(geo, np.uint8, 1)
    torch = torch_cuda()
    for rep in range(2):
        d_in = to_device(np.stack(frames))
        outs, shapes = [None], [None]
        for L, (w, h, _) in enumerate(geo[1:], 1):
            nt = (-(-h // 8)) * (-(-w // 16))
            outs.append(empty_device(2 * nt * 8 * 16))
            shapes.append(nt)
        ds.run_device_batch_tiled(d_in.data_ptr(), 2, [None] + [(8, 16)] * 6,
                                  [0] + [o.data_ptr() for o in outs[1:]], None,
                                  launch_stream())
        torch.cuda.synchronize()
        for k, fr in enumerate(frames):
            ref = oracle.cascade_2d(fr, 7, 1)
            for L in range(1, 7):
                t = from_device(outs[L], np.uint8, (2, shapes[L], 8, 16))
                assert_parity(t[k], oracle.tile_frame(ref[L - 1], 8, 16)[0],
                              f"rep {rep} frame {k} L{L}")
        # streamed frame, taken tiled on demand with ever larger tiles
        ds.add_frame(frames[rep])
        ref = oracle.cascade_2d(frames[rep], 7, 1)
        for L, tile in ((1, (64, 64)), (2, (128, 256))):
            got = ds.take_frame_tiled(L, *tile)
            want_t, want_nz = oracle.tile_frame(ref[L - 1], *tile)
            assert_parity(got[0], want_t, f"rep {rep} take L{L}")
            assert np.array_equal(got[1], want_nz)
        for L in range(3, 7):
            ds.take_frame(L)
    ds.close()
