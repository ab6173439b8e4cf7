"""GPU: c-blosc chunk frames of device-resident chunks (aqz_blosc_compress_device)
against c-blosc 1.21.0 itself (oracle/blosc_ref.py).

The reference's compress_in_place (zarr.common.cpp:106-137) runs
blosc_compress_ctx on every chunk buffer; here the filter runs on the GPU,
the filtered chunks cross PCIe in groups, and host threads run LZ4/zstd.
Every frame must equal libblosc's frame of the same chunk, byte for byte.
"""
import numpy as np
import pytest

import blosc_ref
from gpu_util import empty_device, to_device, torch_cuda

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not blosc_ref.available(), reason="no libblosc")]


def smooth_chunks(rng, n_chunks, h, w, dtype):
    yy, xx = np.mgrid[0:h, 0:w]
    out = np.empty((n_chunks, h, w), dtype)
    for k in range(n_chunks):
        base = 2000 + 500 * np.sin((xx + 13 * k) / 17.0) * np.cos((yy - 5 * k) / 23.0)
        out[k] = (base + rng.normal(0, 4, (h, w))).astype(dtype)
    return out


@pytest.fixture(scope="module")
def ctx(aqz):
    c = aqz.BloscContext(0, 0)
    yield c
    c.close()


def check_frames(frames, chunks_bytes, nbytes, clevel, shuffle, ts, cname):
    for k, fr in enumerate(frames):
        src = chunks_bytes[k * nbytes:(k + 1) * nbytes]
        want = blosc_ref.compress(src, clevel, shuffle, ts, cname)
        assert fr == want, (k, len(fr), len(want), blosc_ref.header(fr), blosc_ref.header(want))


@pytest.mark.parametrize("cname,clevel", [("lz4", 1), ("lz4", 5), ("lz4", 9), ("zstd", 1),
                                          ("zstd", 5)])
@pytest.mark.parametrize("shuffle", [0, 1, 2])
def test_u16_chunks_match_cblosc(aqz, ctx, cname, clevel, shuffle):
    rng = np.random.default_rng(clevel * 7 + shuffle)
    chunks = smooth_chunks(rng, 40, 256, 256, np.uint16)  # 40 x 128 KiB: 2 copy groups
    raw = chunks.view(np.uint8).reshape(-1)
    d = to_device(raw)
    frames = ctx.compress_device(clevel, shuffle, 2, cname, d.data_ptr(), 256 * 256 * 2, 40)
    check_frames(frames, raw, 256 * 256 * 2, clevel, shuffle, 2, cname)


@pytest.mark.parametrize("ts,dtype", [(1, np.uint8), (4, np.float32), (8, np.float64)])
def test_other_typesizes(aqz, ctx, ts, dtype):
    rng = np.random.default_rng(ts)
    chunks = smooth_chunks(rng, 6, 100, 130, dtype)  # leftover blocks, odd sizes
    raw = chunks.view(np.uint8).reshape(-1)
    nbytes = 100 * 130 * ts
    d = to_device(raw)
    for cname, clevel, shuffle in (("lz4", 3, 1), ("zstd", 2, 2), ("lz4", 8, 2)):
        frames = ctx.compress_device(clevel, shuffle, ts, cname, d.data_ptr(), nbytes, 6)
        check_frames(frames, raw, nbytes, clevel, shuffle, ts, cname)


def test_incompressible_chunks_copy_raw(aqz, ctx):
    """Random chunks: c-blosc stores them unfiltered (memcpy flag); the raw
    bytes come straight from the device."""
    rng = np.random.default_rng(3)
    raw = rng.integers(0, 256, 12 * 70000, dtype=np.uint8)
    raw[5 * 70000:6 * 70000] = 7  # one compressible chunk among them
    d = to_device(raw)
    frames = ctx.compress_device(5, 1, 2, "lz4", d.data_ptr(), 70000, 12)
    assert sum(1 for f in frames if f[2] & 0x2) == 11
    check_frames(frames, raw, 70000, 5, 1, 2, "lz4")


@pytest.mark.parametrize("nbytes,clevel", [(100, 5), (5000, 0), (64, 0)])
def test_memcpy_frames(aqz, ctx, nbytes, clevel):
    raw = (np.arange(9 * nbytes) % 13).astype(np.uint8)
    d = to_device(raw)
    frames = ctx.compress_device(clevel, 2, 2, "zstd", d.data_ptr(), nbytes, 9)
    check_frames(frames, raw, nbytes, clevel, 2, 2, "zstd")


def test_tiled_pyramid_chunks(aqz, oracle):
    """Levels written chunk-tiled by the pyramid kernel
    (aqz_ds_run_device_batch_tiled) compressed where they lie: each tile is
    one chunk buffer of a chunk-depth-1 array."""
    torch = torch_cuda()
    W = H = 1024
    tile = 256
    dims = [(aqz.TIME, 0, 1, 1), (aqz.SPACE, H, tile, 1), (aqz.SPACE, W, tile, 1)]
    geo = aqz.level_geometry(aqz.plan_levels(dims))
    rng = np.random.default_rng(11)
    frame = smooth_chunks(rng, 1, H, W, np.uint16)[0]
    ds = aqz.Downsampler(geo, np.uint16, aqz.METHODS["mean"], device=0)
    d_in = to_device(frame)
    n_levels = len(geo)
    tiles_per = [0] + [(-(-w // tile)) * (-(-h // tile)) for w, h, _ in geo[1:]]
    outs = [None] + [empty_device(t * tile * tile * 2) for t in tiles_per[1:]]
    ds.run_device_batch_tiled(d_in.data_ptr(), 1, [(tile, tile)] * n_levels,
                              [0] + [o.data_ptr() for o in outs[1:]])
    torch.cuda.synchronize()
    c = aqz.BloscContext(0, 4)
    ref = oracle.OracleDownsampler(geo, np.uint16, aqz.METHODS["mean"])
    ref.add_frame(frame)
    for L in range(1, n_levels):
        lvl = ref.take_frame(L)
        want_tiles, _ = oracle.tile_frame(lvl, tile, tile)
        want_tiles = want_tiles.view(np.uint8).reshape(-1)
        nb = tile * tile * 2
        frames = c.compress_device(1, 1, 2, "lz4", outs[L].data_ptr(), nb, tiles_per[L])
        check_frames(frames, want_tiles, nb, 1, 1, 2, "lz4")
    c.close()
    ds.close()


def test_errors(aqz, ctx):
    d = empty_device(1024)
    for args in ((10, 1, 2, "lz4"), (5, 3, 2, "lz4"), (5, 1, 0, "lz4"), (5, 1, 2, "snappy")):
        with pytest.raises(aqz.AqzError):
            ctx.compress_device(*args, d.data_ptr(), 512, 2)
    with pytest.raises(aqz.AqzError):  # stride too small
        ctx.compress_device(5, 1, 2, "lz4", d.data_ptr(), 512, 2,
                            host_dst=np.empty(2048, np.uint8), dst_stride=520)
