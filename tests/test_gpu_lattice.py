"""GPU: levels written by the pyramid kernel straight into chunk buffers
(aqz_ds_run_device_batch_chunked), against the oracle pyramid tiled by the
oracle and placed where Array::write_frame_to_chunks_ puts each tile
(array.cpp:563-617: chunks_[t + tile_group_offset] at chunk_internal_offset).

Every lattice buffer is poisoned first: bytes no frame owns must keep the
poison, every byte a frame owns must equal the oracle's.  The full chunks of
a completed layer are then compressed where they lie and checked against
c-blosc itself.

Expected placement never comes from the product: the KAT-dims case takes it
from the reference's own assertions (tests/golden/reference_kats.json,
`addressing`), every other case from the oracle's restatement of
array.dimensions.cpp:232-314 (`oracle.chunk_frame_offsets`), which the CPU
suite pins to those same assertions (tests/test_reference_addressing.py).
"""
import numpy as np
import pytest

import kat_runner
from gpu_util import empty_device, random_frames, to_device, torch_cuda

pytestmark = pytest.mark.gpu

SPACE, CHANNEL, TIME = 0, 1, 2
POISON = 0xA5


def level_dims(dims, geo, L):
    """The level-L dims: the XY sizes of the pyramid level, the rest kept."""
    w, h, _ = geo[L]
    return dims[:-2] + [(SPACE, h, dims[-2][2], 1), (SPACE, w, dims[-1][2], 1)]


def expected_lattices(oracle, dims, geo, frames, dtype, method, first, cap, placement=None):
    ref = oracle.OracleDownsampler(geo, dtype, method)
    bpp = np.dtype(dtype).itemsize
    outs = [None] + [np.full(cap[L], POISON, np.uint8) for L in range(1, len(geo))]
    offs = [None]
    for L in range(1, len(geo)):
        if placement is not None:
            offs.append(placement[L])
            continue
        o, cb, _ = oracle.chunk_frame_offsets(level_dims(dims, geo, L), bpp, first, len(frames))
        offs.append((o, cb))
    for k, fr in enumerate(frames):
        ref.add_frame(fr)
        for L in range(1, len(geo)):
            lvl = ref.take_frame(L)
            tr, tc = dims[-2][2], dims[-1][2]
            tiles, _ = oracle.tile_frame(lvl, tr, tc)
            o, cb = offs[L]
            tb = tr * tc * bpp
            for t in range(tiles.shape[0]):
                at = o[k] + t * cb
                outs[L][at:at + tb] = tiles[t].view(np.uint8).reshape(-1)
    return outs, offs


def run_case(aqz, oracle, dims, dtype, method, first, n, seed, max_levels=0, placement=None):
    """`placement[L]` = (offsets, chunk_bytes, layer_bytes) overrides the
    oracle's addressing for level L."""
    torch = torch_cuda()
    geo = aqz.level_geometry(aqz.plan_levels(dims, max_levels))
    assert len(geo) >= 2
    H, W = dims[-2][1], dims[-1][1]
    rng = np.random.default_rng(seed)
    frames = random_frames(rng, dtype, (n, H, W))
    bpp = np.dtype(dtype).itemsize
    cap = [0]
    for L in range(1, len(geo)):
        if placement is not None:
            o, cb, lb = placement[L]
        else:
            o, cb, lb = oracle.chunk_frame_offsets(level_dims(dims, geo, L), bpp, first, n)
        # the layers this batch touches
        cap.append((max(o) // lb + 1) * lb)
    want, offs = expected_lattices(oracle, dims, geo, list(frames), dtype, method, first,
                                   cap, None if placement is None else
                                   [None] + [placement[L][:2] for L in range(1, len(geo))])
    ds = aqz.Downsampler(geo, dtype, method, device=0)
    d_in = to_device(frames)
    bufs = [None] + [empty_device(cap[L]) for L in range(1, len(geo))]
    for b in bufs[1:]:
        b.fill_(POISON)
    lats = [None] + [(bufs[L].data_ptr(), cap[L], dims[-2][2], dims[-1][2], offs[L][1],
                      offs[L][0]) for L in range(1, len(geo))]
    counts = ds.run_device_batch_chunked(d_in.data_ptr(), n, lats)
    torch.cuda.synchronize()
    assert counts == [n] * len(geo)
    for L in range(1, len(geo)):
        got = bufs[L].cpu().numpy()
        if not np.array_equal(got, want[L]):  # bytes: NaN payloads included
            bad = np.flatnonzero(got != want[L])
            raise AssertionError(f"level {L}: {bad.size} bytes differ, first at {bad[0]}")
    ds.close()
    return geo, bufs, offs, cap


@pytest.mark.parametrize("dtype", [np.uint8, np.uint16, np.float32])
@pytest.mark.parametrize("first", [0, 2])
def test_time_chunks(aqz, oracle, dtype, first):
    """T/Y/X with 3 frames per chunk, ragged XY chunks, a batch starting
    inside a chunk and spanning three layers."""
    dims = [(TIME, 0, 3, 1), (SPACE, 384, 128, 1), (SPACE, 520, 96, 1)]
    run_case(aqz, oracle, dims, dtype, aqz.METHODS["mean"], first, 7, seed=first + 1)


@pytest.mark.parametrize("method", ["decimate", "min", "max"])
def test_channel_chunks(aqz, oracle, method):
    """T/C/Y/X: 3 channels in chunks of 2, frames C-fastest, so a frame's
    chunk and its place in it both depend on the channel."""
    dims = [(TIME, 0, 2, 1), (CHANNEL, 3, 2, 1), (SPACE, 256, 64, 1), (SPACE, 300, 64, 1)]
    run_case(aqz, oracle, dims, np.uint16, aqz.METHODS[method], 1, 9, seed=7)


def kat_placement():
    """Frame k's tile-0 offset in a lattice of the KAT dims (t 0/5, c 3/2,
    z 5/2, y 48/16, x 64/16, u16), built only from the reference's asserted
    values: chunk_lattice_index(k, 0) layers, tile_group_offset(k) chunks and
    chunk_internal_offset(k) bytes (array-dimensions-*.cpp)."""
    kats = {c["function"]: c for c in kat_runner.load()["addressing"]}
    cio = {a["args"][0]: a["expect"] for a in kats["chunk_internal_offset"]["asserts"]}
    tgo = {a["args"][0]: a["expect"] for a in kats["tile_group_offset"]["asserts"]}
    layer = {a["args"][0]: a["expect"] for a in kats["chunk_lattice_index"]["asserts"]
             if a["args"][1] == 0}
    assert kats["chunk_internal_offset"]["dtype"] == 1  # offsets in u16 bytes
    chunk_bytes = 2 * 5 * 2 * 2 * 16 * 16      # bytes_per_chunk_, array.dimensions.cpp:171
    layer_bytes = 2 * 3 * 3 * 4 * chunk_bytes  # number_of_chunks_in_memory_, :175
    frames = sorted(cio)
    assert frames == list(range(76)) and sorted(tgo) == frames
    # the lattice-index KAT names the layer of 17 of these frames; the rest
    # share layer 0 (frames 0..74 are t 0..4, one T chunk)
    offs = [layer.get(k, 0 if k < 75 else None) * layer_bytes + tgo[k] * chunk_bytes + cio[k]
            for k in frames]
    return offs, chunk_bytes, layer_bytes


def test_kat_dims_placement(aqz, oracle):
    """The reference's addressing test dims as a pyramid level: a 96x128 base
    (y/x chunks 16) gives level 1 = t 0/5, c 3/2, z 5/2, y 48/16, x 64/16 —
    the dims of tests/unit-tests/array-dimensions-*.cpp (z is typed Channel so
    the planner keeps its 5 planes; the addressing reads sizes and chunks
    only).  All 76 frames those tests name go in one batch, frame 75 into the
    second layer; every tile must land where the asserted values put it."""
    dims = [(TIME, 0, 5, 1), (CHANNEL, 3, 2, 1), (CHANNEL, 5, 2, 1), (SPACE, 96, 16, 1),
            (SPACE, 128, 16, 1)]
    geo = aqz.level_geometry(aqz.plan_levels(dims, 1))
    assert geo == [(128, 96, 5), (64, 48, 5)]
    run_case(aqz, oracle, dims, np.uint16, aqz.METHODS["mean"], 0, 76, seed=21, max_levels=1,
             placement=[None, kat_placement()])


def test_deep_pyramid_chains(aqz, oracle):
    """Six levels: two fused runs, both writing into the lattice."""
    dims = [(TIME, 0, 2, 1), (SPACE, 1024, 16, 1), (SPACE, 1024, 16, 1)]
    geo, *_ = run_case(aqz, oracle, dims, np.uint16, aqz.METHODS["mean"], 0, 3, seed=3)
    assert len(geo) == 7


def test_rejects_offsets_outside_the_buffer(aqz):
    torch = torch_cuda()
    dims = [(TIME, 0, 2, 1), (SPACE, 256, 128, 1), (SPACE, 256, 128, 1)]
    geo = aqz.level_geometry(aqz.plan_levels(dims))
    ds = aqz.Downsampler(geo, np.uint16, aqz.METHODS["mean"], device=0)
    d_in = empty_device(2 * 256 * 256 * 2)
    o, cb, lb = aqz.chunk_frame_offsets(level_dims(dims, geo, 1), 2, 0, 2)
    buf = empty_device(lb)
    ok = [None, (buf.data_ptr(), lb, 128, 128, cb, o)]
    for bad in ([buf.data_ptr(), lb - 2, 128, 128, cb, o],        # capacity short by a pixel
                [buf.data_ptr(), lb, 128, 128, cb, [o[0], o[1] + 1]],  # misaligned offset
                [buf.data_ptr(), lb, 128, 128, 100, o]):           # stride below a tile
        with pytest.raises(aqz.AqzError):
            ds.run_device_batch_chunked(d_in.data_ptr(), 2, [None, tuple(bad)])
    ds.run_device_batch_chunked(d_in.data_ptr(), 2, ok)
    torch.cuda.synchronize()
    ds.close()


def test_completed_layer_compresses_in_place(aqz, oracle):
    """A batch that fills whole chunk layers: every chunk buffer is then one
    contiguous device span, compressed where it lies; frames must equal
    c-blosc's of the oracle's chunks."""
    import blosc_ref
    if not blosc_ref.available():
        pytest.skip("no libblosc")
    dims = [(TIME, 0, 4, 1), (SPACE, 512, 128, 1), (SPACE, 512, 128, 1)]
    geo, bufs, offs, cap = run_case(aqz, oracle, dims, np.uint16, aqz.METHODS["mean"], 0, 8,
                                    seed=9)
    ctx = aqz.BloscContext(0, 4)
    for L in range(1, len(geo)):
        cb = offs[L][1]
        n_chunks = cap[L] // cb
        host = bufs[L].cpu().numpy()
        frames = ctx.compress_device(1, 1, 2, "lz4", bufs[L].data_ptr(), cb, n_chunks)
        for k in range(n_chunks):
            assert frames[k] == blosc_ref.compress(host[k * cb:(k + 1) * cb], 1, 1, 2, "lz4")
    ctx.close()
