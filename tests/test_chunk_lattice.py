"""CPU: aqz_chunk_frame_offsets — where each frame's tiles go in the chunk
lattice — against an independent N-D formulation of the reference's chunk
addressing.

The reference writes tile t of frame `frame_id` into
chunks_[t + tile_group_offset(frame_id)] at chunk_internal_offset(frame_id)
(array.cpp:563-617), with ArrayDimensions::chunk_lattice_index /
tile_group_offset / chunk_internal_offset (array.dimensions.cpp:232-314) and
one chunk layer of number_of_chunks_in_memory_ chunks of bytes_per_chunk_
(:168-178).  Here the frame id is unravelled into its index along every
non-spatial dimension (storage order, last fastest); the chunk holding the
frame is the index // chunk size along each, its place inside the chunk the
index % chunk size — the same addresses, derived without the reference's
stride loops.
"""
import numpy as np
import pytest


def nd_offsets(dims, bpp, first, n):
    """dims: [(type, array, chunk, shard)], storage order, ndims >= 3."""
    a = [d[1] for d in dims]
    c = [d[2] for d in dims]
    nd = len(dims)
    tile = bpp * c[-1] * c[-2]
    chunk_bytes = bpp * int(np.prod(c))
    counts = [-(-a[i] // c[i]) for i in range(nd)]
    layer_chunks = int(np.prod(counts[1:]))
    # chunk strides (in chunks) inside a layer, dims 1..nd-1 (last fastest)
    cstride = [0] * nd
    acc = 1
    for i in range(nd - 1, 0, -1):
        cstride[i] = acc
        acc *= counts[i]
    inner = a[1:nd - 2]                      # array sizes of dims 1..nd-3
    frames_per_t = int(np.prod(inner)) if inner else 1
    out = []
    for f in range(first, first + n):
        idx = [f // frames_per_t]
        rem = f % frames_per_t
        for j in range(1, nd - 2):
            span = int(np.prod(a[j + 1:nd - 2])) if j + 1 < nd - 2 else 1
            idx.append(rem // span)
            rem %= span
        layer = idx[0] // c[0]
        group = sum((idx[j] // c[j]) * cstride[j] for j in range(1, nd - 2))
        within = 0
        for j in range(0, nd - 2):
            within = within * c[j] + idx[j] % c[j]
        out.append(layer * layer_chunks * chunk_bytes + group * chunk_bytes + within * tile)
    layer0 = (first // frames_per_t) // c[0]
    base = layer0 * layer_chunks * chunk_bytes
    return [o - base for o in out], chunk_bytes, layer_chunks * chunk_bytes


SPACE, CHANNEL, TIME = 0, 1, 2


@pytest.mark.parametrize("dims", [
    [(TIME, 0, 3, 1), (SPACE, 480, 128, 1), (SPACE, 640, 128, 1)],
    [(TIME, 0, 1, 1), (SPACE, 4096, 256, 1), (SPACE, 4096, 256, 1)],
    [(TIME, 0, 2, 1), (CHANNEL, 3, 2, 1), (SPACE, 100, 32, 1), (SPACE, 90, 64, 1)],
    [(TIME, 0, 4, 1), (CHANNEL, 5, 5, 1), (SPACE, 7, 3, 1), (SPACE, 64, 16, 1),
     (SPACE, 48, 16, 1)],
    [(TIME, 0, 1, 1), (CHANNEL, 2, 1, 1), (SPACE, 6, 4, 1), (SPACE, 256, 64, 1),
     (SPACE, 256, 64, 1)],
])
@pytest.mark.parametrize("bpp", [1, 2, 4])
def test_offsets_match_nd_formulation(aqz, dims, bpp):
    for first in (0, 1, 5, 37):
        got, cb, lb = aqz.chunk_frame_offsets(dims, bpp, first, 40)
        want, wcb, wlb = nd_offsets(dims, bpp, first, 40)
        assert (cb, lb) == (wcb, wlb)
        assert got == want, (first, got[:8], want[:8])


def test_random_dimension_sets(aqz):
    rng = np.random.default_rng(4)
    for _ in range(300):
        nd = int(rng.integers(3, 6))
        dims = [(TIME, 0, int(rng.integers(1, 5)), 1)]
        for _ in range(nd - 3):
            size = int(rng.integers(1, 7))
            dims.append((CHANNEL, size, int(rng.integers(1, size + 1)), 1))
        for _ in range(2):
            size = int(rng.integers(1, 300))
            dims.append((SPACE, size, int(rng.integers(1, 80)), 1))
        first = int(rng.integers(0, 50))
        got = aqz.chunk_frame_offsets(dims, 2, first, 25)
        assert got == nd_offsets(dims, 2, first, 25), dims


def test_three_d_is_depth_times_tile(aqz):
    """T/Y/X with a T chunk of D frames: frame k at (k % D) tiles into its
    chunk, a new chunk layer every D frames."""
    D = 3
    dims = [(TIME, 0, D, 1), (SPACE, 500, 128, 1), (SPACE, 300, 128, 1)]
    offs, cb, lb = aqz.chunk_frame_offsets(dims, 2, 4, 8)
    tile = 128 * 128 * 2
    assert cb == D * tile and lb == 4 * 3 * cb
    assert offs == [((4 + k) // D - 1) * lb + ((4 + k) % D) * tile for k in range(8)]


def test_errors(aqz):
    with pytest.raises(aqz.AqzError):
        aqz.chunk_frame_offsets([(SPACE, 10, 5, 1), (SPACE, 10, 5, 1)], 2, 0, 1)
    with pytest.raises(aqz.AqzError):
        aqz.chunk_frame_offsets([(TIME, 0, 0, 1), (SPACE, 10, 5, 1), (SPACE, 10, 5, 1)], 2, 0, 1)
    with pytest.raises(aqz.AqzError):
        aqz.chunk_frame_offsets([(TIME, 0, 1, 1), (CHANNEL, 0, 1, 1), (SPACE, 10, 5, 1),
                                 (SPACE, 10, 5, 1)], 2, 0, 1)
