"""MI355X parity of the codec stages beside the pyramid (SURVEY §8(f) rows
3-4) against the CPU oracle (oracle/codec_oracle.c, pinned in
tests/test_oracle_codecs.py): blosc's per-block shuffle filters and CRC-32C,
through the C ABI (include/aqz_codec.h).  Byte-exact."""
import numpy as np
import pytest

from gpu_util import empty_device, from_device, launch_stream, to_device, torch_cuda

pytestmark = pytest.mark.gpu

FILTER_CASES = [
    # (typesize, blocksize, nbytes, n_buffers)
    (2, 65536, 131072, 4),          # 256x256 u16 chunk: two full blocks
    (2, 65536, 65536 * 3 + 4096, 2),  # leftover block, vector path
    (2, 32768, 1000, 3),            # one short block: generic path
    (1, 4096, 4096 * 5 + 8, 2),     # u8 bitshuffle (G = 16)
    (4, 16384, 16384 * 4, 3),       # u32 / f32
    (8, 16384, 16384 * 2 + 48, 2),  # u64 / f64, leftover of 6 elements
    (16, 8192, 8192 * 2, 2),        # typesize 16
    (3, 3000, 9000 + 7, 2),         # odd typesize: generic kernels, tails
    (2, 4104, 4104 * 2, 1),         # 2052 elements: not a multiple of 8 groups
    (2, 200, 13, 5),                # block of 13 bytes: odd tail byte
    (4, 2, 10, 1),                  # blocksize < typesize
    # bit shuffle rows staged through LDS (a workgroup inside one block)
    (4, 65536, 65536 * 2 + 1024, 2),  # f32 chunk blocks + an unstaged leftover
    (8, 65536, 65536 * 2, 2),       # f64: 2-B rows per thread
    (2, 32768, 32768 * 3, 2),       # exactly 256 threads per block
    # 4- and 8-byte bit shuffle through the 32x32 word transpose: short bit
    # rows, few threads per block, blocks narrower than a wave
    (4, 256, 256 * 5, 2),           # 8-B rows: 2 threads per block
    (4, 384, 384 * 3, 2),           # 12-B rows: 3 threads per block
    (8, 512, 512 * 3 + 72, 3),      # 8-B rows: 4 threads per block; 72-B leftover copied
    (8, 256, 256 * 6, 2),           # 4-B rows: 2 threads per block
    (2, 128 * 3, 128 * 3 * 7, 2),   # u16, 24-B rows: 3 threads per block
    (4, 4096 * 4, 4096 * 4 * 64, 1),  # a 4096-wide f32 level as 16 KiB blocks
]


@pytest.mark.parametrize("shuffle", [0, 1, 2], ids=["noshuffle", "shuffle", "bitshuffle"])
@pytest.mark.parametrize("case", FILTER_CASES, ids=lambda c: f"ts{c[0]}_bs{c[1]}_n{c[2]}x{c[3]}")
def test_blosc_filter_matches_oracle(aqz, oracle, shuffle, case):
    ts, bs, nbytes, nbuf = case
    rng = np.random.default_rng(ts * 1000 + bs + nbytes + shuffle)
    host = rng.integers(0, 256, nbytes * nbuf, dtype=np.uint8)
    host[: nbytes // 3] = 0  # some zero runs
    d_src = to_device(host)
    d_dst = empty_device(host.size)
    aqz.blosc_filter_device(shuffle, ts, bs, d_src.data_ptr(), nbytes, nbuf, d_dst.data_ptr(),
                            launch_stream())
    got = from_device(d_dst, np.uint8, (nbuf, nbytes))
    for k in range(nbuf):
        want = oracle.blosc_filter(host[k * nbytes:(k + 1) * nbytes], shuffle, ts, bs)
        assert np.array_equal(got[k], want), f"buffer {k}"


@pytest.mark.parametrize("shuffle", [1, 2])
def test_blosc_filter_unaligned_buffers(aqz, oracle, shuffle):
    """Pointers off 16-B alignment take the generic kernels; same bytes."""
    torch = torch_cuda()
    rng = np.random.default_rng(3)
    nbytes, ts, bs = 8192 + 40, 2, 4096
    host = rng.integers(0, 256, nbytes, dtype=np.uint8)
    src = torch.empty(nbytes + 1, dtype=torch.uint8, device="cuda")
    src[1:].copy_(torch.from_numpy(host).to("cuda"))
    dst = torch.empty(nbytes + 3, dtype=torch.uint8, device="cuda")
    aqz.blosc_filter_device(shuffle, ts, bs, src.data_ptr() + 1, nbytes, 1, dst.data_ptr() + 3,
                            launch_stream())
    torch.cuda.synchronize()
    got = dst[3:].cpu().numpy()
    assert np.array_equal(got, oracle.blosc_filter(host, shuffle, ts, bs))


def test_blosc_filter_headline_level0_chunks(aqz, oracle):
    """The headline's level-0 frame as 256 chunk-depth-1 chunks of 256x256
    u16 (what aqz_tile_frame_device lays out), bit-shuffled in 64 KiB
    blocks in one launch: every chunk equals the oracle, and the oracle's
    inverse filter restores the tiles."""
    torch = torch_cuda()
    rng = np.random.default_rng(17)
    frame = rng.integers(0, 4096, (4096, 4096), dtype=np.uint16)
    tiles, _ = oracle.tile_frame(frame, 256, 256)
    d_src = to_device(tiles)
    d_dst = empty_device(tiles.nbytes)
    chunk = 256 * 256 * 2
    aqz.blosc_filter_device(2, 2, 65536, d_src.data_ptr(), chunk, 256, d_dst.data_ptr(),
                            launch_stream())
    got = from_device(d_dst, np.uint8, (256, chunk))
    for k in (0, 1, 77, 255):
        raw = tiles[k].view(np.uint8).reshape(-1)
        want = oracle.blosc_filter(raw, 2, 2, 65536)
        assert np.array_equal(got[k], want), f"chunk {k}"
        assert np.array_equal(oracle.blosc_unfilter(got[k], 2, 2, 65536), raw)
    torch.cuda.synchronize()


def test_blosc_filter_errors(aqz):
    d = empty_device(64)
    for args in [(3, 2, 16), (1, 0, 16), (1, 2, 0)]:
        with pytest.raises(aqz.AqzError):
            aqz.blosc_filter_device(args[0], args[1], args[2], d.data_ptr(), 64, 1,
                                    d.data_ptr())


CRC_SIZES = [0, 1, 9, 255, 256, 257, 4099, 16 * 1024 + 4, 1 << 20]


def test_crc32c_rfc3720_vectors_on_gpu(aqz):
    torch = torch_cuda()
    vecs = [(np.zeros(32, np.uint8), 0x8A9136AA), (np.full(32, 0xFF, np.uint8), 0x62A8AB43),
            (np.arange(32, dtype=np.uint8), 0x46DD794E),
            (np.arange(31, -1, -1).astype(np.uint8), 0x113FDB5C)]
    host = np.concatenate([v for v, _ in vecs])
    d = to_device(host)
    out = torch.zeros(4, dtype=torch.int64, device="cuda")
    aqz.crc32c_device(d.data_ptr(), 32, 32, 4, out.data_ptr(), launch_stream())
    got = from_device(out, np.uint32, (8,))[:4]
    assert [int(x) for x in got] == [c for _, c in vecs]


@pytest.mark.parametrize("n", CRC_SIZES)
def test_crc32c_matches_oracle(aqz, oracle, n):
    torch = torch_cuda()
    rng = np.random.default_rng(n + 1)
    nbuf, stride = 3, n + 13
    host = rng.integers(0, 256, nbuf * stride, dtype=np.uint8)
    d = to_device(host)
    out = torch.zeros(nbuf, dtype=torch.int32, device="cuda")
    aqz.crc32c_device(d.data_ptr() if n else d.data_ptr(), n, stride, nbuf, out.data_ptr(),
                      launch_stream())
    got = from_device(out, np.uint32, (nbuf,))
    for k in range(nbuf):
        assert int(got[k]) == oracle.crc32c(host[k * stride:k * stride + n]), f"buffer {k}"


@pytest.mark.parametrize("n", [1, 64, 65, 128, 1000, 1024, 4096, 8193, 16384])
def test_crc32c_packed_small_tables(aqz, oracle, n):
    """Tables of <= 16 KiB pack 256 >> lgp to a workgroup (lanes = next power
    of two of their 64-B segments); 37 tables leave a partial last workgroup,
    and the words after crcs[36] must stay untouched."""
    torch = torch_cuda()
    rng = np.random.default_rng(n + 77)
    nbuf, stride = 37, n + 5
    host = rng.integers(0, 256, nbuf * stride, dtype=np.uint8)
    d = to_device(host)
    out = torch.full((nbuf + 8,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    aqz.crc32c_device(d.data_ptr(), n, stride, nbuf, out.data_ptr(), launch_stream())
    got = from_device(out, np.uint32, (nbuf + 8,))
    for k in range(nbuf):
        assert int(got[k]) == oracle.crc32c(host[k * stride:k * stride + n]), f"buffer {k}"
    assert all(int(x) == 0x5A5A5A5A for x in got[nbuf:])


def test_crc32c_shard_index_tables(aqz, oracle):
    """A batch of shard index tables (Shard::write_table_, shard.cpp:145-166):
    the GPU checksum equals the 4 bytes the reference appends."""
    torch = torch_cuda()
    rng = np.random.default_rng(9)
    n_chunks, n_shards = 1024, 16
    tables = []
    for s in range(n_shards):
        off = rng.integers(0, 1 << 40, n_chunks, dtype=np.uint64)
        ext = rng.integers(0, 1 << 20, n_chunks, dtype=np.uint64)
        off[::7] = np.uint64(2**64 - 1)  # unwritten-chunk sentinels
        tables.append(oracle.shard_index_table(off, ext))
    host = np.stack(tables)
    d = to_device(host)
    out = torch.zeros(n_shards, dtype=torch.int32, device="cuda")
    aqz.crc32c_device(d.data_ptr(), 16 * n_chunks, host.shape[1], n_shards, out.data_ptr(),
                      launch_stream())
    got = from_device(out, np.uint32, (n_shards,))
    for s in range(n_shards):
        assert int(got[s]) == int(host[s, 16 * n_chunks:].view(np.uint32)[0])
