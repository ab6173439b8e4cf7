"""CPU: the blosc frame writer (include/aqz_blosc.h) against c-blosc itself.

The reference compresses each chunk with blosc_compress_ctx(clevel, shuffle,
typesize, nbytes, src, dest, nbytes + 16, "lz4" | "zstd", 0, 1)
(zarr.common.cpp:106-137).  The image carries c-blosc 1.21.0
(oracle/blosc_ref.py), so here:

* the filter restatement (oracle/codec_oracle.c, which the GPU kernels are
  tested against) equals the filtered blocks c-blosc stores raw for
  incompressible data — the shuffle is pinned by the real library;
* aqz_blosc_blocksize equals the block size c-blosc writes in its header;
* aqz_blosc_frame_from_filtered, fed the filtered blocks, writes the frame
  c-blosc writes, byte for byte: compressible, incompressible (raw splits),
  mixed, memcpy fallback, clevel 0, tiny buffers, too-small destinations;
* and the committed fixtures (tests/golden/blosc_frames.npz, made by
  tests/golden/make_blosc_frames.py from the same library) hold where
  libblosc is absent.

No GPU: the host frame writer is called directly.
"""
import os

import numpy as np
import pytest

import blosc_ref

HERE = os.path.dirname(os.path.abspath(__file__))
needs_blosc = pytest.mark.skipif(not blosc_ref.available(), reason="no libblosc in this image")


def data_kinds(n, rng):
    yield "random", rng.integers(0, 256, n, dtype=np.uint8)
    x = np.arange(n)
    yield "smooth", ((x % 251) + rng.integers(0, 4, n)).astype(np.uint8)
    yield "zeros", np.zeros(n, np.uint8)
    m = np.zeros(n, np.uint8)
    m[n // 3:n // 2] = rng.integers(0, 256, n // 2 - n // 3, dtype=np.uint8)
    yield "mixed", m


def product_frame(aqz, oracle, src, clevel, shuffle, ts, cname, destsize=-1):
    bs = aqz.blosc_blocksize(clevel, ts, src.size, cname)
    filt = oracle.blosc_filter(src, shuffle, ts if ts <= 255 else 1, bs)
    return aqz.blosc_frame_from_filtered(clevel, shuffle, ts, cname, filt, src, destsize)[0]


@needs_blosc
def test_libblosc_version():
    assert blosc_ref.version().startswith("1.")


@needs_blosc
@pytest.mark.parametrize("cname", ["lz4", "zstd"])
def test_blocksize_matches_cblosc(aqz, cname):
    bad = []
    for clevel in range(10):
        for ts in (1, 2, 3, 4, 8, 16, 17, 255, 300):
            for n in (1, 2, 15, 127, 128, 1000, 32767, 32768, 70001, 1 << 20, (3 << 20) + 5):
                fr = blosc_ref.compress(np.zeros(n, np.uint8), clevel, 0, ts, cname)
                want = blosc_ref.header(fr)["blocksize"]
                got = aqz.blosc_blocksize(clevel, ts, n, cname)
                if got != want:
                    bad.append((clevel, ts, n, got, want))
    assert not bad, bad[:10]


@needs_blosc
@pytest.mark.parametrize("shuffle", [1, 2])
@pytest.mark.parametrize("ts", [1, 2, 3, 4, 8, 16])
def test_oracle_filter_is_cblosc_filter(oracle, ts, shuffle):
    """Incompressible data with room to spare: c-blosc keeps every split
    raw, so the stored bytes are exactly its filtered blocks."""
    rng = np.random.default_rng(ts * 10 + shuffle)
    for n in (4096 + 24, 65536 * 3 + 17, 300000):
        src = rng.integers(0, 256, n, dtype=np.uint8)
        fr = blosc_ref.compress(src, 5, shuffle, ts, "lz4", destsize=n + (1 << 16))
        h = blosc_ref.header(fr)
        assert not h["flags"] & 0x2
        stored = b"".join(p for blk in blosc_ref.stored_splits(fr) for _, p in blk)
        assert all(c == len(p) for blk in blosc_ref.stored_splits(fr) for c, p in blk)
        mine = oracle.blosc_filter(src, shuffle, ts, h["blocksize"]).tobytes()
        assert stored == mine, (n, h)


@needs_blosc
@pytest.mark.parametrize("cname", ["lz4", "zstd"])
@pytest.mark.parametrize("shuffle", [0, 1, 2])
@pytest.mark.parametrize("ts", [1, 2, 4, 8])
def test_frames_match_cblosc(aqz, oracle, cname, shuffle, ts):
    rng = np.random.default_rng(1000 + ts * 3 + shuffle)
    bad = []
    for clevel in (1, 4, 9) if cname == "zstd" else (1, 2, 5, 7, 9):
        for n in (100, 1000, 4096 * 3 + 5, 65536 * 3 + 17):
            for kind, src in data_kinds(n, rng):
                for extra in (16, 1 << 16, 40):
                    want = blosc_ref.compress(src, clevel, shuffle, ts, cname, n + extra)
                    got = product_frame(aqz, oracle, src, clevel, shuffle, ts, cname, n + extra)
                    want = b"" if isinstance(want, int) else want
                    if got != want:
                        bad.append((clevel, n, kind, extra, len(got), len(want)))
    assert not bad, bad[:10]


@needs_blosc
@pytest.mark.parametrize("cname", ["lz4", "zstd"])
def test_clevel0_small_and_odd_typesizes(aqz, oracle, cname):
    rng = np.random.default_rng(5)
    for ts in (1, 3, 5, 255, 300):
        for n in (1, 7, 127, 128, 129, 5000):
            src = ((np.arange(n) // 7) % 5).astype(np.uint8) ^ rng.integers(0, 2, n).astype(np.uint8)
            for clevel in (0, 1, 6):
                for shuffle in (0, 1, 2):
                    want = blosc_ref.compress(src, clevel, shuffle, ts, cname)
                    got = product_frame(aqz, oracle, src, clevel, shuffle, ts, cname)
                    assert got == want, (ts, n, clevel, shuffle)


@needs_blosc
def test_raw_needed_leaves_copy_to_caller(aqz, oracle):
    src = np.random.default_rng(9).integers(0, 256, 50000, dtype=np.uint8)
    bs = aqz.blosc_blocksize(5, 2, src.size, "lz4")
    filt = oracle.blosc_filter(src, 1, 2, bs)
    head, raw = aqz.blosc_frame_from_filtered(5, 1, 2, "lz4", filt, None)
    assert raw and len(head) == src.size + 16
    frame = head[:16] + src.tobytes()
    assert frame == blosc_ref.compress(src, 5, 1, 2, "lz4")
    # compressible: no raw copy needed, and the frame decompresses to src
    src2 = np.repeat(np.arange(500, dtype=np.uint16), 50)
    b2 = src2.view(np.uint8)
    bs2 = aqz.blosc_blocksize(5, 2, b2.size, "zstd")
    fr2, raw2 = aqz.blosc_frame_from_filtered(5, 1, 2, "zstd", oracle.blosc_filter(b2, 1, 2, bs2), None)
    assert not raw2 and len(fr2) < b2.size
    assert np.array_equal(blosc_ref.decompress(fr2, b2.size), b2)


def test_golden_frames(aqz, oracle):
    """Fixtures from c-blosc 1.21.0 (tests/golden/make_blosc_frames.py)."""
    z = np.load(os.path.join(HERE, "golden", "blosc_frames.npz"))
    keys = [k[len("frame__"):] for k in z.files if k.startswith("frame__")]
    assert len(keys) >= 50
    for key in keys:
        name, cname, clevel, shuffle, ts = key.split("__")
        src = z[f"in__{name}"]
        got = product_frame(aqz, oracle, src, int(clevel), int(shuffle), int(ts), cname)
        assert got == z[f"frame__{key}"].tobytes(), key


def test_invalid_arguments(aqz):
    with pytest.raises(aqz.AqzError):
        aqz.blosc_blocksize(10, 2, 1000, "lz4")
    with pytest.raises(aqz.AqzError):
        aqz.blosc_blocksize(5, 2, 1000, "blosclz")
    with pytest.raises(aqz.AqzError):
        aqz.blosc_blocksize(5, 0, 1000, "zstd")
    with pytest.raises(aqz.AqzError):
        aqz.blosc_frame_from_filtered(5, 3, 2, "lz4", np.zeros(100, np.uint8))
    info = aqz.blosc_codec_info()
    assert info.startswith("lz4 1.") and "; zstd 1." in info, info
