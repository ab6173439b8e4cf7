"""CPU: pins the codec oracle (oracle/codec_oracle.c) used for SURVEY §8(f)
rows 3-4.  c-blosc and google/crc32c are absent from the image, so the
restatements are checked against their published definitions:

* crc32c against the RFC 3720 B.4 test vectors (and the usual "123456789"
  check value);
* the blosc byte/bit shuffle against hand-derived vectors and against an
  independent numpy formulation of the published layouts (byte transpose;
  bit rows j*8+b holding bit b of byte j of every element, LSB-first), with
  c-blosc 1.x's block rules: typesize > 1 for byte shuffle, blocksize >=
  typesize for bit shuffle, element counts that are not a multiple of 8 left
  unshuffled, the blocksize % typesize tail copied, the leftover block
  filtered with its own size.
"""
import numpy as np
import pytest


def np_filter(buf, shuffle, ts, bs):
    buf = np.asarray(buf, np.uint8)
    out = buf.copy()
    for off in range(0, buf.size, bs):
        blk = buf[off:off + bs]
        m = blk.size
        ne = m // ts
        if shuffle == 1 and ts > 1:
            out[off:off + ne * ts] = blk[:ne * ts].reshape(ne, ts).T.reshape(-1)
        elif shuffle == 2 and m >= ts and ne % 8 == 0:
            bits = np.unpackbits(blk[:ne * ts].reshape(ne, ts), axis=1, bitorder="little")
            out[off:off + ne * ts] = np.packbits(bits.T, axis=1,
                                                 bitorder="little").reshape(-1)
    return out


RFC3720 = [
    (np.zeros(32, np.uint8), 0x8A9136AA),
    (np.full(32, 0xFF, np.uint8), 0x62A8AB43),
    (np.arange(32, dtype=np.uint8), 0x46DD794E),
    (np.arange(31, -1, -1).astype(np.uint8), 0x113FDB5C),
    (np.frombuffer(b"123456789", np.uint8), 0xE3069283),
    (np.zeros(0, np.uint8), 0x00000000),
]


@pytest.mark.parametrize("data,want", RFC3720, ids=range(len(RFC3720)))
def test_crc32c_known_answers(oracle, data, want):
    assert oracle.crc32c(data) == want


def test_shard_index_table_layout(oracle):
    """Shard::write_table_ (shard.cpp:145-166): (offset, extent) u64 pairs,
    then the crc32c of those 16*n bytes."""
    off = np.array([0, 100, 2**64 - 1], np.uint64)  # kUnwrittenSentinel is ~0
    ext = np.array([100, 50, 2**64 - 1], np.uint64)
    t = oracle.shard_index_table(off, ext)
    assert t.size == 3 * 16 + 4
    pairs = t[:48].view(np.uint64)
    assert list(pairs) == [0, 100, 100, 50, 2**64 - 1, 2**64 - 1]
    assert int(t[48:].view(np.uint32)[0]) == oracle.crc32c(t[:48])


def test_byte_shuffle_hand_vectors(oracle):
    # typesize 2: [a0 a1 b0 b1 c0 c1] -> [a0 b0 c0 a1 b1 c1]
    src = np.array([1, 2, 3, 4, 5, 6], np.uint8)
    assert list(oracle.blosc_filter(src, 1, 2, 6)) == [1, 3, 5, 2, 4, 6]
    # blocksize 7: the 7th byte is the unshuffled tail
    src = np.array([1, 2, 3, 4, 5, 6, 7], np.uint8)
    assert list(oracle.blosc_filter(src, 1, 2, 7)) == [1, 3, 5, 2, 4, 6, 7]
    # two blocks of 4 with a leftover block of 2
    src = np.arange(10, dtype=np.uint8)
    assert list(oracle.blosc_filter(src, 1, 2, 4)) == [0, 2, 1, 3, 4, 6, 5, 7, 8, 9]
    # typesize 1: no byte shuffle at all
    assert list(oracle.blosc_filter(src, 1, 1, 4)) == list(src)


def test_bit_shuffle_hand_vectors(oracle):
    # 8 u8 elements, only element 0 = 1: bit row 0 = 0b00000001
    src = np.array([1, 0, 0, 0, 0, 0, 0, 0], np.uint8)
    assert list(oracle.blosc_filter(src, 2, 1, 8)) == [1, 0, 0, 0, 0, 0, 0, 0]
    # element 7 = 0x80: bit row 7 gets bit 7
    src = np.array([0, 0, 0, 0, 0, 0, 0, 0x80], np.uint8)
    assert list(oracle.blosc_filter(src, 2, 1, 8)) == [0, 0, 0, 0, 0, 0, 0, 0x80]
    # u16 element 0 = 0x0100 (byte 1 bit 0): row 8 = 0x01
    src = np.zeros(8, np.uint16)
    src[0] = 0x0100
    got = oracle.blosc_filter(src, 2, 2, 16)
    assert list(got) == [0] * 8 + [1] + [0] * 7
    # 7 elements (not a multiple of 8): the block is copied unchanged
    src = np.arange(14, dtype=np.uint8)
    assert list(oracle.blosc_filter(src, 2, 2, 14)) == list(src)
    # blocksize < typesize: no bit shuffle (blosc_c's blocksize >= typesize)
    src = np.arange(3, dtype=np.uint8)
    assert list(oracle.blosc_filter(src, 2, 4, 3)) == list(src)


@pytest.mark.parametrize("ts", [1, 2, 3, 4, 8, 16])
@pytest.mark.parametrize("shuffle", [0, 1, 2])
def test_filters_match_published_layout(oracle, ts, shuffle):
    rng = np.random.default_rng(ts * 10 + shuffle)
    for bs, n in [(64, 64), (128, 1000), (96, 96 * 5 + 13), (4096, 4096 * 3),
                  (8 * ts * 3, 8 * ts * 7 + ts * 3), (1000, 999)]:
        buf = rng.integers(0, 256, n, dtype=np.uint8)
        got = oracle.blosc_filter(buf, shuffle, ts, bs)
        assert np.array_equal(got, np_filter(buf, shuffle, ts, bs)), (bs, n)
        assert np.array_equal(oracle.blosc_unfilter(got, shuffle, ts, bs), buf), (bs, n)
