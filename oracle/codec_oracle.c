/*
 * codec_oracle.c — CPU ORACLE for the byte-level codecs next to the
 * downsampler path.  TEST INFRASTRUCTURE ONLY:
 * loaded by tests/ and bench.py's cpu_baseline legs, never by the product.
 *
 * Both algorithms live in third-party dependencies that are absent from
 * /root/reference, so they are restated from their published definitions and
 * anchored on the reference's call sites:
 *
 *  - blosc shuffle filters: c-blosc, pinned `blosc >= 1.21.5` by
 *    vcpkg.json.  The reference calls blosc_compress_ctx(clevel, shuffle,
 *    typesize = bytes_of_type, nbytes, ..., blocksize = 0, nthreads = 1) from
 *    compress_in_place (zarr.common.cpp:106-137) on every chunk buffer
 *    (chunk.cpp:78-105).  c-blosc splits the buffer into blocks and, in
 *    blosc_c (blosc/blosc.c), filters each block before the codec sees it:
 *      byte shuffle only when typesize > 1   (shuffle-generic.c: shuffle_generic)
 *      bit shuffle only when blocksize >= typesize (shuffle.c: bitshuffle, then
 *        bitshuffle-generic.c: bshuf_trans_bit_elem_scal = byte transpose,
 *        8x8 bit transpose per 8 bytes, bit-row transpose)
 *    The last block is the short leftover block, filtered with its own size.
 *  - crc32c: google/crc32c, pinned `crc32c >= 1.1.2`.  The reference calls
 *    crc32c::Crc32c(table, 16 * n_chunks) on each shard index table
 *    (shard.cpp:145-166).  CRC-32C is the Castagnoli CRC: reflected
 *    polynomial 0x82F63B78, initial value and final xor 0xFFFFFFFF
 *    (RFC 3720 §12.1, B.4).
 *
 * Parity: the filters are pinned by c-blosc itself — the image carries
 * c-blosc 1.21.0 (/opt/conda/lib/libblosc.so.1), and for incompressible data
 * it stores every split raw, i.e. exactly its filtered blocks, which equal
 * these functions' output (tests/test_blosc_frames.py, oracle/blosc_ref.py);
 * also by hand-derived vectors and an independent numpy formulation
 * (tests/test_oracle_codecs.py).  crc32c is pinned by the RFC 3720 B.4 test
 * vectors (google/crc32c is not in the image).
 */
#include "codec_oracle.h"

#include <string.h>

/* shuffle_generic: dest[j*neblock + i] = src[i*typesize + j]; the
 * blocksize % typesize tail is copied unshuffled. */
void
oracle_blosc_shuffle_block(uint32_t typesize, uint32_t blocksize, const uint8_t* src, uint8_t* dst)
{
    const uint32_t neblock = blocksize / typesize;
    const uint32_t rem = blocksize % typesize;
    for (uint32_t j = 0; j < typesize; ++j)
        for (uint32_t i = 0; i < neblock; ++i)
            dst[(size_t)j * neblock + i] = src[(size_t)i * typesize + j];
    memcpy(dst + (blocksize - rem), src + (blocksize - rem), rem);
}

void
oracle_blosc_unshuffle_block(uint32_t typesize, uint32_t blocksize, const uint8_t* src, uint8_t* dst)
{
    const uint32_t neblock = blocksize / typesize;
    const uint32_t rem = blocksize % typesize;
    for (uint32_t i = 0; i < neblock; ++i)
        for (uint32_t j = 0; j < typesize; ++j)
            dst[(size_t)i * typesize + j] = src[(size_t)j * neblock + i];
    memcpy(dst + (blocksize - rem), src + (blocksize - rem), rem);
}

/* The 8x8 bit-matrix transpose of bitshuffle's TRANS_BIT_8X8 (little
 * endian): bit (8r + c) of x moves to bit (8c + r). */
static uint64_t
trans_bit_8x8(uint64_t x)
{
    uint64_t t;
    t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
    x = x ^ t ^ (t << 7);
    t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
    x = x ^ t ^ (t << 14);
    t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
    x = x ^ t ^ (t << 28);
    return x;
}

/* bshuf_trans_bit_elem_scal over `size` elements (size % 8 == 0), written
 * as its three published passes. `tmp` holds size*typesize bytes. */
static void
bshuf_trans_bit_elem(const uint8_t* in, uint8_t* out, size_t size, uint32_t typesize, uint8_t* tmp)
{
    const size_t nbyte = size * typesize;
    const size_t nbyte_row = nbyte / 8;
    /* 1. byte transpose: out[j*size + i] = in[i*typesize + j] */
    for (size_t i = 0; i < size; ++i)
        for (uint32_t j = 0; j < typesize; ++j)
            out[j * size + i] = in[i * typesize + j];
    /* 2. bit transpose of every 8 bytes into 8 bit rows of nbyte/8 bytes */
    for (size_t ii = 0; ii < nbyte_row; ++ii) {
        uint64_t x;
        memcpy(&x, out + ii * 8, 8);
        x = trans_bit_8x8(x);
        for (int kk = 0; kk < 8; ++kk) {
            tmp[kk * nbyte_row + ii] = (uint8_t)x;
            x >>= 8;
        }
    }
    /* 3. bit-row transpose: 8 x typesize matrix of size/8-byte rows,
     * out[(j*8 + kk)] = tmp[(kk*typesize + j)] */
    const size_t row = size / 8;
    for (int kk = 0; kk < 8; ++kk)
        for (uint32_t j = 0; j < typesize; ++j)
            memcpy(out + ((size_t)j * 8 + kk) * row, tmp + ((size_t)kk * typesize + j) * row, row);
}

/* c-blosc 1.x bitshuffle(): whole groups of 8 elements are bit-transposed
 * and the blocksize % typesize tail copied; a block whose element count is
 * not a multiple of 8 is copied unchanged. */
void
oracle_blosc_bitshuffle_block(uint32_t typesize,
                              uint32_t blocksize,
                              const uint8_t* src,
                              uint8_t* dst,
                              uint8_t* tmp)
{
    const size_t size = blocksize / typesize;
    if (size % 8 == 0) {
        bshuf_trans_bit_elem(src, dst, size, typesize, tmp);
        const size_t off = size * typesize;
        memcpy(dst + off, src + off, blocksize - off);
    } else {
        memcpy(dst, src, blocksize);
    }
}

void
oracle_blosc_unbitshuffle_block(uint32_t typesize, uint32_t blocksize, const uint8_t* src, uint8_t* dst)
{
    const size_t size = blocksize / typesize;
    if (size % 8 != 0) {
        memcpy(dst, src, blocksize);
        return;
    }
    const size_t row = size / 8;
    for (size_t i = 0; i < size; ++i)
        for (uint32_t j = 0; j < typesize; ++j) {
            uint8_t v = 0;
            for (int b = 0; b < 8; ++b)
                v |= (uint8_t)(((src[((size_t)j * 8 + b) * row + i / 8] >> (i % 8)) & 1u) << b);
            dst[i * typesize + j] = v;
        }
    const size_t off = size * typesize;
    memcpy(dst + off, src + off, blocksize - off);
}

int
oracle_blosc_filter(int shuffle,
                    uint32_t typesize,
                    uint32_t blocksize,
                    const void* src,
                    size_t nbytes,
                    void* dst,
                    void* tmp)
{
    if (typesize == 0 || blocksize == 0 || shuffle < 0 || shuffle > 2)
        return -1;
    const uint8_t* s = (const uint8_t*)src;
    uint8_t* d = (uint8_t*)dst;
    for (size_t off = 0; off < nbytes; off += blocksize) {
        const uint32_t bs = (uint32_t)(nbytes - off < blocksize ? nbytes - off : blocksize);
        if (shuffle == 1 && typesize > 1)
            oracle_blosc_shuffle_block(typesize, bs, s + off, d + off);
        else if (shuffle == 2 && bs >= typesize)
            oracle_blosc_bitshuffle_block(typesize, bs, s + off, d + off, (uint8_t*)tmp);
        else
            memcpy(d + off, s + off, bs);
    }
    return 0;
}

int
oracle_blosc_unfilter(int shuffle,
                      uint32_t typesize,
                      uint32_t blocksize,
                      const void* src,
                      size_t nbytes,
                      void* dst)
{
    if (typesize == 0 || blocksize == 0 || shuffle < 0 || shuffle > 2)
        return -1;
    const uint8_t* s = (const uint8_t*)src;
    uint8_t* d = (uint8_t*)dst;
    for (size_t off = 0; off < nbytes; off += blocksize) {
        const uint32_t bs = (uint32_t)(nbytes - off < blocksize ? nbytes - off : blocksize);
        if (shuffle == 1 && typesize > 1)
            oracle_blosc_unshuffle_block(typesize, bs, s + off, d + off);
        else if (shuffle == 2 && bs >= typesize)
            oracle_blosc_unbitshuffle_block(typesize, bs, s + off, d + off);
        else
            memcpy(d + off, s + off, bs);
    }
    return 0;
}

/* Bitwise reflected CRC-32C, one byte at a time (no tables: the definition). */
uint32_t
oracle_crc32c(const void* data, size_t n)
{
    const uint8_t* p = (const uint8_t*)data;
    uint32_t crc = 0xFFFFFFFFu;
    for (size_t i = 0; i < n; ++i) {
        crc ^= p[i];
        for (int k = 0; k < 8; ++k)
            crc = (crc >> 1) ^ (0x82F63B78u & (0u - (crc & 1u)));
    }
    return crc ^ 0xFFFFFFFFu;
}

/* Shard::write_table_ (shard.cpp:145-166): n_chunks (offset, extent) u64
 * pairs followed by their crc32c, little endian. */
void
oracle_shard_index_table(const uint64_t* offsets,
                         const uint64_t* extents,
                         size_t n_chunks,
                         uint8_t* out)
{
    for (size_t i = 0; i < n_chunks; ++i) {
        memcpy(out + 16 * i, &offsets[i], 8);
        memcpy(out + 16 * i + 8, &extents[i], 8);
    }
    const uint32_t crc = oracle_crc32c(out, 16 * n_chunks);
    memcpy(out + 16 * n_chunks, &crc, 4);
}
