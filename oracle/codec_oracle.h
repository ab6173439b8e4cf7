/*
 * codec_oracle.h — CPU ORACLE for the blosc shuffle filters and crc32c
 * (SURVEY §8(f) rows 3-4).  TEST INFRASTRUCTURE ONLY; see codec_oracle.c for
 * the third-party algorithms restated and what pins them.
 */
#ifndef CODEC_ORACLE_H
#define CODEC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C"
{
#endif

void oracle_blosc_shuffle_block(uint32_t typesize, uint32_t blocksize, const uint8_t* src,
                                uint8_t* dst);
void oracle_blosc_unshuffle_block(uint32_t typesize, uint32_t blocksize, const uint8_t* src,
                                  uint8_t* dst);
/* tmp: blocksize bytes of scratch */
void oracle_blosc_bitshuffle_block(uint32_t typesize, uint32_t blocksize, const uint8_t* src,
                                   uint8_t* dst, uint8_t* tmp);
void oracle_blosc_unbitshuffle_block(uint32_t typesize, uint32_t blocksize, const uint8_t* src,
                                     uint8_t* dst);

/*
 * The bytes c-blosc hands its codec for each block of an `nbytes` buffer
 * (blosc_c's filter step, shuffle = BLOSC_NOSHUFFLE 0 / BLOSC_SHUFFLE 1 /
 * BLOSC_BITSHUFFLE 2), written block by block into dst; tmp holds
 * `blocksize` bytes of scratch.  Returns 0 / -1.
 */
int oracle_blosc_filter(int shuffle, uint32_t typesize, uint32_t blocksize, const void* src,
                        size_t nbytes, void* dst, void* tmp);
/* Inverse of oracle_blosc_filter (blosc_d's unshuffle step). */
int oracle_blosc_unfilter(int shuffle, uint32_t typesize, uint32_t blocksize,
                          const void* src, size_t nbytes, void* dst);

/* CRC-32C (Castagnoli), as crc32c::Crc32c. */
uint32_t oracle_crc32c(const void* data, size_t n);

/* Shard::write_table_ (shard.cpp:145-166): out = 16*n_chunks + 4 bytes. */
void oracle_shard_index_table(const uint64_t* offsets, const uint64_t* extents,
                              size_t n_chunks, uint8_t* out);

#ifdef __cplusplus
}
#endif

#endif
