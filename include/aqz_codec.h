/*
 * aqz_codec.h — byte-level codec stages on MI355X next to the multiscale
 * downsampler.  Same library
 * (libaqz_downsampler.so) and status codes as aqz_downsampler.h.
 *
 * Both entry points work on device buffers and queue work on a HIP stream
 * without synchronising.  They reproduce third-party algorithms the
 * reference calls (c-blosc's shuffle filters, google/crc32c); the CPU
 * restatement they are tested against is oracle/codec_oracle.c.
 */
#ifndef AQZ_CODEC_H
#define AQZ_CODEC_H

#include "aqz_downsampler.h"

#ifdef __cplusplus
extern "C"
{
#endif

/* BloscCompressionParams::shuffle values (c-blosc's BLOSC_NOSHUFFLE,
 * BLOSC_SHUFFLE, BLOSC_BITSHUFFLE; validated in zarr.stream.cpp:127-136). */
enum
{
    AQZ_BLOSC_NOSHUFFLE = 0,
    AQZ_BLOSC_SHUFFLE = 1,
    AQZ_BLOSC_BITSHUFFLE = 2
};

/*
 * The filter step c-blosc applies to every block of a chunk buffer before
 * its codec (blosc_c in c-blosc 1.x, reached from compress_in_place,
 * zarr.common.cpp:106-137, with typesize = bytes per pixel, for every chunk
 * in Chunk::compress_and_take_buffer, chunk.cpp:78-105).  `n_buffers`
 * buffers of `nbytes` each lie back to back at `device_src` (e.g. the
 * chunk-depth-1 tiles aqz_ds_take_frame_tiled lays out); each is split into
 * `blocksize` blocks, the last one shorter, and every block is written to
 * the same offset of `device_dst` as
 *   AQZ_BLOSC_SHUFFLE, typesize > 1:   byte planes (shuffle_generic), the
 *                                      blocksize % typesize tail copied;
 *   AQZ_BLOSC_BITSHUFFLE, block >= typesize: bit rows (bshuf_trans_bit_elem)
 *                                      when the element count is a multiple
 *                                      of 8, the tail copied; else copied;
 *   otherwise:                         copied.
 * `blocksize` is the one c-blosc chose for the chunk (it depends only on
 * clevel, typesize, nbytes and the codec; blosc_cbuffer_sizes reports it
 * for any compressed chunk).  Returns AQZ_INVALID_ARGUMENT for typesize 0,
 * blocksize 0, an unknown shuffle or n_buffers 0.
 */
int aqz_blosc_filter_device(int shuffle,
                            uint32_t typesize,
                            uint32_t blocksize,
                            const void* device_src,
                            size_t nbytes,
                            uint32_t n_buffers,
                            void* device_dst,
                            void* hip_stream);

/*
 * crc32c::Crc32c (CRC-32C, Castagnoli) of `n_buffers` device buffers of
 * `nbytes`, buffer k at device_data + k * stride, into device_crcs[k] — the
 * checksum Shard::write_table_ appends to each shard index table
 * (shard.cpp:145-166).
 */
int aqz_crc32c_device(const void* device_data,
                      size_t nbytes,
                      size_t stride,
                      uint32_t n_buffers,
                      uint32_t* device_crcs,
                      void* hip_stream);

#ifdef __cplusplus
}
#endif

#endif
