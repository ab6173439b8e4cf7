/*
 * aqz_blosc.h — c-blosc 1.x chunk frames around the GPU byte/bit shuffle
 * (widened to the whole call it feeds).  Same library
 * (libaqz_downsampler.so) and status codes as aqz_downsampler.h.
 *
 * The reference compresses every chunk buffer with
 *   blosc_compress_ctx(clevel, shuffle, typesize = bytes_of_type, nbytes,
 *                      src, dest, destsize = nbytes + BLOSC_MAX_OVERHEAD,
 *                      cname = "lz4" | "zstd", blocksize = 0, nthreads = 1)
 * in compress_in_place (zarr.common.cpp:106-137), called per chunk from
 * Chunk::compress_and_take_buffer (chunk.cpp:78-105); the codec names come
 * from blosc.compression.params.cpp:5-13 and zarr.stream.cpp:115-118.
 *
 * Here the filter stage (the HBM-bound part) runs on the GPU
 * (aqz_blosc_filter_device) and the entropy coder stays on the host: LZ4
 * (LZ4_compress_fast) or zstd (ZSTD_compress), from the same shared
 * libraries c-blosc links (see aqz_blosc_codec_info).  The frames are
 * byte-identical to c-blosc 1.21's: header, block starts, per-split
 * compressed sizes, raw splits for incompressible ones, and the whole-buffer
 * memcpy fallback.  tests/test_blosc_frames.py checks that against the
 * image's libblosc 1.21.0 itself.
 */
#ifndef AQZ_BLOSC_H
#define AQZ_BLOSC_H

#include "aqz_codec.h"

#ifdef __cplusplus
extern "C"
{
#endif

/* BLOSC_MAX_OVERHEAD: the frame header; a destination of nbytes + this
 * always fits (the memcpy fallback). */
#define AQZ_BLOSC_MAX_OVERHEAD 16

/*
 * The block size blosc_compress_ctx picks for (clevel, typesize, nbytes,
 * cname) with blocksize = 0 — c-blosc's compute_blocksize, the value
 * aqz_blosc_filter_device needs.  typesize > 255 counts as 1, as in c-blosc.
 * AQZ_INVALID_ARGUMENT for clevel outside 0..9, typesize 0, an unknown
 * cname (only "lz4" and "zstd", the reference's two) or a null pointer.
 */
int aqz_blosc_blocksize(int clevel,
                        uint32_t typesize,
                        size_t nbytes,
                        const char* cname,
                        uint32_t* blocksize);

/*
 * Host frame writer.  `filtered` holds the `nbytes` chunk already filtered
 * block by block (aqz_blosc_filter_device with aqz_blosc_blocksize's block
 * size, copied to host).  Writes the c-blosc frame blosc_compress_ctx would
 * write for the unfiltered chunk into dest[0, destsize) and sets
 * *frame_bytes (0: it does not fit, c-blosc's return value 0).
 * When c-blosc would store the chunk unfiltered (clevel 0, nbytes < 128, or
 * incompressible as a whole) the frame is the 16-byte header plus the raw
 * chunk: `src` (host, may be NULL) supplies it; with `src` NULL only the
 * header is written, *raw_needed is set to 1 and the caller copies the
 * nbytes raw bytes to dest + 16 itself (e.g. straight from the device).
 * `raw_needed` may be NULL when `src` is given.
 */
int aqz_blosc_frame_from_filtered(int clevel,
                                  int shuffle,
                                  uint32_t typesize,
                                  const char* cname,
                                  const void* filtered,
                                  const void* src,
                                  size_t nbytes,
                                  void* dest,
                                  size_t destsize,
                                  size_t* frame_bytes,
                                  int* raw_needed);

/* Device scratch, pinned staging and host worker threads for
 * aqz_blosc_compress_device.  n_threads 0: min(16, hardware threads).
 * A ctx serves one call at a time: its scratch is shared by every call on
 * it, so two threads must not use one ctx concurrently (one ctx per thread,
 * as the reference's compression jobs would hold one each). */
typedef struct aqz_blosc_ctx aqz_blosc_ctx;

int aqz_blosc_ctx_create(int device, uint32_t n_threads, aqz_blosc_ctx** out);
void aqz_blosc_ctx_destroy(aqz_blosc_ctx* ctx);

/*
 * compress_in_place for `n_buffers` device chunk buffers of `nbytes` each,
 * back to back at `device_src` (e.g. the tiles aqz_ds_run_device_batch_tiled
 * or aqz_ds_take_frame_tiled lay out).  The filter runs on `hip_stream`, the
 * filtered chunks cross PCIe in groups, and host threads compress each group
 * while the next one is in flight.  Frame k is written at
 * host_dst + k * dst_stride (dst_stride >= nbytes + AQZ_BLOSC_MAX_OVERHEAD,
 * so every frame fits, as compress_in_place sizes it) and its size to
 * frame_bytes[k].  Chunks c-blosc would store unfiltered are copied raw from
 * the device.  Returns when every frame is written.
 */
int aqz_blosc_compress_device(aqz_blosc_ctx* ctx,
                              int clevel,
                              int shuffle,
                              uint32_t typesize,
                              const char* cname,
                              const void* device_src,
                              size_t nbytes,
                              uint32_t n_buffers,
                              void* host_dst,
                              size_t dst_stride,
                              size_t* frame_bytes,
                              void* hip_stream);

/* Which LZ4 and zstd libraries the frame writer loaded, with versions
 * ("" entries for a codec that failed to load).  $AQZ_LZ4_LIB and
 * $AQZ_ZSTD_LIB name them explicitly. */
const char* aqz_blosc_codec_info(void);

#ifdef __cplusplus
}
#endif

#endif
