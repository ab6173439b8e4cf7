/*
 * ds_oracle.h — CPU ORACLE for the multiscale downsampler.
 *
 * TEST INFRASTRUCTURE ONLY.  This is a plain-C restatement of the reference
 * algorithm in acquire-zarr v0.8.1 `src/streaming/downsampler.cpp`, used as
 * the parity checker by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg.  The product (acquire-zarr_amd/) never links or calls it.
 *
 * Parity status: pinned by the reference's own known-answer tests
 * (tests/unit-tests/downsampler.cpp, downsampler-odd-z.cpp) and the pixel
 * expectations of python/tests/test_stream.py, restated as fixtures under
 * tests/golden/; the chunk addressing by the 203 assertions of the
 * reference's tests/unit-tests/array-dimensions-*.cpp.  Since round 4 it is
 * also pinned by the REFERENCE ITSELF: oracle/_ref (downsampler.cpp compiled
 * unmodified, `make -C oracle ref`) made tests/golden/reference_vectors.* and
 * reference_digests.json, which this oracle reproduces byte for byte, and is
 * fuzzed against it live (tests/test_reference_pin.py); see DESIGN.md §3.
 */
#ifndef DS_ORACLE_H
#define DS_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C"
{
#endif

typedef struct
{
    int32_t type; /* ZarrDimensionType value */
    uint32_t array_size_px;
    uint32_t chunk_size_px;
    uint32_t shard_size_chunks;
    double scale;
} oracle_dim;

/* bytes_of_type (zarr.common.cpp:48-69); 0 for an invalid dtype. */
size_t oracle_bytes_of_type(int dtype);

/*
 * scale_image<T> (downsampler.cpp:139-206): one 2x2 reduction of a w x h
 * row-major frame into ceil(w/2) x ceil(h/2), odd edges replicated.
 * Returns 0 on success, -1 on invalid dtype/method.
 */
int oracle_scale_image(int dtype,
                       int method,
                       const void* src,
                       size_t width,
                       size_t height,
                       void* dst);

/*
 * average_two_frames<T> (downsampler.cpp:208-246): dst[i] = f(dst[i], src[i])
 * over n pixels; dst holds the earlier plane, src the current one.
 */
int oracle_average_two_frames(int dtype,
                              int method,
                              void* dst,
                              const void* src,
                              size_t n_pixels);

/* The scalar reducers, exposed for known-answer tests on single values.
 * a,b,c,d point at one element each of the dtype; result written to out. */
int oracle_reduce4(int dtype,
                   int method,
                   const void* a,
                   const void* b,
                   const void* c,
                   const void* d,
                   void* out);
int oracle_reduce2(int dtype,
                   int method,
                   const void* a,
                   const void* b,
                   void* out);

/*
 * make_writer_configurations_ (downsampler.cpp:493-597) with
 * downsample_dimension (downsampler.cpp:8-37).  Same contract as
 * aqz_plan_levels in include/aqz_downsampler.h.  Returns 0 / -1 / -2 (cap).
 */
int oracle_plan_levels(const oracle_dim* dims,
                       uint32_t ndims,
                       uint32_t max_levels,
                       oracle_dim* out,
                       uint32_t out_cap_levels,
                       uint32_t* n_levels);

/*
 * Chunk tiling of one frame (§8(f) row 2 oracle): restates
 * Array::write_frame_to_chunks_ (array.cpp:507-622) and
 * Chunk::write_tile_rows (chunk.cpp:17-58) for one row-major frame, written
 * into a zeroed tile-major buffer — tile t = ty*n_tiles_x + tx at
 * t*tile_rows*tile_cols*bpp, rows at tile_cols*bpp — exactly the bytes the
 * reference leaves in each chunk buffer's tile slot.  `nonzero[t]` is the
 * chunk zero scan (any copied byte != 0).  Returns 0 / -1.
 */
int oracle_tile_frame(int dtype,
                      const void* src,
                      uint32_t width,
                      uint32_t height,
                      uint32_t tile_rows,
                      uint32_t tile_cols,
                      void* dst,
                      uint8_t* nonzero);

/*
 * transpose_frame (array.cpp:488-504): the src_rows x src_cols row-major frame
 * transposed into dst (src_cols x src_rows).  Returns 0 / -1.
 */
int oracle_transpose_frame(int dtype,
                           const void* src,
                           uint32_t src_rows,
                           uint32_t src_cols,
                           void* dst);

/*
 * Chunk addressing restated from ArrayDimensions (array.dimensions.cpp:
 * 232-314) over storage-order dims (ndims >= 3, the last two Y and X):
 * chunk_lattice_index (UINT32_MAX on a bad dim index), tile_group_offset (in
 * chunks) and chunk_internal_offset (in bytes).
 */
uint32_t oracle_chunk_lattice_index(const oracle_dim* dims,
                                    uint32_t ndims,
                                    uint64_t frame_id,
                                    uint32_t dim_index);
uint64_t oracle_tile_group_offset(const oracle_dim* dims,
                                  uint32_t ndims,
                                  uint64_t frame_id);
uint64_t oracle_chunk_internal_offset(const oracle_dim* dims,
                                      uint32_t ndims,
                                      uint32_t bytes_per_px,
                                      uint64_t frame_id);

/* Stateful downsampler: Downsampler::add_frame / take_frame
 * (downsampler.cpp:306-414) over per-level (width, height, planes). */
typedef struct oracle_ds oracle_ds;

oracle_ds* oracle_ds_create(const uint32_t* widths,
                            const uint32_t* heights,
                            const uint32_t* planes,
                            uint32_t n_levels,
                            int dtype,
                            int method);
void oracle_ds_destroy(oracle_ds* ds);
/* Returns 0, or -1 on a size mismatch (the reference EXPECT throws). */
int oracle_ds_add_frame(oracle_ds* ds, const void* frame, size_t nbytes);
/* Returns 1 and copies the cached level frame (removing it) if present,
 * 0 if absent, -1 on a bad level or too-small buffer. */
int oracle_ds_take_frame(oracle_ds* ds,
                         uint32_t level,
                         void* dst,
                         size_t cap,
                         size_t* nbytes);
/* Frames emitted so far at `level` (level_frame_count_). */
uint32_t oracle_ds_level_count(const oracle_ds* ds, uint32_t level);

#ifdef __cplusplus
}
#endif

#endif
