/*
 * aqz_downsampler.h — C ABI of the MI355X-native multiscale pyramid
 * downsampler (the acquire-zarr streaming hot path).
 *
 * This header is the drop-in boundary.  It replaces the CPU implementation of
 * `zarr::Downsampler` in the reference
 * (`src/streaming/downsampler.{hh,cpp}`, v0.8.1).  The `zarr::Downsampler`
 * class contract (downsampler.hh:11-64) is kept by a thin C++ adapter
 *  that forwards to the functions below.  Nothing else in the
 * reference changes: `MultiscaleArray` (multiscale.array.cpp:172-189,
 * 291-325) keeps calling add_frame/take_frame, and the public
 * `ZarrStream_*` / `ZarrStreamSettings` surface in include/acquire.zarr.h is
 * untouched.
 *
 * Plain C: no C++ or HIP types cross this boundary.  Streams are passed as
 * `void*` (a hipStream_t).  Enum-valued arguments take the numeric values of
 * the reference's `ZarrDataType`, `ZarrDownsamplingMethod` and
 * `ZarrDimensionType` (include/zarr.types.h:55-97); return values are
 * `ZarrStatusCode` values (zarr.types.h:13-31).
 *
 * Threading: a handle is used by one thread at a time, exactly like the
 * reference Downsampler, which only the stream's frame-queue consumer job
 * touches (zarr.stream.cpp:1616-1630).  Every entry point binds the handle's
 * device first (hipSetDevice), because that consumer thread is not the thread
 * that created the handle.
 */
#ifndef AQZ_DOWNSAMPLER_H
#define AQZ_DOWNSAMPLER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C"
{
#endif

/* Status codes: numerically equal to ZarrStatusCode (zarr.types.h:13-31). */
#define AQZ_OK 0
#define AQZ_INVALID_ARGUMENT 1
#define AQZ_OVERFLOW 2
#define AQZ_INVALID_INDEX 3
#define AQZ_NOT_YET_IMPLEMENTED 4
#define AQZ_INTERNAL_ERROR 5
#define AQZ_OUT_OF_MEMORY 6

/* ZarrDataType values (zarr.types.h:55-68). */
#define AQZ_DTYPE_UINT8 0
#define AQZ_DTYPE_UINT16 1
#define AQZ_DTYPE_UINT32 2
#define AQZ_DTYPE_UINT64 3
#define AQZ_DTYPE_INT8 4
#define AQZ_DTYPE_INT16 5
#define AQZ_DTYPE_INT32 6
#define AQZ_DTYPE_INT64 7
#define AQZ_DTYPE_FLOAT32 8
#define AQZ_DTYPE_FLOAT64 9
#define AQZ_DTYPE_COUNT 10

/* ZarrDownsamplingMethod values (zarr.types.h:90-97). */
#define AQZ_METHOD_DECIMATE 0
#define AQZ_METHOD_MEAN 1
#define AQZ_METHOD_MIN 2
#define AQZ_METHOD_MAX 3
#define AQZ_METHOD_COUNT 4

/* ZarrDimensionType values (zarr.types.h:81-88). */
#define AQZ_DIM_SPACE 0
#define AQZ_DIM_CHANNEL 1
#define AQZ_DIM_TIME 2
#define AQZ_DIM_OTHER 3

/* Upper bounds for the fixed-size tables below. */
#define AQZ_MAX_DIMS 32
#define AQZ_MAX_LEVELS 32

/*
 * One dimension of one pyramid level, in storage order.  Mirrors the numeric
 * fields of the reference's `ZarrDimension` (array.dimensions.hh:12-43); the
 * name and unit strings stay with the caller, since the planner only copies
 * them.
 */
typedef struct
{
    int32_t type;               /* ZarrDimensionType */
    uint32_t array_size_px;     /* 0 = unbounded append dimension */
    uint32_t chunk_size_px;
    uint32_t shard_size_chunks;
    double scale;
} aqz_dimension;

/*
 * Geometry of one pyramid level as the per-frame state machine needs it.
 * Derived from the level's dimensions: `width` = last dim, `height` =
 * second-to-last, `planes` = dim[ndims-3] (downsampler.cpp:311-333).
 */
typedef struct
{
    uint32_t width;
    uint32_t height;
    uint32_t planes;
} aqz_level_desc;

/*
 * Level planner: restates `Downsampler::make_writer_configurations_`
 * (downsampler.cpp:493-597) and `downsample_dimension` (downsampler.cpp:8-37).
 *
 * `dims` are the base (level-0) dimensions in storage order, already carrying
 * the phantom singleton dimension the reference prepends to 2-D arrays
 * (array.dimensions.cpp:149-152), so ndims >= 3.  `max_levels` = 0 means no
 * limit (ArrayConfig::max_levels, array.base.hh:56).
 *
 * Writes `*n_levels` (total levels including level 0) and, if `out` is
 * non-NULL, `out[level * ndims + d]` for every level.  `out_cap_levels` is the
 * number of levels `out` has room for; AQZ_OVERFLOW if too small.
 */
int aqz_plan_levels(const aqz_dimension* dims,
                    uint32_t ndims,
                    uint32_t max_levels,
                    aqz_dimension* out,
                    uint32_t out_cap_levels,
                    uint32_t* n_levels);

/* Opaque downsampler handle: the device-side replacement of zarr::Downsampler. */
typedef struct aqz_ds aqz_ds;

/*
 * Create a downsampler for `n_levels` levels (level 0 = full resolution).
 * Replaces the constructor `Downsampler(config, method)` (downsampler.cpp:
 * 249-304): dtype and method are validated here.  `device` is the HIP
 * ordinal; -1 selects $AQZ_GPU_DEVICE or else the current device.
 * $AQZ_GPU_DEVICE=spread gives each new handle the next visible GPU in turn,
 * so the multiscale arrays of one process spread over a node's GPUs (their
 * frames are independent: no collective).  An ordinal that names no visible
 * device is AQZ_INVALID_ARGUMENT.
 * Allocates the level-0 frame, two slots per level and the stored Z planes
 * on the device up front; pinned memory only for the eager readback of small
 * pyramids and for $AQZ_PINNED_STAGING=1.  Tile scratch, the host-batch
 * pipeline and the upload thread are allocated on first use.
 */
int aqz_ds_create(const aqz_level_desc* levels,
                  uint32_t n_levels,
                  int dtype,
                  int method,
                  int device,
                  aqz_ds** out);

/* Release every device/pinned buffer, stream and event of the handle. */
void aqz_ds_destroy(aqz_ds* ds);

/*
 * Add one full-resolution frame from host memory.  Replaces
 * `Downsampler::add_frame` (downsampler.cpp:306-401): same level cascade, Z
 * pairing, odd-plane pass-through and emit/no-overwrite rules.
 * `nbytes` must equal width*height*bytes_of_type at level 0.
 * The host buffer is read only during the call: it is uploaded straight from
 * the caller's (pageable) memory and the call returns once that upload has
 * completed ($AQZ_PINNED_STAGING=1: staged through a pinned buffer instead),
 * so the caller may reuse it immediately.
 * Kernels and device->host copies are queued asynchronously; the level
 * frames are synchronised in aqz_ds_take_frame.
 */
int aqz_ds_add_frame(aqz_ds* ds, const void* host_frame, size_t nbytes);

/*
 * aqz_ds_add_frame without waiting: validates the size,
 * hands the frame to the handle's upload thread and returns at once, so the
 * caller can chunk the same frame into its level-0 array
 * (`MultiscaleArray::write_frame`, multiscale.array.cpp:57-74, runs
 * `arrays_[0]->write_frame` before `write_multiscale_frames_`) while it
 * crosses PCIe and the pyramid is queued.  `host_frame` must stay valid and
 * unmodified until aqz_ds_wait returns.  Every other call on the handle
 * (except the size queries and aqz_ds_last_error) waits for the pending frame
 * first and, if its add failed, returns that status instead of doing its own
 * work.  At most one frame is pending: a second aqz_ds_add_frame_async waits
 * for the first.
 */
int aqz_ds_add_frame_async(aqz_ds* ds, const void* host_frame, size_t nbytes);

/*
 * Wait for the frame passed to aqz_ds_add_frame_async to be uploaded and its
 * pyramid queued; returns that add's status (AQZ_OK if nothing was pending).
 * After it returns the caller may reuse the frame buffer.
 */
int aqz_ds_wait(aqz_ds* ds);

/*
 * Non-blocking: *done = 1 when no aqz_ds_add_frame_async job is running (the
 * next aqz_ds_wait returns at once), 0 while one is.  Reports nothing else and
 * clears no status: the job's status is still aqz_ds_wait's to return.  No
 * reference counterpart; aqz_node_take_frame uses it to hand out levels as
 * soon as their add has finished.
 */
int aqz_ds_poll(aqz_ds* ds, int* done);

/*
 * Wait only until the pending aqz_ds_add_frame_async[_take] job no longer
 * reads its host frame (the upload is done, or the add failed): the caller
 * may then reuse or free that frame, while the pyramid and the takes may
 * still run.  Returns AQZ_OK (also when nothing is pending) and clears no
 * status: a failed add is still reported by aqz_ds_wait.  No reference
 * counterpart; aqz_node_wait_input is built on it.
 */
int aqz_ds_wait_input(aqz_ds* ds);

/*
 * Non-blocking aqz_ds_wait_input: *pending = 1 while the pending
 * aqz_ds_add_frame_async[_take] job may still read its host frame, 0 once the
 * caller may reuse it (or nothing is pending).  Clears no status.  No
 * reference counterpart; aqz_node_inputs_released is built on it.
 */
int aqz_ds_input_pending(aqz_ds* ds, int* pending);

/*
 * One level's part in aqz_ds_add_frame_async_take.
 *   mode AQZ_TAKE_NONE: nothing (the level is taken later, or not at all);
 *   AQZ_TAKE_INTO: right behind the add, take the level's frame if it has
 *     one — chunk-tiled into `dst` like aqz_ds_take_frame_tiled when
 *     tile_rows/tile_cols are nonzero (`tile_nonzero` optional), row-major
 *     like aqz_ds_take_frame when both are 0 — and report has_frame/nbytes;
 *     `dst` must hold the level's whole (tiled) frame, checked before the job
 *     is queued (AQZ_INVALID_ARGUMENT otherwise, nothing queued);
 *   AQZ_TAKE_HOLD: the caller still holds an untaken frame of this level
 *     from an earlier INTO take, so this add's frame at the level is dropped,
 *     as Downsampler::emplace_downsampled_frame_ drops a frame while one is
 *     cached (downsampler.cpp:599-605).
 */
#define AQZ_TAKE_NONE 0
#define AQZ_TAKE_INTO 1
#define AQZ_TAKE_HOLD 2
typedef struct
{
    int mode;
    uint32_t tile_rows, tile_cols;
    void* dst;
    size_t cap;
    uint8_t* tile_nonzero;
    size_t nbytes;  /* out */
    int has_frame;  /* out */
} aqz_level_take;

/*
 * aqz_ds_add_frame_async plus, in the same background job, the takes
 * MultiscaleArray::write_multiscale_frames_ makes right after add_frame
 * (multiscale.array.cpp:298-325): `takes[L]` for every level L >= 1 (index 0
 * ignored).  The levels' device-to-host copies then overlap the caller's own
 * work as the upload does.  `host_frame`, `takes` and every buffer they name
 * must stay valid until aqz_ds_wait returns; the outputs are valid once it
 * has returned AQZ_OK.  Same results as aqz_ds_add_frame followed by the
 * takes.  aqz_ds_add_frame, _add_frame_async and _add_device_frame end any
 * hold.
 */
int aqz_ds_add_frame_async_take(aqz_ds* ds,
                                const void* host_frame,
                                size_t nbytes,
                                aqz_level_take* takes);

/*
 * Transposed storage order (`transpose_frame`,
 * array.cpp:488-504).  When the array's storage_dimension_order swaps Y and X
 * (`ArrayDimensions::needs_xy_transposition`, array.dimensions.cpp:563-576),
 * `Array::write_frame_to_chunks_` transposes each level-0 frame before
 * chunking it (array.cpp:517-530) and, because it replaces the caller's
 * frame, the downsampler is fed the transposed frame.  With `transpose` = 1
 * the handle takes frames in ACQUISITION order — `levels[0].width` rows of
 * `levels[0].height` pixels (acquisition_frame_rows/cols,
 * array.dimensions.cpp:578-599) — and transposes them on the GPU before the
 * pyramid, so the level geometry stays in storage order, as the reference
 * plans it.  Applies to add_frame, add_frame_async and add_device_frame; the
 * batch entry points return AQZ_INVALID_ARGUMENT while it is set.
 */
int aqz_ds_set_input_transpose(aqz_ds* ds, int transpose);

/*
 * The last level-0 frame added, in storage order (transposed if input
 * transposition is on), copied to `dst`: chunk-tiled like
 * aqz_ds_take_frame_tiled when tile_rows/tile_cols are nonzero (the level-0
 * half of `Array::write_frame_to_chunks_`, array.cpp:507-622, with the zero
 * scan in `tile_nonzero`), or the plain row-major frame when both are 0.
 * One-shot: *has_frame = 0 if no frame was added since the last take (or a
 * batch ran since).  `dst` == NULL reports *nbytes only.  For
 * aqz_ds_add_device_frame without transposition the caller's device frame
 * is read, so it must still be valid.
 */
int aqz_ds_take_input_frame(aqz_ds* ds,
                            uint32_t tile_rows,
                            uint32_t tile_cols,
                            void* dst,
                            size_t cap,
                            uint8_t* tile_nonzero,
                            size_t* nbytes,
                            int* has_frame);

/*
 * `transpose_frame` (array.cpp:488-504) on the device: `device_dst`
 * (cols x rows) = transpose of `device_src` (rows x cols), both row-major of
 * `dtype`.  Queued on `hip_stream` (NULL = default stream), not synchronised.
 */
int aqz_transpose_frame_device(int dtype,
                               const void* device_src,
                               uint32_t rows,
                               uint32_t cols,
                               void* device_dst,
                               void* hip_stream);

/*
 * Same as aqz_ds_add_frame for a frame already resident in device memory
 * (`device_frame` is a device pointer on the handle's device).  The frame
 * must stay valid until the next call on the handle.
 */
int aqz_ds_add_device_frame(aqz_ds* ds, const void* device_frame, size_t nbytes);

/*
 * Take the cached frame of `level` (1..n_levels-1).  Replaces
 * `Downsampler::take_frame` (downsampler.cpp:403-414): if a frame is cached
 * it is copied into `dst` (capacity `cap` bytes), removed from the cache,
 * `*nbytes` is set and `*has_frame` = 1; otherwise `*has_frame` = 0 and
 * nothing is written.  Not idempotent.
 * With `dst` == NULL and has_frame, only `*nbytes` is reported and the frame
 * stays cached (size query).
 */
int aqz_ds_take_frame(aqz_ds* ds,
                      uint32_t level,
                      void* dst,
                      size_t cap,
                      size_t* nbytes,
                      int* has_frame);

/*
 * Chunk-tiled take.  Same as aqz_ds_take_frame, but the
 * frame arrives in the tile order Array::write_frame_to_chunks_ consumes
 * (array.cpp:507-622): tile t = ty*n_tiles_x + tx holds tile_rows x
 * tile_cols pixels row-major, zero-padded where it overhangs the frame —
 * exactly the bytes Chunk::write_tile_rows (chunk.cpp:17-58) leaves in the
 * chunk's tile slot, so each tile is ONE contiguous copy into its chunk
 * buffer.  `tile_nonzero` (optional, n_tiles bytes) receives the chunk zero
 * scan (1 = some copied byte is nonzero).  `*nbytes` = n_tiles * tile_rows *
 * tile_cols * bytes_of_type; dst == NULL is a size query (frame stays).
 */
int aqz_ds_take_frame_tiled(aqz_ds* ds,
                            uint32_t level,
                            uint32_t tile_rows,
                            uint32_t tile_cols,
                            void* dst,
                            size_t cap,
                            uint8_t* tile_nonzero,
                            size_t* nbytes,
                            int* has_frame);

/*
 * Declare level `level`'s chunk tile (its chunk_size_px in y and x — chunks
 * are preserved across levels, downsampler.cpp:16-17).  From then on every
 * frame that becomes the level's cached frame is also tiled on the GPU right
 * behind the pyramid kernels, so aqz_ds_take_frame_tiled with the same tile
 * is a plain device->host copy.  0, 0 switches it off.
 */
int aqz_ds_set_level_tiling(aqz_ds* ds,
                            uint32_t level,
                            uint32_t tile_rows,
                            uint32_t tile_cols);

/*
 * Chunk tiling of a device-resident W x H frame (same layout and scan as
 * aqz_ds_take_frame_tiled) into device memory `device_tiles`;
 * `device_nonzero` receives one uint32 per tile.  Runs on `hip_stream`
 * (NULL = default stream), asynchronous.  For the full-resolution level, whose
 * tiling the reference does on the host (array.cpp:575 OpenMP loop).
 */
int aqz_tile_frame_device(int dtype,
                          const void* device_frame,
                          uint32_t width,
                          uint32_t height,
                          uint32_t tile_rows,
                          uint32_t tile_cols,
                          void* device_tiles,
                          uint32_t* device_nonzero,
                          void* hip_stream);

/*
 * The same tiling with the zero scan split into slices, as the handle's
 * eager tiling runs it: `device_slice_flags` (device or host-mapped memory)
 * receives aqz_tile_slices(tile_rows, tile_cols) bytes per tile, tile-major,
 * each 0 or 1; tile t is nonzero iff any of its slice bytes is.  No
 * pre-clear and no atomics, so it is a single kernel launch.
 */
uint32_t aqz_tile_slices(uint32_t tile_rows, uint32_t tile_cols);
int aqz_tile_frame_device_sliced(int dtype,
                                 const void* device_frame,
                                 uint32_t width,
                                 uint32_t height,
                                 uint32_t tile_rows,
                                 uint32_t tile_cols,
                                 void* device_tiles,
                                 uint8_t* device_slice_flags,
                                 void* hip_stream);

/*
 * Device-resident batch path (benchmark / bulk API).  Equivalent to calling
 * aqz_ds_add_frame on `n_frames` consecutive frames of `device_frames`
 * (frame i at byte offset i*frame_bytes) followed by take_frame on every
 * level, except that nothing leaves the device: the k-th frame emitted at
 * level L is written to `device_out_levels[L] + k * level_bytes(L)`.
 * `device_out_levels[0]` is ignored.  `out_counts` (optional, n_levels
 * entries) receives the number of frames emitted per level.
 * Runs on `hip_stream` (NULL = the handle's own stream) and does not
 * synchronise; pure-2-D pyramids are one fused launch per 4 levels.
 */
int aqz_ds_run_device_batch(aqz_ds* ds,
                            const void* device_frames,
                            uint32_t n_frames,
                            void* const* device_out_levels,
                            uint32_t* out_counts,
                            void* hip_stream);

/*
 * Device-resident batch with every level emitted chunk-tiled by the pyramid
 * kernel itself: the k-th frame of level L is written to
 * `device_out_levels[L] + k * n_tiles(L) * tile_rows[L] * tile_cols[L] *
 * bytes_of_type` in the order Array::write_frame_to_chunks_ fills chunks
 * (array.cpp:507-622): tile t = ty * n_tiles_x + tx holds tile_rows[L] x
 * tile_cols[L] pixels row-major, zero where it overhangs the level — the
 * bytes Chunk::write_tile_rows (chunk.cpp:17-58) leaves in the tile's slot —
 * with n_tiles_x = ceil(width / tile_cols[L]) and n_tiles(L) = n_tiles_x *
 * ceil(height / tile_rows[L]).  `device_tile_nonzero[L]` (optional: the
 * array or any entry may be NULL) receives the chunk zero scan as
 * S = aqz_ds_tiled_flag_slots(ds, L, tile_rows[L], tile_cols[L]) flag bytes
 * per tile (tile-major, n_tiles(L) * S bytes per frame): a tile holds a
 * nonzero byte iff any of its S bytes is nonzero.  Index 0 of every array is
 * ignored.  One kernel per 4 levels writes the levels from registers — no
 * row-major pass, no tiling pass — and its trailing waves zero the tile
 * overhang; when S > 1 every flag byte is written once by the wave that owns
 * it, so nothing is cleared first (S == 1: one byte per tile, cleared by a
 * fill before the kernel).
 * Pure-XY (2-D) pyramids only, frames at least one 16-byte load wide (so
 * is the first level of every later fused run: levels 4, 8, ... of deeper
 * pyramids), no input transposition; anything else is AQZ_INVALID_ARGUMENT
 * (aqz_ds_run_device_batch takes any width).  Runs on
 * `hip_stream` (NULL = the handle's stream) without synchronising;
 * `out_counts` as for aqz_ds_run_device_batch.  Pyramids deeper than 4
 * levels chain runs through handle scratch, so each tiled/chunked batch is
 * ordered behind the handle's previous one whatever stream either ran on
 * (an event wait; no host synchronisation).  A handle is not thread-safe:
 * one caller thread at a time, as for zarr::Downsampler.
 */
int aqz_ds_run_device_batch_tiled(aqz_ds* ds,
                                  const void* device_frames,
                                  uint32_t n_frames,
                                  const uint32_t* tile_rows,
                                  const uint32_t* tile_cols,
                                  void* const* device_out_levels,
                                  uint8_t* const* device_tile_nonzero,
                                  uint32_t* out_counts,
                                  void* hip_stream);

/*
 * Flag bytes per tile that aqz_ds_run_device_batch_tiled writes for level
 * `level` with tile_rows x tile_cols tiles: S > 1 when the kernel's wave
 * blocks tile the chunk tiles exactly (one byte per block), else 1.  0 for a
 * bad level or tile shape.
 */
uint32_t aqz_ds_tiled_flag_slots(const aqz_ds* ds,
                                 uint32_t level,
                                 uint32_t tile_rows,
                                 uint32_t tile_cols);

/*
 * One level's chunk lattice in device memory: the chunk buffers of
 * Array::chunks_ (array.cpp:563-617), `chunk_stride_bytes` apart, so tile
 * t of frame k lands in chunk t + tile_group_offset(k) at
 * chunk_internal_offset(k) (array.dimensions.cpp:265-314).
 * `frame_offset_bytes` (host, n_frames entries) gives, per frame of the
 * batch, where its tile 0 goes: tile_group_offset * chunk_stride_bytes +
 * chunk_internal_offset, plus the layer's base when the buffer holds several
 * chunk layers (aqz_chunk_frame_offsets computes exactly that).
 */
typedef struct
{
    void* device_base;
    size_t capacity_bytes;        /* bytes at device_base: every tile must fit */
    uint32_t tile_rows, tile_cols; /* the level's XY chunk shape */
    size_t chunk_stride_bytes;    /* >= one tile; usually bytes_per_chunk */
    const uint64_t* frame_offset_bytes;
} aqz_chunk_lattice;

/*
 * aqz_ds_run_device_batch_tiled with every tile written straight into its
 * chunk buffer (SURVEY §8(f) row 2 up to whole chunks): `lattices[L]` per
 * level (index 0 ignored); the tiles, zero overhang and zero-scan flags are
 * those of the tiled batch (device_tile_nonzero as there: per frame, not per
 * chunk).  A frame whose tiles would leave the lattice buffer, an offset or
 * stride that is not a multiple of the pixel size, or a stride below one
 * tile is AQZ_INVALID_ARGUMENT before anything runs.  The offsets cross to
 * the device on `hip_stream` with the batch; the call returns without
 * synchronising, and `lattices` may be freed on return.
 */
int aqz_ds_run_device_batch_chunked(aqz_ds* ds,
                                    const void* device_frames,
                                    uint32_t n_frames,
                                    const aqz_chunk_lattice* lattices,
                                    uint8_t* const* device_tile_nonzero,
                                    uint32_t* out_counts,
                                    void* hip_stream);

/*
 * Where frames first_frame .. first_frame + n_frames - 1 of an array with
 * storage-order dimensions `dims` (ndims >= 3, the last two Y and X) put
 * their tile 0 in a lattice of chunk buffers `*chunk_bytes` apart:
 *   (layer(k) - layer(first_frame)) * *layer_bytes
 *     + tile_group_offset(k) * *chunk_bytes + chunk_internal_offset(k)
 * restating ArrayDimensions::chunk_lattice_index / tile_group_offset /
 * chunk_internal_offset (array.dimensions.cpp:232-314); *chunk_bytes =
 * bytes_per_chunk (every dim's chunk size x bytes_per_px), *layer_bytes =
 * the chunks of one append-dimension chunk layer (the buffer Array::chunks_
 * holds) x *chunk_bytes.  Frame ids are in storage order.
 */
int aqz_chunk_frame_offsets(const aqz_dimension* dims,
                            uint32_t ndims,
                            uint32_t bytes_per_px,
                            uint64_t first_frame,
                            uint32_t n_frames,
                            uint64_t* frame_offset_bytes,
                            uint64_t* chunk_bytes,
                            uint64_t* layer_bytes);

/*
 * Host-resident batch, pipelined (overlapping frames).
 * Same results as aqz_ds_add_frame + aqz_ds_take_frame(every level) on each
 * of `n_frames` consecutive frames of `host_frames`: the k-th frame emitted at
 * level L is written to `host_out_levels[L] + k * level_bytes(L)`
 * (`host_out_levels[0]` ignored; `out_counts` optional, n_levels entries).
 * Frames move in double-buffered groups on three streams — upload, kernels,
 * download — so both PCIe directions and the kernels overlap.  Pass pinned
 * (hipHostMalloc'd or registered) buffers for full overlap; pageable memory
 * works but serialises the copies.  Blocks until every level is on the host.
 */
int aqz_ds_run_host_batch(aqz_ds* ds,
                          const void* host_frames,
                          uint32_t n_frames,
                          void* const* host_out_levels,
                          uint32_t* out_counts);

/*
 * Diagnostic: the path the last aqz_ds_run_device_batch[_tiled] took —
 * 0 = per-frame state machine, 1 = fused 2-D cascade, 2 = fused volume
 * (XY + Z), 3 = 2-D batch with some level runs on batched single-level
 * kernels (frames narrower than one 16-byte load, or buffers that are not
 * element-aligned; the fused kernels take any other width and offset),
 * 4 = fused 2-D cascade writing chunk tiles (aqz_ds_run_device_batch_tiled),
 * -1 = none.
 */
int aqz_ds_last_batch_kind(const aqz_ds* ds);

/*
 * Diagnostic: how many runs of pure-XY levels the streaming path (add_frame)
 * has written in ONE tiled-cascade launch — levels row-major into their
 * slots and chunk-tiled, zero scan included, into the tiles
 * aqz_ds_set_level_tiling asked for — instead of the cascade plus a tile pass
 * per level ($AQZ_STREAM_TILE_PASS=1 forces the latter).
 */
uint64_t aqz_ds_stream_tiled_runs(const aqz_ds* ds);

/* HIP ordinal the handle runs on (-1 for a null handle). */
int aqz_ds_device(const aqz_ds* ds);

/* Bytes of one frame at `level` (0 on bad level). */
size_t aqz_ds_level_bytes(const aqz_ds* ds, uint32_t level);

/* Number of levels (including level 0). */
uint32_t aqz_ds_level_count(const aqz_ds* ds);

/* Bytes of device memory held by the handle (reported separately from the
 * reference's host memory estimate, acquire.zarr.cpp:216-314). */
size_t aqz_ds_device_memory_usage(const aqz_ds* ds);

/* Last error message of the handle (never NULL; "" when none). */
const char* aqz_ds_last_error(const aqz_ds* ds);

/* Last error of a failed aqz_ds_create / aqz_plan_levels on this thread. */
const char* aqz_last_error(void);

/*
 * `Downsampler::downsampling_method` (downsampler.cpp:422-437): "decimate",
 * "local_mean", "local_min", "local_max"; NULL for an invalid method.
 */
const char* aqz_method_name(int method);

/*
 * `Downsampler::get_metadata` (downsampler.cpp:440-485) serialised as a
 * compact JSON object; NULL for an invalid method.
 */
const char* aqz_method_metadata_json(int method);

/* Library version string. */
const char* aqz_version(void);

/* ---- Frame sharding over a node's GPUs --------------------
 *
 * Frames of a 2-D pyramid are independent, and so are slabs of a volume that
 * start where add_frame's Z-pairing state is fresh.  An aqz_node deals a host
 * batch over one aqz_ds handle per device entry — contiguous blocks of whole
 * shard units, each handle running aqz_ds_run_host_batch on its own streams
 * and PCIe link in its own host thread — and every block writes its levels at
 * its frames' place in the outputs, so the caller receives each level in
 * frame-id order, as `Array::write_frame` requires (array.cpp:179-189).  No
 * collective: nothing is exchanged between GPUs.
 */

/*
 * The shard unit of a pyramid: the fewest level-0 frames (planes) after which
 * add_frame's state (downsampler.cpp:306-401: stored Z planes and the
 * odd-stack pass-through count) is back at a fresh handle's.  1 when no level
 * halves Z; 2^h when h levels halve Z and the planes divide by 2^h; else the
 * whole stack.  `frames_per_unit` (optional, n_levels entries) receives the
 * frames each level emits per unit.  Host-only (no device call).
 */
int aqz_shard_unit(const aqz_level_desc* levels,
                   uint32_t n_levels,
                   uint32_t* unit,
                   uint32_t* frames_per_unit);

typedef struct aqz_node aqz_node;

/*
 * One aqz_ds handle per entry of `devices` (HIP ordinals; an ordinal may
 * repeat, giving several handles on one GPU).  Validation as aqz_ds_create.
 * Like an aqz_ds, a node serves one caller thread at a time.
 */
int aqz_node_create(const aqz_level_desc* levels,
                    uint32_t n_levels,
                    int dtype,
                    int method,
                    const int* devices,
                    uint32_t n_devices,
                    aqz_node** out);

void aqz_node_destroy(aqz_node* node);

/* Number of handles, and handle `i` (NULL when out of range): per-device
 * diagnostics (aqz_ds_device, aqz_ds_device_memory_usage). */
uint32_t aqz_node_handle_count(const aqz_node* node);
aqz_ds* aqz_node_handle(aqz_node* node, uint32_t i);

/*
 * aqz_ds_run_host_batch over the node: same results, layout and counts as one
 * handle running the whole batch, with `n_frames` a whole number of shard
 * units, starting where the stream (aqz_node_add_frame) stands on a unit
 * boundary (else AQZ_INVALID_ARGUMENT before anything runs); adds in flight
 * are flushed first.  Blocks until every handle has finished; a failing
 * handle's status and message are returned after all handles have drained.
 */
int aqz_node_run_host_batch(aqz_node* node,
                            const void* host_frames,
                            uint32_t n_frames,
                            void* const* host_out_levels,
                            uint32_t* out_counts);

/* aqz_node_run_device_batch flag: stage every block through the handle's
 * own buffers even on the batch's GPU (tests the xGMI path on one GPU). */
#define AQZ_NODE_STAGE_ALL 1u

/*
 * Device-resident batch over the node's GPUs (BASELINE config F: frame
 * batches sharded across GPUs over xGMI).  `device_frames` and every
 * `device_out_levels[L]` (index 0 ignored) live on HIP device `src_device`;
 * results, layout and counts are those of aqz_ds_run_device_batch on one
 * handle: the k-th frame emitted at level L at `device_out_levels[L] +
 * k * level_bytes(L)`, so every level comes back in frame-id order, as
 * Array::write_frame requires (array.cpp:179-189).  `n_frames` is a whole
 * number of shard units and the node's stream stands on a unit boundary
 * (else AQZ_INVALID_ARGUMENT before anything runs); adds in flight are
 * flushed first.  Contiguous blocks of whole units go one per handle: a
 * handle on `src_device` runs its block in place on `hip_stream`; a handle on
 * another GPU pulls its block into its own staging by peer copy (xGMI DMA),
 * runs it there and pushes each level back, in sub-batches of at most
 * $AQZ_NODE_STAGE_MB MiB per staging slot (default 256) so that pull,
 * pyramid and push overlap.  Asynchronous: the blocks start behind the work
 * already on `hip_stream` (NULL = the null stream of `src_device`), and
 * `hip_stream` waits for every block before its later work runs; the call
 * returns without a host synchronisation.  `flags`: 0 or AQZ_NODE_STAGE_ALL.
 * The caller's current device is unchanged on return.
 */
int aqz_node_run_device_batch(aqz_node* node,
                              const void* device_frames,
                              int src_device,
                              uint32_t n_frames,
                              void* const* device_out_levels,
                              uint32_t* out_counts,
                              void* hip_stream,
                              uint32_t flags);

/*
 * Streaming over the node: several frames in flight, one per handle.  Frame k
 * goes to handle (k / unit) % n_handles as an aqz_ds_add_frame_async_take that
 * takes every level into node-owned buffers; the call returns once the frame
 * is handed to that handle's upload thread (after settling the handle's
 * previous add).  `host_frame` must stay valid and unchanged until the handle
 * is used again (unit x n_handles frames later) or aqz_node_flush returns.
 * Same frames, in the same per-level order, as one Downsampler fed the stream
 * with every level taken after every frame (the MultiscaleArray caller,
 * multiscale.array.cpp:298-325) — the emplace rule never applies, since the
 * node takes every frame.
 */
int aqz_node_add_frame(aqz_node* node, const void* host_frame, size_t nbytes);

/*
 * The next level-`level` frame in emission order, if its add has completed
 * (non-blocking: finished adds are settled through aqz_ds_poll, and
 * *has_frame = 0 when the frame's add, or an earlier one, still runs;
 * aqz_node_flush makes every frame of the adds so far ready).  `dst` NULL: size query, the frame
 * stays queued.
 */
int aqz_node_take_frame(aqz_node* node,
                        uint32_t level,
                        void* dst,
                        size_t cap,
                        size_t* nbytes,
                        int* has_frame);

/*
 * Streaming takes of `level` chunk-tiled (tile_rows x tile_cols, the layout
 * of aqz_ds_take_frame_tiled, zero overhang included) instead of row-major:
 * aqz_node_take_frame then hands out the tiled frame.  Each handle tiles on
 * its GPU right behind the pyramid (aqz_ds_set_level_tiling).  Before the
 * first add only; (0, 0) restores row-major.
 */
int aqz_node_set_level_tiling(aqz_node* node,
                              uint32_t level,
                              uint32_t tile_rows,
                              uint32_t tile_cols);

/* Wait for every add in flight; their level frames become takeable. */
int aqz_node_flush(aqz_node* node);

/*
 * Wait until no add in flight still reads its host frame (aqz_ds_wait_input
 * on every handle): every frame handed to aqz_node_add_frame so far may then
 * be reused, while their pyramids and level copies still run.  A failed add
 * is reported by the take or flush that settles it.  The drop-in
 * (integration/src/streaming/downsampler.hip.cpp, node mode) calls it where
 * the single-handle adapter waits for the whole add.
 */
int aqz_node_wait_input(aqz_node* node);

/*
 * Non-blocking: *released = the number of frames, counted from the node's
 * first aqz_node_add_frame, that no add in flight still reads — every frame
 * before the earliest one whose upload may still run (all of them when none
 * is).  A caller that owns the frames' buffers recycles each one whose index
 * is below *released; the drop-in's node mode keeps the consumer's frame
 * buffers this way instead of waiting for every upload
 * (integration/src/streaming/downsampler.hip.cpp, Downsampler::release_frame;
 * the buffers are the frame queue's, which FrameQueue::pop hands over by swap,
 * frame.queue.cpp:48-74).
 */
int aqz_node_inputs_released(aqz_node* node, uint64_t* released);

/* Last error message of the node (never NULL; "" when none). */
const char* aqz_node_last_error(const aqz_node* node);

#ifdef __cplusplus
}
#endif

#endif /* AQZ_DOWNSAMPLER_H */
