// ds_kernels.hh — launchers for the MI355X pyramid kernels (ds_kernels.hip).
//
// Three kernels cover the reference's two hot loops
// (src/streaming/downsampler.cpp):
//   * cascade   — scale_image<T> (:139-206) applied 1..4 times in one pass:
//                 each wave reads a 2^NL-row base tile once and writes every
//                 level of the run; odd edges replicated per level.
//   * xy_generic — one scale_image<T> level, one output pixel per lane; used
//                 by the general state machine and for frames narrower than
//                 one vector load.
//   * zpair     — average_two_frames<T> (:208-246), out = f(earlier, current).
//   * volume    — both of the above fused for pyramids whose levels halve XY
//                 and Z (3-D stacks): 2^NL planes x 2^NL rows per wave, every
//                 level written from registers.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace aqz {

constexpr int kMaxFusedLevels = 4;
constexpr int kMaxVolumeLevels = 2;

// One output level of a cascade launch.  `frame_elems` is the element stride
// between consecutive frames of that level (w*h for densely packed batches).
struct LevelOut
{
    void* ptr;
    uint64_t frame_elems;
    uint32_t w, h;
};

size_t dtype_bytes(int dtype);
bool dtype_valid(int dtype);
bool method_valid(int method);

// Columns per lane the fused cascade would use for this run of levels (0:
// unsupported).  Any width and byte offset works as long as the buffers are
// element-aligned, a row holds at least one 16-byte (narrow tiles: 8-byte)
// load, and each output level is exactly ceil(in/2) of the one before.
uint32_t cascade_pick_cols(int dtype,
                           const void* src,
                           uint64_t src_frame_elems,
                           uint32_t W,
                           uint32_t H,
                           const LevelOut* outs,
                           int n_out);
bool cascade_supported(int dtype,
                       const void* src,
                       uint64_t src_frame_elems,
                       uint32_t W,
                       uint32_t H,
                       const LevelOut* outs,
                       int n_out);

// Fused multi-level XY reduction of `n_frames` frames (frame i at
// src + i*src_frame_elems).  n_out in [1, kMaxFusedLevels].
hipError_t launch_cascade(int dtype,
                          int method,
                          const void* src,
                          uint64_t src_frame_elems,
                          uint32_t W,
                          uint32_t H,
                          const LevelOut* outs,
                          int n_out,
                          uint32_t n_frames,
                          hipStream_t stream);

// Chunk-tiled output of one cascade level: frame k of
// the level at ptr + k * n_tiles * tile_rows * tile_cols elements, tile
// t = ty * n_tiles_x + tx holding tile_rows x tile_cols elements row-major,
// zero where it overhangs the level — the layout Array::write_frame_to_chunks_
// fills (array.cpp:507-622, chunk.cpp:17-58).  `nonzero` (optional, device)
// receives the chunk zero scan as flag bytes (cascade_tiled_slots).
// Chunk lattice instead (frame_offsets non-null, device): frame k's tile t at
// ptr + frame_offsets[k] + t * tile_stride elements — every tile straight
// into its chunk buffer at the frame's place in it.
struct TiledOut
{
    void* ptr;
    uint32_t tile_rows, tile_cols;
    uint8_t* nonzero;
    const uint64_t* frame_offsets = nullptr; // elements, n_frames entries
    uint64_t tile_stride = 0;                // elements (with frame_offsets)
};

// Columns per lane launch_cascade_tiled uses for W-wide frames of `dtype`
// (cascade_pick_cols for element-aligned buffers).
uint32_t cascade_tiled_cols(int dtype, uint32_t W);

// Zero-scan flag bytes per tile that launch_cascade_tiled writes for level
// `level` (1-based within a launch of n_out levels over W-wide frames): when
// the kernel's wave blocks tile the chunk tiles exactly, `slots` bytes per
// tile (*slots_x across), each written once by the wave owning that block —
// the tile is nonzero iff any of its slots is; returns 0 otherwise (one byte
// per tile, cleared before the launch).
uint32_t cascade_tiled_slots(int dtype,
                             uint32_t W,
                             int n_out,
                             int level,
                             uint32_t tile_rows,
                             uint32_t tile_cols,
                             uint32_t* slots_x);

// launch_cascade with every level written chunk-tiled from registers: one
// kernel, whose trailing waves zero-fill the tile overhang past the frame
// (plus one flag clear per level whose tiles do not hold whole wave blocks).
// touts[i].nonzero then holds n_frames * n_tiles * max(1, slots) bytes.
// outs[i] gives level i's geometry; its ptr, when non-null, also receives the
// level row-major (the input of a following launch).  Same geometry rules as
// launch_cascade.
hipError_t launch_cascade_tiled(int dtype,
                                int method,
                                const void* src,
                                uint64_t src_frame_elems,
                                uint32_t W,
                                uint32_t H,
                                const LevelOut* outs,
                                const TiledOut* touts,
                                int n_out,
                                uint32_t n_frames,
                                hipStream_t stream);

// Fused 2x2x2 (XY reduce, then Z pair) over `n_planes` consecutive planes for
// pyramids whose levels all halve both XY and Z; n_planes must be a multiple
// of 2^n_out, n_out in [1, kMaxVolumeLevels].  Level L receives
// n_planes >> L frames.
bool volume_supported(int dtype,
                      const void* src,
                      uint32_t W,
                      uint32_t H,
                      const LevelOut* outs,
                      int n_out);
hipError_t launch_volume(int dtype,
                         int method,
                         const void* src,
                         uint64_t src_frame_elems,
                         uint32_t W,
                         uint32_t H,
                         const LevelOut* outs,
                         int n_out,
                         uint32_t n_planes,
                         hipStream_t stream);

// One XY level, any width/alignment.
// (The dtype-dispatching launchers below are defined per build shard in
// ds_kernels.hip and routed by ds_dispatch.cpp.)
hipError_t launch_xy_generic(int dtype,
                             int method,
                             const void* src,
                             uint64_t src_frame_elems,
                             uint32_t w,
                             uint32_t h,
                             const LevelOut& out,
                             uint32_t n_frames,
                             hipStream_t stream);

// out[i] = reduce2(earlier[i], current[i]) over n elements; `out` may alias
// either input.  16-byte vectors when all pointers are aligned, else scalar.
hipError_t launch_zpair(int dtype,
                        int method,
                        void* out,
                        const void* earlier,
                        const void* current,
                        uint64_t n,
                        hipStream_t stream);

// Chunk tiling of one W x H frame (array.cpp:507-622 / chunk.cpp:17-58):
// transpose_frame (array.cpp:488-504): `dst` (cols x rows, row-major)
// receives the transpose of `src` (rows x cols, row-major).
hipError_t launch_transpose(int dtype,
                            const void* src,
                            uint32_t rows,
                            uint32_t cols,
                            void* dst,
                            hipStream_t stream);

// `dst` receives n_tiles x tile_rows x tile_cols elements, tile-major,
// zero-padded; `nonzero[t]` (device, one u32 per tile, cleared here) is set
// when tile t holds any nonzero byte.
hipError_t launch_tile_frame(int dtype,
                             const void* src,
                             uint32_t W,
                             uint32_t H,
                             uint32_t tile_rows,
                             uint32_t tile_cols,
                             void* dst,
                             uint32_t* nonzero,
                             hipStream_t stream);

// Same tiling with one flag byte per (tile, slice): slice_flags holds
// n_tiles * tile_slices(tile_rows, tile_cols) bytes (tile-major), written
// without atomics or a pre-clear; a tile is nonzero iff any of its slices is.
uint32_t tile_slices(uint32_t tile_rows, uint32_t tile_cols);
hipError_t launch_tile_frame_sliced(int dtype,
                                    const void* src,
                                    uint32_t W,
                                    uint32_t H,
                                    uint32_t tile_rows,
                                    uint32_t tile_cols,
                                    void* dst,
                                    uint8_t* slice_flags,
                                    hipStream_t stream);

} // namespace aqz
