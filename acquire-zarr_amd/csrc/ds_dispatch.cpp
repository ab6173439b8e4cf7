// ds_dispatch.cpp — routes each dtype-dispatching launcher of ds_kernels.hh
// to the build shard that instantiates that dtype's kernels.
//
// ds_kernels.hip is compiled AQZ_SHARDS times (acquire-zarr_amd/Makefile);
// shard k holds the kernels of the dtypes whose code % AQZ_SHARDS == k and
// names its launchers <launcher>_shard<k>.  This file is compiled once.
#include "ds_kernels.hh"

#ifndef AQZ_SHARDS
#error "ds_dispatch.cpp is built with -DAQZ_SHARDS=<n> (acquire-zarr_amd/Makefile)"
#endif
#if AQZ_SHARDS != 8
#error "ds_dispatch.cpp routes to exactly 8 shards"
#endif

namespace aqz {

#define AQZ_DECLARE_SHARDS(name, params)                                       \
    hipError_t name##_shard0 params;                                           \
    hipError_t name##_shard1 params;                                           \
    hipError_t name##_shard2 params;                                           \
    hipError_t name##_shard3 params;                                           \
    hipError_t name##_shard4 params;                                           \
    hipError_t name##_shard5 params;                                           \
    hipError_t name##_shard6 params;                                           \
    hipError_t name##_shard7 params;

#define AQZ_ROUTE(name, dtype, args)                                           \
    do {                                                                       \
        if (!dtype_valid(dtype))                                               \
            return hipErrorInvalidValue;                                       \
        switch ((dtype) % AQZ_SHARDS) {                                        \
            case 0:                                                            \
                return name##_shard0 args;                                     \
            case 1:                                                            \
                return name##_shard1 args;                                     \
            case 2:                                                            \
                return name##_shard2 args;                                     \
            case 3:                                                            \
                return name##_shard3 args;                                     \
            case 4:                                                            \
                return name##_shard4 args;                                     \
            case 5:                                                            \
                return name##_shard5 args;                                     \
            case 6:                                                            \
                return name##_shard6 args;                                     \
            default:                                                           \
                return name##_shard7 args;                                     \
        }                                                                      \
    } while (0)

AQZ_DECLARE_SHARDS(launch_cascade,
                   (int, int, const void*, uint64_t, uint32_t, uint32_t, const LevelOut*, int,
                    uint32_t, hipStream_t))
AQZ_DECLARE_SHARDS(launch_cascade_tiled,
                   (int, int, const void*, uint64_t, uint32_t, uint32_t, const LevelOut*,
                    const TiledOut*, int, uint32_t, hipStream_t))
AQZ_DECLARE_SHARDS(launch_volume,
                   (int, int, const void*, uint64_t, uint32_t, uint32_t, const LevelOut*, int,
                    uint32_t, hipStream_t))
AQZ_DECLARE_SHARDS(launch_xy_generic,
                   (int, int, const void*, uint64_t, uint32_t, uint32_t, const LevelOut&,
                    uint32_t, hipStream_t))
AQZ_DECLARE_SHARDS(launch_zpair,
                   (int, int, void*, const void*, const void*, uint64_t, hipStream_t))
AQZ_DECLARE_SHARDS(launch_transpose,
                   (int, const void*, uint32_t, uint32_t, void*, hipStream_t))
AQZ_DECLARE_SHARDS(launch_tile_frame,
                   (int, const void*, uint32_t, uint32_t, uint32_t, uint32_t, void*, uint32_t*,
                    hipStream_t))
AQZ_DECLARE_SHARDS(launch_tile_frame_sliced,
                   (int, const void*, uint32_t, uint32_t, uint32_t, uint32_t, void*, uint8_t*,
                    hipStream_t))

hipError_t
launch_cascade(int dtype,
               int method,
               const void* src,
               uint64_t src_frame_elems,
               uint32_t W,
               uint32_t H,
               const LevelOut* outs,
               int n_out,
               uint32_t n_frames,
               hipStream_t stream)
{
    AQZ_ROUTE(launch_cascade, dtype,
              (dtype, method, src, src_frame_elems, W, H, outs, n_out, n_frames, stream));
}

hipError_t
launch_cascade_tiled(int dtype,
                     int method,
                     const void* src,
                     uint64_t src_frame_elems,
                     uint32_t W,
                     uint32_t H,
                     const LevelOut* outs,
                     const TiledOut* touts,
                     int n_out,
                     uint32_t n_frames,
                     hipStream_t stream)
{
    AQZ_ROUTE(launch_cascade_tiled, dtype,
              (dtype, method, src, src_frame_elems, W, H, outs, touts, n_out, n_frames, stream));
}

hipError_t
launch_volume(int dtype,
              int method,
              const void* src,
              uint64_t src_frame_elems,
              uint32_t W,
              uint32_t H,
              const LevelOut* outs,
              int n_out,
              uint32_t n_planes,
              hipStream_t stream)
{
    AQZ_ROUTE(launch_volume, dtype,
              (dtype, method, src, src_frame_elems, W, H, outs, n_out, n_planes, stream));
}

hipError_t
launch_xy_generic(int dtype,
                  int method,
                  const void* src,
                  uint64_t src_frame_elems,
                  uint32_t w,
                  uint32_t h,
                  const LevelOut& out,
                  uint32_t n_frames,
                  hipStream_t stream)
{
    AQZ_ROUTE(launch_xy_generic, dtype,
              (dtype, method, src, src_frame_elems, w, h, out, n_frames, stream));
}

hipError_t
launch_zpair(int dtype,
             int method,
             void* out,
             const void* earlier,
             const void* current,
             uint64_t n,
             hipStream_t stream)
{
    AQZ_ROUTE(launch_zpair, dtype, (dtype, method, out, earlier, current, n, stream));
}

hipError_t
launch_transpose(int dtype,
                 const void* src,
                 uint32_t rows,
                 uint32_t cols,
                 void* dst,
                 hipStream_t stream)
{
    AQZ_ROUTE(launch_transpose, dtype, (dtype, src, rows, cols, dst, stream));
}

hipError_t
launch_tile_frame(int dtype,
                  const void* src,
                  uint32_t W,
                  uint32_t H,
                  uint32_t tile_rows,
                  uint32_t tile_cols,
                  void* dst,
                  uint32_t* nonzero,
                  hipStream_t stream)
{
    AQZ_ROUTE(launch_tile_frame, dtype,
              (dtype, src, W, H, tile_rows, tile_cols, dst, nonzero, stream));
}

hipError_t
launch_tile_frame_sliced(int dtype,
                         const void* src,
                         uint32_t W,
                         uint32_t H,
                         uint32_t tile_rows,
                         uint32_t tile_cols,
                         void* dst,
                         uint8_t* slice_flags,
                         hipStream_t stream)
{
    AQZ_ROUTE(launch_tile_frame_sliced, dtype,
              (dtype, src, W, H, tile_rows, tile_cols, dst, slice_flags, stream));
}

} // namespace aqz
