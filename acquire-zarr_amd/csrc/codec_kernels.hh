// codec_kernels.hh — launchers for the blosc filter and crc32c kernels
// (codec_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace aqz {

// blosc_c's filter step on `n_buffers` buffers of `nbytes` each, back to
// back: every `blocksize` block (the last one shorter) byte-shuffled
// (shuffle 1, typesize > 1), bit-shuffled (2, block >= typesize) or copied.
hipError_t launch_blosc_filter(int shuffle,
                               uint32_t typesize,
                               uint32_t blocksize,
                               const void* src,
                               uint64_t nbytes,
                               uint32_t n_buffers,
                               void* dst,
                               hipStream_t stream);

// CRC-32C of `n_buffers` buffers of `nbytes`, buffer k at k * stride.
hipError_t launch_crc32c(const void* data,
                         uint64_t nbytes,
                         uint64_t stride,
                         uint32_t n_buffers,
                         uint32_t* crcs,
                         hipStream_t stream);

} // namespace aqz
