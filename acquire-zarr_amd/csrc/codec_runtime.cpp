// codec_runtime.cpp — C ABI of include/aqz_codec.h over codec_kernels.hip.
#include "aqz_codec.h"
#include "abi_guard.hh"
#include "codec_kernels.hh"

#include <hip/hip_runtime.h>

#include <string>

namespace {

int
status_of(hipError_t e, const char* who)
{
    if (e == hipSuccess)
        return AQZ_OK;
    aqz::set_last_error(std::string(who) + ": " + hipGetErrorString(e));
    return e == hipErrorInvalidValue ? AQZ_INVALID_ARGUMENT : AQZ_INTERNAL_ERROR;
}

} // namespace

extern "C" {

int
aqz_blosc_filter_device(int shuffle,
                        uint32_t typesize,
                        uint32_t blocksize,
                        const void* device_src,
                        size_t nbytes,
                        uint32_t n_buffers,
                        void* device_dst,
                        void* hip_stream)
{
    try {
        if (!device_src || !device_dst || typesize == 0 || blocksize == 0 || n_buffers == 0 ||
            shuffle < AQZ_BLOSC_NOSHUFFLE || shuffle > AQZ_BLOSC_BITSHUFFLE) {
            aqz::set_last_error("blosc_filter_device: invalid argument");
            return AQZ_INVALID_ARGUMENT;
        }
        return status_of(aqz::launch_blosc_filter(shuffle, typesize, blocksize, device_src, nbytes,
                                                  n_buffers, device_dst,
                                                  static_cast<hipStream_t>(hip_stream)),
                         "blosc_filter_device");
    } catch (...) {
        return ABI_GUARD_FAIL(nullptr);
    }
}

int
aqz_crc32c_device(const void* device_data,
                  size_t nbytes,
                  size_t stride,
                  uint32_t n_buffers,
                  uint32_t* device_crcs,
                  void* hip_stream)
{
    try {
        if ((!device_data && nbytes) || !device_crcs || n_buffers == 0 ||
            (n_buffers > 1 && stride < nbytes)) {
            aqz::set_last_error("crc32c_device: invalid argument");
            return AQZ_INVALID_ARGUMENT;
        }
        return status_of(aqz::launch_crc32c(device_data, nbytes, stride, n_buffers, device_crcs,
                                            static_cast<hipStream_t>(hip_stream)),
                         "crc32c_device");
    } catch (...) {
        return ABI_GUARD_FAIL(nullptr);
    }
}

} // extern "C"
