// tools/hbm_probe.hip — measured HBM ceilings for bench.py (not product).
//
// libaqz_hbm_probe.so exports one launcher: a contiguous, non-temporal
// read + write stream with a fixed read:write byte ratio (RD:WR 4 KiB
// blocks per 256-thread workgroup, one round per workgroup, every load of a
// wave instruction one contiguous KiB).  tools/readbench.hip and
// tools/variants.hip measured this shape as the fastest way to move bytes
// on MI355X (7.08 TB/s read-only against 6.14 TB/s for a grid-stride loop),
// so it is the ceiling a kernel with the same byte mix is held to.
// bench.py times it beside the product kernel, on the same input buffer and
// stream, and reports roofline.same_mix_ceiling.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template<int RD, int WR>
__global__ __launch_bounds__(256) void
mix_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint32_t* sink)
{
    const uint64_t rb = uint64_t(blockIdx.x) * 256 * RD + threadIdx.x;
    u32x4 v[RD];
#pragma unroll
    for (int k = 0; k < RD; ++k)
        v[k] = __builtin_nontemporal_load(src + rb + k * 256);
    if constexpr (WR == 0) {
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < RD; ++k)
            acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
        if (acc == 0x12345678u)
            sink[0] = acc;
    } else {
        const uint64_t wb = uint64_t(blockIdx.x) * 256 * WR + threadIdx.x;
#pragma unroll
        for (int k = 0; k < WR; ++k) {
            u32x4 a = v[k];
#pragma unroll
            for (int j = k + WR; j < RD; j += WR)
                a ^= v[j];
            __builtin_nontemporal_store(a, dst + wb + k * 256);
        }
    }
}

} // namespace

extern "C" {

// Moves blocks * RD * 4 KiB in and blocks * WR * 4 KiB out, blocks =
// src_bytes / (RD * 4 KiB).  `dst` must hold blocks * WR * 4 KiB; `sink`
// 4 bytes.  Supported RD:WR = 16:0, 12:4, 13:3, 14:2, 10:6, 9:7.  Returns 0 or a
// hipError_t; *moved_bytes = bytes read + written.
int
aqz_hbm_probe(const void* src, uint64_t src_bytes, void* dst, void* sink, int rd, int wr,
              void* stream, uint64_t* moved_bytes)
{
    if (!src || !sink || (wr && !dst) || rd <= 0)
        return int(hipErrorInvalidValue);
    const uint64_t blocks = src_bytes / (uint64_t(rd) * 4096);
    if (blocks == 0 || blocks >= (1ull << 31))
        return int(hipErrorInvalidValue);
    const auto s = static_cast<hipStream_t>(stream);
    const auto* in = static_cast<const u32x4*>(src);
    auto* out = static_cast<u32x4*>(dst);
    auto* sk = static_cast<uint32_t*>(sink);
    if (rd == 16 && wr == 0)
        hipLaunchKernelGGL((mix_kernel<16, 0>), dim3(blocks), dim3(256), 0, s, in, out, sk);
    else if (rd == 12 && wr == 4)
        hipLaunchKernelGGL((mix_kernel<12, 4>), dim3(blocks), dim3(256), 0, s, in, out, sk);
    else if (rd == 13 && wr == 3)
        hipLaunchKernelGGL((mix_kernel<13, 3>), dim3(blocks), dim3(256), 0, s, in, out, sk);
    else if (rd == 14 && wr == 2)
        hipLaunchKernelGGL((mix_kernel<14, 2>), dim3(blocks), dim3(256), 0, s, in, out, sk);
    else if (rd == 10 && wr == 6) // Decimate's mix: half the rows read
        hipLaunchKernelGGL((mix_kernel<10, 6>), dim3(blocks), dim3(256), 0, s, in, out, sk);
    else if (rd == 9 && wr == 7)
        hipLaunchKernelGGL((mix_kernel<9, 7>), dim3(blocks), dim3(256), 0, s, in, out, sk);
    else
        return int(hipErrorInvalidValue);
    if (moved_bytes)
        *moved_bytes = blocks * uint64_t(rd + wr) * 4096;
    return int(hipGetLastError());
}

} // extern "C"
