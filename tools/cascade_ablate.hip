// tools/cascade_ablate.hip — where the headline cascade's time goes (not product).
//
// Headline batch (64 frames of 4096^2 u16, 5 levels, Mean), interleaved
// medians over 3 x 20 launches:
//   product          : launch_cascade as shipped
//   ablate mask M    : the same tiles, loads and reductions, storing only the
//                      levels in bit mask M (bit l-1 = level l); the rest are
//                      folded into a never-true predicate so nothing is DCE'd
//   oneshot read     : contiguous 32 KiB per block read ceiling
//   oneshot r3w1     : contiguous 48 KiB read + 16 KiB nt write per block
//                      (the cascade's 3:1 byte mix at the best access shape)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 -I include
//          -I acquire-zarr_amd/csrc tools/cascade_ablate.hip -o tools/cascade_ablate
#include "../acquire-zarr_amd/csrc/ds_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CHECK(x)                                                               \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,     \
                         hipGetErrorString(e_));                               \
            std::exit(2);                                                      \
        }                                                                      \
    } while (0)

namespace aqz {
namespace {

__global__ void
fill_kernel(uint32_t* p, uint64_t n)
{
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n;
         i += uint64_t(gridDim.x) * blockDim.x)
        p[i] = uint32_t((i * 0x9E3779B97F4A7C15ull) >> 29);
}

template<int MASK, int C, int J, int NL, int RI, int CI>
__device__ __forceinline__ void
ablate_level(const CascadeParams& p, const uint16_t (&in)[RI][CI], uint32_t f, uint32_t row0,
             uint32_t col0, int lane, uint32_t& acc)
{
    using T = uint16_t;
    constexpr int RO = RI / 2;
    constexpr int CO = (CI >= 2) ? CI / 2 : 1;
    const uint32_t win = (J == 1) ? p.W : p.w[J - 2];
    const uint32_t hin = (J == 1) ? p.H : p.h[J - 2];
    T out[RO][CO];
    xy_step<T, kMean, C, J, RI, CI, false>(in, out, win, hin, col0 >> (J - 1),
                                           row0 >> (J - 1));
    if constexpr ((MASK >> (J - 1)) & 1) {
        T* dst = reinterpret_cast<T*>(p.dst[J - 1]) + uint64_t(f) * p.dst_frame_elems[J - 1];
        store_level<T, C, J, RO, CO, false, true>(dst, out, p.w[J - 1], p.h[J - 1], col0, row0,
                                                  lane);
    } else {
#pragma unroll
        for (int r = 0; r < RO; ++r)
#pragma unroll
            for (int c = 0; c < CO; ++c)
                acc ^= out[r][c];
    }
    if constexpr (J < NL)
        ablate_level<MASK, C, J + 1, NL, RO, CO>(p, out, f, row0, col0, lane, acc);
}

template<int MASK>
__global__ __launch_bounds__(256) void
cascade_ablate(CascadeParams p, uint32_t* sink)
{
    using T = uint16_t;
    constexpr int NL = 4, R = 16, C = 8;
    const int lane = threadIdx.x & 63;
    const uint32_t u = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (u >= p.total_units)
        return;
    const uint32_t ux = u % p.units_x;
    const uint32_t t = u / p.units_x;
    const uint32_t row0 = (t % p.units_y) * R;
    const uint32_t f = t / p.units_y;
    const uint32_t col0 = ux * (64u * C) + uint32_t(lane) * C;
    const T* src = reinterpret_cast<const T*>(p.src) + uint64_t(f) * p.src_frame_elems;
    T v[R][C];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const u32x4 q = __builtin_nontemporal_load(
          reinterpret_cast<const u32x4*>(src + uint64_t(row0 + r) * p.W + col0));
        __builtin_memcpy(&v[r][0], &q, 16);
    }
    uint32_t acc = 0;
    ablate_level<MASK, C, 1, NL, R, C>(p, v, f, row0, col0, lane, acc);
    if (acc == 0xBEEFu) // u16 xors stay below 2^16
        sink[0] = acc;
}

template<int U>
__global__ __launch_bounds__(256) void
oneshot_read(const u32x4* p, uint32_t* sink)
{
    const uint64_t base = uint64_t(blockIdx.x) * 256 * U + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k)
        v[k] = __builtin_nontemporal_load(p + base + k * 256);
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < U; ++k)
        acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    if (acc == 0x12345678u)
        sink[0] = acc;
}

// 12 x 4 KiB read, 4 x 4 KiB written per block, both contiguous
__global__ __launch_bounds__(256) void
oneshot_r3w1(const u32x4* p, u32x4* out)
{
    const uint64_t rb = uint64_t(blockIdx.x) * 256 * 12 + threadIdx.x;
    const uint64_t wb = uint64_t(blockIdx.x) * 256 * 4 + threadIdx.x;
    u32x4 v[12];
#pragma unroll
    for (int k = 0; k < 12; ++k)
        v[k] = __builtin_nontemporal_load(p + rb + k * 256);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        __builtin_nontemporal_store(v[3 * k] ^ v[3 * k + 1] ^ v[3 * k + 2], out + wb + k * 256);
}

} // namespace
} // namespace aqz

using namespace aqz;

int
main(int argc, char** argv)
{
    const uint32_t W = 4096, H = 4096, B = argc > 1 ? std::atoi(argv[1]) : 64;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 20;
    const uint64_t frame = uint64_t(W) * H;
    const uint64_t in_bytes = frame * B * 2;
    uint16_t* d_in;
    CHECK(hipMalloc(&d_in, in_bytes));
    hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0,
                       reinterpret_cast<uint32_t*>(d_in), in_bytes / 4);
    uint32_t w[4], h[4];
    uint64_t lvl_bytes = 0;
    for (int i = 0; i < 4; ++i) {
        w[i] = W >> (i + 1);
        h[i] = H >> (i + 1);
        lvl_bytes += uint64_t(w[i]) * h[i] * 2;
    }
    const uint64_t alg = in_bytes + lvl_bytes * B;
    void* outs[4];
    for (int i = 0; i < 4; ++i)
        CHECK(hipMalloc(&outs[i], uint64_t(w[i]) * h[i] * 2 * B));
    uint32_t* sink;
    CHECK(hipMalloc(&sink, 64));
    u32x4* mix_out;
    const uint64_t mix_blocks = in_bytes / (12 * 4096);
    CHECK(hipMalloc(&mix_out, mix_blocks * 4 * 4096));

    CascadeParams p{};
    p.src = reinterpret_cast<const uint8_t*>(d_in);
    p.src_frame_elems = frame;
    p.W = W;
    p.H = H;
    p.units_x = W / 512;
    p.units_y = H / 16;
    p.total_units = p.units_x * p.units_y * B;
    for (int i = 0; i < 4; ++i) {
        p.dst[i] = static_cast<uint8_t*>(outs[i]);
        p.dst_frame_elems[i] = uint64_t(w[i]) * h[i];
        p.w[i] = w[i];
        p.h[i] = h[i];
    }
    const uint32_t grid = p.total_units / 4;

    struct V
    {
        std::string name;
        uint64_t bytes;
        std::function<void()> run;
        std::vector<float> us;
    };
    std::vector<V> vs;
    vs.push_back({ "product", alg, [&] {
                      LevelOut o[4];
                      for (int i = 0; i < 4; ++i)
                          o[i] = { outs[i], uint64_t(w[i]) * h[i], w[i], h[i] };
                      CHECK(launch_cascade(1, 1, d_in, frame, W, H, o, 4, B, 0));
                  }, {} });
#define ABL(M)                                                                 \
    vs.push_back({ "ablate mask " #M, alg, [&] {                               \
                      hipLaunchKernelGGL(cascade_ablate<M>, dim3(grid), dim3(256), 0, 0, p, sink); \
                  }, {} })
    ABL(15);
    ABL(0);
    ABL(1);
    ABL(3);
    ABL(7);
    ABL(14);
    vs.push_back({ "oneshot read", in_bytes, [&] {
                      hipLaunchKernelGGL(oneshot_read<8>, dim3(in_bytes / (16 * 256 * 8)),
                                         dim3(256), 0, 0,
                                         reinterpret_cast<const u32x4*>(d_in), sink);
                  }, {} });
    vs.push_back({ "oneshot r3w1", mix_blocks * 16 * 4096, [&] {
                      hipLaunchKernelGGL(oneshot_r3w1, dim3(mix_blocks), dim3(256), 0, 0,
                                         reinterpret_cast<const u32x4*>(d_in), mix_out);
                  }, {} });

    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (auto& v : vs)
        for (int i = 0; i < 2; ++i)
            v.run();
    CHECK(hipDeviceSynchronize());
    for (int r = 0; r < 3; ++r)
        for (auto& v : vs)
            for (int i = 0; i < reps; ++i) {
                CHECK(hipEventRecord(e0, 0));
                v.run();
                CHECK(hipEventRecord(e1, 0));
                CHECK(hipEventSynchronize(e1));
                float ms;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                v.us.push_back(ms * 1e3f);
            }
    std::printf("batch %u frames of %ux%u u16, alg bytes %.1f MB (read %.1f MB)\n", B, W, H,
                alg / 1e6, in_bytes / 1e6);
    for (auto& v : vs) {
        std::sort(v.us.begin(), v.us.end());
        const float med = v.us[v.us.size() / 2];
        std::printf("%-18s median %8.1f us  min %8.1f us  %7.1f GB/s of %7.1f MB (%.1f%%)\n",
                    v.name.c_str(), med, v.us[0], v.bytes / (med * 1e3), v.bytes / 1e6,
                    100.0 * v.bytes / (med * 1e3) / 8000.0);
    }
    return 0;
}
