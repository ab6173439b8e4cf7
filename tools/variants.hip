// tools/variants.hip — same-box A/B of the fused kernels against HBM
// ceilings of the same byte mix (not product).
//
// Workloads (device-resident, as bench.py runs them):
//   u16 : 64 frames of 4096^2 uint16, 5 levels (headline)
//   f32 : 64 frames of 4096^2 float32, 5 levels (config F)
//   vol : 1024^2 x 256 uint16 volume, 3 levels (config V)
// Variants:
//   product      : launch_cascade / launch_volume as shipped
//   CcUu         : C columns per lane, U adjacent column tiles per wave, all
//                  U tiles' loads issued before any arithmetic (U = 1 is the
//                  product's wave shape at that C)
// Ceilings (contiguous, nt, one round per block): read of the input bytes,
// and read + write in the workload's own read:write byte ratio.
// Every variant's levels are compared with the product's (bit-exact).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 -I include
//          -I acquire-zarr_amd/csrc tools/variants.hip -o tools/variants
#include "../acquire-zarr_amd/csrc/ds_kernels.hip"
#include "aqz_downsampler.h"

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
fill_u32(uint32_t* p, uint64_t n, bool as_f32)
{
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n;
         i += uint64_t(gridDim.x) * blockDim.x) {
        uint64_t x = i * 0x9E3779B97F4A7C15ull;
        x ^= x >> 31;
        x *= 0xBF58476D1CE4E5B9ull;
        const uint32_t r = uint32_t(x >> 32);
        if (as_f32) {
            const float f = (float(r) / 4294967296.0f) * 2000.0f - 1000.0f;
            __builtin_memcpy(&p[i], &f, 4);
        } else {
            p[i] = r;
        }
    }
}

__global__ void
count_diff(const uint8_t* a, const uint8_t* b, uint64_t n, unsigned long long* bad)
{
    unsigned long long c = 0;
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n;
         i += uint64_t(gridDim.x) * blockDim.x)
        c += a[i] != b[i];
    if (c)
        atomicAdd(bad, c);
}

// 2-D: U adjacent column tiles per wave (interior frames only)
template<typename T, int C, int U>
__global__ __launch_bounds__(256) void
cascade_multi(CascadeParams p)
{
    constexpr int NL = 4, R = 16;
    constexpr int V = C * int(sizeof(T)) / 16;
    constexpr int E = 16 / int(sizeof(T));
    const int lane = threadIdx.x & 63;
    const uint32_t u = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t gx = p.units_x / U;
    if (u >= p.total_units / U)
        return;
    const uint32_t ux = (u % gx) * U;
    const uint32_t t = u / gx;
    const uint32_t row0 = (t % p.units_y) * R;
    const uint32_t f = t / p.units_y;
    const T* src = reinterpret_cast<const T*>(p.src) + uint64_t(f) * p.src_frame_elems;
    T v[U][R][C];
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint32_t col0 = (ux + j) * (64u * C) + uint32_t(lane) * C;
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int k = 0; k < V; ++k) {
                const u32x4 q = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(
                  src + uint64_t(row0 + r) * p.W + col0 + k * E));
                __builtin_memcpy(&v[j][r][k * E], &q, 16);
            }
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint32_t col0 = (ux + j) * (64u * C) + uint32_t(lane) * C;
        cascade_level<T, kMean, C, 1, NL, R, C, false, true>(p, v[j], f, row0, col0, lane);
    }
}

// 2-D, one tile per wave, frame index fastest in the unit order (waves in
// flight spread over every frame of the batch instead of one frame's bands)
template<typename T, int C>
__global__ __launch_bounds__(256) void
cascade_frame_fast(CascadeParams p, uint32_t n_frames)
{
    constexpr int NL = 4, R = 16;
    constexpr int V = C * int(sizeof(T)) / 16;
    constexpr int E = 16 / int(sizeof(T));
    const int lane = threadIdx.x & 63;
    const uint32_t u = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (u >= p.total_units)
        return;
    const uint32_t f = u % n_frames;
    const uint32_t t = u / n_frames;
    const uint32_t ux = t % p.units_x;
    const uint32_t row0 = (t / p.units_x) * R;
    const T* src = reinterpret_cast<const T*>(p.src) + uint64_t(f) * p.src_frame_elems;
    const uint32_t col0 = ux * (64u * C) + uint32_t(lane) * C;
    T v[R][C];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int k = 0; k < V; ++k) {
            const u32x4 q = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(
              src + uint64_t(row0 + r) * p.W + col0 + k * E));
            __builtin_memcpy(&v[r][k * E], &q, 16);
        }
    cascade_level<T, kMean, C, 1, NL, R, C, false, true>(p, v, f, row0, col0, lane);
}

// 3-D (NL = 2): U adjacent column tiles per wave
template<int C, int U>
__global__ __launch_bounds__(256) void
volume_multi(VolumeParams p)
{
    using T = uint16_t;
    constexpr int NL = 2, R = 4, Z = 4;
    constexpr int V = C * 2 / 16;
    const int lane = threadIdx.x & 63;
    const uint32_t u = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t gx = p.units_x / U;
    if (u >= p.total_units / U)
        return;
    const uint32_t ux = (u % gx) * U;
    const uint32_t t = u / gx;
    const uint32_t row0 = (t % p.units_y) * R;
    const uint32_t g = t / p.units_y;
    T v[U][Z][R][C];
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint32_t col0 = (ux + j) * (64u * C) + uint32_t(lane) * C;
#pragma unroll
        for (int z = 0; z < Z; ++z) {
            const T* src = reinterpret_cast<const T*>(p.src) +
                           (uint64_t(g) * Z + z) * p.src_frame_elems;
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int k = 0; k < V; ++k) {
                    const u32x4 q = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(
                      src + uint64_t(row0 + r) * p.W + col0 + k * 8));
                    __builtin_memcpy(&v[j][z][r][k * 8], &q, 16);
                }
        }
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
        const uint32_t col0 = (ux + j) * (64u * C) + uint32_t(lane) * C;
        volume_level<T, kMean, C, 1, NL, Z, R, C, false, true>(p, v[j], g, row0, col0, lane);
    }
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

// RD x 4 KiB read, WR x 4 KiB written per block, both contiguous, nt
template<int RD, int WR>
__global__ __launch_bounds__(256) void
oneshot_mix(const u32x4* p, u32x4* out)
{
    const uint64_t rb = uint64_t(blockIdx.x) * 256 * RD + threadIdx.x;
    const uint64_t wb = uint64_t(blockIdx.x) * 256 * WR + threadIdx.x;
    u32x4 v[RD];
#pragma unroll
    for (int k = 0; k < RD; ++k)
        v[k] = __builtin_nontemporal_load(p + rb + k * 256);
#pragma unroll
    for (int k = 0; k < WR; ++k) {
        u32x4 a = v[k];
#pragma unroll
        for (int j = k + WR; j < RD; j += WR)
            a ^= v[j];
        __builtin_nontemporal_store(a, out + wb + k * 256);
    }
}

struct V
{
    std::string name;
    uint64_t bytes;
    std::function<void()> run;
    bool checked;
    std::vector<float> us;
};

void
time_all(std::vector<V>& vs, int reps)
{
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
}

} // namespace
} // namespace aqz

using namespace aqz;

int
main(int argc, char** argv)
{
    const std::string which = argc > 1 ? argv[1] : "u16";
    const int reps = argc > 2 ? std::atoi(argv[2]) : 20;
    const bool vol = which == "vol";
    const bool f32 = which == "f32";
    const int dtype = f32 ? AQZ_DTYPE_FLOAT32 : AQZ_DTYPE_UINT16;
    const uint32_t bpp = f32 ? 4 : 2;
    const uint32_t W = vol ? 1024 : 4096, H = W;
    const uint32_t B = vol ? 256 : 64; // frames or planes
    const int nl = vol ? 2 : 4;
    const uint64_t frame = uint64_t(W) * H;
    const uint64_t in_bytes = frame * B * bpp;
    void* d_in;
    CHECK(hipMalloc(&d_in, in_bytes));
    hipLaunchKernelGGL(fill_u32, dim3(8192), dim3(256), 0, 0, static_cast<uint32_t*>(d_in),
                       in_bytes / 4, f32);
    uint32_t w[4], h[4], nlv[4];
    uint64_t out_bytes = 0;
    void* ref[4];
    void* var[4];
    for (int i = 0; i < nl; ++i) {
        w[i] = W >> (i + 1);
        h[i] = H >> (i + 1);
        nlv[i] = vol ? (B >> (i + 1)) : B;
        const uint64_t b = uint64_t(w[i]) * h[i] * bpp * nlv[i];
        out_bytes += b;
        CHECK(hipMalloc(&ref[i], b));
        CHECK(hipMalloc(&var[i], b));
    }
    const uint64_t alg = in_bytes + out_bytes;
    uint32_t* sink;
    CHECK(hipMalloc(&sink, 64));
    LevelOut ro[4];
    for (int i = 0; i < nl; ++i)
        ro[i] = { ref[i], uint64_t(w[i]) * h[i], w[i], h[i] };

    std::vector<V> vs;
    vs.push_back({ "product", alg, [&] {
                      if (vol)
                          CHECK(launch_volume(dtype, AQZ_METHOD_MEAN, d_in, frame, W, H, ro, nl, B, 0));
                      else
                          CHECK(launch_cascade(dtype, AQZ_METHOD_MEAN, d_in, frame, W, H, ro, nl, B, 0));
                  }, false, {} });

    auto cparams = [&](uint32_t C) {
        CascadeParams p{};
        p.src = static_cast<const uint8_t*>(d_in);
        p.src_frame_elems = frame;
        p.W = W;
        p.H = H;
        p.units_x = W / (64 * C);
        p.units_y = H / 16;
        p.total_units = p.units_x * p.units_y * B;
        for (int i = 0; i < nl; ++i) {
            p.dst[i] = static_cast<uint8_t*>(var[i]);
            p.dst_frame_elems[i] = uint64_t(w[i]) * h[i];
            p.w[i] = w[i];
            p.h[i] = h[i];
        }
        return p;
    };
    auto vparams = [&](uint32_t C) {
        VolumeParams p{};
        p.src = static_cast<const uint8_t*>(d_in);
        p.src_frame_elems = frame;
        p.W = W;
        p.H = H;
        p.units_x = W / (64 * C);
        p.units_y = H / 4;
        p.total_units = p.units_x * p.units_y * (B / 4);
        for (int i = 0; i < nl; ++i) {
            p.dst[i] = static_cast<uint8_t*>(var[i]);
            p.dst_frame_elems[i] = uint64_t(w[i]) * h[i];
            p.w[i] = w[i];
            p.h[i] = h[i];
        }
        return p;
    };
#define C2D(T, C, U)                                                           \
    vs.push_back({ "C" #C "U" #U, alg, [&] {                                   \
                      CascadeParams p = cparams(C);                            \
                      const uint32_t waves = p.total_units / U;                \
                      hipLaunchKernelGGL((cascade_multi<T, C, U>), dim3((waves + 3) / 4), \
                                         dim3(256), 0, 0, p);                  \
                  }, true, {} })
#define C3D(C, U)                                                              \
    vs.push_back({ "vol C" #C "U" #U, alg, [&] {                               \
                      VolumeParams p = vparams(C);                             \
                      const uint32_t waves = p.total_units / U;                \
                      hipLaunchKernelGGL((volume_multi<C, U>), dim3((waves + 3) / 4), \
                                         dim3(256), 0, 0, p);                  \
                  }, true, {} })
    if (vol) {
        C3D(8, 1);
        C3D(8, 2);
        C3D(16, 1);
    } else if (f32) {
        C2D(float, 8, 1);
        C2D(float, 4, 1);
        C2D(float, 4, 2);
        C2D(float, 8, 2);
    } else {
        C2D(uint16_t, 8, 1);
        C2D(uint16_t, 8, 2);
        C2D(uint16_t, 16, 1);
        vs.push_back({ "C8 frame-fastest", alg, [&] {
                          CascadeParams p = cparams(8);
                          hipLaunchKernelGGL((cascade_frame_fast<uint16_t, 8>),
                                             dim3((p.total_units + 3) / 4), dim3(256), 0, 0, p, B);
                      }, true, {} });
    }
    // ceilings of the same byte mix
    vs.push_back({ "ceiling read", in_bytes, [&] {
                      hipLaunchKernelGGL(oneshot_read<8>, dim3(in_bytes / (16 * 256 * 8)),
                                         dim3(256), 0, 0, static_cast<const u32x4*>(d_in), sink);
                  }, false, {} });
    u32x4* mix;
    CHECK(hipMalloc(&mix, in_bytes / 3 + 65536));
    if (vol) {
        // 512 MiB read : 72 MiB written ~ 7:1
        const uint64_t blocks = in_bytes / (14 * 4096);
        vs.push_back({ "ceiling r7w1 (14:2)", blocks * 16 * 4096, [&, blocks] {
                          hipLaunchKernelGGL((oneshot_mix<14, 2>), dim3(blocks), dim3(256), 0, 0,
                                             static_cast<const u32x4*>(d_in), mix);
                      }, false, {} });
    } else {
        const uint64_t blocks = in_bytes / (12 * 4096);
        vs.push_back({ "ceiling r3w1 (12:4)", blocks * 16 * 4096, [&, blocks] {
                          hipLaunchKernelGGL((oneshot_mix<12, 4>), dim3(blocks), dim3(256), 0, 0,
                                             static_cast<const u32x4*>(d_in), mix);
                      }, false, {} });
    }
    time_all(vs, reps);

    unsigned long long* bad;
    CHECK(hipMalloc(&bad, 8));
    std::printf("%s: %u x %ux%u, %d levels after the base, alg %.1f MB (read %.1f MB)\n",
                which.c_str(), B, W, H, nl, alg / 1e6, in_bytes / 1e6);
    for (auto& v : vs) {
        std::sort(v.us.begin(), v.us.end());
        const float med = v.us[v.us.size() / 2];
        std::string verdict;
        if (v.checked) {
            for (int i = 0; i < nl; ++i)
                CHECK(hipMemset(var[i], 0xA5, uint64_t(w[i]) * h[i] * bpp * nlv[i]));
            v.run();
            CHECK(hipMemset(bad, 0, 8));
            for (int i = 0; i < nl; ++i)
                hipLaunchKernelGGL(count_diff, dim3(2048), dim3(256), 0, 0,
                                   static_cast<uint8_t*>(var[i]), static_cast<uint8_t*>(ref[i]),
                                   uint64_t(w[i]) * h[i] * bpp * nlv[i], bad);
            unsigned long long nb;
            CHECK(hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost));
            verdict = nb ? " MISMATCH" : " (== product)";
        }
        std::printf("%-20s median %8.1f us  min %8.1f us  %7.1f GB/s of %8.1f MB (%.1f%%)%s\n",
                    v.name.c_str(), med, v.us[0], v.bytes / (med * 1e3), v.bytes / 1e6,
                    100.0 * v.bytes / (med * 1e3) / 8000.0, verdict.c_str());
    }
    return 0;
}
