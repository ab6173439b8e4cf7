// tools/mixbench.hip — can any cache policy or burst shape move a 3:1
// read:write byte mix faster than tools/hbm_probe.hip's? (not product)
//
// Every variant reads the same 2 GiB buffer (one round per 256-thread
// workgroup, contiguous 4 KiB blocks per load instruction group) and, unless
// read-only, writes a third of that.  Policies on the gfx950 global memory
// instructions: nt (streaming), sc0/sc1 (scope bits).  Inline-asm variants
// wait vmcnt(0) explicitly before using loaded data.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/mixbench.hip -o tools/mixbench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
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

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void
fill_kernel(uint32_t* p, uint64_t n)
{
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n;
         i += uint64_t(gridDim.x) * blockDim.x)
        p[i] = uint32_t((i * 0x9E3779B97F4A7C15ull) >> 32);
}

// LP: 0 plain, 1 nt (builtin), 2 asm "nt sc0 sc1"
// SP: 0 plain, 1 nt (builtin), 2 asm "nt sc1", 3 asm "sc0 sc1", 4 asm "nt sc0 sc1"
template<int LP>
__device__ __forceinline__ u32x4
load(const u32x4* p)
{
    if constexpr (LP == 0) {
        return *p;
    } else if constexpr (LP == 1) {
        return __builtin_nontemporal_load(p);
    } else {
        u32x4 v;
        asm volatile("global_load_dwordx4 %0, %1, off nt sc0 sc1" : "=v"(v) : "v"(p) : "memory");
        return v;
    }
}

template<int SP>
__device__ __forceinline__ void
store(u32x4* p, u32x4 v)
{
    if constexpr (SP == 0) {
        *p = v;
    } else if constexpr (SP == 1) {
        __builtin_nontemporal_store(v, p);
    } else if constexpr (SP == 2) {
        asm volatile("global_store_dwordx4 %0, %1, off nt sc1" ::"v"(p), "v"(v) : "memory");
    } else if constexpr (SP == 3) {
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
    } else {
        asm volatile("global_store_dwordx4 %0, %1, off nt sc0 sc1" ::"v"(p), "v"(v) : "memory");
    }
}

template<int RD, int WR, int LP, int SP>
__global__ __launch_bounds__(256) void
mix(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint32_t* sink)
{
    const uint64_t rb = uint64_t(blockIdx.x) * 256 * RD + threadIdx.x;
    u32x4 v[RD];
#pragma unroll
    for (int k = 0; k < RD; ++k)
        v[k] = load<LP>(src + rb + k * 256);
    if constexpr (LP == 2)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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
            store<SP>(dst + wb + k * 256, a);
        }
    }
}

// write-only: W x 4 KiB per workgroup
template<int W, int SP>
__global__ __launch_bounds__(256) void
write_only(u32x4* __restrict__ dst)
{
    const uint64_t wb = uint64_t(blockIdx.x) * 256 * W + threadIdx.x;
    u32x4 a = { blockIdx.x, threadIdx.x, 1u, 2u };
#pragma unroll
    for (int k = 0; k < W; ++k)
        store<SP>(dst + wb + k * 256, a + k);
}

int
main(int argc, char** argv)
{
    const uint64_t bytes = uint64_t(argc > 1 ? std::atoi(argv[1]) : 2048) << 20;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 20;
    u32x4 *src, *dst;
    uint32_t* sink;
    CHECK(hipMalloc(&src, bytes));
    CHECK(hipMalloc(&dst, bytes / 2));
    CHECK(hipMalloc(&sink, 64));
    hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0, reinterpret_cast<uint32_t*>(src),
                       bytes / 4);
    struct V
    {
        std::string name;
        uint64_t moved;
        std::function<void()> run;
        std::vector<float> us;
    };
    std::vector<V> vs;
#define MIX(RD, WR, LP, SP, NAME)                                              \
    {                                                                          \
        const uint64_t blocks = bytes / (uint64_t(RD) * 4096);                 \
        vs.push_back({ NAME, blocks * (RD + WR) * 4096, [=] {                  \
                          hipLaunchKernelGGL((mix<RD, WR, LP, SP>), dim3(blocks), dim3(256), 0, 0, \
                                             src, dst, sink);                  \
                      }, {} });                                                \
    }
    MIX(12, 4, 1, 1, "12:4 nt / nt (probe)");
    MIX(12, 4, 1, 0, "12:4 nt / plain");
    MIX(12, 4, 0, 1, "12:4 plain / nt");
    MIX(12, 4, 1, 2, "12:4 nt / nt sc1");
    MIX(12, 4, 1, 3, "12:4 nt / sc0 sc1");
    MIX(12, 4, 1, 4, "12:4 nt / nt sc0 sc1");
    MIX(12, 4, 2, 1, "12:4 nt sc0 sc1 / nt");
    MIX(24, 8, 1, 1, "24:8 nt / nt");
    MIX(6, 2, 1, 1, "6:2 nt / nt");
    MIX(16, 0, 1, 1, "read only nt");
    {
        const uint64_t blocks = bytes / 3 / (4 * 4096);
        vs.push_back({ "write only nt (1/3 size)", blocks * 4 * 4096, [=] {
                          hipLaunchKernelGGL((write_only<4, 1>), dim3(blocks), dim3(256), 0, 0, dst);
                      }, {} });
        vs.push_back({ "write only plain (1/3)", blocks * 4 * 4096, [=] {
                          hipLaunchKernelGGL((write_only<4, 0>), dim3(blocks), dim3(256), 0, 0, dst);
                      }, {} });
    }
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
    std::printf("source %.0f MiB\n", bytes / 1048576.0);
    for (auto& v : vs) {
        std::sort(v.us.begin(), v.us.end());
        const float med = v.us[v.us.size() / 2];
        std::printf("%-28s median %8.1f us  min %8.1f us  %7.1f GB/s moved (%.1f%% of 8 TB/s)\n",
                    v.name.c_str(), med, v.us[0], v.moved / (med * 1e3),
                    100.0 * v.moved / (med * 1e3) / 8000.0);
    }
    return 0;
}
