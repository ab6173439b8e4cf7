// tools/readbench.hip — read-side HBM ceiling probe on MI355X (not product).
//
// The fused cascade moves 2 GiB in + 0.68 GB out per headline launch and sits
// at the rate of tools/microbench.hip's plain streaming read.  This probe asks
// whether any load scheme reads a 2 GiB buffer faster than that, so a cascade
// rewrite around it would pay:
//   reg  U/G     : U x 16 B register loads per lane per round, grid G blocks
//                  of 256 threads, grid-stride loop (G = 0: one round per
//                  thread, no loop, like the cascade's one-tile-per-wave grid)
//   pipe U/G     : the same with the next round's U loads issued before the
//                  current round is consumed
//   glds D/G     : LDS-DMA (global_load_lds_dwordx4) into a per-wave ring of
//                  16 x 1 KiB slots, one load per step, at most D in flight
//                  (s_waitcnt vmcnt(D)), nothing read back from LDS
// nt = non-temporal policy (aux 2 for LDS-DMA).  Medians over 3 x 20
// interleaved launches.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/readbench.hip -o tools/readbench
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

template<bool NT>
__device__ __forceinline__ u32x4
ld(const u32x4* p)
{
    if constexpr (NT)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}

// grid-stride, U loads then consume
template<int U, bool NT>
__global__ __launch_bounds__(256) void
read_reg(const u32x4* p, uint64_t n, uint32_t* sink)
{
    uint32_t acc = 0;
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i + (U - 1) * stride < n;
         i += U * stride) {
        u32x4 v[U];
#pragma unroll
        for (int k = 0; k < U; ++k)
            v[k] = ld<NT>(p + i + k * stride);
#pragma unroll
        for (int k = 0; k < U; ++k)
            acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    if (acc == 0x12345678u)
        sink[0] = acc;
}

// one round per thread: block b reads a contiguous U x 4 KiB span, each
// load instruction of a wave covering 1 KiB contiguous (cascade-like)
template<int U, bool NT>
__global__ __launch_bounds__(256) void
read_oneshot(const u32x4* p, uint32_t* sink)
{
    const uint64_t base = uint64_t(blockIdx.x) * 256 * U + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k)
        v[k] = ld<NT>(p + base + k * 256);
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < U; ++k)
        acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    if (acc == 0x12345678u)
        sink[0] = acc;
}

// software-pipelined grid-stride: next U issued before current consumed
template<int U, bool NT>
__global__ __launch_bounds__(256) void
read_pipe(const u32x4* p, uint64_t n, uint32_t* sink)
{
    uint32_t acc = 0;
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x;
    u32x4 a[U], b[U];
    if (i + (U - 1) * stride >= n)
        return;
#pragma unroll
    for (int k = 0; k < U; ++k)
        a[k] = ld<NT>(p + i + k * stride);
    i += U * stride;
    while (true) {
        const bool more = i + (U - 1) * stride < n;
        if (more) {
#pragma unroll
            for (int k = 0; k < U; ++k)
                b[k] = ld<NT>(p + i + k * stride);
        }
#pragma unroll
        for (int k = 0; k < U; ++k)
            acc ^= a[k].x ^ a[k].y ^ a[k].z ^ a[k].w;
        if (!more)
            break;
#pragma unroll
        for (int k = 0; k < U; ++k)
            a[k] = b[k];
        i += U * stride;
    }
    if (acc == 0x12345678u)
        sink[0] = acc;
}

// LDS-DMA stream: one 1 KiB load per step into a 16-slot per-wave ring, at
// most D outstanding.  Each wave walks its own contiguous span.
template<int D, int AUX>
__global__ __launch_bounds__(256) void
read_glds(const u32x4* p, uint64_t n, uint32_t* sink)
{
    __shared__ u32x4 ring[4][16][64];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const uint64_t waves = uint64_t(gridDim.x) * 4;
    const uint64_t wid = uint64_t(blockIdx.x) * 4 + w;
    const uint64_t per = n / 64 / waves; // 1 KiB steps per wave
    const u32x4* q = p + wid * per * 64 + lane;
    for (uint64_t s = 0; s < per; ++s) {
        __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(q + s * 64),
          (__attribute__((address_space(3))) void*)(&ring[w][s & 15][0]), 16, 0, AUX);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (ring[w][0][lane].x == 0x12345678u && ring[w][1][lane].y == 0x9u)
        sink[0] = 1;
}

int
main(int argc, char** argv)
{
    const uint64_t bytes = uint64_t(argc > 1 ? std::atoi(argv[1]) : 2048) << 20;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 20;
    const uint64_t n = bytes / 16;
    u32x4* d;
    uint32_t* sink;
    CHECK(hipMalloc(&d, bytes));
    CHECK(hipMalloc(&sink, 64));
    hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0,
                       reinterpret_cast<uint32_t*>(d), bytes / 4);

    struct V
    {
        std::string name;
        std::function<void()> run;
        std::vector<float> us;
    };
    std::vector<V> vs;
    auto add = [&](std::string name, std::function<void()> f) {
        vs.push_back({ name, f, {} });
    };
#define REG(U, NT, G)                                                          \
    add(std::string("reg U" #U " G" #G) + (NT ? " nt" : ""), [&] {                            \
        hipLaunchKernelGGL((read_reg<U, NT>), dim3(G), dim3(256), 0, 0, d, n, sink); \
    })
#define ONE(U, NT)                                                             \
    add(std::string("oneshot U" #U) + (NT ? " nt" : ""), [&] {                                \
        hipLaunchKernelGGL((read_oneshot<U, NT>), dim3(n / (256 * U)), dim3(256), 0, 0, d, sink); \
    })
#define PIPE(U, NT, G)                                                         \
    add(std::string("pipe U" #U " G" #G) + (NT ? " nt" : ""), [&] {                           \
        hipLaunchKernelGGL((read_pipe<U, NT>), dim3(G), dim3(256), 0, 0, d, n, sink); \
    })
#define GLDS(D, AUX, G)                                                        \
    add(std::string("glds D" #D " G" #G) + (AUX ? " nt" : ""), [&] {                          \
        hipLaunchKernelGGL((read_glds<D, AUX>), dim3(G), dim3(256), 0, 0, d, n, sink); \
    })
    REG(8, true, 4096);
    REG(8, false, 4096);
    REG(8, true, 2048);
    REG(8, true, 8192);
    REG(16, true, 2048);
    REG(16, true, 4096);
    REG(4, true, 4096);
    ONE(8, true);
    ONE(16, true);
    ONE(4, true);
    ONE(16, false);
    PIPE(8, true, 1024);
    PIPE(8, true, 2048);
    PIPE(4, true, 2048);
    GLDS(8, 2, 512);
    GLDS(12, 2, 512);
    GLDS(15, 2, 512);
    GLDS(8, 2, 1024);
    GLDS(12, 2, 1024);
    GLDS(15, 2, 1024);
    GLDS(12, 0, 1024);
    GLDS(15, 2, 2048);

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
    std::printf("read of %.0f MiB\n", bytes / 1048576.0);
    for (auto& v : vs) {
        std::sort(v.us.begin(), v.us.end());
        const float med = v.us[v.us.size() / 2];
        std::printf("%-22s median %8.1f us  min %8.1f us  %7.1f GB/s (%.1f%% of 8 TB/s)\n",
                    v.name.c_str(), med, v.us[0], bytes / (med * 1e3),
                    100.0 * bytes / (med * 1e3) / 8000.0);
    }
    return 0;
}
