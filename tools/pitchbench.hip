// tools/pitchbench.hip — cost of row pitches that split 64/128-byte lines
// (not product).
//
// The cascade's level-1 stores are 512 B per wave instruction (64 lanes x
// 8 B) at row pitch 2*w1 bytes; its loads are 1 KiB per instruction at the
// input pitch.  This probe writes (or reads) ~768 MB as rows of a frame batch
// with a given pitch, each wave owning a 512-B (1 KiB) column segment of 8
// (16) consecutive rows, as the cascade's waves do, and reports GB/s for
// pitches that are / are not multiples of 64 and 128 bytes.
// Usage: tools/pitchbench [MiB] [reps] [policy]  (policy: also write-back
// stores and the XCD-contiguous block order)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/pitchbench.hip -o tools/pitchbench
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

typedef uint64_t u64_u __attribute__((aligned(1)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_u __attribute__((aligned(1)));

// segs_per_row segments of 512 B per row (the last one clipped to the row).
// NT: non-temporal stores (the product's), else plain write-back stores.
// REMAP: consecutive logical blocks on one XCD (hardware block b runs on
// XCD b % 8), so the waves that share a partial 64-B burst at a segment
// boundary usually write it through the same L2.
template<bool NT, bool REMAP>
__global__ __launch_bounds__(256) void
write_rows(uint8_t* dst, uint32_t pitch, uint32_t segs_per_row, uint32_t bands)
{
    const uint32_t lane = threadIdx.x & 63;
    uint32_t b = blockIdx.x;
    if constexpr (REMAP) {
        const uint32_t per = gridDim.x / 8; // gridDim.x is a multiple of 8 here
        b = (b % 8) * per + b / 8;
    }
    const uint32_t u = b * 4 + (threadIdx.x >> 6);
    if (u >= segs_per_row * bands)
        return;
    const uint32_t seg = u % segs_per_row, band = u / segs_per_row;
    const uint32_t col = seg * 512 + lane * 8;
    if (col + 8 > pitch)
        return;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        u64_u* p = reinterpret_cast<u64_u*>(dst + (uint64_t(band) * 8 + r) * pitch + col);
        if constexpr (NT)
            __builtin_nontemporal_store(uint64_t(u * 8 + r), p);
        else
            *p = uint64_t(u * 8 + r);
    }
}

__global__ __launch_bounds__(256) void
read_rows(const uint8_t* src, uint32_t pitch, uint32_t segs_per_row, uint32_t bands,
          uint32_t* sink)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t u = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (u >= segs_per_row * bands)
        return;
    const uint32_t seg = u % segs_per_row, band = u / segs_per_row;
    const uint32_t col = seg * 1024 + lane * 16;
    if (col + 16 > pitch)
        return;
    u32x4 v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r)
        v[r] = __builtin_nontemporal_load(
          reinterpret_cast<const u32x4_u*>(src + (uint64_t(band) * 16 + r) * pitch + col));
    uint32_t acc = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r)
        acc ^= v[r].x ^ v[r].y ^ v[r].z ^ v[r].w;
    if (acc == 0x12345678u)
        sink[0] = acc;
}

int
main(int argc, char** argv)
{
    const uint64_t bytes = uint64_t(argc > 1 ? std::atoi(argv[1]) : 768) << 20;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 20;
    uint8_t* buf;
    uint32_t* sink;
    CHECK(hipMalloc(&buf, bytes + 4096));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(buf, 1, bytes + 4096));
    struct V
    {
        std::string name;
        uint64_t moved;
        std::function<void()> run;
        std::vector<float> us;
    };
    std::vector<V> vs;
    const bool policies = argc > 3 && std::string(argv[3]) == "policy";
    for (uint32_t pitch : { 2048u, 2176u, 2112u, 2016u, 2032u, 2040u, 2000u }) {
        const uint32_t segs = (pitch + 511) / 512;
        const uint32_t bands = uint32_t(bytes / (uint64_t(pitch) * 8));
        const uint64_t moved = uint64_t(bands) * 8 * (pitch / 8 * 8);
        const uint32_t blocks = ((segs * bands + 3) / 4 + 7) / 8 * 8;
        auto add = [&](const char* tag, auto kern) {
            vs.push_back({ std::string("write ") + tag + " pitch " + std::to_string(pitch), moved,
                           [=] {
                               hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, buf, pitch,
                                                  segs, bands);
                           },
                           {} });
        };
        add("nt", write_rows<true, false>);
        if (policies) {
            add("wb", write_rows<false, false>);
            add("nt-xcd", write_rows<true, true>);
            add("wb-xcd", write_rows<false, true>);
        }
    }
    for (uint32_t pitch : { 4096u, 4352u, 4224u, 4032u, 4064u, 4080u, 4000u, 8192u, 8320u,
                            8448u, 8704u, 12288u, 16384u, 16512u }) {
        if (policies)
            break;
        const uint32_t segs = (pitch + 1023) / 1024;
        const uint32_t bands = uint32_t(bytes / (uint64_t(pitch) * 16));
        const uint64_t moved = uint64_t(bands) * 16 * (pitch / 16 * 16);
        vs.push_back({ "read pitch " + std::to_string(pitch), moved, [=] {
                          const uint32_t waves = segs * bands;
                          hipLaunchKernelGGL(read_rows, dim3((waves + 3) / 4), dim3(256), 0, 0,
                                             buf, pitch, segs, bands, sink);
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
    std::printf("%.0f MiB per pass; pitch %% 64 / %% 128 shown\n", bytes / 1048576.0);
    for (auto& v : vs) {
        std::sort(v.us.begin(), v.us.end());
        const float med = v.us[v.us.size() / 2];
        const uint32_t pitch = uint32_t(std::atoi(v.name.c_str() + v.name.rfind(' ') + 1));
        std::printf("%-24s (%%64=%2u %%128=%3u) median %8.1f us  %7.1f GB/s\n", v.name.c_str(),
                    pitch % 64, pitch % 128, med, v.moved / (med * 1e3));
    }
    return 0;
}
