// tools/e2e_probe.cpp — component timings of the host->GPU->host path for one
// 4096^2 u16 frame (33.5 MB in, 11.1 MB of levels out).  Not product code.
// Build: hipcc -O2 -std=c++20 tools/e2e_probe.cpp -o tools/e2e_probe -lpthread
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CHECK(x)                                                               \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
            std::exit(2);                                                      \
        }                                                                      \
    } while (0)

using clk = std::chrono::steady_clock;

template<typename F>
double
best_ms(F&& f, int reps = 7)
{
    double best = 1e30;
    for (int i = 0; i < reps; ++i) {
        auto t0 = clk::now();
        f();
        const double ms =
          std::chrono::duration<double, std::milli>(clk::now() - t0).count();
        best = std::min(best, ms);
    }
    return best;
}

void
par_memcpy(void* dst, const void* src, size_t n, int threads)
{
    std::vector<std::thread> ts;
    const size_t per = (n / threads + 4095) & ~size_t(4095);
    for (int t = 0; t < threads; ++t) {
        const size_t off = per * t;
        if (off >= n)
            break;
        const size_t len = std::min(per, n - off);
        ts.emplace_back([=] {
            std::memcpy(static_cast<char*>(dst) + off,
                        static_cast<const char*>(src) + off, len);
        });
    }
    for (auto& t : ts)
        t.join();
}

int
main()
{
    const size_t in = size_t(4096) * 4096 * 2;
    const size_t out = 11141120;
    std::vector<uint8_t> pageable(in), pageable_out(out);
    for (size_t i = 0; i < in; ++i)
        pageable[i] = uint8_t(i * 131);
    void *pinned, *pinned_out, *dev, *dev_out;
    CHECK(hipHostMalloc(&pinned, in, hipHostMallocDefault));
    CHECK(hipHostMalloc(&pinned_out, out, hipHostMallocDefault));
    CHECK(hipMalloc(&dev, in));
    CHECK(hipMalloc(&dev_out, out));
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));

    std::printf("memcpy pageable->pinned 1 thread : %7.3f ms\n",
                best_ms([&] { std::memcpy(pinned, pageable.data(), in); }));
    for (int t : { 2, 4, 8 })
        std::printf("memcpy pageable->pinned %d threads: %7.3f ms\n", t,
                    best_ms([&] { par_memcpy(pinned, pageable.data(), in, t); }));
    std::printf("H2D pinned 33.5 MB              : %7.3f ms\n", best_ms([&] {
                    CHECK(hipMemcpyAsync(dev, pinned, in, hipMemcpyHostToDevice, s));
                    CHECK(hipStreamSynchronize(s));
                }));
    std::printf("H2D pageable 33.5 MB            : %7.3f ms\n", best_ms([&] {
                    CHECK(hipMemcpyAsync(dev, pageable.data(), in,
                                         hipMemcpyHostToDevice, s));
                    CHECK(hipStreamSynchronize(s));
                }));
    std::printf("D2H pinned 11.1 MB              : %7.3f ms\n", best_ms([&] {
                    CHECK(hipMemcpyAsync(pinned_out, dev_out, out,
                                         hipMemcpyDeviceToHost, s));
                    CHECK(hipStreamSynchronize(s));
                }));
    std::printf("memcpy pinned->pageable 11.1 MB : %7.3f ms\n",
                best_ms([&] { std::memcpy(pageable_out.data(), pinned_out, out); }));
    std::printf("hipHostRegister+Unregister 33.5 MB: %7.3f ms\n", best_ms([&] {
                    CHECK(hipHostRegister(pageable.data(), in, hipHostRegisterDefault));
                    CHECK(hipHostUnregister(pageable.data()));
                }, 3));
    CHECK(hipHostRegister(pageable.data(), in, hipHostRegisterDefault));
    std::printf("H2D registered 33.5 MB          : %7.3f ms\n", best_ms([&] {
                    CHECK(hipMemcpyAsync(dev, pageable.data(), in,
                                         hipMemcpyHostToDevice, s));
                    CHECK(hipStreamSynchronize(s));
                }));
    CHECK(hipHostUnregister(pageable.data()));
    // chunked: memcpy chunk k+1 while chunk k is in flight
    for (int chunks : { 4, 8, 16 }) {
        const size_t cs = in / chunks;
        std::printf("chunked stage+H2D (%2d chunks)    : %7.3f ms\n", chunks,
                    best_ms([&] {
                        for (int k = 0; k < chunks; ++k) {
                            std::memcpy(static_cast<char*>(pinned) + k * cs,
                                        pageable.data() + k * cs, cs);
                            CHECK(hipMemcpyAsync(static_cast<char*>(dev) + k * cs,
                                                 static_cast<char*>(pinned) + k * cs,
                                                 cs, hipMemcpyHostToDevice, s));
                        }
                        CHECK(hipStreamSynchronize(s));
                    }));
    }
    return 0;
}
