// blosc_frame.cpp — c-blosc 1.x chunk frames around the GPU filter
// (include/aqz_blosc.h).
//
// Replaces, for the blosc codecs, the per-chunk call the reference makes in
// compress_in_place (zarr.common.cpp:106-137):
//   blosc_compress_ctx(clevel, shuffle, typesize, nbytes, src, dest,
//                      nbytes + 16, cname, blocksize 0, nthreads 1)
// The filter (byte / bit shuffle per block) is the GPU kernel behind
// aqz_blosc_filter_device; what stays on the host is the entropy coder and
// the frame layout, written here to produce c-blosc 1.21's bytes:
//   - compute_blocksize: 32 KiB base (x2 for zstd), scaled by clevel, then for
//     split codecs min(bs, 256 KiB) * typesize clamped to [64 KiB, 1 MiB];
//     capped at nbytes and rounded down to a typesize multiple;
//   - blocks are split into `typesize` streams (lz4; never zstd) unless the
//     block is the short leftover one or has < 128 elements;
//   - header: version 2, versionlz 1, flags (shuffle 0x1 / bitshuffle 0x4,
//     0x10 = not split, codec format << 5, memcpy 0x2), typesize, nbytes,
//     blocksize, total bytes; then one int32 start offset per block;
//   - every split: int32 size + codec output, compressed into at most the
//     split's own size (LZ4_compress_fast with acceleration 10 - clevel;
//     ZSTD_compress at 2*clevel - 1, clevel 9 -> ZSTD_maxCLevel()); a split
//     the codec cannot shrink is stored raw (filtered);
//   - a chunk that does not fit into the destination that way, clevel 0, or
//     nbytes < 128, is stored unfiltered after a header with 0x2 set.
// These rules were pinned against the image's libblosc 1.21.0 (which links
// the same liblz4 / libzstd this file loads) byte for byte:
// tests/test_blosc_frames.py.
#include "aqz_blosc.h"
#include "abi_guard.hh"
#include "codec_kernels.hh"

#include <hip/hip_runtime.h>

#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr size_t kHeader = 16;       // BLOSC_MAX_OVERHEAD
constexpr size_t kMinBuffer = 128;   // MIN_BUFFERSIZE
constexpr uint32_t kMaxSplits = 16;  // MAX_SPLITS
constexpr size_t kMaxBuffer = 0x7FFFFFFFu - kHeader; // BLOSC_MAX_BUFFERSIZE

enum Codec
{
    CODEC_LZ4 = 1, // BLOSC_LZ4_FORMAT
    CODEC_ZSTD = 4 // BLOSC_ZSTD_FORMAT
};

int
codec_of(const char* cname)
{
    if (!cname)
        return -1;
    if (std::strcmp(cname, "lz4") == 0)
        return CODEC_LZ4;
    if (std::strcmp(cname, "zstd") == 0)
        return CODEC_ZSTD;
    return -1;
}

// ---- codec libraries -------------------------------------------------------

struct CodecLibs
{
    int (*lz4_compress_fast)(const char*, char*, int, int, int) = nullptr;
    int (*lz4_version)(void) = nullptr;
    size_t (*zstd_compress)(void*, size_t, const void*, size_t, int) = nullptr;
    unsigned (*zstd_is_error)(size_t) = nullptr;
    int (*zstd_max_clevel)(void) = nullptr;
    unsigned (*zstd_version)(void) = nullptr;
    std::string info;
};

void*
open_first(const char* env, const char* const* names, std::string* which)
{
    std::vector<const char*> tries;
    if (const char* e = std::getenv(env); e && *e)
        tries.push_back(e);
    for (const char* const* n = names; *n; ++n)
        tries.push_back(*n);
    for (const char* t : tries)
        if (void* h = dlopen(t, RTLD_NOW | RTLD_LOCAL)) {
            *which = t;
            return h;
        }
    return nullptr;
}

const CodecLibs&
codec_libs()
{
    static const CodecLibs libs = [] {
        CodecLibs c;
        // c-blosc's own codec libraries first (the image's libblosc links
        // these), then whatever the loader finds.
        static const char* const lz4_names[] = { "/opt/conda/lib/liblz4.so.1", "liblz4.so.1",
                                                 nullptr };
        static const char* const zstd_names[] = { "/opt/conda/lib/libzstd.so.1", "libzstd.so.1",
                                                  nullptr };
        std::string lz4_path, zstd_path;
        if (void* h = open_first("AQZ_LZ4_LIB", lz4_names, &lz4_path)) {
            c.lz4_compress_fast =
              reinterpret_cast<decltype(c.lz4_compress_fast)>(dlsym(h, "LZ4_compress_fast"));
            c.lz4_version = reinterpret_cast<decltype(c.lz4_version)>(dlsym(h, "LZ4_versionNumber"));
        }
        if (void* h = open_first("AQZ_ZSTD_LIB", zstd_names, &zstd_path)) {
            c.zstd_compress = reinterpret_cast<decltype(c.zstd_compress)>(dlsym(h, "ZSTD_compress"));
            c.zstd_is_error = reinterpret_cast<decltype(c.zstd_is_error)>(dlsym(h, "ZSTD_isError"));
            c.zstd_max_clevel =
              reinterpret_cast<decltype(c.zstd_max_clevel)>(dlsym(h, "ZSTD_maxCLevel"));
            c.zstd_version = reinterpret_cast<decltype(c.zstd_version)>(dlsym(h, "ZSTD_versionNumber"));
        }
        auto ver = [](unsigned v) {
            return std::to_string(v / 10000) + "." + std::to_string(v / 100 % 100) + "." +
                   std::to_string(v % 100);
        };
        c.info = "lz4 " + (c.lz4_compress_fast && c.lz4_version
                             ? ver(static_cast<unsigned>(c.lz4_version())) + " (" + lz4_path + ")"
                             : std::string()) +
                 "; zstd " +
                 (c.zstd_compress && c.zstd_is_error && c.zstd_max_clevel && c.zstd_version
                    ? ver(c.zstd_version()) + " (" + zstd_path + ")"
                    : std::string());
        return c;
    }();
    return libs;
}

bool
codec_ready(int codec)
{
    const CodecLibs& c = codec_libs();
    if (codec == CODEC_LZ4)
        return c.lz4_compress_fast != nullptr;
    return c.zstd_compress && c.zstd_is_error && c.zstd_max_clevel;
}

// One split through the codec into at most `maxout` bytes; 0 when it does
// not fit (blosc_c's lz4_wrap_compress / zstd_wrap_compress).
size_t
compress_split(int codec, int clevel, const uint8_t* in, size_t n, uint8_t* out, size_t maxout)
{
    const CodecLibs& c = codec_libs();
    if (codec == CODEC_LZ4) {
        const int r = c.lz4_compress_fast(reinterpret_cast<const char*>(in),
                                          reinterpret_cast<char*>(out), static_cast<int>(n),
                                          static_cast<int>(maxout), 10 - clevel);
        return r > 0 ? static_cast<size_t>(r) : 0;
    }
    const int level = clevel < 9 ? 2 * clevel - 1 : c.zstd_max_clevel();
    const size_t r = c.zstd_compress(out, maxout, in, n, level);
    return c.zstd_is_error(r) ? 0 : r;
}

// ---- frame layout ----------------------------------------------------------

struct Params
{
    int clevel;
    int shuffle;
    uint32_t typesize;
    int codec;
};

bool
split_block(int codec, uint32_t typesize, size_t blocksize)
{
    return codec != CODEC_ZSTD && typesize <= kMaxSplits && blocksize / typesize >= kMinBuffer;
}

size_t
compute_blocksize(const Params& p, size_t nbytes)
{
    if (nbytes < p.typesize)
        return 1;
    size_t bs = nbytes;
    if (nbytes >= 32 * 1024) {
        bs = 32 * 1024;
        const bool hcr = p.codec == CODEC_ZSTD;
        if (hcr)
            bs *= 2;
        switch (p.clevel) {
            case 0: bs /= 4; break;
            case 1: bs /= 2; break;
            case 2: break;
            case 3: bs *= 2; break;
            case 4:
            case 5: bs *= 4; break;
            case 6:
            case 7:
            case 8: bs *= 8; break;
            default: bs *= hcr ? 16 : 8; break;
        }
    }
    if (p.clevel > 0 && split_block(p.codec, p.typesize, bs)) {
        bs = std::min<size_t>(bs, 1u << 18) * p.typesize;
        bs = std::max<size_t>(bs, 1u << 16);
        bs = std::min<size_t>(bs, 1u << 20);
    }
    bs = std::min(bs, nbytes);
    if (bs > p.typesize)
        bs = bs / p.typesize * p.typesize;
    return bs;
}

uint8_t
header_flags(const Params& p, size_t blocksize)
{
    uint8_t f = static_cast<uint8_t>(p.codec << 5);
    if (p.shuffle == AQZ_BLOSC_SHUFFLE)
        f |= 0x1;
    else if (p.shuffle == AQZ_BLOSC_BITSHUFFLE)
        f |= 0x4;
    if (!split_block(p.codec, p.typesize, blocksize))
        f |= 0x10;
    return f;
}

void
put32(uint8_t* d, uint32_t v)
{
    d[0] = static_cast<uint8_t>(v);
    d[1] = static_cast<uint8_t>(v >> 8);
    d[2] = static_cast<uint8_t>(v >> 16);
    d[3] = static_cast<uint8_t>(v >> 24);
}

void
put_header(uint8_t* d, const Params& p, uint8_t flags, size_t nbytes, size_t bs, size_t total)
{
    d[0] = 2; // BLOSC_VERSION_FORMAT
    d[1] = 1; // versionlz of lz4 and zstd
    d[2] = flags;
    d[3] = static_cast<uint8_t>(p.typesize);
    put32(d + 4, static_cast<uint32_t>(nbytes));
    put32(d + 8, static_cast<uint32_t>(bs));
    put32(d + 12, static_cast<uint32_t>(total));
}

// The filtered-block frame; returns its size, or 0 when c-blosc would fall
// back to storing the chunk unfiltered (or nothing fits).
size_t
blocks_frame(const Params& p, const uint8_t* filt, size_t nbytes, size_t bs, uint8_t* dest,
             size_t destsize)
{
    const size_t nblocks = (nbytes + bs - 1) / bs;
    size_t nt = kHeader + 4 * nblocks;
    if (nt > destsize)
        return 0;
    const bool split = split_block(p.codec, p.typesize, bs);
    for (size_t b = 0; b < nblocks; ++b) {
        const size_t off = b * bs;
        const size_t bsize = std::min(bs, nbytes - off);
        const bool leftover = bsize < bs;
        const size_t nsplits = (split && !leftover) ? p.typesize : 1;
        const size_t neb = bsize / nsplits;
        put32(dest + kHeader + 4 * b, static_cast<uint32_t>(nt));
        for (size_t j = 0; j < nsplits; ++j) {
            const uint8_t* piece = filt + off + j * neb;
            nt += 4;
            if (nt >= destsize)
                return 0;
            const size_t maxout = std::min(neb, destsize - nt);
            size_t c = compress_split(p.codec, p.clevel, piece, neb, dest + nt, maxout);
            if (c == 0 || c == neb) {
                if (nt + neb > destsize)
                    return 0;
                std::memcpy(dest + nt, piece, neb);
                c = neb;
            }
            put32(dest + nt - 4, static_cast<uint32_t>(c));
            nt += c;
        }
    }
    put_header(dest, p, header_flags(p, bs), nbytes, bs, nt);
    return nt;
}

// Frame of one chunk; *raw set when the caller must put the unfiltered
// chunk at dest + 16 (the header is written).  Returns 0 when nothing fits.
size_t
write_frame(const Params& p, const uint8_t* filt, size_t nbytes, uint8_t* dest, size_t destsize,
            bool* raw)
{
    *raw = false;
    const size_t bs = compute_blocksize(p, nbytes);
    if (p.clevel != 0 && nbytes >= kMinBuffer) {
        if (const size_t n = blocks_frame(p, filt, nbytes, bs, dest, destsize))
            return n;
    }
    if (destsize < nbytes + kHeader)
        return 0;
    put_header(dest, p, static_cast<uint8_t>(header_flags(p, bs) | 0x2), nbytes, bs,
               nbytes + kHeader);
    *raw = true;
    return nbytes + kHeader;
}

int
check_params(int clevel, int shuffle, uint32_t typesize, const char* cname, Params* p)
{
    const int codec = codec_of(cname);
    if (clevel < 0 || clevel > 9 || typesize == 0 || codec < 0 || shuffle < AQZ_BLOSC_NOSHUFFLE ||
        shuffle > AQZ_BLOSC_BITSHUFFLE) {
        aqz::set_last_error("blosc: invalid clevel, shuffle, typesize or codec name");
        return AQZ_INVALID_ARGUMENT;
    }
    if (!codec_ready(codec)) {
        aqz::set_last_error(std::string("blosc: codec library not loaded: ") +
                            codec_libs().info);
        return AQZ_INTERNAL_ERROR;
    }
    *p = Params{ clevel, shuffle, typesize > 255 ? 1u : typesize, codec };
    return AQZ_OK;
}

} // namespace

struct aqz_blosc_ctx
{
    int device = 0;
    unsigned n_threads = 1;
    void* d_filtered = nullptr;
    size_t d_cap = 0;
    uint8_t* h_filtered = nullptr; // pinned
    size_t h_cap = 0;
    std::vector<hipEvent_t> events; // one per D2H group
};

namespace {

void
release(aqz_blosc_ctx* c)
{
    for (hipEvent_t e : c->events)
        (void)hipEventDestroy(e);
    c->events.clear();
    if (c->d_filtered)
        (void)hipFree(c->d_filtered);
    if (c->h_filtered)
        (void)hipHostFree(c->h_filtered);
    c->d_filtered = nullptr;
    c->h_filtered = nullptr;
    c->d_cap = c->h_cap = 0;
}

int
hip_status(hipError_t e, const char* who)
{
    if (e == hipSuccess)
        return AQZ_OK;
    aqz::set_last_error(std::string("blosc_compress_device: ") + who + ": " +
                        hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? AQZ_OUT_OF_MEMORY : AQZ_INTERNAL_ERROR;
}

#define BLOSC_HIP(call, who)                                                                       \
    do {                                                                                           \
        const int rc_ = hip_status((call), who);                                                   \
        if (rc_ != AQZ_OK)                                                                         \
            return rc_;                                                                            \
    } while (0)

// Raw (unfiltered) device chunks into their frames, after the header.
int
copy_raw(const uint8_t* d_src, size_t nbytes, uint8_t* host_dst, size_t stride,
         const std::vector<uint32_t>& which)
{
    for (uint32_t k : which)
        BLOSC_HIP(hipMemcpy(host_dst + k * stride + kHeader, d_src + k * nbytes, nbytes,
                            hipMemcpyDeviceToHost),
                  "raw copy");
    return AQZ_OK;
}

} // namespace

extern "C" {

int
aqz_blosc_blocksize(int clevel, uint32_t typesize, size_t nbytes, const char* cname,
                    uint32_t* blocksize)
{
    try {
        const int codec = codec_of(cname);
        if (!blocksize || clevel < 0 || clevel > 9 || typesize == 0 || codec < 0 ||
            nbytes > kMaxBuffer) {
            aqz::set_last_error("blosc_blocksize: invalid argument");
            return AQZ_INVALID_ARGUMENT;
        }
        const Params p{ clevel, 0, typesize > 255 ? 1u : typesize, codec };
        *blocksize = static_cast<uint32_t>(compute_blocksize(p, nbytes));
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(nullptr);
    }
}

int
aqz_blosc_frame_from_filtered(int clevel, int shuffle, uint32_t typesize, const char* cname,
                              const void* filtered, const void* src, size_t nbytes, void* dest,
                              size_t destsize, size_t* frame_bytes, int* raw_needed)
{
    try {
        if (!frame_bytes || !dest || (!filtered && nbytes) || (!src && !raw_needed) ||
            nbytes == 0 || nbytes > kMaxBuffer) {
            aqz::set_last_error("blosc_frame_from_filtered: invalid argument");
            return AQZ_INVALID_ARGUMENT;
        }
        Params p{};
        if (const int rc = check_params(clevel, shuffle, typesize, cname, &p); rc != AQZ_OK)
            return rc;
        bool raw = false;
        auto* d = static_cast<uint8_t*>(dest);
        *frame_bytes = write_frame(p, static_cast<const uint8_t*>(filtered), nbytes, d, destsize,
                                   &raw);
        if (raw && src)
            std::memcpy(d + kHeader, src, nbytes);
        if (raw_needed)
            *raw_needed = raw && !src;
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(nullptr);
    }
}

int
aqz_blosc_ctx_create(int device, uint32_t n_threads, aqz_blosc_ctx** out)
{
    try {
        if (!out) {
            aqz::set_last_error("blosc_ctx_create: null out");
            return AQZ_INVALID_ARGUMENT;
        }
        *out = nullptr;
        int n_dev = 0;
        if (hipGetDeviceCount(&n_dev) != hipSuccess || device < 0 || device >= n_dev) {
            aqz::set_last_error("blosc_ctx_create: no such device");
            return AQZ_INVALID_ARGUMENT;
        }
        auto* c = new aqz_blosc_ctx;
        c->device = device;
        const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
        c->n_threads = n_threads ? n_threads : std::min(16u, hw);
        *out = c;
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(nullptr);
    }
}

void
aqz_blosc_ctx_destroy(aqz_blosc_ctx* ctx)
{
    if (!ctx)
        return;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(ctx->device);
    release(ctx);
    (void)hipSetDevice(prev);
    delete ctx;
}

int
aqz_blosc_compress_device(aqz_blosc_ctx* ctx, int clevel, int shuffle, uint32_t typesize,
                          const char* cname, const void* device_src, size_t nbytes,
                          uint32_t n_buffers, void* host_dst, size_t dst_stride,
                          size_t* frame_bytes, void* hip_stream)
{
    try {
        if (!ctx || !device_src || !host_dst || !frame_bytes || n_buffers == 0 || nbytes == 0 ||
            nbytes > kMaxBuffer || dst_stride < nbytes + kHeader) {
            aqz::set_last_error("blosc_compress_device: invalid argument");
            return AQZ_INVALID_ARGUMENT;
        }
        Params p{};
        if (const int rc = check_params(clevel, shuffle, typesize, cname, &p); rc != AQZ_OK)
            return rc;
        int prev = 0;
        (void)hipGetDevice(&prev);
        struct Restore
        {
            int d;
            ~Restore() { (void)hipSetDevice(d); }
        } restore{ prev };
        BLOSC_HIP(hipSetDevice(ctx->device), "set device");
        auto stream = static_cast<hipStream_t>(hip_stream);
        const auto* src = static_cast<const uint8_t*>(device_src);
        auto* dst = static_cast<uint8_t*>(host_dst);
        const size_t bs = compute_blocksize(p, nbytes);

        if (clevel == 0 || nbytes < kMinBuffer) {
            // c-blosc stores these unfiltered: header + one strided D2H
            bool raw = false;
            for (uint32_t k = 0; k < n_buffers; ++k)
                frame_bytes[k] = write_frame(p, nullptr, nbytes, dst + k * dst_stride, dst_stride,
                                             &raw);
            BLOSC_HIP(hipMemcpy2DAsync(dst + kHeader, dst_stride, src, nbytes, nbytes, n_buffers,
                                       hipMemcpyDeviceToHost, stream),
                      "raw copy");
            BLOSC_HIP(hipStreamSynchronize(stream), "sync");
            return AQZ_OK;
        }

        const size_t total = nbytes * n_buffers;
        if (ctx->d_cap < total) {
            if (ctx->d_filtered)
                BLOSC_HIP(hipFree(ctx->d_filtered), "free");
            ctx->d_filtered = nullptr;
            ctx->d_cap = 0;
            BLOSC_HIP(hipMalloc(&ctx->d_filtered, total), "device scratch");
            ctx->d_cap = total;
        }
        if (ctx->h_cap < total) {
            if (ctx->h_filtered)
                BLOSC_HIP(hipHostFree(ctx->h_filtered), "free pinned");
            ctx->h_filtered = nullptr;
            ctx->h_cap = 0;
            BLOSC_HIP(hipHostMalloc(reinterpret_cast<void**>(&ctx->h_filtered), total), "pinned staging");
            ctx->h_cap = total;
        }
        // groups of about 4 MiB cross PCIe one after another; the host
        // compresses a group as soon as its copy has landed
        const uint32_t per_group =
          static_cast<uint32_t>(std::clamp<size_t>((4u << 20) / nbytes, 1, n_buffers));
        const uint32_t n_groups = (n_buffers + per_group - 1) / per_group;
        while (ctx->events.size() < n_groups) {
            hipEvent_t e;
            BLOSC_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
            ctx->events.push_back(e);
        }
        // From the filter launch on, work that reads or writes ctx's scratch
        // is queued on `stream`: every exit drains it first, so a failed call
        // never leaves a copy into h_filtered in flight for the next one.
        struct Drain
        {
            hipStream_t s;
            ~Drain() { (void)hipStreamSynchronize(s); }
        } drain{ stream };
        BLOSC_HIP(aqz::launch_blosc_filter(shuffle, p.typesize, static_cast<uint32_t>(bs), src,
                                           nbytes, n_buffers, ctx->d_filtered, stream),
                  "filter");
        const auto* dfilt = static_cast<const uint8_t*>(ctx->d_filtered);
        for (uint32_t g = 0; g < n_groups; ++g) {
            const size_t k0 = static_cast<size_t>(g) * per_group;
            const size_t kn = std::min<size_t>(per_group, n_buffers - k0);
            BLOSC_HIP(hipMemcpyAsync(ctx->h_filtered + k0 * nbytes, dfilt + k0 * nbytes,
                                     kn * nbytes, hipMemcpyDeviceToHost, stream),
                      "copy");
            BLOSC_HIP(hipEventRecord(ctx->events[g], stream), "record");
        }

        std::atomic<uint32_t> next{ 0 };
        std::atomic<int> failed{ AQZ_OK };
        std::mutex raw_mu;
        std::vector<uint32_t> raw_ids;
        auto work = [&] {
            for (;;) {
                const uint32_t k = next.fetch_add(1);
                if (k >= n_buffers || failed.load() != AQZ_OK)
                    return;
                if (hipEventSynchronize(ctx->events[k / per_group]) != hipSuccess) {
                    failed.store(AQZ_INTERNAL_ERROR);
                    return;
                }
                bool raw = false;
                frame_bytes[k] = write_frame(p, ctx->h_filtered + static_cast<size_t>(k) * nbytes,
                                             nbytes, dst + k * dst_stride, dst_stride, &raw);
                if (raw) {
                    std::lock_guard<std::mutex> lock(raw_mu);
                    raw_ids.push_back(k);
                }
            }
        };
        const unsigned nt = std::min<unsigned>(ctx->n_threads, n_buffers);
        std::vector<std::thread> pool;
        pool.reserve(nt > 0 ? nt - 1 : 0);
        for (unsigned t = 1; t < nt; ++t)
            pool.emplace_back(work);
        work();
        for (auto& t : pool)
            t.join();
        if (failed.load() != AQZ_OK) {
            // the later groups' copies into ctx->h_filtered may still be
            // queued: drain `stream` here (Drain does it again on the way
            // out) so the ctx can be reused or destroyed at once
            (void)hipStreamSynchronize(stream);
            aqz::set_last_error("blosc_compress_device: staged copy failed");
            return failed.load();
        }
        // chunks c-blosc would store unfiltered (incompressible ones)
        return copy_raw(src, nbytes, dst, dst_stride, raw_ids);
    } catch (...) {
        return ABI_GUARD_FAIL(nullptr);
    }
}

const char*
aqz_blosc_codec_info(void)
{
    try {
        return codec_libs().info.c_str();
    } catch (...) {
        return "";
    }
}

} // extern "C"
