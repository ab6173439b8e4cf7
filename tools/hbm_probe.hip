// tools/hbm_probe.hip — measured HBM ceilings for bench.py (not product).
//
// libaqz_hbm_probe.so exports one launcher: a contiguous read + write stream
// (non-temporal stores; loads non-temporal or plain, aqz_hbm_probe_ld) with a
// fixed read:write byte ratio (RD:WR 4 KiB
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

template<int RD, int WR, bool NTL = true>
__global__ __launch_bounds__(256) void
mix_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst, uint32_t* sink)
{
    const uint64_t rb = uint64_t(blockIdx.x) * 256 * RD + threadIdx.x;
    u32x4 v[RD];
#pragma unroll
    for (int k = 0; k < RD; ++k) {
        if constexpr (NTL)
            v[k] = __builtin_nontemporal_load(src + rb + k * 256);
        else
            v[k] = src[rb + k * 256];
    }
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

// Row-shaped probe: the cascade's read pattern without its arithmetic.  One
// wave per (frame, 16-row band, 1 KiB row segment) unit, four waves per
// workgroup; each lane loads 16 B from each of the band's 16 rows at
// row_bytes pitch (lanes past the row end idle, rows past the frame end
// skipped) and stores WR x 1 KiB contiguous, in unit order, with
// nontemporal stores.  At row_bytes = 8192 it is the headline's pattern; at
// 6000 or 10944 the rows split 128-B lines the way 3000^2 and 5472x3648
// frames do, so the two rates isolate what the frame pitch alone costs.
template<bool NTLOAD, int WR>
__global__ __launch_bounds__(256) void
rows_kernel(const uint8_t* __restrict__ src, uint32_t row_bytes, uint64_t pitch, uint32_t rows,
            uint64_t frame_stride, uint32_t bands, uint32_t segs, uint64_t units,
            u32x4* __restrict__ dst, uint32_t* sink)
{
    const uint64_t u = uint64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
    if (u >= units)
        return;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t seg = uint32_t(u % segs);
    const uint64_t fb = u / segs;
    const uint32_t band = uint32_t(fb % bands);
    const uint64_t frame = fb / bands;
    const uint32_t col = seg * 1024 + lane * 16;
    const uint8_t* base = src + frame * frame_stride + uint64_t(band) * 16 * pitch + col;
    const uint32_t nrows = min(16u, rows - band * 16);
    u32x4 v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        v[r] = u32x4{ 0, 0, 0, 0 };
        if (col < row_bytes && uint32_t(r) < nrows) {
            const auto* p = reinterpret_cast<const u32x4*>(base + uint64_t(r) * pitch);
            v[r] = NTLOAD ? __builtin_nontemporal_load(p) : *p;
        }
    }
    if constexpr (WR == 0) {
        uint32_t acc = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r)
            acc ^= v[r].x ^ v[r].y ^ v[r].z ^ v[r].w;
        if (acc == 0x12345678u)
            sink[0] = acc;
    } else {
        u32x4* o = dst + u * (64 * WR) + lane;
#pragma unroll
        for (int k = 0; k < WR; ++k) {
            u32x4 a = v[k];
#pragma unroll
            for (int j = k + WR; j < 16; j += WR)
                a ^= v[j];
            __builtin_nontemporal_store(a, o + k * 64);
        }
    }
}

} // namespace

extern "C" {

// Row-shaped probe (rows_kernel above) over `frames` frames of `rows` rows of
// `row_bytes` bytes (a multiple of 16), `pitch` bytes apart (>= row_bytes;
// twice row_bytes reads every other row, as Decimate does), frames
// `frame_stride` bytes apart (>= rows * pitch).  wr = 0 (read only) or 5
// (16:5, the cascade's 3:1 mix); `dst` must hold units * wr KiB, units =
// frames * ceil(rows/16) * ceil(row_bytes/1024).  nt_load picks
// nontemporal loads.  *moved_bytes = bytes read + bytes written.
int
aqz_hbm_probe_rows(const void* src, uint32_t row_bytes, uint64_t pitch, uint32_t rows,
                   uint64_t frame_stride, uint32_t frames, void* dst, void* sink, int wr,
                   int nt_load, void* stream, uint64_t* moved_bytes)
{
    if (!src || !sink || (wr && !dst) || row_bytes == 0 || row_bytes % 16 || rows == 0 ||
        frames == 0 || (wr != 0 && wr != 5) || pitch < row_bytes || pitch % 16 ||
        frame_stride < uint64_t(rows) * pitch)
        return int(hipErrorInvalidValue);
    const uint32_t bands = (rows + 15) / 16, segs = (row_bytes + 1023) / 1024;
    const uint64_t units = uint64_t(frames) * bands * segs;
    const uint64_t blocks = (units + 3) / 4;
    if (blocks >= (1ull << 31))
        return int(hipErrorInvalidValue);
    const auto s = static_cast<hipStream_t>(stream);
    const auto* in = static_cast<const uint8_t*>(src);
    auto* out = static_cast<u32x4*>(dst);
    auto* sk = static_cast<uint32_t*>(sink);
#define AQZ_ROWS(NT, W)                                                                 \
    hipLaunchKernelGGL((rows_kernel<NT, W>), dim3(blocks), dim3(256), 0, s, in, row_bytes, \
                       pitch, rows, frame_stride, bands, segs, units, out, sk)
    if (nt_load && wr)
        AQZ_ROWS(true, 5);
    else if (nt_load)
        AQZ_ROWS(true, 0);
    else if (wr)
        AQZ_ROWS(false, 5);
    else
        AQZ_ROWS(false, 0);
#undef AQZ_ROWS
    if (moved_bytes)
        *moved_bytes = uint64_t(frames) * rows * row_bytes + units * uint64_t(wr) * 1024;
    return int(hipGetLastError());
}

// Moves blocks * RD * 4 KiB in and blocks * WR * 4 KiB out, blocks =
// src_bytes / (RD * 4 KiB).  `dst` must hold blocks * WR * 4 KiB; `sink`
// 4 bytes.  Supported RD:WR = 16:0, 12:4, 13:3, 14:2, 10:6, 9:7.  Returns 0 or a
// hipError_t; *moved_bytes = bytes read + written.
int
aqz_hbm_probe_ld(const void* src, uint64_t src_bytes, void* dst, void* sink, int rd, int wr,
                 int nt_load, void* stream, uint64_t* moved_bytes)
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
#define AQZ_MIX(R, W)                                                                     \
    if (rd == R && wr == W) {                                                            \
        if (nt_load)                                                                     \
            hipLaunchKernelGGL((mix_kernel<R, W, true>), dim3(blocks), dim3(256), 0, s, in, \
                               out, sk);                                                 \
        else                                                                             \
            hipLaunchKernelGGL((mix_kernel<R, W, false>), dim3(blocks), dim3(256), 0, s, \
                               in, out, sk);                                             \
        if (moved_bytes)                                                                 \
            *moved_bytes = blocks * uint64_t(rd + wr) * 4096;                            \
        return int(hipGetLastError());                                                   \
    }
    AQZ_MIX(16, 0)
    AQZ_MIX(12, 4)
    AQZ_MIX(13, 3)
    AQZ_MIX(14, 2)
    AQZ_MIX(10, 6) // Decimate's mix: half the rows read
    AQZ_MIX(9, 7)
#undef AQZ_MIX
    return int(hipErrorInvalidValue);
}

// aqz_hbm_probe_ld with nontemporal loads (the round-1..4 ceiling).
int
aqz_hbm_probe(const void* src, uint64_t src_bytes, void* dst, void* sink, int rd, int wr,
              void* stream, uint64_t* moved_bytes)
{
    return aqz_hbm_probe_ld(src, src_bytes, dst, sink, rd, wr, 1, stream, moved_bytes);
}

} // extern "C"
