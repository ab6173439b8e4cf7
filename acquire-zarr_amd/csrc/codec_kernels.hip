// codec_kernels.hip — byte-level codec stages beside the pyramid on gfx950
// (SURVEY §8(f) rows 3-4), behind include/aqz_codec.h.
//
//  * blosc filters: the bytes c-blosc hands its codec for every block of a
//    chunk buffer (blosc_c's shuffle step; the reference calls
//    blosc_compress_ctx from compress_in_place, zarr.common.cpp:106-137, on
//    each chunk, chunk.cpp:78-105).  Byte shuffle gathers byte j of every
//    element into plane j; bit shuffle (bitshuffle's bshuf_trans_bit_elem)
//    writes bit row j*8+b = bit b of byte j of every element, LSB first.
//    Both are pure permutations: HBM-bound, nbytes read + nbytes written.
//  * crc32c: the Castagnoli CRC of a shard index table (shard.cpp:145-166),
//    batched over many buffers: 16 KiB of a buffer per workgroup, or several
//    small buffers packed into one workgroup.
//
// Restated from the published algorithms (c-blosc 1.21 shuffle-generic.c /
// bitshuffle-generic.c; RFC 3720 CRC-32C); the CPU restatement the tests
// compare against is oracle/codec_oracle.c.
#include "codec_kernels.hh"

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

namespace aqz {

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_u __attribute__((aligned(1))); // any byte alignment (gfx950 global loads)

// A run of equally sized blocks: block g of the run starts at
// (g / per) * stride + first + (g % per) * bs.  A launch covers blocks
// g0 .. g0 + n_blocks - 1 and fewer than 2^31 threads, so thread ids and
// in-launch divisions stay 32-bit.
struct BlockRun
{
    uint64_t stride; // bytes between buffers
    uint64_t first;  // offset of the run's first block within a buffer
    uint32_t per;    // blocks of the run per buffer
    uint32_t bs;     // block size in bytes
    uint32_t g0;     // first block of this launch
};

__device__ __forceinline__ uint64_t
block_base(const BlockRun& r, uint32_t g)
{
    g += r.g0;
    return uint64_t(g / r.per) * r.stride + r.first + uint64_t(g % r.per) * r.bs;
}

// 8x8 bit-matrix transpose (bitshuffle's TRANS_BIT_8X8): bit 8r+c -> 8c+r
__device__ __forceinline__ uint64_t
trans_bit_8x8(uint64_t x)
{
    uint64_t t;
    t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
    x = x ^ t ^ (t << 7);
    t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
    x = x ^ t ^ (t << 14);
    t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
    x = x ^ t ^ (t << 28);
    return x;
}

// ---- byte shuffle -----------------------------------------------------------

// Vector form, TS in {2, 4, 8, 16}: one thread = 8 elements (8*TS bytes in,
// TS 8-byte stores out, lanes contiguous per plane).  Needs every block of
// the run to hold a multiple of 8 elements and 16-B aligned block bases.
template<int TS>
__global__ __launch_bounds__(256) void
shuffle_vec_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, BlockRun run,
                   uint32_t n_blocks)
{
    const uint32_t groups = run.bs / (8 * TS); // 8-element groups per block
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= groups * n_blocks)
        return;
    const uint32_t g = gid / groups;
    const uint32_t q = gid % groups;
    const uint64_t base = block_base(run, g);
    const uint32_t ne = run.bs / TS;
    constexpr int NV = (8 * TS) / 16; // 16-B loads per thread
    u32x4 v[NV];
    const auto* s = reinterpret_cast<const u32x4*>(src + base + uint64_t(q) * 8 * TS);
#pragma unroll
    for (int k = 0; k < NV; ++k)
        v[k] = __builtin_nontemporal_load(s + k);
    uint8_t e[8 * TS];
    __builtin_memcpy(e, v, sizeof(e));
#pragma unroll
    for (int j = 0; j < TS; ++j) {
        uint64_t w = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            w |= uint64_t(e[k * TS + j]) << (8 * k);
        __builtin_nontemporal_store(
          w, reinterpret_cast<uint64_t*>(dst + base + uint64_t(j) * ne + uint64_t(q) * 8));
    }
}

// Any typesize and block size: one thread per output byte (shuffle_generic).
__global__ __launch_bounds__(256) void
shuffle_generic_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, BlockRun run,
                       uint32_t n_blocks, uint32_t ts)
{
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= run.bs * n_blocks)
        return;
    const uint32_t g = gid / run.bs;
    const uint32_t o = gid % run.bs;
    const uint64_t base = block_base(run, g);
    const uint32_t ne = run.bs / ts;
    uint8_t v;
    if (o < ne * ts) {
        const uint32_t j = o / ne, i = o % ne;
        v = src[base + uint64_t(i) * ts + j];
    } else {
        v = src[base + o]; // blocksize % typesize tail
    }
    dst[base + o] = v;
}

// ---- bit shuffle ------------------------------------------------------------

// Vector form, TS in {1, 2, 4, 8}: one thread = G groups of 8 elements
// (128 contiguous input bytes); for each of the 8*TS bit rows it writes G
// bytes.  Needs (elements/8) % G == 0 per block, so row stores stay aligned.
template<int TS>
constexpr int kBitGroups = 16 / TS;

// 32x32 bit-matrix transpose in registers, LSB first: afterwards bit e of
// a[r] is what bit r of a[e] was.  Five block-swap stages of 16 word pairs.
__device__ __forceinline__ void
transpose_bits_32(uint32_t (&a)[32])
{
#pragma unroll
    for (int st = 0; st < 5; ++st) {
        const int s = 16 >> st;
        const uint32_t m = st == 0   ? 0x0000FFFFu
                           : st == 1 ? 0x00FF00FFu
                           : st == 2 ? 0x0F0F0F0Fu
                           : st == 3 ? 0x33333333u
                                     : 0x55555555u;
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            if (i & s)
                continue;
            const uint32_t t = ((a[i] >> s) ^ a[i + s]) & m;
            a[i + s] ^= t;
            a[i] ^= t << s;
        }
    }
}

template<int TS, int WAVES = 4, bool WORDS = true>
__global__ __launch_bounds__(64 * WAVES) void
bitshuffle_vec_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, BlockRun run,
                      uint32_t n_blocks)
{
    constexpr int G = kBitGroups<TS>;
    // Per wave: 64 threads x 128 input bytes, one 16-B pad per thread row so
    // the per-thread reads below are bank-conflict free.
    __shared__ u32x4 stage[WAVES][64][9];
    const uint32_t ne = run.bs / TS;
    const uint32_t row = ne / 8;          // bytes per bit row
    const uint32_t per_thread = row / G;  // threads per block
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = gid < per_thread * n_blocks;
    const uint32_t g = active ? gid / per_thread : 0;
    const uint32_t t = active ? gid % per_thread : 0;
    const uint64_t base = block_base(run, g);
    // Coalesced staging: load k of lane l fetches 16 B (l % 8) of thread
    // 8k + l/8's 128 input bytes, so each load instruction reads 8 whole
    // 128-B segments (1 KiB contiguous when the threads' segments are) instead
    // of 64 scattered 16-B pieces.  Measured on MI355X: 18.7 -> see DESIGN.
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const uint64_t sp = active ? reinterpret_cast<uint64_t>(src + base + uint64_t(t) * 128) : 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int owner = k * 8 + (lane >> 3);
        const uint64_t osp = __shfl(static_cast<unsigned long long>(sp), owner);
        u32x4 q = { 0u, 0u, 0u, 0u };
        if (osp)
            q = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(osp) + (lane & 7));
        stage[w][owner][lane & 7] = q;
    }
    __syncthreads();
    if (!active)
        return;
    u32x4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
        v[k] = stage[w][lane][k];
    if constexpr (WORDS && TS >= 2) {
        // The thread's 128 B as one 32x32 bit matrix whose transpose holds
        // every bit row (bit r of element e is bit e of bit row r, LSB first):
        //  TS = 4: 32 elements, a[e] = element e, row r = a[r];
        //  TS = 8: 16 elements, a[e] / a[16 + e] = low / high word of element
        //          e, rows r and 32 + r = low / high half of a[r];
        //  TS = 2: 64 elements, a[e] = element e | element 32 + e << 16,
        //          row r = a[r] | a[16 + r] << 32.
        // About a third of the per-byte gather, transpose and scatter work.
        uint32_t wd[32];
        __builtin_memcpy(wd, v, sizeof(wd));
        uint32_t a[32];
#pragma unroll
        for (int e = 0; e < 32; ++e) {
            if constexpr (TS == 4)
                a[e] = wd[e];
            else if constexpr (TS == 8)
                a[e] = e < 16 ? wd[2 * e] : wd[2 * (e - 16) + 1];
            else
                a[e] = (e & 1) ? (wd[e / 2] >> 16) | (wd[16 + e / 2] & 0xFFFF0000u)
                               : (wd[e / 2] & 0xFFFFu) | (wd[16 + e / 2] << 16);
        }
        transpose_bits_32(a);
        uint8_t* d = dst + base + uint64_t(t) * G;
        if constexpr (TS == 4) {
#pragma unroll
            for (int r = 0; r < 32; ++r)
                __builtin_nontemporal_store(a[r], reinterpret_cast<uint32_t*>(d + uint64_t(r) * row));
        } else if constexpr (TS == 8) {
#pragma unroll
            for (int r = 0; r < 32; ++r) {
                __builtin_nontemporal_store(uint16_t(a[r]),
                                            reinterpret_cast<uint16_t*>(d + uint64_t(r) * row));
                __builtin_nontemporal_store(
                  uint16_t(a[r] >> 16), reinterpret_cast<uint16_t*>(d + uint64_t(32 + r) * row));
            }
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r)
                __builtin_nontemporal_store(uint64_t(a[r]) | (uint64_t(a[16 + r]) << 32),
                                            reinterpret_cast<uint64_t*>(d + uint64_t(r) * row));
        }
        return;
    }
    uint8_t e[128];
    __builtin_memcpy(e, v, sizeof(e));
    // out[r] collects G bytes of bit row r (byte gi = group gi of this thread)
    uint64_t out[8 * TS][(G + 7) / 8];
#pragma unroll
    for (int r = 0; r < 8 * TS; ++r)
#pragma unroll
        for (int w = 0; w < (G + 7) / 8; ++w)
            out[r][w] = 0;
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
#pragma unroll
        for (int j = 0; j < TS; ++j) {
            uint64_t x = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k)
                x |= uint64_t(e[(gi * 8 + k) * TS + j]) << (8 * k);
            x = trans_bit_8x8(x);
#pragma unroll
            for (int b = 0; b < 8; ++b)
                out[j * 8 + b][gi / 8] |= ((x >> (8 * b)) & 0xFFull) << (8 * (gi % 8));
        }
    }
#pragma unroll
    for (int r = 0; r < 8 * TS; ++r) {
        uint8_t* d = dst + base + uint64_t(r) * row + uint64_t(t) * G;
        if constexpr (G == 16) {
            u32x4 q;
            __builtin_memcpy(&q, out[r], 16);
            __builtin_nontemporal_store(q, reinterpret_cast<u32x4*>(d));
        } else if constexpr (G == 8) {
            __builtin_nontemporal_store(out[r][0], reinterpret_cast<uint64_t*>(d));
        } else if constexpr (G == 4) {
            __builtin_nontemporal_store(uint32_t(out[r][0]), reinterpret_cast<uint32_t*>(d));
        } else {
            __builtin_nontemporal_store(uint16_t(out[r][0]), reinterpret_cast<uint16_t*>(d));
        }
    }
}

// Any typesize: one thread per output byte.  Blocks whose element count is
// not a multiple of 8 are copied (c-blosc 1.x bitshuffle()).
__global__ __launch_bounds__(256) void
bitshuffle_generic_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, BlockRun run,
                          uint32_t n_blocks, uint32_t ts)
{
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= run.bs * n_blocks)
        return;
    const uint32_t g = gid / run.bs;
    const uint32_t o = gid % run.bs;
    const uint64_t base = block_base(run, g);
    const uint32_t ne = run.bs / ts;
    uint8_t v;
    if (ne % 8 != 0 || o >= ne * ts) {
        v = src[base + o];
    } else {
        const uint32_t row = ne / 8;
        const uint32_t r = o / row, m = o % row;
        const uint32_t j = r / 8, b = r % 8;
        uint32_t acc = 0;
        for (uint32_t k = 0; k < 8; ++k)
            acc |= ((uint32_t(src[base + uint64_t(8 * m + k) * ts + j]) >> b) & 1u) << k;
        v = uint8_t(acc);
    }
    dst[base + o] = v;
}

__global__ __launch_bounds__(256) void
copy_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, BlockRun run,
            uint32_t n_blocks)
{
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= run.bs * n_blocks)
        return;
    const uint32_t g = gid / run.bs;
    const uint32_t o = gid % run.bs;
    const uint64_t base = block_base(run, g);
    dst[base + o] = src[base + o];
}

// Launch one kernel over blocks [g0, g0 + n) of a run; `threads_per_block`
// threads per data block.
template<typename L>
hipError_t
split_launch(BlockRun run, uint32_t n_blocks, uint64_t threads_per_block, L&& launch)
{
    if (threads_per_block == 0)
        return hipSuccess;
    const uint64_t cap = (1ull << 31) / threads_per_block; // blocks per launch
    if (cap == 0)
        return hipErrorInvalidValue;
    for (uint64_t g = 0; g < n_blocks; g += cap) {
        const uint32_t n = uint32_t(n_blocks - g < cap ? n_blocks - g : cap);
        run.g0 = uint32_t(g);
        launch(run, n, uint32_t((threads_per_block * n + 255) / 256));
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess)
            return e;
    }
    return hipSuccess;
}

// One run of equal blocks through the right kernel for `shuffle`.
hipError_t
filter_run(int shuffle, uint32_t ts, const uint8_t* src, uint8_t* dst, const BlockRun& run,
           uint32_t n_blocks, bool aligned, hipStream_t stream)
{
    if (n_blocks == 0 || run.bs == 0)
        return hipSuccess;
    const uint32_t ne = run.bs / ts;
    const bool doshuffle = shuffle == 1 && ts > 1;
    const bool dobit = shuffle == 2 && run.bs >= ts;
    auto generic = [&](auto kernel) {
        return split_launch(run, n_blocks, run.bs, [&](BlockRun r, uint32_t n, uint32_t grid) {
            hipLaunchKernelGGL(kernel, dim3(grid), dim3(256), 0, stream, src, dst, r, n, ts);
        });
    };
    if (doshuffle) {
        const bool vec = aligned && run.bs % 16 == 0 && run.bs % ts == 0 && ne % 8 == 0 &&
                         (ts == 2 || ts == 4 || ts == 8 || ts == 16);
        if (!vec)
            return generic(shuffle_generic_kernel);
        return split_launch(run, n_blocks, run.bs / (8 * ts),
                            [&](BlockRun r, uint32_t n, uint32_t grid) {
            switch (ts) {
                case 2:
                    hipLaunchKernelGGL(shuffle_vec_kernel<2>, dim3(grid), dim3(256), 0, stream,
                                       src, dst, r, n);
                    break;
                case 4:
                    hipLaunchKernelGGL(shuffle_vec_kernel<4>, dim3(grid), dim3(256), 0, stream,
                                       src, dst, r, n);
                    break;
                case 8:
                    hipLaunchKernelGGL(shuffle_vec_kernel<8>, dim3(grid), dim3(256), 0, stream,
                                       src, dst, r, n);
                    break;
                default:
                    hipLaunchKernelGGL(shuffle_vec_kernel<16>, dim3(grid), dim3(256), 0, stream,
                                       src, dst, r, n);
                    break;
            }
        });
    }
    if (dobit) {
        const int G = (ts == 1 || ts == 2 || ts == 4 || ts == 8) ? int(16 / ts) : 0;
        const bool vec = aligned && G > 0 && run.bs % ts == 0 && ne % 8 == 0 &&
                         (ne / 8) % uint32_t(G) == 0 && run.bs % 16 == 0;
        if (!vec)
            return generic(bitshuffle_generic_kernel);
        // One-wave workgroups for 1-byte types (the staging barrier then
        // spans one wave), four for the word-transpose types: with the
        // transpose, u16 runs at 104-106% of a same-size copy with 4 waves
        // against 94% with one (profiles/r02/bitshuffle_waves_word_transpose.log).
        // $AQZ_BITSHUFFLE_WAVES = 1, 2 or 4 overrides (A/B only).
        static const int waves_env = [] {
            const char* e = std::getenv("AQZ_BITSHUFFLE_WAVES");
            const int v = e ? std::atoi(e) : 0;
            return (v == 1 || v == 2 || v == 4) ? v : 0;
        }();
        const int waves = waves_env ? waves_env : (ts == 1 ? 1 : 4);
        // $AQZ_BITSHUFFLE_BYTES=1: the per-byte gather form the word transpose
        // replaced (A/B only)
        static const bool bytes_env = [] {
            const char* e = std::getenv("AQZ_BITSHUFFLE_BYTES");
            return e && *e == '1';
        }();
        if (bytes_env && ts >= 2) {
            const uint32_t per = ne / 8 / G;
            const uint32_t wv = ts <= 2 ? 1 : 4;
            return split_launch(run, n_blocks, per, [&](BlockRun r, uint32_t n, uint32_t) {
                const uint32_t grid = uint32_t((uint64_t(per) * n + 64 * wv - 1) / (64 * wv));
                if (ts == 2)
                    hipLaunchKernelGGL((bitshuffle_vec_kernel<2, 1, false>), dim3(grid), dim3(64),
                                       0, stream, src, dst, r, n);
                else if (ts == 4)
                    hipLaunchKernelGGL((bitshuffle_vec_kernel<4, 4, false>), dim3(grid), dim3(256),
                                       0, stream, src, dst, r, n);
                else
                    hipLaunchKernelGGL((bitshuffle_vec_kernel<8, 4, false>), dim3(grid), dim3(256),
                                       0, stream, src, dst, r, n);
            });
        }
        if (waves != 4) {
            const uint32_t per = ne / 8 / G;
            return split_launch(run, n_blocks, per, [&](BlockRun r, uint32_t n, uint32_t) {
                const uint32_t grid = uint32_t((uint64_t(per) * n + 64 * waves - 1) / (64 * waves));
                auto go = [&](auto kern) {
                    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * waves), 0, stream, src, dst, r, n);
                };
                if (waves == 1) {
                    if (ts == 1) go(bitshuffle_vec_kernel<1, 1>);
                    else if (ts == 2) go(bitshuffle_vec_kernel<2, 1>);
                    else if (ts == 4) go(bitshuffle_vec_kernel<4, 1>);
                    else go(bitshuffle_vec_kernel<8, 1>);
                } else {
                    if (ts == 1) go(bitshuffle_vec_kernel<1, 2>);
                    else if (ts == 2) go(bitshuffle_vec_kernel<2, 2>);
                    else if (ts == 4) go(bitshuffle_vec_kernel<4, 2>);
                    else go(bitshuffle_vec_kernel<8, 2>);
                }
            });
        }
        return split_launch(run, n_blocks, ne / 8 / G,
                            [&](BlockRun r, uint32_t n, uint32_t grid) {
            switch (ts) {
                case 1:
                    hipLaunchKernelGGL(bitshuffle_vec_kernel<1>, dim3(grid), dim3(256), 0,
                                       stream, src, dst, r, n);
                    break;
                case 2:
                    hipLaunchKernelGGL(bitshuffle_vec_kernel<2>, dim3(grid), dim3(256), 0,
                                       stream, src, dst, r, n);
                    break;
                case 4:
                    hipLaunchKernelGGL(bitshuffle_vec_kernel<4>, dim3(grid), dim3(256), 0,
                                       stream, src, dst, r, n);
                    break;
                default:
                    hipLaunchKernelGGL(bitshuffle_vec_kernel<8>, dim3(grid), dim3(256), 0,
                                       stream, src, dst, r, n);
                    break;
            }
        });
    }
    return split_launch(run, n_blocks, run.bs, [&](BlockRun r, uint32_t n, uint32_t grid) {
        hipLaunchKernelGGL(copy_kernel, dim3(grid), dim3(256), 0, stream, src, dst, r, n);
    });
}

// ---- crc32c -----------------------------------------------------------------

constexpr uint32_t kCrc32cPoly = 0x82F63B78u; // reflected Castagnoli

// a * b mod P over GF(2), reflected bit order (zlib's multmodp), branch-free
__host__ __device__ inline uint32_t
multmodp(uint32_t a, uint32_t b)
{
    uint32_t p = 0;
    for (int k = 31; k >= 0; --k) {
        p ^= b & (0u - ((a >> k) & 1u));
        b = (b >> 1) ^ (kCrc32cPoly & (0u - (b & 1u)));
    }
    return p;
}

// x^(8n) mod P (host side, once per launch)
uint32_t
x8nmodp(uint64_t n)
{
    uint32_t sq = 1u << 30;   // x^1, squared up to x^(2^k)
    for (int k = 0; k < 3; ++k)
        sq = multmodp(sq, sq); // x^8
    uint32_t p = 1u << 31;    // x^0
    while (n) {
        if (n & 1)
            p = multmodp(sq, p);
        sq = multmodp(sq, sq);
        n >>= 1;
    }
    return p;
}

// Shift tables for crc32c_kernel, passed by value as a kernel argument.
constexpr int kCrcThreadsPerWg = 256;
constexpr uint32_t kCrcSeg = 64;                                  // bytes per thread
constexpr uint32_t kCrcWgBytes = kCrcThreadsPerWg * kCrcSeg;      // 16 KiB per workgroup
constexpr int kCrcWgLevels = 16;                                  // up to 2^16 workgroups a buffer

struct CrcPow
{
    uint32_t seg[kCrcThreadsPerWg]; // x^(8 * 64 * t) mod P
    uint32_t wg[kCrcWgLevels];      // x^(8 * 16 KiB * 2^l) mod P
};

// CRC-32C of many equal-length buffers, 16 KiB of a buffer per workgroup.
// The buffer is cut into 64-byte segments aligned to its END; segment j
// (counted from the end) belongs to thread j % 256 of workgroup j / 256.
// By linearity of the CRC register update over GF(2):
//   CRC(M) = R0(M) ^ R_init(0^n) ^ ~0,   R0(M) = XOR_j R0(seg_j) * x^(8*64*j)
// where R0 is the register after a zero-initialised run (zlib's
// crc32_combine identity).  Each thread shifts its segment's R0 by its
// place in the workgroup (one table multiply), the workgroup XOR-reduces
// them, shifts the result by the workgroup's place (binary powers), and
// XORs it into crcs[b] atomically; crcs[b] was preset to R_init(0^n) ^ ~0
// on the host side of the launch.  No ordering between workgroups is
// needed, so every CU works on a table at once.  A table of at most 16 KiB
// (Single, the common shard index size) needs no atomic and no preset fill:
// it gets the next power of two of its segment count in lanes, so small
// tables pack 256 >> lgp to a workgroup (1 KiB tables: 16), and its first
// lane stores R0(M) ^ preset after a lane-group XOR.
template <bool Single>
__global__ __launch_bounds__(kCrcThreadsPerWg) void
crc32c_kernel(const uint8_t* __restrict__ data, uint64_t nbytes, uint64_t stride, uint32_t wgs,
              uint32_t n_buffers, uint32_t lgp, CrcPow pw, uint32_t preset,
              uint32_t* __restrict__ crcs)
{
    __shared__ uint32_t table[8][256];
    __shared__ uint32_t wave_x[kCrcThreadsPerWg / 64];
    const uint32_t tid = threadIdx.x;
    {
        uint32_t c = tid;
        for (int k = 0; k < 8; ++k)
            c = (c >> 1) ^ (kCrc32cPoly & (0u - (c & 1u)));
        table[0][tid] = c;
    }
    __syncthreads();
    for (int k = 1; k < 8; ++k) {
        const uint32_t prev = table[k - 1][tid];
        table[k][tid] = (prev >> 8) ^ table[0][prev & 0xFFu];
    }
    __syncthreads();

    // Single: 2^lgp lanes per table (lgp <= 8), 256 >> lgp tables per workgroup
    const uint32_t lanes = Single ? (1u << lgp) : uint32_t(kCrcThreadsPerWg);
    const uint32_t b = Single ? blockIdx.x * (kCrcThreadsPerWg >> lgp) + (tid >> lgp)
                              : blockIdx.x / wgs;
    const uint32_t q = Single ? 0u : blockIdx.x % wgs;
    const uint32_t js = tid & (lanes - 1);                   // segment within the workgroup
    const uint8_t* buf = data + uint64_t(b) * stride;
    const uint64_t j = uint64_t(q) * kCrcThreadsPerWg + js; // segment, from the end
    uint32_t c = 0;                                          // zero-initialised register
    auto step8 = [&](const uint8_t* v) {                     // slicing-by-8
        const uint32_t lo = c ^ (uint32_t(v[0]) | uint32_t(v[1]) << 8 | uint32_t(v[2]) << 16 |
                                 uint32_t(v[3]) << 24);
        c = table[7][lo & 0xFFu] ^ table[6][(lo >> 8) & 0xFFu] ^ table[5][(lo >> 16) & 0xFFu] ^
            table[4][lo >> 24] ^ table[3][v[4]] ^ table[2][v[5]] ^ table[1][v[6]] ^
            table[0][v[7]];
    };
    if (b < n_buffers && kCrcSeg * j < nbytes) {
        const uint64_t end = nbytes - kCrcSeg * j;
        if (end >= kCrcSeg) {
            // a whole segment: four 16-byte loads in flight, any alignment
            // (shard index tables sit at 4-byte offsets after their CRC)
            const uint8_t* s = buf + end - kCrcSeg;
            u32x4 w[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                w[k] = *reinterpret_cast<const u32x4_u*>(s + 16 * k);
            uint8_t v[64];
            __builtin_memcpy(v, w, 64);
#pragma unroll
            for (int k = 0; k < 8; ++k)
                step8(v + 8 * k);
        } else {
            // the buffer's first, short segment
            for (uint64_t i = 0; i < end; ++i)
                c = (c >> 8) ^ table[0][(c ^ buf[i]) & 0xFFu];
        }
        c = multmodp(pw.seg[js], c); // shift by the segments after it in this workgroup
    }
    // XOR over each table's lanes (the whole wave when a table spans waves)
#pragma unroll
    for (uint32_t d = 32; d >= 1; d >>= 1)
        if (d < lanes)
            c ^= __shfl_xor(c, d);
    if (Single && lanes <= 64) {
        if (js == 0 && b < n_buffers)
            crcs[b] = c ^ preset;
        return;
    }
    if ((tid & 63) == 0)
        wave_x[tid >> 6] = c;
    __syncthreads();
    const uint32_t wpt = lanes / 64; // waves per table
    if (tid < kCrcThreadsPerWg / 64 / wpt) {
        uint32_t v = 0;
        for (uint32_t k = 0; k < wpt; ++k)
            v ^= wave_x[tid * wpt + k];
        if constexpr (Single) {
            const uint32_t bt = blockIdx.x * (kCrcThreadsPerWg >> lgp) + tid;
            if (bt < n_buffers)
                crcs[bt] = v ^ preset;
        } else {
            // shift by the workgroups after this one: x^(8 * 16 KiB * q)
            for (int l = 0; l < kCrcWgLevels; ++l)
                if ((q >> l) & 1u)
                    v = multmodp(pw.wg[l], v);
            atomicXor(crcs + b, v);
        }
    }
}

} // namespace

hipError_t
launch_blosc_filter(int shuffle,
                    uint32_t typesize,
                    uint32_t blocksize,
                    const void* src,
                    uint64_t nbytes,
                    uint32_t n_buffers,
                    void* dst,
                    hipStream_t stream)
{
    if (typesize == 0 || blocksize == 0 || shuffle < 0 || shuffle > 2 || n_buffers == 0)
        return hipErrorInvalidValue;
    if (nbytes == 0)
        return hipSuccess;
    const auto* s = static_cast<const uint8_t*>(src);
    auto* d = static_cast<uint8_t*>(dst);
    const bool aligned = reinterpret_cast<uintptr_t>(s) % 16 == 0 &&
                         reinterpret_cast<uintptr_t>(d) % 16 == 0 &&
                         (n_buffers == 1 || nbytes % 16 == 0);
    const uint64_t full = nbytes / blocksize;
    const uint32_t leftover = uint32_t(nbytes % blocksize);
    if (full * n_buffers >= (1ull << 32))
        return hipErrorInvalidValue;
    if (full) {
        const BlockRun run{ nbytes, 0, uint32_t(full), blocksize, 0 };
        hipError_t e = filter_run(shuffle, typesize, s, d, run, uint32_t(full * n_buffers),
                                  aligned, stream);
        if (e != hipSuccess)
            return e;
    }
    if (leftover) {
        const BlockRun run{ nbytes, full * blocksize, 1, leftover, 0 };
        return filter_run(shuffle, typesize, s, d, run, n_buffers,
                          aligned && (full * blocksize) % 16 == 0, stream);
    }
    return hipSuccess;
}

hipError_t
launch_crc32c(const void* data, uint64_t nbytes, uint64_t stride, uint32_t n_buffers,
              uint32_t* crcs, hipStream_t stream)
{
    if (n_buffers == 0 || n_buffers >= (1u << 31))
        return hipErrorInvalidValue;
    const uint64_t wgs = (nbytes + kCrcWgBytes - 1) / kCrcWgBytes;
    if (wgs >= (1ull << kCrcWgLevels) || wgs * n_buffers >= (1ull << 31))
        return hipErrorInvalidValue;
    // crcs[b] = R_init(0^n) ^ ~0; the kernel XORs R0(M) in
    const uint32_t preset = multmodp(x8nmodp(nbytes), 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
    if (wgs <= 1) {
        // empty tables: the CRC is the preset; else one workgroup per table
        // writes R0(M) ^ preset and nothing needs filling first
        if (wgs == 0)
            return hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(crcs), int(preset),
                                     n_buffers, stream);
    } else {
        hipError_t e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(crcs), int(preset),
                                         n_buffers, stream);
        if (e != hipSuccess)
            return e;
    }
    // the shift powers do not depend on the launch: computed once
    static const CrcPow pw = [] {
        CrcPow p;
        const uint32_t seg = x8nmodp(kCrcSeg);
        p.seg[0] = 1u << 31; // x^0
        for (int t = 1; t < kCrcThreadsPerWg; ++t)
            p.seg[t] = multmodp(seg, p.seg[t - 1]);
        p.wg[0] = x8nmodp(kCrcWgBytes);
        for (int l = 1; l < kCrcWgLevels; ++l)
            p.wg[l] = multmodp(p.wg[l - 1], p.wg[l - 1]);
        return p;
    }();
    if (wgs == 1) {
        uint32_t lgp = 0; // lanes per table: next power of two of its segments
        while ((uint64_t(kCrcSeg) << lgp) < nbytes)
            ++lgp;
        const uint32_t per_wg = uint32_t(kCrcThreadsPerWg) >> lgp;
        hipLaunchKernelGGL(crc32c_kernel<true>, dim3((n_buffers + per_wg - 1) / per_wg),
                           dim3(kCrcThreadsPerWg), 0, stream,
                           static_cast<const uint8_t*>(data), nbytes, stride, uint32_t(wgs),
                           n_buffers, lgp, pw, preset, crcs);
    } else {
        hipLaunchKernelGGL(crc32c_kernel<false>, dim3(uint32_t(wgs * n_buffers)),
                           dim3(kCrcThreadsPerWg), 0, stream, static_cast<const uint8_t*>(data),
                           nbytes, stride, uint32_t(wgs), n_buffers, 8u, pw, preset, crcs);
    }
    return hipGetLastError();
}

} // namespace aqz
