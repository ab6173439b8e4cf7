// ds_kernels.hip — CDNA4 (gfx950) kernels for the acquire-zarr multiscale
// pyramid.  See ds_kernels.hh for the contract and DESIGN.md for the
// roofline analysis.
//
// Semantics restated from acquire-zarr v0.8.1 src/streaming/downsampler.cpp:
//   reducers        :39-137 (decimate/mean/min/max, 4- and 2-operand forms)
//   scale_image<T>  :139-206 (2x2 reduce, odd right/bottom edge replicated)
//   average_two_frames<T> :208-246 (dst = f(earlier, current))
// The arithmetic is bit-exact with the reference binary: narrow integers are
// promoted to int, 32/64-bit integer sums wrap, floats sum left to right and
// divide by 4 (exact as a multiply by 0.25), min/max are compare-select
// chains seeded with the first operand so NaN order matches.
//
// Design: this is an HBM-bound stencil, not a contraction — no MFMA.  Each
// wave owns a tile of 64 lanes x 16 bytes wide and 2^NL rows tall, issues
// all 2^NL row loads (16 B per lane, 1 KiB per wave instruction) before any
// arithmetic, and reduces the pyramid in registers: in-lane while a lane
// still holds >= 2 columns of a level, then across lanes with __shfl_down at
// doubling strides.  Every level of the run is written from the same pass,
// so the base frame is read exactly once.  LDS only assembles stores: the
// band kernels (cascade_band_kernel) stage each level's rows of a whole row
// band in LDS so that they leave as full 64-byte bursts, and
// transpose_kernel turns its tiles through LDS.
#include "ds_kernels.hh"

// Build sharding (acquire-zarr_amd/Makefile): the library compiles this file
// AQZ_SHARDS times; shard k instantiates the kernels of the dtypes whose
// code % AQZ_SHARDS == k, and its dtype-dispatching launchers are named
// <launcher>_shard<k>.  ds_dispatch.cpp routes each call to its shard, and
// shard 0 alone defines the dtype-independent helpers.  The shards compile
// in parallel: one unit held over a thousand kernel instantiations.  Included
// directly (the tools/ probes), the file builds unsharded.
#ifndef AQZ_SHARDS
#define AQZ_SHARDS 1
#endif
#ifndef AQZ_SHARD
#define AQZ_SHARD 0
#endif
#if AQZ_SHARDS > 1
#define AQZ_CAT2_(a, b) a##b
#define AQZ_CAT_(a, b) AQZ_CAT2_(a, b)
#define AQZ_SHARDED(name) AQZ_CAT_(name##_shard, AQZ_SHARD)
#else
#define AQZ_SHARDED(name) name
#endif

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace aqz {
namespace {

// Native 16-byte vector (HIP's uint4 is a struct; the builtins want this).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// The same widths at byte alignment, for the fused kernels' frame accesses:
// a batch of odd-width frames puts rows (and frames) at any byte offset.
// gfx950 global loads/stores take unaligned addresses (the compiler emits the
// same global_load_dwordx4 / global_store_dwordx2 for these types); the
// bytes a wave touches are unchanged, so HBM traffic is unchanged.
typedef u32x4 u32x4_u __attribute__((aligned(1)));
typedef uint64_t u64_u __attribute__((aligned(1)));
typedef uint32_t u32_u __attribute__((aligned(1)));
typedef uint16_t u16_u __attribute__((aligned(1)));

enum
{
    kDecimate = 0,
    kMean = 1,
    kMin = 2,
    kMax = 3
};

// ---- reducers --------------------------------------------------------------

// NaN payloads exactly as the reference binary makes them.  IEEE 754 leaves
// a NaN result's payload open; the reference's compiled float mean (x86 SSE
// addss/divss, downsampler.cpp:48-51,108-112) returns the FIRST source
// operand's NaN, quieted, when it is a NaN, else the second's, and for an
// invalid sum (inf + -inf) the negative "default NaN" (sign and quiet bits
// set, zero payload).  gfx950's v_add/v_div pick differently (inf - inf
// gives the positive quiet NaN), so the kernels keep
// the plain arithmetic and rebuild the bits only where the result is a NaN:
// one compare per output in the common case, the walk below when a wave has
// a NaN lane.  The walk selects on bits (integer ops) so nothing
// canonicalises the payload; divide by 4 or 2 keeps a quiet NaN unchanged on
// x86.  The
// oracle states the same rule (oracle/ds_oracle.c add_<T>).
template<typename T>
struct float_bits;
template<>
struct float_bits<float>
{
    using U = uint32_t;
    static constexpr U quiet() { return 0x00400000u; }
    static constexpr U default_nan() { return 0xFFC00000u; }
};
template<>
struct float_bits<double>
{
    using U = uint64_t;
    static constexpr U quiet() { return 0x0008000000000000ull; }
    static constexpr U default_nan() { return 0xFFF8000000000000ull; }
};

// x86 `x + y` with its NaN rule (x the first source), as selects on bits.
template<typename T>
__device__ __forceinline__ T
x86_add(T x, T y)
{
    using FB = float_bits<T>;
    using U = typename FB::U;
    const T s = x + y;
    const U bx = __builtin_bit_cast(U, x) | FB::quiet();
    const U by = __builtin_bit_cast(U, y) | FB::quiet();
    const U bs = (s != s) ? FB::default_nan() : __builtin_bit_cast(U, s);
    return __builtin_bit_cast(T, (x != x) ? bx : ((y != y) ? by : bs));
}

// Whether any lane of the wave holds a NaN result.  The fix-up runs behind a
// wave-uniform branch.  A lane-divergent one (only the NaN lanes inside) gave
// wrong outputs in edge tiles of 16-byte f32 tiles on 4 of 256 fuzz cases
// (round 5): in-range lanes read the next row's chunk as zero or stale bits.
// Round 6 (tools/divergent/) narrowed it to the divergent
// branch together with exec-masked edge loads (load_chunk); either one alone
// is exact, and tests/test_gpu_divergent.py reruns round 5's launch.
__device__ __forceinline__ bool
wave_any(bool p)
{
    return __builtin_amdgcn_ballot_w64(p) != 0;
}

#ifdef AQZ_NAN_FIXUP_DIVERGENT
// The round-5 lane-divergent form (branches on the NaN lanes only), kept for
// the regression probe (tools/divergent/, tests/test_gpu_divergent.py).
template<typename T>
__device__ __forceinline__ T
x86_add_branchy(T x, T y)
{
    using FB = float_bits<T>;
    using U = typename FB::U;
    const T s = x + y;
    U r;
    if (x != x)
        r = __builtin_bit_cast(U, x) | FB::quiet();
    else if (y != y)
        r = __builtin_bit_cast(U, y) | FB::quiet();
    else if (s != s)
        r = FB::default_nan();
    else
        return s;
    return __builtin_bit_cast(T, r);
}
#endif

template<typename T>
__device__ __forceinline__ T
mean4(T a, T b, T c, T d)
{
    if constexpr (std::is_floating_point_v<T>) {
        const T r = (((a + b) + c) + d) / T(4);
#ifdef AQZ_NAN_FIXUP_DIVERGENT
        if (__builtin_expect(r != r, 0))
            return x86_add_branchy(x86_add_branchy(x86_add_branchy(a, b), c), d);
        return r;
#endif
        if (__builtin_expect(wave_any(r != r), 0)) {
            // the chain's first NaN is the value (x86 keeps it through the
            // later adds and the divide); other lanes keep theirs
            const T n = x86_add(x86_add(x86_add(a, b), c), d);
            return (r != r) ? n : r;
        }
        return r;
    } else if constexpr (sizeof(T) < sizeof(int)) {
        return T((int(a) + int(b) + int(c) + int(d)) / 4);
    } else {
        using U = std::make_unsigned_t<T>;
        const T s = T(U(a) + U(b) + U(c) + U(d));
        return T(s / T(4));
    }
}

template<typename T>
__device__ __forceinline__ T
mean2(T a, T b)
{
    if constexpr (std::is_floating_point_v<T>) {
        const T r = (a + b) / T(2);
#ifdef AQZ_NAN_FIXUP_DIVERGENT
        if (__builtin_expect(r != r, 0))
            return x86_add_branchy(a, b);
        return r;
#endif
        if (__builtin_expect(wave_any(r != r), 0)) {
            const T n = x86_add(a, b);
            return (r != r) ? n : r;
        }
        return r;
    } else if constexpr (sizeof(T) < sizeof(int)) {
        return T((int(a) + int(b)) / 2);
    } else {
        using U = std::make_unsigned_t<T>;
        const T s = T(U(a) + U(b));
        return T(s / T(2));
    }
}

template<typename T, int M>
__device__ __forceinline__ T
reduce4(T a, T b, T c, T d)
{
    if constexpr (M == kDecimate) {
        return a;
    } else if constexpr (M == kMean) {
        return mean4(a, b, c, d);
    } else if constexpr (M == kMin) {
        T v = a;
        v = (b < v) ? b : v;
        v = (c < v) ? c : v;
        v = (d < v) ? d : v;
        return v;
    } else {
        T v = a;
        v = (b > v) ? b : v;
        v = (c > v) ? c : v;
        v = (d > v) ? d : v;
        return v;
    }
}

template<typename T, int M>
__device__ __forceinline__ T
reduce2(T a, T b)
{
    if constexpr (M == kDecimate) {
        return a;
    } else if constexpr (M == kMean) {
        return mean2(a, b);
    } else if constexpr (M == kMin) {
        return a < b ? a : b;
    } else {
        return a > b ? a : b;
    }
}

// ---- cross-lane move of any 1/2/4/8-byte element ---------------------------

template<typename T>
__device__ __forceinline__ T
shfl_down_any(T v, int delta)
{
    if constexpr (sizeof(T) <= 4) {
        uint32_t x = 0;
        __builtin_memcpy(&x, &v, sizeof(T));
        x = __shfl_down(x, (unsigned)delta);
        T r;
        __builtin_memcpy(&r, &x, sizeof(T));
        return r;
    } else {
        unsigned long long x;
        __builtin_memcpy(&x, &v, 8);
        x = __shfl_down(x, (unsigned)delta);
        T r;
        __builtin_memcpy(&r, &x, 8);
        return r;
    }
}

// Store N contiguous elements of T as one access at any byte alignment
// (optionally non-temporal: write-once pyramid levels).
template<typename T, int N, bool NT = false>
__device__ __forceinline__ void
store_vec(T* dst, const T (&v)[N])
{
    constexpr int B = int(sizeof(T)) * N;
    static_assert(B == 1 || B == 2 || B == 4 || B == 8 || B == 16, "width");
    if constexpr (B == 16) {
        u32x4 q;
        __builtin_memcpy(&q, v, 16);
        u32x4_u* d = reinterpret_cast<u32x4_u*>(dst); // typedef keeps align 1
        if constexpr (NT)
            __builtin_nontemporal_store(q, d);
        else
            *d = q;
    } else if constexpr (B == 8) {
        uint64_t q;
        __builtin_memcpy(&q, v, 8);
        u64_u* d = reinterpret_cast<u64_u*>(dst); // typedef keeps align 1
        if constexpr (NT)
            __builtin_nontemporal_store(q, d);
        else
            *d = q;
    } else if constexpr (B == 4) {
        uint32_t q;
        __builtin_memcpy(&q, v, 4);
        u32_u* d = reinterpret_cast<u32_u*>(dst); // typedef keeps align 1
        if constexpr (NT)
            __builtin_nontemporal_store(q, d);
        else
            *d = q;
    } else if constexpr (B == 2) {
        uint16_t q;
        __builtin_memcpy(&q, v, 2);
        u16_u* d = reinterpret_cast<u16_u*>(dst); // typedef keeps align 1
        if constexpr (NT)
            __builtin_nontemporal_store(q, d);
        else
            *d = q;
    } else {
        uint8_t q;
        __builtin_memcpy(&q, v, 1);
        uint8_t* d = reinterpret_cast<uint8_t*>(dst);
        if constexpr (NT)
            __builtin_nontemporal_store(q, d);
        else
            *d = q;
    }
}

#ifdef AQZ_EDGE_SHIFT_ASM
// probe variants (tools/divergent): the 64-bit shifts as
// inline asm, =2 with two wait states after each one
__device__ __forceinline__ uint64_t
probe_shr64(uint64_t x, uint32_t n)
{
    uint64_t r;
#if AQZ_EDGE_SHIFT_ASM == 2
    asm volatile("v_lshrrev_b64 %0, %1, %2\n\ts_nop 1" : "=v"(r) : "v"(n), "v"(x));
#else
    asm volatile("v_lshrrev_b64 %0, %1, %2" : "=v"(r) : "v"(n), "v"(x));
#endif
    return r;
}
__device__ __forceinline__ uint64_t
probe_shl64(uint64_t x, uint32_t n)
{
    uint64_t r;
#if AQZ_EDGE_SHIFT_ASM == 2
    asm volatile("v_lshlrev_b64 %0, %1, %2\n\ts_nop 1" : "=v"(r) : "v"(n), "v"(x));
#else
    asm volatile("v_lshlrev_b64 %0, %1, %2" : "=v"(r) : "v"(n), "v"(x));
#endif
    return r;
}
#endif

// Shift a little-endian LB-byte vector down by `bytes` (0 <= bytes < LB).
template<int LB>
__device__ __forceinline__ void
shift_down(uint64_t (&q)[LB / 8], uint32_t bytes)
{
#ifdef AQZ_EDGE_SHIFT32
    // probe variant (tools/divergent): the same shift in
    // 32-bit words, no 64-bit shifts; `bytes` >= LB gives zero
    if constexpr (LB == 16) {
        uint32_t w[4], o[4];
        __builtin_memcpy(w, q, 16);
        const uint32_t k = bytes >> 2, r = (bytes & 3u) * 8u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t j = uint32_t(i) + k;
            const uint32_t a = j == 0 ? w[0] : j == 1 ? w[1] : j == 2 ? w[2] : j == 3 ? w[3] : 0u;
            const uint32_t b = j == 0 ? w[1] : j == 1 ? w[2] : j == 2 ? w[3] : 0u;
            o[i] = r ? (a >> r) | (b << (32u - r)) : a;
        }
        __builtin_memcpy(q, o, 16);
        return;
    }
#endif
    const uint32_t n = 8 * bytes;
#ifdef AQZ_EDGE_SHIFT_ASM
    if constexpr (LB == 16) {
        uint64_t lo = q[0], hi = q[1];
        if (n >= 64) {
            lo = probe_shr64(hi, n - 64);
            hi = 0;
        } else if (n) {
            lo = probe_shr64(lo, n) | probe_shl64(hi, 64 - n);
            hi = probe_shr64(hi, n);
        }
        q[0] = lo;
        q[1] = hi;
        return;
    }
#endif
    if constexpr (LB == 8) {
        q[0] = n ? q[0] >> n : q[0];
    } else {
        uint64_t lo = q[0], hi = q[1];
        if (n >= 64) {
            lo = hi >> (n - 64);
            hi = 0;
        } else if (n) {
            lo = (lo >> n) | (hi << (64 - n));
            hi >>= n;
        }
        q[0] = lo;
        q[1] = hi;
    }
}

// E elements of T from row `row` starting at column `col`, as one LB-byte
// vector load at any alignment.  EDGE (tiles that touch the frame's right or
// bottom edge): rows past the frame (`row_ok` false) and chunks starting at
// or past `W` read as zero.  A chunk that straddles the row end is loaded
// whole when the bytes past the row end are still inside the buffer
// (`tail_safe`: they belong to the next row or frame; the kernel replaces
// those columns by edge replication anyway).  On the batch's last row it is
// loaded instead as the row's last E elements and shifted down in registers,
// so nothing outside the buffer is read.  Needs W >= E (cascade_fits).
// Every lane issues one vector load either way: no divergent element loads,
// and the edge path costs the interior path no registers.
//
// Out-of-range chunks (rows past the frame, columns past W) are skipped by
// an exec-masked load and read as zero.  AQZ_EDGE_LOAD_SELECT (probe builds,
// tools/divergent/) loads on every lane instead — from the row's last chunk,
// or from `safe` (the frame's first elements) for rows past the frame — and
// selects the zero afterwards.  That form cures the round-5 divergent-branch
// build, but it gave one wrong pixel in one default fuzz
// run, so the product keeps the masked form with its long clean record.
template<typename T, int E, bool NT, bool EDGE>
__device__ __forceinline__ void
load_chunk(T* out, const T* row, uint32_t col, uint32_t W, bool row_ok, bool tail_safe,
           const T* safe)
{
    constexpr int LB = E * int(sizeof(T));
    static_assert(LB == 16 || LB == 8, "fused loads are 8 or 16 bytes");
    uint32_t at = col;
    bool ok = true;
    if constexpr (EDGE) {
        ok = row_ok && col < W;
        if (col + E > W && !tail_safe)
            at = W - E;
    }
    uint64_t q[LB / 8] = {};
#ifdef AQZ_EDGE_LOAD_SELECT
    if constexpr (EDGE) {
        // past the row end: the row's last chunk, whose line the wave's last
        // in-range lane reads anyway (=1), or `safe` (=2); past the frame's
        // last row: `safe`
        const T* a0 = ok ? row + at : (row_ok && AQZ_EDGE_LOAD_SELECT == 1) ? row + (W - E) : safe;
        uint64_t w[LB / 8];
        if constexpr (LB == 16) {
            const u32x4 v = NT ? __builtin_nontemporal_load(reinterpret_cast<const u32x4_u*>(a0))
                               : *reinterpret_cast<const u32x4_u*>(a0);
            __builtin_memcpy(w, &v, 16);
        } else {
            w[0] = NT ? __builtin_nontemporal_load(reinterpret_cast<const u64_u*>(a0))
                      : *reinterpret_cast<const u64_u*>(a0);
        }
#pragma unroll
        for (int i = 0; i < LB / 8; ++i)
            q[i] = ok ? w[i] : 0ull;
        shift_down<LB>(q, (col - at) * uint32_t(sizeof(T)));
        __builtin_memcpy(out, q, LB);
        return;
    }
#endif
    (void)safe;
    if (ok) {
        // explicit byte-aligned pointer types (a template argument would drop
        // the typedef's alignment)
        if constexpr (LB == 16) {
            const u32x4_u* a = reinterpret_cast<const u32x4_u*>(row + at);
            const u32x4 v = NT ? __builtin_nontemporal_load(a) : *a;
            __builtin_memcpy(q, &v, 16);
        } else {
            const u64_u* a = reinterpret_cast<const u64_u*>(row + at);
            q[0] = NT ? __builtin_nontemporal_load(a) : *a;
        }
    }
#ifdef AQZ_EDGE_DEBUG
    // probe variant (tools/divergent): report in-range edge chunks that
    // loaded as all-zero bits (the round-5 failure's signature)
    if constexpr (EDGE) {
        bool zero = true;
#pragma unroll
        for (int i = 0; i < LB / 8; ++i)
            zero = zero && q[i] == 0;
        if (ok && zero)
            printf("AQZDBG blk %u lane %u row %p col %u at %u W %u tail %d\n", blockIdx.x,
                   threadIdx.x, (const void*)row, col, at, W, int(tail_safe));
    }
#endif
    if constexpr (EDGE)
        shift_down<LB>(q, (col - at) * uint32_t(sizeof(T)));
    __builtin_memcpy(out, q, LB);
}

// ---- fused cascade ---------------------------------------------------------

// Division by a runtime constant as a multiply-high and shifts (Granlund &
// Montgomery; exact for every 32-bit n).  The tiled stores divide row and
// column indices by the chunk shape: per block, not per element, but on
// small frames a block is a few KiB and a 32-bit division's ~40 scalar
// instructions showed up (512^2 u8 tiled).
struct FastDiv
{
    uint32_t d = 1, m = 0, s = 0; // d == 1: m = 0, q = n

    static FastDiv make(uint32_t d)
    {
        FastDiv f;
        f.d = d ? d : 1;
        if (f.d == 1)
            return f;
        uint32_t l = 0;
        while ((1ull << l) < f.d)
            ++l;
        f.m = uint32_t(((uint64_t(1) << 32) * ((uint64_t(1) << l) - f.d)) / f.d + 1);
        f.s = l - 1;
        return f;
    }
    __device__ __forceinline__ uint32_t div(uint32_t n) const
    {
        if (d == 1)
            return n;
        const uint32_t t = __umulhi(n, m);
        return (t + ((n - t) >> 1)) >> s;
    }
};

// One chunk-tiled output level of the tiled cascade.  Frame f's tile
// t = ty * ntx + tx (tr x tc elements, row-major; the padded level is pw x ph)
// at tdst + base(f) + t * tstride, where base(f) = f * tframe_elems and
// tstride = tr * tc (tiles back to back), or — for a chunk lattice
// (launch_cascade_tiled with TiledOut::frame_offsets) — base(f) = foff[f] and
// tstride = the distance between neighbouring chunks: the reference's
// chunks_[tile + tile_group_offset(f)] at chunk_internal_offset(f)
// (array.cpp:563-617, array.dimensions.cpp:265-314).
// Zero scan.  slots > 0 (wave blocks and tiles nest): tile t owns `slots`
// flag bytes, one per (block, tile) pair (slots_x across), and every byte is
// written exactly once — by its wave, or as 0 by the zero-fill waves for
// blocks past the grid — so nothing is cleared first.  slots == 0: one byte
// per tile, cleared before the launch, set to 1 by every wave storing a
// nonzero byte into the tile.
// Zero-fill waves (wave ids past the grid's blocks): the padded area the
// blocks do not reach — columns >= cov_w, and rows >= cov_h — per
// (frame, level, padded row) item (zrows items per frame here), plus the
// slot flags of those blocks.
struct TiledLevel
{
    uint8_t* tdst;
    uint8_t* flags;
    uint64_t tframe_elems;
    const uint64_t* foff; // per-frame element offsets (chunk lattice), or null
    uint64_t tstride;     // elements from one tile to the next
    uint32_t tr, tc, ntx, pw, ph;
    uint32_t slots, slots_x, flags_frame;
    uint32_t cov_w, cov_h, zrows;
    FastDiv dr, dc; // by tr, by tc
};

// Element offset of frame f's tile 0 (wave-uniform f: a scalar load).
__device__ __forceinline__ uint64_t
tiled_frame_base(const TiledLevel& t, uint32_t f)
{
    return t.foff ? t.foff[f] : uint64_t(f) * t.tframe_elems;
}

struct CascadeParams
{
    const uint8_t* src;
    uint64_t src_frame_elems;
    uint32_t W, H;         // input level geometry
    uint32_t units_x;      // column tiles per frame
    uint32_t units_y;      // row tiles per frame
    uint32_t total_units;  // units_x * units_y * n_frames
    uint8_t* dst[kMaxFusedLevels];
    uint64_t dst_frame_elems[kMaxFusedLevels];
    uint32_t w[kMaxFusedLevels];
    uint32_t h[kMaxFusedLevels];
    // Chunk-tiled outputs (cascade_kernel<..., TILED>, launch_cascade_tiled), one
    // TiledLevel per level; dst[J-1] may then be null (no row-major copy).
    TiledLevel tl[kMaxFusedLevels];
    uint32_t zitems;                 // items per frame, all levels
    FastDiv zdiv;                    // by zitems
    uint32_t zwaves;                 // zero-fill waves: the grid's first zwaves / (waves per block) blocks
    uint32_t main_blocks;            // blocks of cascade waves after them
    uint32_t remap;                  // 1: XCD-contiguous block order (cascade_kernel)
    uint32_t wb;                     // bit J-1: level J's row-major stores write-back, not nt
    uint32_t order;                  // unit order: 0 columns fastest, 1 frames, 2 row bands
    uint32_t seg_w;                  // > 0: a workgroup is seg_w column tiles of one row band
    uint32_t nt;                     // launcher's choice of load policy (load_nt)
    uint32_t band_last;              // K > 0: the band's last K waves to finish store it (no barrier)
    uint32_t seg_rowwise;            // 1: band segments of misaligned rows (StageCtx::rowb)
    uint32_t upw;                    // units per wave (cascade_kernel, columns-fastest order)
};

// $AQZ_LOAD_NT: 1 / 0 forces the fused cascade's loads with / without the
// non-temporal hint (A/B only); unset (-1): the launcher decides.
inline int
load_nt_env()
{
    static const int v = [] {
        const char* e = std::getenv("AQZ_LOAD_NT");
        return (e && *e) ? std::atoi(e) : -1;
    }();
    return v;
}

// Non-temporal loads unless the frame rows are not whole 128-B lines: there a
// line straddles two waves' row segments, and without the streaming hint the
// second wave finds it in L2 (3000^2 u16: 2.7% fewer read requests, 4%
// faster; aligned rows lose 6% without the hint; profiles/r02/loadnt_ab.log).
inline uint32_t
load_nt(uint32_t W, size_t bpp)
{
    if (load_nt_env() >= 0)
        return load_nt_env() != 0;
    return (uint64_t(W) * bpp) % 128 == 0;
}

// $AQZ_TILED_ZWAVES: unset = the launcher's count of zero-fill waves, else
// that count (A/B only; 0 skips the zero fill and leaves the overhang
// unwritten).
inline int
tiled_zwaves_env()
{
    static const int v = [] {
        const char* e = std::getenv("AQZ_TILED_ZWAVES");
        return (e && *e) ? std::atoi(e) : -1;
    }();
    return v;
}

// $AQZ_STORE_WB: unset = the launcher's default, else a level bit mask
// (bit J-1 = level J) of row-major stores issued write-back instead of
// non-temporal (A/B).
inline int
store_wb_env()
{
    static const int v = [] {
        const char* e = std::getenv("AQZ_STORE_WB");
        return (e && *e) ? std::atoi(e) : -1;
    }();
    return v;
}

// $AQZ_UNIT_ORDER (0 columns fastest = default, 1 frames fastest, 2 row bands
// fastest) and $AQZ_CASCADE_WAVES (waves per workgroup, 4 = default, up to
// 8): A/B switches of the row-major cascade's unit-to-wave mapping.
inline int
int_env(const char* name, int dflt)
{
    const char* e = std::getenv(name);
    return (e && *e) ? std::atoi(e) : dflt;
}

// $AQZ_SPLIT_LOADS: 1 / 0 = band kernels of 4- and 8-byte types load each
// row's 2 KiB wave segment as two contiguous halves (cascade_unit SPLIT) or
// as 32 bytes per lane; unset: the launcher's default.
inline bool
split_loads()
{
    static const bool v = [] {
        const char* e = std::getenv("AQZ_SPLIT_LOADS");
        return (e && *e) ? std::atoi(e) != 0 : false;
    }();
    return v;
}

// $AQZ_XCD_REMAP: unset = the launcher's default, 0 = off, 1 = on (A/B only).
inline int
xcd_remap_env()
{
    static const int v = [] {
        const char* e = std::getenv("AQZ_XCD_REMAP");
        return (e && *e) ? std::atoi(e) : -1;
    }();
    return v;
}

// Columns of T per lane in the fused cascade: 16 bytes for 1- and 2-byte
// types, 32 bytes (two 16-byte loads per row) for 4- and 8-byte types, which
// keeps levels 1-3 in-lane and halves the cross-lane shuffles.  A/B on
// MI355X (tools/microbench.hip f32): 4096^2 f32 x64 batch 1083 -> 975 us,
// bit-identical; the same widening measured slower for u16 (562 vs 470 us).
template<typename T>
constexpr int kCascadeCols = sizeof(T) >= 4 ? 32 / int(sizeof(T)) : 16 / int(sizeof(T));

inline uint32_t
cascade_cols(size_t bpp)
{
    return uint32_t((bpp >= 4 ? 32 : 16) / bpp);
}

// Lanes per column group at level J when each lane starts with C columns.
template<int C, int J>
constexpr int kLaneStride = ((1 << J) >= C) ? ((1 << J) / C) : 1;

// One XY level in registers: level J (1-based within the run) from level J-1
// held as RI rows x CI columns per lane.  CI == 1 means the lane holds one
// column of a column group spread over kLaneStride<C, J-1> lanes (only the
// group's first lane is meaningful); the right-hand neighbour then comes
// from that many lanes up.  `win`/`hin` are level J-1's size, `cin0`/`rin0`
// the lane's first column/row there (edge replication needs them).
template<typename T, int M, int C, int J, int RI, int CI, bool EDGE>
__device__ __forceinline__ void
xy_step(const T (&in)[RI][CI],
        T (&out)[RI / 2][(CI >= 2) ? CI / 2 : 1],
        uint32_t win,
        uint32_t hin,
        uint32_t cin0,
        uint32_t rin0)
{
    constexpr int RO = RI / 2;
    constexpr bool kInLane = CI >= 2;
    constexpr int CO = kInLane ? CI / 2 : 1;
    constexpr int SI = kLaneStride<C, J - 1>;
#pragma unroll
    for (int r = 0; r < RO; ++r) {
#pragma unroll
        for (int c = 0; c < CO; ++c) {
            T here, right, down, diag;
            if constexpr (kInLane) {
                here = in[2 * r][2 * c];
                right = in[2 * r][2 * c + 1];
                down = in[2 * r + 1][2 * c];
                diag = in[2 * r + 1][2 * c + 1];
            } else {
                here = in[2 * r][0];
                down = in[2 * r + 1][0];
                right = shfl_down_any(here, SI);
                diag = shfl_down_any(down, SI);
            }
            if constexpr (EDGE) {
                // scale_image edge replication (downsampler.cpp:186-197):
                // last column of an odd width / last row of an odd height.
                const uint32_t col = cin0 + (kInLane ? 2u * c : 0u);
                const bool pw = col + 1 >= win;
                const bool ph = rin0 + 2u * r + 1 >= hin;
                const T r_ = pw ? here : right;
                const T g_ = ph ? r_ : (pw ? down : diag);
                const T d_ = ph ? here : down;
                right = r_;
                down = d_;
                diag = g_;
            }
            out[r][c] = reduce4<T, M>(here, right, down, diag);
        }
    }
}

// Write the lane's RO x CO block of level J (frame base `dst`, row pitch
// `wout`); only column-group leaders store, edge tiles clip to the level.
template<typename T, int C, int J, int RO, int CO, bool EDGE, bool NTS>
__device__ __forceinline__ void
store_level(T* dst,
            const T (&out)[RO][CO],
            uint32_t wout,
            uint32_t hout,
            uint32_t col0,
            uint32_t row0,
            int lane)
{
    constexpr int SO = kLaneStride<C, J>;
    const uint32_t cout0 = col0 >> J;
    const uint32_t rout0 = row0 >> J;
    const bool leader = (SO == 1) || ((lane & (SO - 1)) == 0);
#pragma unroll
    for (int r = 0; r < RO; ++r) {
        bool ok = leader;
        if constexpr (EDGE) {
            ok = ok && (rout0 + r < hout) && (cout0 < wout);
        }
        if (!ok)
            continue;
        T* d = dst + uint64_t(rout0 + r) * wout + cout0;
        if (!EDGE || cout0 + CO <= wout) {
            store_vec<T, CO, NTS>(d, out[r]);
        } else {
            // the lane's block overhangs the row end (any-width frames)
#pragma unroll
            for (int c = 0; c < CO; ++c) {
                if (cout0 + c < wout) {
                    const T one[1] = { out[r][c] };
                    store_vec<T, 1, NTS>(d + c, one);
                }
            }
        }
    }
}

// Any nonzero byte (the chunk zero scan is byte-wise: -0.0 counts).
template<typename T>
__device__ __forceinline__ bool
nonzero_bits(T x)
{
    if constexpr (sizeof(T) == 8) {
        uint64_t b;
        __builtin_memcpy(&b, &x, 8);
        return b != 0;
    } else {
        uint32_t b = 0;
        __builtin_memcpy(&b, &x, sizeof(T));
        return b != 0;
    }
}

// Write the lane's RO x CO block of level J in chunk-tile order (the layout
// Array::write_frame_to_chunks_ fills, array.cpp:507-622): element (row, col)
// goes to tile (row / tr, col / tc) at (row % tr) * tc + col % tc.  Positions
// past the level inside the padded pw x ph area are stored as zero — the
// bytes Chunk::write_tile_rows leaves in an overhanging tile slot
// (chunk.cpp:17-58) — and positions past the padding are skipped.  `wc0` is
// the wave's first level-0 column (uniform).  Flags: see CascadeParams.
template<typename T, int C, int J, int RO, int CO, bool EDGE, int MODE>
__device__ __forceinline__ void
store_level_tiled(const CascadeParams& p,
                  const T (&out)[RO][CO],
                  uint32_t f,
                  uint32_t wc0,
                  uint32_t row0,
                  int lane)
{
    constexpr int SO = kLaneStride<C, J>;
    constexpr int I = J - 1;
    const TiledLevel t = p.tl[I]; // one kernarg block load
    const uint32_t w = p.w[I], h = p.h[I], tr = t.tr, tc = t.tc;
    const uint32_t pw = t.pw, ph = t.ph;
    const uint32_t lc = (uint32_t(lane) * C) >> J; // lane's column offset in the block
    const uint32_t bc = wc0 >> J;                    // block's first level column (uniform)
    const uint32_t br = row0 >> J;                   // block's first level row (uniform)
    const uint32_t cout0 = bc + lc;
    const bool leader = (SO == 1) || ((lane & (SO - 1)) == 0);
    const uint64_t tile_elems = t.tstride;
    T* base = reinterpret_cast<T*>(t.tdst) + tiled_frame_base(t, f);
    uint8_t* flags = t.flags ? t.flags + uint64_t(f) * t.flags_frame : nullptr;
    auto nested = [&]() {
        const uint32_t K = t.slots;
        // Blocks and tiles nest: the block lies in one tile (its columns at
        // offset bx there), or spans whole tiles side by side (bx = 0).
        // Row and tile coordinates are wave-uniform; lanes add their column.
        constexpr uint32_t BW = (64u * C) >> J; // block columns at this level
        if (br >= ph || bc >= pw)
            return; // past the padding (uniform): no tile, no slot
        const uint32_t ty = t.dr.div(br), tx0 = t.dc.div(bc);
        const uint32_t ry0 = br - ty * tr, bx = bc - tx0 * tc;
        const uint32_t ltx = BW > tc ? t.dc.div(lc) : 0u; // lane's tile within the block
        const uint32_t cx = bx + lc - ltx * tc;
        T* tile = base + (uint64_t(ty) * t.ntx + tx0 + ltx) * tile_elems;
        const bool in_pad = cout0 < pw; // a block spanning tiles may pass the padding
        const bool act = leader && in_pad;
        // Values (zero past the level) and the vote first, so the flag store
        // goes out ahead of the block's data stores: a wave with little data
        // retires only when its last store completes.
        T v[RO][CO];
        bool nz = false;
#pragma unroll
        for (int r = 0; r < RO; ++r) {
#pragma unroll
            for (int c = 0; c < CO; ++c) {
                T x = out[r][c];
                if constexpr (EDGE) {
                    if (br + r >= h || cout0 + c >= w)
                        x = T(0);
                }
                v[r][c] = x;
                nz = nz || (act && nonzero_bits(x));
            }
        }
        const uint64_t votes = __ballot(nz); // every lane reaches the vote
        if (flags && lane == 0) {
            const uint32_t srow = (ry0 / RO) * t.slots_x;
            uint8_t* f0 = flags + (uint64_t(ty) * t.ntx + tx0) * K + srow;
            if (BW <= tc) {
                f0[bx / BW] = votes != 0 ? 1 : 0;
            } else {
                // one slot per tile the block spans: the lanes of tile q are
                // those whose columns fall in [q * tc, (q + 1) * tc)
                const uint32_t lanes = (tc << J) / C; // lanes per tile (<= 64)
                const uint64_t m = lanes >= 64 ? ~0ull : ((1ull << lanes) - 1);
                for (uint32_t q = 0; q * lanes < 64 && tx0 + q < t.ntx; ++q)
                    f0[uint64_t(q) * K] = ((votes >> (q * lanes)) & m) != 0 ? 1 : 0;
            }
        }
        if (act) {
#pragma unroll
            for (int r = 0; r < RO; ++r)
                store_vec<T, CO, true>(tile + uint64_t(ry0 + r) * tc + cx, v[r]);
        }
    };
    auto general = [&]() {
    // General geometry: per-row tile coordinates, per-lane tile columns.
    const uint32_t tx = t.dc.div(cout0);
    const uint32_t cx = cout0 - tx * tc;
#pragma unroll
    for (int r = 0; r < RO; ++r) {
        const uint32_t row = br + r;
        bool ok = leader;
        if constexpr (EDGE) {
            ok = ok && row < ph && cout0 < pw;
        }
        if (!ok)
            continue;
        const uint32_t ty = t.dr.div(row);
        T* trow = base + uint64_t(ty) * t.ntx * tile_elems + uint64_t(row - ty * tr) * tc;
        T v[CO];
        bool rnz = false;
#pragma unroll
        for (int c = 0; c < CO; ++c) {
            T x = out[r][c];
            if constexpr (EDGE) {
                if (row >= h || cout0 + c >= w)
                    x = T(0);
            }
            v[c] = x;
            rnz = rnz || nonzero_bits(x);
        }
        if (cx + CO <= tc) {
            store_vec<T, CO, true>(trow + tx * tile_elems + cx, v);
            if (rnz && flags)
                flags[ty * t.ntx + tx] = 1;
        } else {
            // the lane's columns cross a tile edge (tc not a multiple of CO)
#pragma unroll
            for (int c = 0; c < CO; ++c) {
                const uint32_t col = cout0 + c;
                if (col >= pw)
                    continue;
                const uint32_t ctx = t.dc.div(col);
                const T one[1] = { v[c] };
                store_vec<T, 1, true>(trow + ctx * tile_elems + (col - ctx * tc), one);
                if (flags && nonzero_bits(v[c]))
                    flags[ty * t.ntx + ctx] = 1;
            }
        }
    }

    };
    if constexpr (MODE == 1) {
        nested();
    } else {
        // per level: nested blocks keep their clear-free slots
        if (t.slots)
            nested();
        else
            general();
    }
}

// Level I's TiledLevel with compile-time kernarg offsets (indexing p.tl with
// a runtime I would copy the array to scratch).
__device__ __forceinline__ TiledLevel
tiled_level(const CascadeParams& p, int I)
{
    static_assert(kMaxFusedLevels == 4, "tiled_level");
    return I == 0 ? p.tl[0] : I == 1 ? p.tl[1] : I == 2 ? p.tl[2] : p.tl[3];
}

template<typename T>
__device__ __forceinline__ void
zero_fill_tiled(const CascadeParams& p, uint32_t z, uint32_t nz, int lane, int n_out,
                uint32_t n_frames)
{
    constexpr int E = 16 / int(sizeof(T));
    const uint32_t items = p.zitems * n_frames; // < 2^32: checked at launch
    for (uint32_t it = z; it < items; it += nz) {
        const uint32_t f = p.zdiv.div(it);
        uint32_t rem = it - f * p.zitems;
        int I = 0;
#pragma unroll
        for (int k = 0; k < kMaxFusedLevels - 1; ++k) {
            const uint32_t zr = k == 0 ? p.tl[0].zrows : k == 1 ? p.tl[1].zrows : p.tl[2].zrows;
            if (I == k && I + 1 < n_out && rem >= zr) {
                rem -= zr;
                ++I;
            }
        }
        const TiledLevel t = tiled_level(p, I);
        const uint32_t tr = t.tr, tc = t.tc, pw = t.pw;
        const uint32_t cw = min(t.cov_w, pw), chh = min(t.cov_h, t.ph);
        const uint32_t row = cw < pw ? rem : chh + rem;
        const uint32_t a = row >= chh ? 0u : cw;
        const uint64_t tile_elems = t.tstride;
        const uint32_t ty = t.dr.div(row);
        T* trow = reinterpret_cast<T*>(t.tdst) + tiled_frame_base(t, f) +
                  uint64_t(ty) * t.ntx * tile_elems + uint64_t(row - ty * tr) * tc;
        for (uint32_t tx = t.dc.div(a); tx * tc < pw; ++tx) {
            const uint32_t c0 = max(a, tx * tc) - tx * tc; // segment [c0, tc) in the tile row
            T* seg = trow + tx * tile_elems + c0;
            const uint32_t len = tc - c0;
            for (uint32_t i = uint32_t(lane) * E; i < len; i += 64u * E) {
                if (i + E <= len) {
                    const T zeros[E] = {};
                    store_vec<T, E, true>(seg + i, zeros);
                } else {
                    for (uint32_t k = i; k < len; ++k) {
                        const T zero[1] = { T(0) };
                        store_vec<T, 1, true>(seg + k, zero);
                    }
                }
            }
        }
    }
    // slot flags of blocks no wave of the grid owns (rows >= cov_h or
    // columns >= cov_w at their level)
#pragma unroll
    for (int I = 0; I < kMaxFusedLevels; ++I) {
        if (I >= n_out)
            break;
        const TiledLevel t = p.tl[I];
        if (!t.slots || !t.flags || (t.cov_w >= t.pw && t.cov_h >= t.ph))
            continue;
        const uint32_t K = t.slots, kx = t.slots_x, ky = K / kx;
        const uint32_t bh = t.tr / ky, bw = t.tc / kx; // slot size at the level
        const uint64_t per_frame = t.flags_frame;
        const uint64_t total = per_frame * n_frames;
        for (uint64_t q = uint64_t(z) * 64 + lane; q < total; q += uint64_t(nz) * 64) {
            const uint32_t f = uint32_t(q / per_frame);
            const uint32_t s = uint32_t(q - uint64_t(f) * per_frame);
            const uint32_t tile = s / K, slot = s - tile * K;
            const uint32_t ty = tile / t.ntx, tx = tile - ty * t.ntx;
            const uint32_t r0 = ty * t.tr + (slot / kx) * bh;
            const uint32_t c0 = tx * t.tc + (slot % kx) * bw;
            if (r0 >= t.cov_h || c0 >= t.cov_w)
                t.flags[q] = 0;
        }
    }
}

// Row-band staging (cascade_band_kernel): levels whose rows split 64-byte
// DRAM bursts are written to LDS first, so that one workgroup — which owns
// a whole row band of the frame — stores each level's band as one
// contiguous span in whole 16-byte chunks.  lds[J-1] maps byte 0 to the
// span start rounded down to 16 bytes (`head` bytes before the span).
struct StageCtx
{
    uint8_t* lds[kMaxFusedLevels];
    uint32_t head[kMaxFusedLevels];
    uint32_t mask; // bit J-1: level J is staged
    // LDS row stride (elements) and first staged column per level: the
    // level width and 0 for a whole band, the segment's for a segmented one
    uint32_t stride[kMaxFusedLevels];
    uint32_t scol[kMaxFusedLevels];
    // Misaligned segments (rowb > 0): each level row of the segment is its
    // own piece in LDS, rowb bytes apart, placed at the same offset modulo
    // 16 as its global address, so that it leaves in aligned 16-byte chunks:
    // row r's piece starts (head + r * hstep) % 16 bytes into its slot.
    uint32_t rowb[kMaxFusedLevels];
    uint32_t hstep[kMaxFusedLevels];
};

template<typename T, int C, int J, int RO, int CO, bool EDGE, bool ROWS = false>
__device__ __forceinline__ void
stage_level(const StageCtx& sc,
            const T (&out)[RO][CO],
            uint32_t wout,
            uint32_t hout,
            uint32_t col0,
            uint32_t row0,
            uint32_t band_row0,
            int lane)
{
    constexpr int SO = kLaneStride<C, J>;
    const uint32_t cout0 = col0 >> J;
    const uint32_t rout0 = row0 >> J;
    const bool leader = (SO == 1) || ((lane & (SO - 1)) == 0);
    uint8_t* base = sc.lds[J - 1] + sc.head[J - 1];
#pragma unroll
    for (int r = 0; r < RO; ++r) {
        bool ok = leader;
        if constexpr (EDGE) {
            ok = ok && (rout0 + r < hout) && (cout0 < wout);
        }
        if (!ok)
            continue;
        const uint32_t rr = rout0 + r - (band_row0 >> J); // row within the band
        T* d;
        if constexpr (ROWS) {
            d = reinterpret_cast<T*>(sc.lds[J - 1] + rr * sc.rowb[J - 1] +
                                     ((sc.head[J - 1] + rr * sc.hstep[J - 1]) & 15u)) +
                (cout0 - sc.scol[J - 1]);
        } else {
            d = reinterpret_cast<T*>(base) + uint64_t(rr) * sc.stride[J - 1] +
                (cout0 - sc.scol[J - 1]);
        }
        // A lane's CO elements as one LDS vector write where they are whole
        // and aligned (every row of an aligned band): element writes put the
        // lanes 16 B apart for f32 level 1, a 4-way bank conflict (60% of
        // LDS cycles, profiles/r03/f32/); the element path stays for edges
        // and unaligned bands.
        constexpr int VB = CO * int(sizeof(T));
        if constexpr (VB == 16 || VB == 8 || VB == 4) {
            if ((!EDGE || cout0 + CO <= wout) &&
                (reinterpret_cast<uintptr_t>(d) & uintptr_t(VB - 1)) == 0) {
                if constexpr (VB == 16) {
                    u32x4 v;
                    __builtin_memcpy(&v, out[r], 16);
                    *reinterpret_cast<u32x4*>(d) = v;
                } else if constexpr (VB == 8) {
                    uint64_t v;
                    __builtin_memcpy(&v, out[r], 8);
                    *reinterpret_cast<uint64_t*>(d) = v;
                } else {
                    uint32_t v;
                    __builtin_memcpy(&v, out[r], 4);
                    *reinterpret_cast<uint32_t*>(d) = v;
                }
                continue;
            }
        }
#pragma unroll
        for (int c = 0; c < CO; ++c) {
            if (!EDGE || cout0 + c < wout)
                d[c] = out[r][c];
        }
    }
}

// Level J of the 2-D cascade: reduce, store, recurse to J+1.
template<typename T, int M, int C, int J, int NL, int RI, int CI, bool EDGE,
         bool NTS = false, int STAGED = 0, int TILED = 0>
__device__ __forceinline__ void
cascade_level(const CascadeParams& p,
              const T (&in)[RI][CI],
              uint32_t f,
              uint32_t row0,
              uint32_t col0,
              int lane,
              const StageCtx* sc = nullptr)
{
    constexpr int RO = RI / 2;
    constexpr int CO = (CI >= 2) ? CI / 2 : 1;
    const uint32_t win = (J == 1) ? p.W : p.w[J - 2];
    const uint32_t hin = (J == 1) ? p.H : p.h[J - 2];

    T out[RO][CO];
    xy_step<T, M, C, J, RI, CI, EDGE>(in, out, win, hin, col0 >> (J - 1),
                                      row0 >> (J - 1));
    T* dst = reinterpret_cast<T*>(p.dst[J - 1]) +
             uint64_t(f) * p.dst_frame_elems[J - 1];
    if constexpr (TILED) {
        // a row-major copy only where the next launch reads this level
        if (p.dst[J - 1])
            store_level<T, C, J, RO, CO, EDGE, NTS>(dst, out, p.w[J - 1], p.h[J - 1],
                                                    col0, row0, lane);
        store_level_tiled<T, C, J, RO, CO, EDGE, TILED>(p, out, f, col0 - uint32_t(lane) * C,
                                                        row0, lane);
    } else if constexpr (STAGED) {
        if ((sc->mask >> (J - 1)) & 1u) {
            // the band's rows start at row0 - row0 % 2^NL: one band per block
            stage_level<T, C, J, RO, CO, EDGE, STAGED == 2>(*sc, out, p.w[J - 1], p.h[J - 1],
                                                            col0, row0,
                                                            row0 & ~((1u << NL) - 1u), lane);
        } else {
            store_level<T, C, J, RO, CO, EDGE, NTS>(dst, out, p.w[J - 1], p.h[J - 1],
                                                    col0, row0, lane);
        }
    } else if ((p.wb >> (J - 1)) & 1u) {
        // write-back: partial 64-B bursts of neighbouring waves merge in L2
        store_level<T, C, J, RO, CO, EDGE, false>(dst, out, p.w[J - 1], p.h[J - 1], col0, row0,
                                                  lane);
    } else {
        store_level<T, C, J, RO, CO, EDGE, NTS>(dst, out, p.w[J - 1], p.h[J - 1],
                                                col0, row0, lane);
    }
    if constexpr (J < NL) {
        cascade_level<T, M, C, J + 1, NL, RO, CO, EDGE, NTS, STAGED, TILED>(p, out, f, row0,
                                                                           col0, lane, sc);
    }
}

// C = columns per lane (a multiple of 16 bytes of T); NT / NTS = non-temporal
// loads / stores.  Every byte of the pyramid is touched exactly once, so both
// streams are marked non-temporal: measured on MI355X (tools/microbench.hip,
// profiles/r01) the headline batch drops from ~530 to ~475 us with NT stores.
//
// SPLIT (two 16-byte loads per lane and row, i.e. 4- and 8-byte types at the
// wide tile): the wave's 64 x 32-byte row segment is loaded as two halves of
// 64 x 16 contiguous bytes — load k covers bytes [k KiB, (k+1) KiB) of the
// segment, lane i bytes 16i.. of it — instead of lane i taking bytes 32i..
// in both loads.  Each load instruction then reads whole 128-byte lines, and
// no line is requested by two instructions, which L2 did not always merge
// (F config Min/Max fetched 2.3-2.7% more than the frame).
// The halves are two tiles of E columns per lane, reduced and stored
// (staged) one after the other by the E-column cascade.
template<typename T, int M, int NL, int C, bool NT, bool EDGE, bool NTS = true,
         int STAGED = 0, int TILED = 0, bool SPLIT = false>
__device__ __forceinline__ void
cascade_unit(const CascadeParams& p,
             uint32_t f,
             uint32_t row0,
             uint32_t col0,
             int lane,
             const StageCtx* sc = nullptr)
{
    constexpr int R = 1 << NL;
    constexpr int RB = C * int(sizeof(T));   // bytes per lane per row
    constexpr int LB = RB >= 16 ? 16 : RB;   // bytes per load (8 for narrow tiles)
    constexpr int V = RB / LB;               // loads per row
    constexpr int E = LB / int(sizeof(T));   // elements per load
    const T* src =
      reinterpret_cast<const T*>(p.src) + uint64_t(f) * p.src_frame_elems;
    if constexpr (SPLIT) {
        static_assert(V == 2 && TILED == 0, "SPLIT: two loads per row, row-major/staged levels");
        const uint32_t wc0 = col0 - uint32_t(lane) * C; // the wave's first column
        const bool last_frame = f + 1 == p.total_units / (p.units_x * p.units_y);
        T h[2][R][E];
#pragma unroll
        for (int r = 0; r < R; ++r) {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                load_chunk<T, E, NT, EDGE>(&h[k][r][0], src + uint64_t(row0 + r) * p.W,
                                           wc0 + uint32_t(k) * 64u * E + uint32_t(lane) * E, p.W,
                                           row0 + r < p.H, !last_frame || row0 + r + 1 < p.H, src);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            cascade_level<T, M, E, 1, NL, R, E, EDGE, NTS, STAGED, TILED>(
              p, h[k], f, row0, wc0 + uint32_t(k) * 64u * E + uint32_t(lane) * E, lane, sc);
        }
        return;
    }

    T v[R][C];
    // All row loads are issued before any arithmetic: 2^NL * V outstanding
    // loads per lane (1 KiB per wave instruction at 16 B).
    // reading past a row end stays in the buffer except on the batch's last row
    const bool last_frame = f + 1 == p.total_units / (p.units_x * p.units_y);
#pragma unroll
    for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int k = 0; k < V; ++k) {
            load_chunk<T, E, NT, EDGE>(&v[r][k * E], src + uint64_t(row0 + r) * p.W,
                                       col0 + uint32_t(k) * E, p.W, row0 + r < p.H,
                                       !last_frame || row0 + r + 1 < p.H, src);
        }
    }
    // keep every load above the reductions (the scheduler would otherwise
    // hold back the last rows' loads to save registers)
    __builtin_amdgcn_sched_barrier(0);
    cascade_level<T, M, C, 1, NL, R, C, EDGE, NTS, STAGED, TILED>(p, v, f, row0, col0, lane,
                                                                   sc);
}

// TILED (1: blocks and tiles nest, 2: any chunk shape): every level goes out
// in chunk-tile order (store_level_tiled); the grid's first blocks zero-fill
// the tile overhang its cascade blocks do not reach (zero_fill_tiled).
template<typename T, int M, int NL, int C = kCascadeCols<T>, bool NT = true, int TILED = 0>
__global__ __launch_bounds__(512) void
cascade_kernel(CascadeParams p)
{
    // one tile per wave, the grid covers every tile (no grid-stride loop:
    // measured 2-4% faster for f32 than the looped form), except that small
    // units go p.upw consecutive ones per wave (below)
    constexpr int R = 1 << NL;
    const int lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t blk = blockIdx.x;
    if constexpr (TILED) {
        // The first blocks zero-fill the tile overhang (dispatched round-robin
        // over the XCDs like any blocks); the cascade blocks follow.
        const uint32_t wpb = blockDim.x >> 6;
        const uint32_t zb = p.zwaves / wpb;
        if (blk < zb) {
            zero_fill_tiled<T>(p, blk * wpb + wave, p.zwaves, lane, NL,
                               p.total_units / (p.units_x * p.units_y));
            return;
        }
        blk -= zb;
    }
    if (p.remap) {
        // XCD-contiguous order ($AQZ_XCD_REMAP=1, off by default): workgroup
        // i runs on XCD i % 8, so remapping i to (i % 8) * (n / 8) + i / 8
        // gives XCD x a contiguous eighth of the units (whole frames for
        // batches of >= 8).  Same-box A/B (profiles/r02/remap_ab.log): +2-4%
        // for 5472x3648, -1-5% for 3000^2, within noise at the headline.
        const uint32_t nb8 = p.main_blocks & ~7u;
        if (blk < nb8)
            blk = (blk & 7u) * (nb8 >> 3) + (blk >> 3);
    }
    if constexpr (TILED) {
        // one unit per wave (the loop below, even run once, cost the tiled
        // instantiations 40-70% more VGPRs: headline 60 -> 100, half the
        // occupancy, 3000^2 tiled 539 -> 710 us)
        uint32_t ux, uy, f;
        if (p.seg_w) {
            // band-aligned workgroups (rows that split 128-B lines): the
            // waves sharing a line run on one CU, so it is fetched once
            const uint32_t segs = (p.units_x + p.seg_w - 1) / p.seg_w;
            const uint32_t band = blk / segs;
            ux = (blk - band * segs) * p.seg_w + wave;
            if (ux >= p.units_x || band >= p.total_units / p.units_x)
                return;
            uy = band % p.units_y;
            f = band / p.units_y;
        } else {
            const uint32_t u = blk * (blockDim.x >> 6) + wave;
            if (u >= p.total_units)
                return;
            ux = u % p.units_x;
            const uint32_t t = u / p.units_x;
            uy = t % p.units_y;
            f = t / p.units_y;
        }
        const uint32_t row0 = uy * R;
        const uint32_t tile_col0 = ux * (64u * C);
        const uint32_t col0 = tile_col0 + uint32_t(lane) * C;
        if ((tile_col0 + 64u * C <= p.W) && (row0 + R <= p.H))
            cascade_unit<T, M, NL, C, NT, false, true, 0, TILED>(p, f, row0, col0, lane);
        else
            cascade_unit<T, M, NL, C, NT, true, true, 0, TILED>(p, f, row0, col0, lane);
        return;
    }
    // p.upw > 1 (columns-fastest order, no band workgroups): each wave takes
    // that many consecutive units, for launches whose units move only a few
    // KiB (Decimate of narrow frames reads 2 of 4 rows of 512 B)
    const uint32_t upw = (!p.seg_w && p.order == 0) ? max(p.upw, 1u) : 1u;
    for (uint32_t it = 0; it < upw; ++it) {
        uint32_t ux, uy, f;
        if (p.seg_w) {
            // band-aligned workgroups: the waves that share a row's partial
            // 64-B bursts run on one CU, so the halves meet in its L2
            const uint32_t segs = (p.units_x + p.seg_w - 1) / p.seg_w;
            const uint32_t band = blk / segs;
            ux = (blk - band * segs) * p.seg_w + wave;
            if (ux >= p.units_x || band >= p.total_units / p.units_x)
                return;
            uy = band % p.units_y;
            f = band / p.units_y;
        } else if (const uint32_t u = (blk * (blockDim.x >> 6) + wave) * upw + it;
                   u >= p.total_units) {
            return;
        } else if (p.order == 0) {
            ux = u % p.units_x;
            const uint32_t t = u / p.units_x;
            uy = t % p.units_y;
            f = t / p.units_y;
        } else if (p.order == 1) {
            const uint32_t nf = p.total_units / (p.units_x * p.units_y);
            f = u % nf;
            const uint32_t t = u / nf;
            ux = t % p.units_x;
            uy = t / p.units_x;
        } else {
            uy = u % p.units_y;
            const uint32_t t = u / p.units_y;
            ux = t % p.units_x;
            f = t / p.units_x;
        }
        const uint32_t row0 = uy * R;
        const uint32_t tile_col0 = ux * (64u * C);
        const uint32_t col0 = tile_col0 + uint32_t(lane) * C;
        // wave-uniform: interior tiles take the edge-free path
        if ((tile_col0 + 64u * C <= p.W) && (row0 + R <= p.H)) {
            cascade_unit<T, M, NL, C, NT, false, true, 0, 0>(p, f, row0, col0, lane);
        } else {
            cascade_unit<T, M, NL, C, NT, true, true, 0, 0>(p, f, row0, col0, lane);
        }
    }
}

// Band-staged cascade: one workgroup per row band of one frame, one wave per
// column tile.  Staged levels (StageCtx) go to LDS; after one barrier the
// workgroup writes each staged level's band — consecutive level rows are
// adjacent in memory — as one span of whole, 16-byte-aligned chunks, so only
// the span's first and last chunk share bursts with the neighbouring bands.
// Used for frames whose level rows split 64-byte bursts (widths like 2000 or
// 3000 px, bands of <= 4 tiles, <= 6 for 2-byte types: partial-burst writes
// measured 30% slower than whole ones, tools/pitchbench.hip), where the
// band's last wave stores it instead of a barrier (CascadeParams::band_last),
// and for aligned bands of 5-8 tiles (row-major rows at >= 4 KiB pitch
// written 512 B per wave ran 15% slow on most boxes).  seg_tiles > 0
// (aligned frames only): a band wider than that
// is split into segments of seg_tiles tiles, one workgroup each, every level
// row of a segment one contiguous piece; waves past the last tile only join
// the barrier.
template<typename T, int M, int NL, int C, bool NT = true, bool ROWS = false, bool SPLIT = false>
__global__ __launch_bounds__(512)
// 2-byte Min / Max on line-aligned rows (NT loads): held to 80 VGPRs, 6
// waves per SIMD instead of 5 at 81 (headline Min 481 -> 470 us, Max 483
// -> 470); the same hint on misaligned bands stored by their last wave cost
// 3000^2 Max 546 -> 584 us, and Mean would spill at 80
// (profiles/r03/occupancy/)
__attribute__((amdgpu_waves_per_eu(
  sizeof(T) == 2 && (M == kMin || M == kMax) && NT ? 6 : 1))) void
cascade_band_kernel(CascadeParams p, uint32_t stage_mask, uint32_t seg_tiles)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t band_lds[];
    constexpr int R = 1 << NL;
    const int lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t segs = seg_tiles ? (p.units_x + seg_tiles - 1) / seg_tiles : 1u;
    const uint32_t seg = blockIdx.x % segs;
    const uint32_t band = blockIdx.x / segs;
    const uint32_t uy = band % p.units_y;
    const uint32_t f = band / p.units_y;
    const uint32_t row0 = uy * R;
    const uint32_t ux = seg * seg_tiles + wave;
    const uint32_t seg_col0 = seg * seg_tiles * 64u * C; // level-0 column

    // LDS regions of the staged levels (same arithmetic in every thread)
    StageCtx sc{};
    sc.mask = stage_mask;
    uint32_t len[kMaxFusedLevels] = {};  // bytes per level row piece x rows
    uint32_t rows_of[kMaxFusedLevels] = {};
    uint32_t piece[kMaxFusedLevels] = {}; // bytes of one row's piece (segmented)
    uint8_t* span[kMaxFusedLevels] = {};
    uint32_t off = 0;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
        if (!((stage_mask >> i) & 1u))
            continue;
        const uint32_t r0 = row0 >> (i + 1);
        const uint32_t rows = min(uint32_t(R >> (i + 1)), p.h[i] - min(r0, p.h[i]));
        rows_of[i] = rows;
        if (seg_tiles) {
            const uint32_t c0 = seg_col0 >> (i + 1);
            const uint32_t cw = min((seg_tiles * 64u * C) >> (i + 1), p.w[i] - min(c0, p.w[i]));
            sc.stride[i] = cw;
            sc.scol[i] = c0;
            piece[i] = cw * uint32_t(sizeof(T));
            span[i] = p.dst[i] +
                      (uint64_t(f) * p.dst_frame_elems[i] + uint64_t(r0) * p.w[i] + c0) * sizeof(T);
            len[i] = rows * piece[i];
            if constexpr (ROWS) {
                // misaligned rows: one LDS slot per row (StageCtx::rowb)
                sc.head[i] = uint32_t(reinterpret_cast<uintptr_t>(span[i]) & 15u);
                sc.hstep[i] = (p.w[i] * uint32_t(sizeof(T))) & 15u;
                sc.rowb[i] = (piece[i] + 30u) & ~15u;
                sc.lds[i] = band_lds + off;
                off += rows * sc.rowb[i];
                continue;
            }
            sc.head[i] = 0; // aligned frames: every piece starts on 16 bytes
        } else {
            sc.stride[i] = p.w[i];
            sc.scol[i] = 0;
            span[i] = p.dst[i] + (uint64_t(f) * p.dst_frame_elems[i] + uint64_t(r0) * p.w[i]) *
                                   sizeof(T);
            len[i] = rows * p.w[i] * uint32_t(sizeof(T));
            sc.head[i] = uint32_t(reinterpret_cast<uintptr_t>(span[i]) & 15u);
        }
        sc.lds[i] = band_lds + off;
        off += (sc.head[i] + len[i] + 15u) & ~15u;
    }

    // p.band_last: no barrier before the stores.  Each wave counts itself
    // in once its LDS writes are done, and the last one to arrive stores the
    // whole band, so no wave waits for a slower one (the band's partial edge
    // tile; profiles/r02/band8/misaligned_pmc/).
    __shared__ uint32_t band_arrivals;
    const bool last_mode = p.band_last != 0; // uniform
    if (last_mode) {
        if (threadIdx.x == 0)
            band_arrivals = 0;
        __syncthreads();
    }

    if (ux < p.units_x) { // wave-uniform
        const uint32_t col0 = ux * (64u * C) + uint32_t(lane) * C;
        const bool interior = (ux * 64u * C + 64u * C <= p.W) && (row0 + R <= p.H);
        if (interior)
            cascade_unit<T, M, NL, C, NT, false, true, ROWS ? 2 : 1, 0, SPLIT>(p, f, row0, col0,
                                                                           lane, &sc);
        else
            cascade_unit<T, M, NL, C, NT, true, true, ROWS ? 2 : 1, 0, SPLIT>(p, f, row0, col0,
                                                                          lane, &sc);
    }
    uint32_t tid = threadIdx.x, nth = blockDim.x;
    if (last_mode) {
        // release: this wave's LDS writes complete before its count lands;
        // acquire: the storing waves then see every other wave's.  The last
        // K = p.band_last waves to arrive store the band together; all but
        // the very last wait for the stragglers among them (the workgroup's
        // waves are co-resident, so the count always completes).
        const uint32_t nw = blockDim.x >> 6;
        const uint32_t K = min(p.band_last, nw);
        uint32_t old = 0;
        if (lane == 0)
            old = __hip_atomic_fetch_add(&band_arrivals, 1u, __ATOMIC_ACQ_REL,
                                         __HIP_MEMORY_SCOPE_WORKGROUP);
        old = __builtin_amdgcn_readfirstlane(old);
        if (old + K < nw)
            return;
        if (old + 1u < nw) {
            while (__hip_atomic_load(&band_arrivals, __ATOMIC_ACQUIRE,
                                     __HIP_MEMORY_SCOPE_WORKGROUP) < nw)
                __builtin_amdgcn_s_sleep(1);
        }
        tid = (old + K - nw) * 64u + uint32_t(lane);
        nth = K * 64u;
    } else {
        __syncthreads();
    }

#pragma unroll
    for (int i = 0; i < NL; ++i) {
        if (!((stage_mask >> i) & 1u) || len[i] == 0)
            continue;
        if constexpr (ROWS) {
            // misaligned segment: row r's piece leaves in the 16-byte chunks
            // of its own global span, whole ones as vectors, the two ends
            // (shared with the neighbouring segments) byte by byte
            const uint32_t cmax = sc.rowb[i] / 16u;
            const uint32_t chunks = rows_of[i] * cmax;
            const uint64_t pitch = uint64_t(p.w[i]) * sizeof(T);
            for (uint32_t k = tid; k < chunks; k += nth) {
                const uint32_t r = k / cmax, c = k - r * cmax;
                const uint32_t h = (sc.head[i] + r * sc.hstep[i]) & 15u;
                const uint32_t end = h + piece[i];
                const uint32_t a = c * 16u, b = a + 16u;
                if (a >= end)
                    continue;
                const uint8_t* l = sc.lds[i] + r * sc.rowb[i];
                uint8_t* g = span[i] + r * pitch - h;
                if (a >= h && b <= end) {
                    const u32x4 v = *reinterpret_cast<const u32x4*>(l + a);
                    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(g + a));
                } else {
                    for (uint32_t x = max(a, h); x < min(b, end); ++x)
                        g[x] = l[x];
                }
            }
            continue;
        }
        if (seg_tiles) {
            // rows_of[i] pieces of piece[i] bytes, level pitch apart
            const uint32_t cpr = piece[i] / 16u;
            const uint32_t chunks = rows_of[i] * cpr;
            const uint64_t pitch = uint64_t(p.w[i]) * sizeof(T);
            for (uint32_t k = tid; k < chunks; k += nth) {
                const uint32_t r = k / cpr, c = k - r * cpr;
                const u32x4 v = *reinterpret_cast<const u32x4*>(sc.lds[i] + r * piece[i] + c * 16u);
                __builtin_nontemporal_store(
                  v, reinterpret_cast<u32x4*>(span[i] + r * pitch + c * 16u));
            }
            continue;
        }
        const uint32_t head = sc.head[i];
        const uint32_t end = head + len[i];
        const uint32_t chunks = (end + 15u) / 16u;
        uint8_t* g = span[i] - head;
        for (uint32_t k = tid; k < chunks; k += nth) {
            const uint32_t a = k * 16u, b = a + 16u;
            if (a >= head && b <= end) {
                const u32x4 v = *reinterpret_cast<const u32x4*>(sc.lds[i] + a);
                __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(g + a));
            } else {
                // first / last chunk of the span: only the band's own bytes
                for (uint32_t x = max(a, head); x < min(b, end); ++x)
                    g[x] = sc.lds[i][x];
            }
        }
    }
}

// LDS a band workgroup may use: the device's per-workgroup maximum (160 KiB
// on gfx950, so f32 bands of 8 waves, 85 KiB, fit), 64 KiB if the query
// fails; $AQZ_BAND_LDS_CAP (bytes) lowers it for A/B.
inline uint32_t
band_lds_cap()
{
    static const uint32_t cap = [] {
        int dev = 0, v = 0;
        uint32_t c = 65536;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) ==
              hipSuccess &&
            v > 16)
            c = uint32_t(v) - 16u; // the kernel's static arrival counter
        const int e = int_env("AQZ_BAND_LDS_CAP", 0);
        return e > 0 ? std::min(c, uint32_t(e)) : c;
    }();
    return cap;
}

// Bytes of LDS cascade_band_kernel needs for a band (upper bound over
// bands; 0 if no level is staged).
inline uint32_t
band_lds_bytes(size_t b, const LevelOut* outs, int n_out, uint32_t stage_mask,
               uint32_t seg_cols = 0, bool rowwise = false)
{
    uint64_t total = 0;
    for (int i = 0; i < n_out; ++i) {
        if ((stage_mask >> i) & 1u) {
            const uint64_t rows = uint64_t(1) << (n_out - i - 1);
            const uint64_t w = seg_cols ? std::min<uint64_t>(seg_cols >> (i + 1), outs[i].w)
                                        : outs[i].w;
            if (rowwise)
                total += rows * ((w * b + 30) & ~uint64_t(15)); // StageCtx::rowb slots
            else
                total += (15 + rows * w * b + 15) & ~uint64_t(15);
        }
    }
    return total > (1u << 30) ? (1u << 30) : uint32_t(total);
}

// ---- fused volume (2x2x2, two-stage) ----------------------------------------
//
// For pyramids whose every level halves XY *and* Z (3-D stacks, BASELINE
// config V): the reference reduces each plane 2x2 in XY (scale_image), then
// pairs consecutive reduced planes (average_two_frames, dst = earlier plane,
// src = current) — two truncations, not an 8-way mean.
// One wave owns 2^NL planes x 2^NL rows x (64 lanes x 16 B) and produces
// every level of the run from registers.

struct VolumeParams
{
    const uint8_t* src;
    uint64_t src_frame_elems;
    uint32_t W, H;
    uint32_t units_x;
    uint32_t units_y;
    uint32_t total_units; // units_x * units_y * plane groups
    uint8_t* dst[kMaxVolumeLevels];
    uint64_t dst_frame_elems[kMaxVolumeLevels];
    uint32_t w[kMaxVolumeLevels];
    uint32_t h[kMaxVolumeLevels];
};

template<typename T, int M, int C, int J, int NL, int ZI, int RI, int CI,
         bool EDGE, bool NTS>
__device__ __forceinline__ void
volume_level(const VolumeParams& p,
             const T (&in)[ZI][RI][CI],
             uint32_t g,
             uint32_t row0,
             uint32_t col0,
             int lane)
{
    constexpr int RO = RI / 2;
    constexpr int CO = (CI >= 2) ? CI / 2 : 1;
    constexpr int ZO = ZI / 2;
    const uint32_t win = (J == 1) ? p.W : p.w[J - 2];
    const uint32_t hin = (J == 1) ? p.H : p.h[J - 2];

    T xy[ZI][RO][CO];
#pragma unroll
    for (int z = 0; z < ZI; ++z) {
        xy_step<T, M, C, J, RI, CI, EDGE>(in[z], xy[z], win, hin,
                                          col0 >> (J - 1), row0 >> (J - 1));
    }
    T out[ZO][RO][CO];
#pragma unroll
    for (int z = 0; z < ZO; ++z) {
#pragma unroll
        for (int r = 0; r < RO; ++r) {
#pragma unroll
            for (int c = 0; c < CO; ++c) {
                out[z][r][c] = reduce2<T, M>(xy[2 * z][r][c], xy[2 * z + 1][r][c]);
            }
        }
    }
#pragma unroll
    for (int z = 0; z < ZO; ++z) {
        // level-J frame index: plane group g covers 2^(NL-J) frames there
        T* dst = reinterpret_cast<T*>(p.dst[J - 1]) +
                 (uint64_t(g) * ZO + z) * p.dst_frame_elems[J - 1];
        store_level<T, C, J, RO, CO, EDGE, NTS>(dst, out[z], p.w[J - 1],
                                                p.h[J - 1], col0, row0, lane);
    }
    if constexpr (J < NL) {
        volume_level<T, M, C, J + 1, NL, ZO, RO, CO, EDGE, NTS>(p, out, g, row0,
                                                               col0, lane);
    }
}

// C = columns per lane (V = C*sizeof(T)/16 loads per row).  NTL: loads
// nontemporal.  Decimate reads planes 0 and 2 and rows 0 and 2 of the unit
// only (the other loads have no use and are dropped by the compiler).
template<typename T, int M, int NL, int C, bool EDGE, bool NTL>
__device__ __forceinline__ void
volume_load(const VolumeParams& p,
            uint32_t g,
            uint32_t row0,
            uint32_t col0,
            T (&v)[1 << NL][1 << NL][C])
{
    constexpr int R = 1 << NL;
    constexpr int Z = 1 << NL;
    constexpr int V = C * int(sizeof(T)) / 16;
    const bool last_group = g + 1 == p.total_units / (p.units_x * p.units_y);
#pragma unroll
    for (int z = 0; z < Z; ++z) {
        const T* src = reinterpret_cast<const T*>(p.src) +
                       (uint64_t(g) * Z + z) * p.src_frame_elems;
#pragma unroll
        for (int r = 0; r < R; ++r) {
#pragma unroll
            for (int k = 0; k < V; ++k) {
                constexpr int E = 16 / int(sizeof(T));
                load_chunk<T, E, NTL, EDGE>(&v[z][r][k * E], src + uint64_t(row0 + r) * p.W,
                                            col0 + uint32_t(k) * E, p.W, row0 + r < p.H,
                                            !(last_group && z == Z - 1) ||
                                              row0 + r + 1 < p.H,
                                            src);
            }
        }
    }
}

template<typename T, int M, int NL, int C, bool EDGE, bool NTL>
__device__ __forceinline__ void
volume_unit(const VolumeParams& p,
            uint32_t g,
            uint32_t row0,
            uint32_t col0,
            int lane)
{
    constexpr int R = 1 << NL;
    T v[R][R][C];
    volume_load<T, M, NL, C, EDGE, NTL>(p, g, row0, col0, v);
    volume_level<T, M, C, 1, NL, R, R, C, EDGE, true>(p, v, g, row0, col0, lane);
}

// Unit u's plane group, first row and this lane's first column; true when
// the unit lies wholly inside the frame.  ZFAST puts the plane group
// innermost in the unit order.
template<int NL, int C, bool ZFAST>
__device__ __forceinline__ bool
volume_coords(const VolumeParams& p, uint32_t u, int lane, uint32_t& g, uint32_t& row0,
              uint32_t& col0)
{
    uint32_t ux, uy;
    if constexpr (ZFAST) {
        const uint32_t groups = p.total_units / (p.units_x * p.units_y);
        g = u % groups;
        const uint32_t t = u / groups;
        ux = t % p.units_x;
        uy = t / p.units_x;
    } else {
        ux = u % p.units_x;
        const uint32_t t = u / p.units_x;
        uy = t % p.units_y;
        g = t / p.units_y;
    }
    row0 = uy * (1u << NL);
    const uint32_t tile_col0 = ux * (64u * C);
    col0 = tile_col0 + uint32_t(lane) * C;
    return (tile_col0 + 64u * C <= p.W) && (row0 + (1u << NL) <= p.H);
}

// NTL: nontemporal loads.  UPW units per wave (consecutive, columns first):
// with UPW > 1 and every unit inside the frame, all of them are loaded
// before the first is reduced, so a wave has UPW units' loads in flight —
// Decimate's units read only 4 KiB.  Round 5: with the
// volume in HBM, Decimate's launch runs at 0.59-0.60 of spec with
// nontemporal loads and 0.55-0.56 with plain ones; the 0.82 once measured
// with plain loads came from the Infinity Cache holding the launch's
// 128 MiB read set between launches.
template<typename T, int M, int NL, bool NTL, int UPW, int C = 16 / int(sizeof(T)),
         bool ZFAST = false>
__global__ __launch_bounds__(256) void
volume_kernel(VolumeParams p)
{
    const int lane = threadIdx.x & 63;
    const uint32_t w =
      blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if constexpr (UPW == 1) {
        if (w >= p.total_units)
            return;
        uint32_t g, row0, col0;
        if (volume_coords<NL, C, ZFAST>(p, w, lane, g, row0, col0))
            volume_unit<T, M, NL, C, false, NTL>(p, g, row0, col0, lane);
        else
            volume_unit<T, M, NL, C, true, NTL>(p, g, row0, col0, lane);
    } else {
        constexpr int R = 1 << NL;
        const uint32_t u0 = w * UPW;
        if (u0 >= p.total_units)
            return;
        uint32_t g[UPW], row0[UPW], col0[UPW];
        bool inside = u0 + UPW <= p.total_units;
#pragma unroll
        for (int i = 0; i < UPW; ++i) {
            const uint32_t u = min(u0 + uint32_t(i), p.total_units - 1);
            inside = volume_coords<NL, C, ZFAST>(p, u, lane, g[i], row0[i], col0[i]) && inside;
        }
        if (inside) {
            T v[UPW][R][R][C];
#pragma unroll
            for (int i = 0; i < UPW; ++i)
                volume_load<T, M, NL, C, false, NTL>(p, g[i], row0[i], col0[i], v[i]);
#pragma unroll
            for (int i = 0; i < UPW; ++i)
                volume_level<T, M, C, 1, NL, R, R, C, false, true>(p, v[i], g[i], row0[i],
                                                                   col0[i], lane);
        } else {
            for (int i = 0; i < UPW && u0 + uint32_t(i) < p.total_units; ++i) {
                uint32_t gg, r0, c0;
                if (volume_coords<NL, C, ZFAST>(p, u0 + uint32_t(i), lane, gg, r0, c0))
                    volume_unit<T, M, NL, C, false, NTL>(p, gg, r0, c0, lane);
                else
                    volume_unit<T, M, NL, C, true, NTL>(p, gg, r0, c0, lane);
            }
        }
    }
}

// ---- generic single level --------------------------------------------------

template<typename T, int M>
__global__ __launch_bounds__(256) void
xy_generic_kernel(const T* __restrict__ src,
                  uint64_t src_frame_elems,
                  uint32_t w,
                  uint32_t h,
                  T* __restrict__ dst,
                  uint64_t dst_frame_elems,
                  uint32_t wo,
                  uint32_t ho,
                  uint64_t total)
{
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
         i += uint64_t(gridDim.x) * blockDim.x) {
        const uint32_t c = uint32_t(i % wo);
        const uint64_t t = i / wo;
        const uint32_t r = uint32_t(t % ho);
        const uint64_t f = t / ho;
        const uint32_t col = 2 * c, row = 2 * r;
        const bool pw = col + 1 >= w;
        const bool ph = row + 1 >= h;
        const T* s = src + f * src_frame_elems + uint64_t(row) * w + col;
        const uint32_t dr = pw ? 0 : 1;
        const uint64_t dd = ph ? 0 : w;
        const T here = s[0];
        const T right = s[dr];
        const T down = s[dd];
        const T diag = s[dd + dr];
        dst[f * dst_frame_elems + uint64_t(r) * wo + c] =
          reduce4<T, M>(here, right, down, diag);
    }
}

// ---- Z pair ----------------------------------------------------------------

template<typename T, int M, bool VEC>
__global__ __launch_bounds__(256) void
zpair_kernel(T* out, const T* earlier, const T* current, uint64_t n)
{
    constexpr int C = 16 / int(sizeof(T));
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    const uint64_t tid = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    uint64_t done = 0;
    if constexpr (VEC) {
        // all three pointers 16-byte aligned: 16 B per lane per operand
        const uint64_t nvec = n / C;
        for (uint64_t i = tid; i < nvec; i += stride) {
            const u32x4 qa = reinterpret_cast<const u32x4*>(earlier)[i];
            const u32x4 qb = reinterpret_cast<const u32x4*>(current)[i];
            T a[C], b[C], o[C];
            __builtin_memcpy(a, &qa, 16);
            __builtin_memcpy(b, &qb, 16);
#pragma unroll
            for (int k = 0; k < C; ++k) {
                o[k] = reduce2<T, M>(a[k], b[k]);
            }
            store_vec<T, C>(out + i * C, o);
        }
        done = nvec * C;
    }
    for (uint64_t i = done + tid; i < n; i += stride) {
        out[i] = reduce2<T, M>(earlier[i], current[i]);
    }
}

// ---- chunk tiling --------------------------------------
//
// Array::write_frame_to_chunks_ (array.cpp:507-622) copies each frame tile's
// rows into its chunk buffer at stride tile_cols*bpp (Chunk::write_tile_rows,
// chunk.cpp:17-58), leaving the overhang zero, and byte-scans the copied rows
// for the all-zero-chunk skip.  This kernel emits the frame already in that
// tile order (zero-padded) plus the scan result, so the host does one
// contiguous copy per tile and no scan.  Grid: `slices` blocks per tile, one
// block-wide OR per block.

// SLICE_FLAGS: every block writes its own flag byte (flags[t*slices + s]),
// no atomics and no pre-clear; otherwise one u32 per tile, OR-ed atomically
// (the caller clears it).
template<typename T, bool SLICE_FLAGS>
__global__ __launch_bounds__(256) void
tile_kernel(const T* __restrict__ src,
            uint32_t W,
            uint32_t H,
            uint32_t tile_rows,
            uint32_t tile_cols,
            uint32_t n_tiles_x,
            uint32_t slices,
            T* __restrict__ dst,
            void* __restrict__ flags)
{
    const uint32_t t = blockIdx.x / slices;
    const uint32_t s = blockIdx.x % slices;
    const uint32_t ty = t / n_tiles_x, tx = t % n_tiles_x;
    const uint32_t tile_elems = tile_rows * tile_cols; // < 2^31, checked by the launcher
    const uint32_t per = (tile_elems + slices - 1) / slices;
    const uint32_t e0 = s * per;
    const uint32_t e1 = e0 + per < tile_elems ? e0 + per : tile_elems;
    T* out = dst + uint64_t(t) * tile_elems;
    bool any = false;
    for (uint32_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
        const uint32_t r = e / tile_cols;
        const uint32_t c = e % tile_cols;
        const uint32_t row = ty * tile_rows + r;
        const uint32_t col = tx * tile_cols + c;
        T v = T(0);
        if (row < H && col < W) {
            v = src[uint64_t(row) * W + col];
            any = any || nonzero_bits(v);
        }
        out[e] = v;
    }
    const bool block_any = __syncthreads_or(any);
    if (threadIdx.x == 0) {
        if constexpr (SLICE_FLAGS) {
            static_cast<uint8_t*>(flags)[blockIdx.x] = block_any ? 1 : 0;
        } else if (block_any) {
            atomicOr(static_cast<uint32_t*>(flags) + t, 1u);
        }
    }
}

// 16-B vector form for frames whose rows and tiles are 16-B multiples (so a
// vector is entirely inside or entirely outside the frame): block = one
// (tile, slice of rows); lane = one 16-B vector of a tile row.
__device__ __forceinline__ bool
nonzero_vec(u32x4 v)
{
    return (v.x | v.y | v.z | v.w) != 0;
}

template<bool SLICE_FLAGS>
__global__ __launch_bounds__(256) void
tile_kernel_vec(const u32x4* __restrict__ src,
                uint32_t row_vecs,   // W * bpp / 16
                uint32_t H,
                uint32_t tile_rows,
                uint32_t tile_vecs,  // tile_cols * bpp / 16
                uint32_t n_tiles_x,
                uint32_t slices,
                u32x4* __restrict__ dst,
                void* __restrict__ flags)
{
    const uint32_t t = blockIdx.x / slices;
    const uint32_t s = blockIdx.x % slices;
    const uint32_t ty = t / n_tiles_x, tx = t % n_tiles_x;
    const uint32_t rows_per = (tile_rows + slices - 1) / slices;
    const uint32_t r0 = s * rows_per;
    const uint32_t r1 = r0 + rows_per < tile_rows ? r0 + rows_per : tile_rows;
    // 32-bit in-slice indices (the launcher keeps a tile below 2^31 vectors)
    const uint32_t n = (r1 > r0 ? r1 - r0 : 0) * tile_vecs;
    u32x4* out = dst + uint64_t(t) * tile_rows * tile_vecs + uint64_t(r0) * tile_vecs;
    const uint32_t col_v0 = tx * tile_vecs;
    bool any = false;
    // U vectors per lane per round, all loads issued before the stores
    constexpr uint32_t U = 8;
    for (uint32_t e0 = threadIdx.x; e0 < n; e0 += U * blockDim.x) {
        u32x4 v[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t e = e0 + u * blockDim.x;
            const uint32_t r = r0 + e / tile_vecs;
            const uint32_t cv = col_v0 + e % tile_vecs;
            const uint32_t row = ty * tile_rows + r;
            v[u] = u32x4{ 0u, 0u, 0u, 0u };
            if (e < n && row < H && cv < row_vecs)
                v[u] = __builtin_nontemporal_load(src + uint64_t(row) * row_vecs + cv);
        }
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t e = e0 + u * blockDim.x;
            if (e < n) {
                any = any || nonzero_vec(v[u]);
                __builtin_nontemporal_store(v[u], out + e);
            }
        }
    }
    const bool block_any = __syncthreads_or(any);
    if (threadIdx.x == 0) {
        if constexpr (SLICE_FLAGS) {
            static_cast<uint8_t*>(flags)[blockIdx.x] = block_any ? 1 : 0;
        } else if (block_any) {
            atomicOr(static_cast<uint32_t*>(flags) + t, 1u);
        }
    }
}

// ---- transpose_frame (array.cpp:488-504) ------------------------------------
//
// Y x X -> X x Y of a row-major `rows` x `cols` frame, for arrays whose
// storage order swaps the two spatial dimensions (Array::write_frame_to_chunks_
// transposes level 0 before chunking, array.cpp:517-530, and the downsampler
// then sees the transposed frame).  Pure data movement, HBM-bound:
// 2 * rows * cols * sizeof(T) bytes.  One block per kTransposeSub tiles of
// kTransposeTile^2 elements,
// staged through LDS so both the global reads (source rows) and the global
// writes (destination rows) are contiguous; with VEC each lane moves 16 B per
// access on interior tiles.  Edge tiles (and VEC=false frames, whose rows are
// not 16-B aligned) move one element per access.

// tile edge in elements: 256-B row segments on both sides (128 B for u8)
template<typename T>
constexpr int kTransposeTile = sizeof(T) == 1 ? 128 : 256 / int(sizeof(T));

template<typename T>
constexpr int kTransposePitch = kTransposeTile<T> + (sizeof(T) >= 4 ? 1 : 4 / int(sizeof(T)));

// tiles per block, stacked along the source rows: 32 KiB per block for every
// dtype (a lone 64 x 64 f32 tile moved 16 KiB and measured 84% of a D2D copy)
template<typename T>
constexpr int kTransposeSub =
  32768 / (kTransposeTile<T> * kTransposeTile<T> * int(sizeof(T))) > 1
    ? 32768 / (kTransposeTile<T> * kTransposeTile<T> * int(sizeof(T)))
    : 1;

template<typename T, bool VEC>
__global__ __launch_bounds__(256) void
transpose_kernel(const T* __restrict__ src, uint32_t rows, uint32_t cols, T* __restrict__ dst)
{
    constexpr int TD = kTransposeTile<T>;
    constexpr int P = kTransposePitch<T>;
    constexpr int S = kTransposeSub<T>;
    __shared__ T tile[S][TD * P];
    const uint32_t c0 = blockIdx.x * TD;     // source columns = destination rows
    const uint32_t rb = blockIdx.y * TD * S; // source rows = destination columns
    const int tid = threadIdx.x;
    const bool interior = VEC && rb + TD * S <= rows && c0 + TD <= cols;
    if (interior) {
        constexpr int V = 16 / int(sizeof(T));
        constexpr int VPR = TD / V;       // vectors per tile row
        constexpr int RPP = 256 / VPR;    // tile rows per pass
        const int v = tid % VPR;
        if constexpr (S > 1) {
            // every sub-tile's loads before the first LDS store (f32 84% ->
            // 91% of a D2D copy, u8 likewise; the lone u16 tile measured
            // faster with each load followed by its LDS store, below)
            u32x4 x[S][TD / RPP];
#pragma unroll
            for (int t = 0; t < S; ++t) {
#pragma unroll
                for (int i = 0; i < TD / RPP; ++i) {
                    const int r = tid / VPR + i * RPP;
                    x[t][i] = __builtin_nontemporal_load(
                      reinterpret_cast<const u32x4*>(src + uint64_t(rb + t * TD + r) * cols + c0) +
                      v);
                }
            }
#pragma unroll
            for (int t = 0; t < S; ++t) {
#pragma unroll
                for (int i = 0; i < TD / RPP; ++i) {
                    const int r = tid / VPR + i * RPP;
                    T e[V];
                    __builtin_memcpy(e, &x[t][i], 16);
#pragma unroll
                    for (int k = 0; k < V; ++k)
                        tile[t][r * P + v * V + k] = e[k];
                }
            }
        } else {
#pragma unroll
            for (int r = tid / VPR; r < TD; r += RPP) {
                const u32x4 x = __builtin_nontemporal_load(
                  reinterpret_cast<const u32x4*>(src + uint64_t(rb + r) * cols + c0) + v);
                T e[V];
                __builtin_memcpy(e, &x, 16);
#pragma unroll
                for (int k = 0; k < V; ++k)
                    tile[0][r * P + v * V + k] = e[k];
            }
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < S; ++t) {
#pragma unroll
            for (int c = tid / VPR; c < TD; c += RPP) {
                T e[V];
#pragma unroll
                for (int k = 0; k < V; ++k)
                    e[k] = tile[t][(v * V + k) * P + c];
                u32x4 y;
                __builtin_memcpy(&y, e, 16);
                auto* q =
                  reinterpret_cast<u32x4*>(dst + uint64_t(c0 + c) * rows + rb + t * TD) + v;
                __builtin_nontemporal_store(y, q);
            }
        }
    } else {
        // one element per access; lanes sweep rows so accesses stay contiguous
        const int x = tid % TD;
        for (int t = 0; t < S; ++t) {
            const uint32_t r0 = rb + t * TD;
            for (int r = tid / TD; r < TD; r += 256 / TD) {
                if (r0 + r < rows && c0 + x < cols)
                    tile[t][r * P + x] = src[uint64_t(r0 + r) * cols + c0 + x];
            }
        }
        __syncthreads();
        for (int t = 0; t < S; ++t) {
            const uint32_t r0 = rb + t * TD;
            for (int c = tid / TD; c < TD; c += 256 / TD) {
                if (c0 + c < cols && r0 + x < rows)
                    dst[uint64_t(c0 + c) * rows + r0 + x] = tile[t][x * P + c];
            }
        }
    }
}

// ---- dispatch ---------------------------------------------------------------

template<typename F>
hipError_t
with_dtype(int dtype, F&& f)
{
    // only this shard's dtypes are instantiated
    switch (dtype) {
        case 0:
            if constexpr (0 % AQZ_SHARDS == AQZ_SHARD)
                return f(uint8_t{});
            return hipErrorInvalidValue;
        case 1:
            if constexpr (1 % AQZ_SHARDS == AQZ_SHARD)
                return f(uint16_t{});
            return hipErrorInvalidValue;
        case 2:
            if constexpr (2 % AQZ_SHARDS == AQZ_SHARD)
                return f(uint32_t{});
            return hipErrorInvalidValue;
        case 3:
            if constexpr (3 % AQZ_SHARDS == AQZ_SHARD)
                return f(uint64_t{});
            return hipErrorInvalidValue;
        case 4:
            if constexpr (4 % AQZ_SHARDS == AQZ_SHARD)
                return f(int8_t{});
            return hipErrorInvalidValue;
        case 5:
            if constexpr (5 % AQZ_SHARDS == AQZ_SHARD)
                return f(int16_t{});
            return hipErrorInvalidValue;
        case 6:
            if constexpr (6 % AQZ_SHARDS == AQZ_SHARD)
                return f(int32_t{});
            return hipErrorInvalidValue;
        case 7:
            if constexpr (7 % AQZ_SHARDS == AQZ_SHARD)
                return f(int64_t{});
            return hipErrorInvalidValue;
        case 8:
            if constexpr (8 % AQZ_SHARDS == AQZ_SHARD)
                return f(float{});
            return hipErrorInvalidValue;
        case 9:
            if constexpr (9 % AQZ_SHARDS == AQZ_SHARD)
                return f(double{});
            return hipErrorInvalidValue;
        default:
            return hipErrorInvalidValue;
    }
}

template<typename F>
hipError_t
with_method(int method, F&& f)
{
    switch (method) {
        case kDecimate:
            return f(std::integral_constant<int, kDecimate>{});
        case kMean:
            return f(std::integral_constant<int, kMean>{});
        case kMin:
            return f(std::integral_constant<int, kMin>{});
        case kMax:
            return f(std::integral_constant<int, kMax>{});
        default:
            return hipErrorInvalidValue;
    }
}


uint32_t
grid_for(uint64_t work_items, uint32_t per_block, uint32_t cap)
{
    uint64_t blocks = (work_items + per_block - 1) / per_block;
    if (blocks < 1)
        blocks = 1;
    if (cap && blocks > cap)
        blocks = cap;
    return uint32_t(blocks);
}

} // namespace
#if AQZ_SHARD == 0

size_t
dtype_bytes(int dtype)
{
    switch (dtype) {
        case 0:
        case 4:
            return 1;
        case 1:
        case 5:
            return 2;
        case 2:
        case 6:
        case 8:
            return 4;
        case 3:
        case 7:
        case 9:
            return 8;
        default:
            return 0;
    }
}
#endif
#if AQZ_SHARD == 0

bool
dtype_valid(int dtype)
{
    return dtype_bytes(dtype) != 0;
}
#endif
#if AQZ_SHARD == 0

bool
method_valid(int method)
{
    return method >= kDecimate && method <= kMax;
}
#endif


#if AQZ_SHARD == 0
namespace {

// Can the fused cascade run this level run with C columns per lane?
bool
cascade_fits(size_t b,
             const void* src,
             uint64_t src_frame_elems,
             uint32_t W,
             uint32_t H,
             const LevelOut* outs,
             int n_out,
             uint32_t C)
{
    if (!b || C == 0 || n_out < 1 || n_out > kMaxFusedLevels || W == 0 || H == 0)
        return false;
    // Frames of any width and byte offset: loads and stores take any
    // alignment; a lane straddling a row end loads one vector (load_chunk)
    // and stores element by element (store_level).  Needs element-aligned
    // buffers and a row of at least one load (E elements); narrower frames
    // take the single-level kernels.
    const size_t lb = std::min<size_t>(16, size_t(C) * b);
    if (reinterpret_cast<uintptr_t>(src) % b != 0 || W < lb / b)
        return false;
    uint32_t w = W, h = H;
    for (int i = 0; i < n_out; ++i) {
        w = (w + 1) / 2;
        h = (h + 1) / 2;
        if (outs[i].w != w || outs[i].h != h)
            return false;
        if (reinterpret_cast<uintptr_t>(outs[i].ptr) % b != 0)
            return false;
    }
    return true;
}

} // namespace
#endif
#if AQZ_SHARD == 0

// 16-byte tiles for 4- and 8-byte types: rows whose level 1-4 rows are all
// whole 64-B bursts (cascade_pick_cols, cascade_tiled_cols)
static bool
narrow_rows(size_t b, uint32_t W)
{
    return b >= 4 && (uint64_t(W) * b) % 1024 == 0;
}

uint32_t
cascade_pick_cols(int dtype,
                  const void* src,
                  uint64_t src_frame_elems,
                  uint32_t W,
                  uint32_t H,
                  const LevelOut* outs,
                  int n_out)
{
    const size_t b = dtype_bytes(dtype);
    if (!b)
        return 0;
    // wide tiles (kCascadeCols) where a wave's 64 lanes fit in the frame;
    // half-width tiles for narrower frames (a 512-px u8 frame would leave half
    // of every wide wave idle on the edge path) and for widths only the
    // narrow tile divides
    const uint32_t cw = cascade_cols(b), cn = cw / 2;
    const bool wide = cascade_fits(b, src, src_frame_elems, W, H, outs, n_out, cw);
    const bool narrow = cascade_fits(b, src, src_frame_elems, W, H, outs, n_out, cn);
    // 4-byte types on rows of whole 128-B lines take 16-byte tiles too (4
    // columns per lane: 73 VGPRs, 6 waves per SIMD, against 138 VGPRs and 3
    // waves for 32-byte tiles) now that such rows leave through LDS-staged
    // bands: 4096^2 f32 Mean 985 -> 948 us, Max 992 -> 946, Decimate 604 ->
    // 583, 8192x2048 947 -> 903, 3072^2 1105 -> 1018 (profiles/r05/narrow/;
    // round 1, before band staging, had measured the opposite, 1083 -> 975
    // us for the wide tiles).  Rows that split lines keep the wide tiles and
    // their misaligned segments: 5472x3648 1091 against 1206 us narrow,
    // 6000x4000 1049 against 1150, 2000^2 1085 against 1123.  The same holds
    // for the other 4- and 8-byte types at 4096^2: u32 Mean 994 -> 947 us,
    // f64 Mean 1034 -> 884, f64 Max 1056 -> 889 (profiles/r05/widths/).
    // "Whole lines" must hold for the levels too, not only level 0: f32
    // 5472x3648 (21888-B rows, level 2 splits bursts) ran 1155 us narrow
    // against 1065-1091 wide (profiles/r05/shapes/), so the rule asks for
    // W * b a multiple of 1024 (levels 1-4 rows whole 64-B bursts).
    // $AQZ_CASCADE_NARROW=0/1 (A/B) forces wide / narrow for 4- and 8-byte
    // types.
    static const int narrow_env = int_env("AQZ_CASCADE_NARROW", -1);
    const bool prefer_narrow = narrow_env >= 0 ? (narrow_env != 0 && b >= 4)
                                               : narrow_rows(b, W);
    if (prefer_narrow && narrow)
        return cn;
    if (wide && W >= 64 * cw)
        return cw;
    if (narrow)
        return cn;
    return wide ? cw : 0;
}
#endif
#if AQZ_SHARD == 0

bool
cascade_supported(int dtype,
                  const void* src,
                  uint64_t src_frame_elems,
                  uint32_t W,
                  uint32_t H,
                  const LevelOut* outs,
                  int n_out)
{
    return cascade_pick_cols(dtype, src, src_frame_elems, W, H, outs, n_out) != 0;
}
#endif

hipError_t
AQZ_SHARDED(launch_cascade)(int dtype,
               int method,
               const void* src,
               uint64_t src_frame_elems,
               uint32_t W,
               uint32_t H,
               const LevelOut* outs,
               int n_out,
               uint32_t n_frames,
               hipStream_t stream)
{
    const uint32_t cols = cascade_pick_cols(dtype, src, src_frame_elems, W, H, outs, n_out);
    if (cols == 0 || n_frames == 0)
        return hipErrorInvalidValue;

    return with_dtype(dtype, [&](auto tag) -> hipError_t {
        using T = decltype(tag);
        constexpr uint32_t CW = kCascadeCols<T>;
        constexpr uint32_t CN = CW / 2;
        CascadeParams p{};
        p.src = static_cast<const uint8_t*>(src);
        p.src_frame_elems = src_frame_elems;
        p.W = W;
        p.H = H;
        p.units_x = (W + 64 * cols - 1) / (64 * cols);
        const uint32_t R = 1u << n_out;
        p.units_y = (H + R - 1) / R;
        const uint64_t total = uint64_t(p.units_x) * p.units_y * n_frames;
        if (total >= (1ull << 31))
            return hipErrorInvalidValue;
        p.total_units = uint32_t(total);
        for (int i = 0; i < n_out; ++i) {
            p.dst[i] = static_cast<uint8_t*>(outs[i].ptr);
            p.dst_frame_elems[i] = outs[i].frame_elems;
            p.w[i] = outs[i].w;
            p.h[i] = outs[i].h;
        }
        // 4 waves per block, one tile per wave per iteration.
        static const uint32_t wpb = uint32_t(std::clamp(int_env("AQZ_CASCADE_WAVES", 4), 1, 8));
        static const uint32_t order = uint32_t(std::clamp(int_env("AQZ_UNIT_ORDER", 0), 0, 2));
        // Units per wave (cascade_kernel's loop): a Decimate wave whose unit
        // reads under 4 KiB takes 2, 4 or 8 consecutive units, so that it
        // moves at least that much: 512^2 u8 Decimate (1 KiB read per unit)
        // 55.3 -> 40.7 us with 4 (8: 45.8).  Other methods keep one unit per
        // wave and, where that unit is under 4 KiB, load plain: 512^2 u8
        // Mean 61.4-62.0 -> 59.4-59.8 us, Max 61.8 -> 60.6-61.2 against two
        // units with nontemporal loads.  Round 5, with the input and output
        // in HBM (rotating buffer sets); round 4's
        // two-unit Mean/Max choice had been timed with the whole read set
        // resident in the Infinity Cache.  2048^2 u16 Decimate (4 KiB units)
        // keeps 1 (two: 76.5 -> 78.8-80.1 us).  $AQZ_UNITS_PER_WAVE=k forces k.
        static const int upw_env = int_env("AQZ_UNITS_PER_WAVE", 0);
        uint32_t upw = 1;
        bool small_plain = false;
        if (upw_env > 0) {
            upw = uint32_t(std::min(upw_env, 16));
        } else {
            const uint64_t unit_bytes = (uint64_t(R) * 64u * cols * sizeof(T)) >>
                                        (method == kDecimate ? 1 : 0);
            if (method == kDecimate) {
                while (upw < 8 && unit_bytes * upw < 4096)
                    upw *= 2;
            } else {
                small_plain = unit_bytes < 4096;
            }
        }
        p.upw = order == 0 ? upw : 1u;
        const uint32_t grid = grid_for((total + p.upw - 1) / p.upw, wpb, 0);
        p.main_blocks = grid;
        p.order = order;
        p.remap = xcd_remap_env() == 1;
        p.wb = store_wb_env() >= 0 ? uint32_t(store_wb_env()) : 0u;
        p.nt = load_nt(W, sizeof(T));
        // Loads keep the nontemporal hint on aligned rows, Decimate's looped
        // small units included (512^2 u8 Decimate 40.7 us against 42.1-42.5
        // plain, with the data in HBM; the round-5 plain-load rule had been
        // timed with its 128 MiB read set resident in the Infinity Cache,
        // DESIGN.md §11.11), except the small single units above.
        if (load_nt_env() < 0 && small_plain)
            p.nt = 0;
        // Band staging when some level's rows are not whole 64-byte bursts
        // and a row band is at most 4 tiles, 6 for 2-byte types
        // ($AQZ_BAND_STAGING=0: never; $AQZ_BAND_MIS_MAX: the widest such
        // band).  These bands are stored by their last wave to finish
        // (p.band_last = 1), not after a barrier: any wait for the band's
        // slowest wave cost more than staging saves (u16 3000^2 805 us with
        // a barrier, 594 / 676 us with the last two / three waves storing,
        // 546 us with the last one, against 575 us for direct stores;
        // profiles/r03/misaligned/last_wave_ab.log).  Against the barrier
        // form of <= 4 tiles and direct stores above (mis6_edges_ab.log):
        // u16 2000^2 570 -> 523 us, 2304^2 565 -> 498, 3000^2 575 -> 549,
        // 2600^2 538 -> 547; u8 3000^2 104 -> 85; f32 2000^2 unchanged.
        // One wave storing a wider band is too slow: u16 4000x3000 (8 tiles)
        // 557 -> 627 us, u8 5000x4000 (5 tiles) 91 -> 101, f32 3000^2 (6
        // tiles, 64 KiB) 1095 -> 1442, so those keep direct stores.  Aligned
        // bands keep the barrier, where all waves share the stores (4096^2
        // f32 987 us against 1026 / 1058 us).  $AQZ_BAND_LAST=K forces the
        // last K waves to store every band (0: the barrier).  Also tried and
        // dropped: waves storing the bursts inside their own tile from
        // registers and the last wave only the shared ones (5-27% slower).
        static const int band_last_env = int_env("AQZ_BAND_LAST", -1);
        static const int mis_max_env = int_env("AQZ_BAND_MIS_MAX", -1);
        // 16-byte tiles of 4-byte types move 1 KiB per row per wave, as the
        // 2-byte tiles do, so they share the 2-byte thresholds
        const bool tile16 = sizeof(T) == 2 || (sizeof(T) == 4 && cols == CN);
        const uint32_t mis_max = mis_max_env >= 0 ? uint32_t(std::min(mis_max_env, 8))
                                                  : (tile16 ? 6u : 4u);
        static const int mis_seg_env = std::min(int_env("AQZ_BAND_MIS_SEG", -1), 8);
        uint32_t stage_mask = 0;
        for (int i = 0; i < n_out; ++i) {
            const bool whole = (uint64_t(outs[i].w) * sizeof(T)) % 64 == 0 &&
                               (outs[i].frame_elems * sizeof(T)) % 64 == 0 &&
                               reinterpret_cast<uintptr_t>(outs[i].ptr) % 64 == 0;
            if (!whole)
                stage_mask |= 1u << i;
        }
        static const bool band_off = [] {
            const char* v = std::getenv("AQZ_BAND_STAGING");
            return v && std::strcmp(v, "0") == 0;
        }();
        // Aligned frames of 4-8 tiles per row band (the headline's 4096 u16
        // pixels, 3072, 4096 f32, config C2's 2048 u16) stage every level
        // too, in workgroups of one wave per tile, so each level's band
        // leaves as one contiguous span.  4-tile bands joined in round 5,
        // timed with the data in HBM (rotating buffer sets): C2 Mean 123.0-
        // 123.5 -> 118.1-118.4 us, Decimate 76.7-76.9 -> 72.1-72.4
        // (profiles/r05/c2knobs/ab.log).
        // On most MI355X boxes tried, row-major level rows at a >= 4 KiB
        // pitch written 512 B per wave ran 15-20% below the same kernel with
        // tile-order stores; staged bands remove that (headline 535 -> 463
        // us, 3072^2 541 -> 448 us; profiles/r02/band8_*).
        // $AQZ_BAND_ALIGNED=0 turns this off; $AQZ_BAND_FORCE (A/B) stages a
        // level mask whatever the alignment, in bands of up to 8 waves.
        // Aligned bands wider than 8 tiles go in 8-tile segments, one
        // workgroup each, every level row of a segment one contiguous piece:
        // 8192x2048 u16 517 -> 485 us, 8704x2040 532 -> 447 us, 6144x3072
        // 531 -> 516 us, 8192x2048 f32 1012 -> 962 us
        // (profiles/r02/band8/segments_ab.log); $AQZ_BAND_SEGMENTS=0: off.
        static const uint32_t band_force = uint32_t(int_env("AQZ_BAND_FORCE", 0));
        static const bool band_aligned = int_env("AQZ_BAND_ALIGNED", 1) != 0;
        static const bool band_segments = int_env("AQZ_BAND_SEGMENTS", 1) != 0;
        uint32_t band_waves = p.units_x;
        const uint32_t all_levels = (1u << n_out) - 1u;
        uint32_t wide_max = mis_max, seg_tiles = 0;
        const bool misaligned = stage_mask != 0;
        p.band_last = band_last_env >= 0 ? uint32_t(std::min(band_last_env, 8))
                                         : (misaligned ? 1u : 0u);
        if (band_force) {
            stage_mask |= band_force & all_levels;
            wide_max = 8;
        } else if (band_aligned && stage_mask == 0 && band_waves >= 4 && band_waves <= 8 &&
                   band_lds_bytes(sizeof(T), outs, n_out, all_levels) <= band_lds_cap()) {
            stage_mask = all_levels;
            wide_max = 8;
            // 8-tile bands go in segments (first measured as two of 4 tiles,
            // below): a whole 4096 f32 band
            // needs 85 KiB of LDS, one workgroup per CU, whose loads and
            // stores then never overlap; segments fit two or three.  Same
            // box, two rounds (profiles/r03/f32/band_seg4_ab.log): f32 Max
            // 1062 -> 999 us, Mean 1042 -> 991, Min 1064 -> 998, the headline
            // 478 -> 473; 6-tile bands lost (3072^2 470 -> 510), so only
            // bands of 8.  $AQZ_BAND_SEG4=0 / 1: never / always.
            // Tiles per segment: 3 (segments of 3, 3, 2) for 2-byte Mean and
            // for Decimate, 4 otherwise.  Same box, two rounds each
            // (profiles/r03/f32/segment_tiles_ab*.log): headline (u16 Mean)
            // 473-475 -> 462-463 us, 4096x2160 469-473 -> 461-462, u16
            // Decimate 297 -> 294, f32 Decimate 644-652 -> 607-608; but u16
            // Min/Max 472-474 -> 480-483 and f32 Mean/Min/Max 990-1000 ->
            // 1027-1030, which keep 4.  $AQZ_BAND_SEGN overrides (A/B).
            static const int seg4 = int_env("AQZ_BAND_SEG4", -1);
            static const int segn_env = int_env("AQZ_BAND_SEGN", 0);
            const uint32_t segn = segn_env > 0 ? uint32_t(std::min(segn_env, 8))
                                  : (method == kDecimate || (method == kMean && sizeof(T) == 2))
                                    ? 3u : 4u;
            if (seg4 == 1 || (seg4 < 0 && band_waves == 8)) {
                seg_tiles = segn;
                band_waves = segn;
            }
        } else if (band_aligned && band_segments && stage_mask == 0 && band_waves > 8 &&
                   band_lds_bytes(sizeof(T), outs, n_out, all_levels, 8u * 64u * cols) <=
                     band_lds_cap()) {
            stage_mask = all_levels;
            seg_tiles = 8;
            band_waves = 8;
            wide_max = 8;
        } else if (misaligned && band_waves > mis_max && (sizeof(T) == 2 || sizeof(T) == 4) &&
                   // exactly the tiles the dispatch below builds a rowwise
                   // (RW) band kernel for (2-byte narrow tiles
                   // have none)
                   (cols == CW || (sizeof(T) == 4 && cols == CN)) &&
                   (mis_seg_env > 0 || (mis_seg_env < 0 && band_waves > 8))) {
            // Misaligned bands of more than 8 tiles (2- and 4-byte types, wide
            // tiles): balanced segments of at most 4 tiles
            // ($AQZ_BAND_MIS_SEG: any band of those types wider than one
            // wave may store, segments of that many tiles; 0: never), each staged and stored by its last wave,
            // every level row of a segment its own piece (StageCtx::rowb);
            // only the pieces' ends share bursts with the neighbouring
            // segments.  Same box, two rounds, against band workgroups with
            // direct stores (profiles/r03/misaligned/mis_segments_ab*.log):
            // f32 5472x3648 1264 -> 1092 us, 6000x4000 1167 -> 1104, 4100^2
            // 1150 -> 1077; u16 6000x4000 585 -> 557, 5472x3648 534 -> 530.
            // Narrower bands lost or tied (u16 4000x3000 557 -> 612 us, f32
            // 3000^2 1099 -> 1428), and u8 gained only at exactly 6 tiles in
            // 2-tile segments, so those keep direct stores.
            const uint32_t mis_seg = mis_seg_env > 0 ? uint32_t(mis_seg_env) : 4u;
            const uint32_t nseg = (p.units_x + mis_seg - 1) / mis_seg;
            seg_tiles = (p.units_x + nseg - 1) / nseg;
            band_waves = seg_tiles;
            p.seg_rowwise = 1;
            // these segments are stored by their last two waves when level
            // 1's rows split bursts: u16 6000x4000 556 -> 543 us, 5472x3648
            // 535 -> 523, 4100^2 597 -> 582, f32 6000x4000 1085 -> 1045,
            // 4100^2 1074 -> 1060; but f32 5472x3648 (level 1 whole bursts)
            // 1087 -> 1117, so it keeps one (same box, two rounds,
            // profiles/r04/misseg/).  Whole misaligned bands of <= 6 tiles
            // keep one too (3000^2 548-550 -> 600 us with two).
            if (band_last_env < 0)
                p.band_last = (stage_mask & 1u) ? 2u : 1u;
        }
        const uint32_t lds = band_lds_bytes(sizeof(T), outs, n_out, stage_mask,
                                            seg_tiles * 64u * cols, p.seg_rowwise != 0);
        const bool band = stage_mask && !band_off &&
                          band_waves <= wide_max && lds <= band_lds_cap() &&
                          total < (1ull << 31);
        const uint32_t segs = seg_tiles ? (p.units_x + seg_tiles - 1) / seg_tiles : 1u;
        const uint32_t bands = p.units_y * n_frames * segs;
        // Direct stores of rows that split 64-B bursts, bands wider than the
        // staged form takes: one workgroup per band (or per balanced piece
        // of <= 8 tiles), so a burst shared by neighbouring waves is written
        // through one L2.  3000^2 622 -> 576 us, 2600^2 601 -> 540 us,
        // 5472x3648 571 -> 540 us against 4-wave blocks that straddle bands
        // (profiles/r03/misaligned/); $AQZ_BAND_WG=0: off.
        static const bool band_wg = int_env("AQZ_BAND_WG", 1) != 0;
        uint32_t wpb_run = wpb;
        uint32_t grid_run = grid;
        if (!band && band_wg && stage_mask && !band_force && p.order == 0 && p.units_x > 4) {
            const uint32_t nseg = (p.units_x + 7) / 8;
            p.seg_w = (p.units_x + nseg - 1) / nseg;
            wpb_run = p.seg_w;
            grid_run = nseg * p.units_y * n_frames;
            p.main_blocks = grid_run;
        }
        return with_method(method, [&](auto mtag) -> hipError_t {
            constexpr int M = decltype(mtag)::value;
            auto go = [&](auto ctag, auto nttag) {
                constexpr int C = decltype(ctag)::value;
                constexpr bool NT = decltype(nttag)::value;
                if (band) {
                    const dim3 blk(64 * band_waves);
                    auto launch_band = [&](auto rtag, auto stag) {
                        constexpr bool RW = decltype(rtag)::value;
                        constexpr bool SP = decltype(stag)::value;
                        auto one = [&](auto ltag) {
                            constexpr int NLV = decltype(ltag)::value;
                            if (lds > 65536) // above the default per-workgroup LDS
                                (void)hipFuncSetAttribute(
                                  reinterpret_cast<const void*>(
                                    &cascade_band_kernel<T, M, NLV, C, NT, RW, SP>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
                            hipLaunchKernelGGL((cascade_band_kernel<T, M, NLV, C, NT, RW, SP>),
                                               dim3(bands), blk, lds, stream, p, stage_mask,
                                               seg_tiles);
                        };
                        switch (n_out) {
                            case 1: one(std::integral_constant<int, 1>{}); break;
                            case 2: one(std::integral_constant<int, 2>{}); break;
                            case 3: one(std::integral_constant<int, 3>{}); break;
                            default: one(std::integral_constant<int, 4>{}); break;
                        }
                    };
                    // misaligned segments: a separate instantiation, so that
                    // whole bands keep their code (a runtime branch per row
                    // cost 3000^2 / 2600^2 u16 8-9%), for 2- and 4-byte types
                    // at the wide tile only (where the launcher picks them)
                    if constexpr ((sizeof(T) == 2 || sizeof(T) == 4) &&
                                  (C == int(CW) || (sizeof(T) == 4 && C == int(CN)))) {
                        if (p.seg_rowwise) {
                            launch_band(std::true_type{}, std::false_type{});
                            return;
                        }
                    }
                    // whole-line loads for 4- and 8-byte types at the wide
                    // tile (cascade_unit SPLIT); $AQZ_SPLIT_LOADS=0 / 1 (A/B)
                    if constexpr (sizeof(T) >= 4 && C == int(CW)) {
                        if (split_loads()) {
                            launch_band(std::false_type{}, std::true_type{});
                            return;
                        }
                    }
                    launch_band(std::false_type{}, std::false_type{});
                    return;
                }
                switch (n_out) {
                    case 1:
                        hipLaunchKernelGGL((cascade_kernel<T, M, 1, C, NT>), dim3(grid_run), dim3(64 * wpb_run),
                                           0, stream, p);
                        break;
                    case 2:
                        hipLaunchKernelGGL((cascade_kernel<T, M, 2, C, NT>), dim3(grid_run), dim3(64 * wpb_run),
                                           0, stream, p);
                        break;
                    case 3:
                        hipLaunchKernelGGL((cascade_kernel<T, M, 3, C, NT>), dim3(grid_run), dim3(64 * wpb_run),
                                           0, stream, p);
                        break;
                    default:
                        hipLaunchKernelGGL((cascade_kernel<T, M, 4, C, NT>), dim3(grid_run), dim3(64 * wpb_run),
                                           0, stream, p);
                        break;
                }
            };
            auto go_c = [&](auto nttag) {
                if (cols == CW)
                    go(std::integral_constant<int, int(CW)>{}, nttag);
                else
                    go(std::integral_constant<int, int(CN)>{}, nttag);
            };
            if (p.nt)
                go_c(std::true_type{});
            else
                go_c(std::false_type{});
            return hipGetLastError();
        });
    });
}

#if AQZ_SHARD == 0

uint32_t
cascade_tiled_cols(int dtype, uint32_t W)
{
    // cascade_pick_cols for element-aligned buffers: wide tiles once a wave's
    // 64 lanes fit in the frame, half-width ones below
    const size_t b = dtype_bytes(dtype);
    if (!b)
        return 0;
    const uint32_t cw = cascade_cols(b);
    // $AQZ_TILED_NARROW (A/B): 1 half-width tiles wherever they fit, 0 wide;
    // unset: half-width for 4- and 8-byte types on rows whose levels are
    // whole bursts (narrow_rows), as cascade_pick_cols (the streaming path writes a run tiled in one launch
    // only when both agree): chunk-tiled 4096^2 f32 964-979 against
    // 995-1033 us wide; 5472x3648, 6000x4000 and 2000^2 keep wide tiles
    // (1113 / 990 / 1031 against 1129 / 1074 / 1055 us narrow;
    // profiles/r05/narrow/ab_shapes.log)
    static const int narrow = int_env("AQZ_TILED_NARROW", -1);
    if ((narrow == 1 || (narrow < 0 && narrow_rows(b, W))) &&
        W >= 64 * (cw / 2))
        return cw / 2;
    return W >= 64 * cw ? cw : cw / 2;
}

uint32_t
cascade_tiled_slots(int dtype,
                    uint32_t W,
                    int n_out,
                    int level,
                    uint32_t tile_rows,
                    uint32_t tile_cols,
                    uint32_t* slots_x)
{
    const uint32_t cols = cascade_tiled_cols(dtype, W);
    const uint32_t cw = (64u * cols) >> level;       // level columns per wave block
    const uint32_t rh = (1u << n_out) >> level;      // level rows per wave block
    const uint32_t co = std::max(1u, cols >> level); // columns per lane store
    if (slots_x)
        *slots_x = 1;
    if (cols == 0 || level < 1 || level > n_out || tile_rows == 0 || tile_cols == 0 ||
        tile_rows % rh != 0)
        return 0;
    // blocks inside tiles: one slot per block; blocks spanning whole tiles
    // (and lane stores inside one tile): one slot per (tile, block row)
    uint32_t sx = 0;
    if (tile_cols % cw == 0)
        sx = tile_cols / cw;
    else if (cw % tile_cols == 0 && tile_cols % co == 0)
        sx = 1;
    if (sx == 0)
        return 0;
    if (slots_x)
        *slots_x = sx;
    return (tile_rows / rh) * sx;
}
#endif

hipError_t
AQZ_SHARDED(launch_cascade_tiled)(int dtype,
                                  int method,
                                  const void* src,
                                  uint64_t src_frame_elems,
                                  uint32_t W,
                                  uint32_t H,
                                  const LevelOut* outs,
                                  const TiledOut* touts,
                                  int n_out,
                                  uint32_t n_frames,
                                  hipStream_t stream)
{
    // the flag layout (cascade_tiled_slots) assumes the geometry-only choice;
    // cascade_pick_cols != 0 says the buffers and level sizes fit the fused
    // cascade (its conditions do not depend on the tile width)
    const uint32_t cols = cascade_tiled_cols(dtype, W);
    const size_t b = dtype_bytes(dtype);
    if (cols == 0 || n_frames == 0 ||
        cascade_pick_cols(dtype, src, src_frame_elems, W, H, outs, n_out) == 0)
        return hipErrorInvalidValue;
    const uint32_t R = 1u << n_out;
    CascadeParams p{};
    p.src = static_cast<const uint8_t*>(src);
    p.src_frame_elems = src_frame_elems;
    p.W = W;
    p.H = H;
    // The grid's blocks cover the frame; zero-fill waves cover the rest of
    // the padded tile area.
    p.units_x = (W + 64 * cols - 1) / (64 * cols);
    p.units_y = (H + R - 1) / R;
    const uint64_t total = uint64_t(p.units_x) * p.units_y * n_frames;
    if (total >= (1ull << 30))
        return hipErrorInvalidValue;
    p.total_units = uint32_t(total);
    bool flag_fill = false;
    bool nested = true; // every level's wave blocks and tiles nest: mode 1
    for (int i = 0; i < n_out; ++i) {
        const TiledOut& t = touts[i];
        if (!t.ptr || t.tile_rows == 0 || t.tile_cols == 0 ||
            reinterpret_cast<uintptr_t>(t.ptr) % b != 0)
            return hipErrorInvalidValue;
        const uint32_t ntx = (outs[i].w + t.tile_cols - 1) / t.tile_cols;
        const uint32_t nty = (outs[i].h + t.tile_rows - 1) / t.tile_rows;
        const uint64_t pw = uint64_t(ntx) * t.tile_cols, ph = uint64_t(nty) * t.tile_rows;
        if (pw >= (1ull << 31) || ph >= (1ull << 31))
            return hipErrorInvalidValue;
        p.dst[i] = static_cast<uint8_t*>(outs[i].ptr);
        p.dst_frame_elems[i] = outs[i].frame_elems;
        p.w[i] = outs[i].w;
        p.h[i] = outs[i].h;
        TiledLevel& q = p.tl[i];
        q.tdst = static_cast<uint8_t*>(t.ptr);
        q.tframe_elems = pw * ph;
        q.foff = t.frame_offsets;
        q.tstride = t.frame_offsets ? t.tile_stride : uint64_t(t.tile_rows) * t.tile_cols;
        if (q.tstride < uint64_t(t.tile_rows) * t.tile_cols)
            return hipErrorInvalidValue;
        q.tr = t.tile_rows;
        q.tc = t.tile_cols;
        q.dr = FastDiv::make(t.tile_rows);
        q.dc = FastDiv::make(t.tile_cols);
        q.ntx = ntx;
        q.pw = uint32_t(pw);
        q.ph = uint32_t(ph);
        q.cov_w = p.units_x * ((64u * cols) >> (i + 1));
        q.cov_h = p.units_y * (R >> (i + 1));
        q.zrows = q.cov_w < pw ? uint32_t(ph) : (q.cov_h < ph ? uint32_t(ph) - q.cov_h : 0u);
        p.zitems += q.zrows;
        q.slots = cascade_tiled_slots(dtype, W, n_out, i + 1, t.tile_rows, t.tile_cols,
                                      &q.slots_x);
        if (!q.slots)
            nested = false;
        q.flags = t.nonzero;
        q.flags_frame = ntx * nty * std::max<uint32_t>(1, q.slots);
        if (t.nonzero && q.slots && (q.cov_w < pw || q.cov_h < ph))
            flag_fill = true;
        if (t.nonzero && !q.slots) {
            // one flag per tile, OR-ed by plain stores of 1: cleared first
            const hipError_t e =
              hipMemsetAsync(t.nonzero, 0, size_t(n_frames) * ntx * nty, stream);
            if (e != hipSuccess)
                return e;
        }
    }
    // zero-fill waves: a whole number of 8-block (one per XCD) groups
    const uint64_t zitems = uint64_t(p.zitems) * n_frames;
    if (zitems >= (1ull << 32))
        return hipErrorInvalidValue;
    p.zdiv = FastDiv::make(p.zitems ? p.zitems : 1);
    // One zero-fill wave per 128 KiB of overhang (64..4096).  The waves run
    // first and hold their slots while the cascade blocks start; one per
    // item (up to 4096) cost 4-5% at 3000^2 and 5472x3648 against 512, and
    // putting them after the cascade blocks made them the kernel's tail
    // (profiles/r02/tiled_zero_fill_ab.log).
    uint64_t zbytes = 0;
    for (int i = 0; i < n_out; ++i) {
        const TiledLevel& q = p.tl[i];
        const uint64_t cw = std::min(q.cov_w, q.pw), chh = std::min(q.cov_h, q.ph);
        zbytes += (uint64_t(q.pw) * q.ph - cw * chh) * b;
    }
    zbytes *= n_frames;
    // ... and for 1-byte types at most ZI = 32 overhang rows per wave: each
    // row is a short dependent loop, and the byte rule left u8 pyramids
    // (chunk 128, rows of a few dozen bytes) with thousands of rows per
    // wave, the kernel's tail.  Same box (profiles/r04/zrows/ab.log): u8
    // 2600^2 262 -> 111 us, 2304^2 273 -> 131, 1500^2 189 -> 113, 3000^2
    // 141 -> 93, 5000x4000 100 -> 81; the same cap cost u16 2-4% (3000^2
    // 516-519 -> 528-531 us), so wider types keep the byte rule.
    // $AQZ_TILED_ZROWS_PER_WAVE: ZI for every type (0: the byte rule alone).
    static const int zi_env = int_env("AQZ_TILED_ZROWS_PER_WAVE", -1);
    const int zi = zi_env >= 0 ? zi_env : (b == 1 ? 32 : 0);
    uint64_t zw = (zbytes >> 17) + 1;
    if (zi > 0)
        zw = std::max<uint64_t>(zw, (zitems + zi - 1) / uint64_t(zi));
    p.zwaves = (zitems || flag_fill)
                 ? uint32_t(std::min<uint64_t>(std::max<uint64_t>(zw, 64), 4096))
                 : 0u;
    if (const int zw = tiled_zwaves_env(); zw >= 0)
        p.zwaves = uint32_t(zw); // A/B only: 0 leaves the overhang unwritten
    p.remap = xcd_remap_env() == 1;
    // Nontemporal loads on aligned rows for every unit size: with the data
    // in HBM (rotating buffer sets) chunk-tiled 2048^2
    // u16 Decimate runs 73.8-73.9 us with them against 79.0-79.7 plain, and
    // 512^2 u8 Decimate / Mean 73.1-73.5 / 82.6-82.7 against 74.1 / 83.4-
    // 84.8.  (A round-5 plain-load rule for units of <= 4 KiB had been timed
    // with the read set resident in the Infinity Cache.)
    p.nt = load_nt(W, b);
    // $AQZ_TILED_BAND_WG=1 (A/B, off by default): on rows that split 128-B
    // lines, one workgroup per row band (or balanced piece of <= 8 tiles), as
    // the row-major launcher does, so that the two waves sharing a line read
    // it through one L2.  Reads drop to 1.00-1.01x the frame (from 1.02-1.05x)
    // but every shape got slower: u16 3000^2 543 -> 615 us, 5472x3648 517 ->
    // 610, 6000x4000 503 -> 597, 2000^2 507 -> 511, f32 6000x4000 990 -> 1111
    // (same box, two rounds, profiles/r04/tiledwg/).
    static const bool band_wg = int_env("AQZ_TILED_BAND_WG", 0) != 0;
    uint32_t wpb = 4;
    if (band_wg && !p.remap && (uint64_t(W) * b) % 128 != 0 && p.units_x > 1) {
        const uint32_t nseg = (p.units_x + 7) / 8;
        p.seg_w = (p.units_x + nseg - 1) / nseg;
        wpb = p.seg_w;
        p.main_blocks = nseg * p.units_y * n_frames;
    } else {
        // Waves per workgroup: 4 when a row band's tile count divides by 4,
        // else 2.  Same box, two rounds (profiles/r04/tiledwaves/): u16
        // 3000^2 541-549 -> 518-521 us, 2304^2 614-621 -> 576-577, 3500^2
        // 552 -> 519, 4600x3000 531 -> 510, f32 5472x3648 1191-1193 -> 1116-
        // 1118, u8 6000x4000 89-96 -> 80-85; but 2-wave blocks lose where 4
        // divide the band (u16 2000^2 505 -> 580, 6000x4000 505 -> 546-550,
        // f32 6000x4000 989 -> 1063), and 3-wave blocks lose on 6 tiles
        // (3000^2 574-576).  $AQZ_TILED_WAVES (1..8) forces a count (A/B).
        static const int tw = int_env("AQZ_TILED_WAVES", 0);
        wpb = tw > 0 ? uint32_t(std::min(tw, 8)) : (p.units_x % 4 == 0 ? 4u : 2u);
        p.main_blocks = grid_for(total, wpb, 0);
    }
    // zero-fill blocks: a whole number of 8-block (one per XCD) groups
    const uint32_t zblocks = ((p.zwaves + wpb - 1) / wpb + 7) & ~7u;
    p.zwaves = zblocks * wpb;
    const uint32_t grid = zblocks + p.main_blocks;

    return with_dtype(dtype, [&](auto tag) -> hipError_t {
        using T = decltype(tag);
        constexpr uint32_t CW = kCascadeCols<T>;
        constexpr uint32_t CN = CW / 2;
        return with_method(method, [&](auto mtag) -> hipError_t {
            constexpr int M = decltype(mtag)::value;
            auto go_m = [&](auto ctag, auto nttag, auto mdtag) {
                constexpr int C = decltype(ctag)::value;
                constexpr bool NT = decltype(nttag)::value;
                constexpr int MD = decltype(mdtag)::value;
                switch (n_out) {
                    case 1:
                        hipLaunchKernelGGL((cascade_kernel<T, M, 1, C, NT, MD>), dim3(grid),
                                           dim3(64 * wpb), 0, stream, p);
                        break;
                    case 2:
                        hipLaunchKernelGGL((cascade_kernel<T, M, 2, C, NT, MD>), dim3(grid),
                                           dim3(64 * wpb), 0, stream, p);
                        break;
                    case 3:
                        hipLaunchKernelGGL((cascade_kernel<T, M, 3, C, NT, MD>), dim3(grid),
                                           dim3(64 * wpb), 0, stream, p);
                        break;
                    default:
                        hipLaunchKernelGGL((cascade_kernel<T, M, 4, C, NT, MD>), dim3(grid),
                                           dim3(64 * wpb), 0, stream, p);
                        break;
                }
            };
            auto go = [&](auto ctag, auto nttag) {
                if (nested)
                    go_m(ctag, nttag, std::integral_constant<int, 1>{});
                else
                    go_m(ctag, nttag, std::integral_constant<int, 2>{});
            };
            auto go_c = [&](auto nttag) {
                if (cols == CW)
                    go(std::integral_constant<int, int(CW)>{}, nttag);
                else
                    go(std::integral_constant<int, int(CN)>{}, nttag);
            };
            if (p.nt)
                go_c(std::true_type{});
            else
                go_c(std::false_type{});
            return hipGetLastError();
        });
    });
}
#if AQZ_SHARD == 0

bool
volume_supported(int dtype,
                 const void* src,
                 uint32_t W,
                 uint32_t H,
                 const LevelOut* outs,
                 int n_out)
{
    return n_out >= 1 && n_out <= kMaxVolumeLevels &&
           cascade_fits(dtype_bytes(dtype), src, uint64_t(W) * H, W, H, outs, n_out,
                        cascade_cols(dtype_bytes(dtype)));
}
#endif

hipError_t
AQZ_SHARDED(launch_volume)(int dtype,
              int method,
              const void* src,
              uint64_t src_frame_elems,
              uint32_t W,
              uint32_t H,
              const LevelOut* outs,
              int n_out,
              uint32_t n_planes,
              hipStream_t stream)
{
    if (!volume_supported(dtype, src, W, H, outs, n_out) || n_planes == 0 ||
        n_planes % (1u << n_out) != 0)
        return hipErrorInvalidValue;
    return with_dtype(dtype, [&](auto tag) -> hipError_t {
        using T = decltype(tag);
        constexpr uint32_t C = 16 / sizeof(T);
        VolumeParams p{};
        p.src = static_cast<const uint8_t*>(src);
        p.src_frame_elems = src_frame_elems;
        p.W = W;
        p.H = H;
        const uint32_t R = 1u << n_out;
        p.units_x = (W + 64 * C - 1) / (64 * C);
        p.units_y = (H + R - 1) / R;
        const uint64_t total =
          uint64_t(p.units_x) * p.units_y * (n_planes >> n_out);
        if (total >= (1ull << 31))
            return hipErrorInvalidValue;
        p.total_units = uint32_t(total);
        for (int i = 0; i < n_out; ++i) {
            p.dst[i] = static_cast<uint8_t*>(outs[i].ptr);
            p.dst_frame_elems[i] = outs[i].frame_elems;
            p.w[i] = outs[i].w;
            p.h[i] = outs[i].h;
        }
        // Load policy and units per wave: with the
        // volume in HBM (rotating buffer sets) nontemporal loads beat plain
        // ones for every method, Decimate's every-other-row, every-other-
        // plane reads included (44.0-44.4 against 46.7-47.4 us); Decimate's
        // 4-KiB units go two to a wave (one ties).  The plain-load choice of
        // §11.2 had been timed with Decimate's 128 MiB read set resident in
        // the Infinity Cache.  $AQZ_VOLUME_NT=0/1 and $AQZ_VOLUME_UPW=1/2
        // (Decimate) override.
        static const int nt_env = int_env("AQZ_VOLUME_NT", -1);
        static const int upw_env = int_env("AQZ_VOLUME_UPW", 0);
        return with_method(method, [&](auto mtag) -> hipError_t {
            constexpr int M = decltype(mtag)::value;
            const bool ntl = nt_env >= 0 ? nt_env != 0 : true;
            // $AQZ_VOLUME_UPW=4 (A/B, Decimate, nontemporal loads): four
            // units per wave, 16 KiB of loads in flight per wave
            const int upw = M == kDecimate ? (upw_env >= 4 ? 4 : upw_env > 0 ? std::min(upw_env, 2) : 2)
                                           : 1;
            const uint32_t grid = grid_for((total + upw - 1) / upw, 4, 0);
#define AQZ_VOL(NL, NTL, UPW)                                                          \
    hipLaunchKernelGGL((volume_kernel<T, M, NL, NTL, UPW>), dim3(grid), dim3(256), 0, \
                       stream, p)
            // Decimate launches of 128 or more plane groups (two or more
            // config-V volumes) take the plane groups fastest in the unit
            // order, so the units in flight spread over many planes: four
            // 1024^2 x 256 volumes 172.1-172.3 -> 148.1-149.0 us, data in HBM
            // (profiles/r05/vzfast/ab.log); one volume (64 groups) loses
            // 1-2% that way and keeps columns fastest.  Its reads never set
            // the address bits of odd rows and odd planes.
            // $AQZ_VOLUME_ZFAST=0 / 1: never / always (nontemporal loads).
            static const int zf_env = int_env("AQZ_VOLUME_ZFAST", -1);
            const bool zfast = zf_env >= 0 ? zf_env != 0 : (n_planes >> n_out) >= 128;
            if constexpr (M == kDecimate) {
                if (upw == 4 && ntl) {
                    constexpr int CZ = 16 / int(sizeof(T));
                    if (zfast && n_out == 1)
                        hipLaunchKernelGGL((volume_kernel<T, M, 1, true, 4, CZ, true>), dim3(grid),
                                           dim3(256), 0, stream, p);
                    else if (zfast)
                        hipLaunchKernelGGL((volume_kernel<T, M, 2, true, 4, CZ, true>), dim3(grid),
                                           dim3(256), 0, stream, p);
                    else if (n_out == 1)
                        AQZ_VOL(1, true, 4);
                    else
                        AQZ_VOL(2, true, 4);
                    return hipGetLastError();
                }
                if (upw == 2 && zfast && ntl) {
                    constexpr int CZ = 16 / int(sizeof(T));
                    if (n_out == 1)
                        hipLaunchKernelGGL((volume_kernel<T, M, 1, true, 2, CZ, true>), dim3(grid),
                                           dim3(256), 0, stream, p);
                    else
                        hipLaunchKernelGGL((volume_kernel<T, M, 2, true, 2, CZ, true>), dim3(grid),
                                           dim3(256), 0, stream, p);
                    return hipGetLastError();
                }
                if (upw == 2) {
                    if (n_out == 1 && ntl)
                        AQZ_VOL(1, true, 2);
                    else if (n_out == 1)
                        AQZ_VOL(1, false, 2);
                    else if (ntl)
                        AQZ_VOL(2, true, 2);
                    else
                        AQZ_VOL(2, false, 2);
                    return hipGetLastError();
                }
            }
            if (n_out == 1 && ntl)
                AQZ_VOL(1, true, 1);
            else if (n_out == 1)
                AQZ_VOL(1, false, 1);
            else if (ntl)
                AQZ_VOL(2, true, 1);
            else
                AQZ_VOL(2, false, 1);
#undef AQZ_VOL
            return hipGetLastError();
        });
    });
}
#if AQZ_SHARD == 0

uint32_t
tile_slices(uint32_t tile_rows, uint32_t tile_cols)
{
    // ~8 K elements per block, at most 64 blocks per tile
    const uint64_t tile_elems = uint64_t(tile_rows) * tile_cols;
    return uint32_t(std::min<uint64_t>(64, std::max<uint64_t>(1, tile_elems / 8192)));
}
#endif

namespace {

hipError_t
launch_tile_impl(int dtype,
                 const void* src,
                 uint32_t W,
                 uint32_t H,
                 uint32_t tile_rows,
                 uint32_t tile_cols,
                 void* dst,
                 void* flags,
                 bool slice_flags,
                 hipStream_t stream)
{
    if (W == 0 || H == 0 || tile_rows == 0 || tile_cols == 0 ||
        uint64_t(tile_rows) * tile_cols >= (1ull << 31))
        return hipErrorInvalidValue;
    const uint32_t ntx = (W + tile_cols - 1) / tile_cols;
    const uint32_t nty = (H + tile_rows - 1) / tile_rows;
    const uint32_t slices = tile_slices(tile_rows, tile_cols);
    const uint64_t blocks = uint64_t(ntx) * nty * slices;
    if (blocks >= (1ull << 31))
        return hipErrorInvalidValue;
    if (!slice_flags) {
        hipError_t e = hipMemsetAsync(flags, 0, sizeof(uint32_t) * ntx * nty, stream);
        if (e != hipSuccess)
            return e;
    }
    const size_t bpp = dtype_bytes(dtype);
    if ((uint64_t(W) * bpp) % 16 == 0 && (uint64_t(tile_cols) * bpp) % 16 == 0 &&
        reinterpret_cast<uintptr_t>(src) % 16 == 0 &&
        reinterpret_cast<uintptr_t>(dst) % 16 == 0) {
        const uint32_t rv = uint32_t(uint64_t(W) * bpp / 16);
        const uint32_t tv = uint32_t(uint64_t(tile_cols) * bpp / 16);
        const auto* s16 = static_cast<const u32x4*>(src);
        auto* d16 = static_cast<u32x4*>(dst);
        if (slice_flags)
            hipLaunchKernelGGL((tile_kernel_vec<true>), dim3(uint32_t(blocks)), dim3(256), 0,
                               stream, s16, rv, H, tile_rows, tv, ntx, slices, d16, flags);
        else
            hipLaunchKernelGGL((tile_kernel_vec<false>), dim3(uint32_t(blocks)), dim3(256), 0,
                               stream, s16, rv, H, tile_rows, tv, ntx, slices, d16, flags);
        return hipGetLastError();
    }
    return with_dtype(dtype, [&](auto tag) -> hipError_t {
        using T = decltype(tag);
        if (slice_flags)
            hipLaunchKernelGGL((tile_kernel<T, true>), dim3(uint32_t(blocks)), dim3(256),
                               0, stream, static_cast<const T*>(src), W, H, tile_rows,
                               tile_cols, ntx, slices, static_cast<T*>(dst), flags);
        else
            hipLaunchKernelGGL((tile_kernel<T, false>), dim3(uint32_t(blocks)), dim3(256),
                               0, stream, static_cast<const T*>(src), W, H, tile_rows,
                               tile_cols, ntx, slices, static_cast<T*>(dst), flags);
        return hipGetLastError();
    });
}

} // namespace

hipError_t
AQZ_SHARDED(launch_tile_frame)(int dtype,
                  const void* src,
                  uint32_t W,
                  uint32_t H,
                  uint32_t tile_rows,
                  uint32_t tile_cols,
                  void* dst,
                  uint32_t* nonzero,
                  hipStream_t stream)
{
    return launch_tile_impl(dtype, src, W, H, tile_rows, tile_cols, dst, nonzero,
                            false, stream);
}

hipError_t
AQZ_SHARDED(launch_tile_frame_sliced)(int dtype,
                         const void* src,
                         uint32_t W,
                         uint32_t H,
                         uint32_t tile_rows,
                         uint32_t tile_cols,
                         void* dst,
                         uint8_t* slice_flags,
                         hipStream_t stream)
{
    return launch_tile_impl(dtype, src, W, H, tile_rows, tile_cols, dst, slice_flags,
                            true, stream);
}

hipError_t
AQZ_SHARDED(launch_transpose)(int dtype,
                 const void* src,
                 uint32_t rows,
                 uint32_t cols,
                 void* dst,
                 hipStream_t stream)
{
    if (rows == 0 || cols == 0)
        return hipErrorInvalidValue;
    return with_dtype(dtype, [&](auto tag) -> hipError_t {
        using T = decltype(tag);
        constexpr uint32_t TD = kTransposeTile<T>;
        constexpr uint32_t TR = TD * kTransposeSub<T>; // source rows per block
        const uint32_t bx = (cols + TD - 1) / TD;
        const uint32_t by = (rows + TR - 1) / TR;
        if (by > 65535)
            return hipErrorInvalidValue;
        // 16-B vectors need 16-B aligned bases and row pitches on both sides
        const bool vec = (reinterpret_cast<uintptr_t>(src) % 16) == 0 &&
                         (reinterpret_cast<uintptr_t>(dst) % 16) == 0 &&
                         (uint64_t(cols) * sizeof(T)) % 16 == 0 &&
                         (uint64_t(rows) * sizeof(T)) % 16 == 0;
        if (vec)
            hipLaunchKernelGGL((transpose_kernel<T, true>), dim3(bx, by), dim3(256), 0,
                               stream, static_cast<const T*>(src), rows, cols,
                               static_cast<T*>(dst));
        else
            hipLaunchKernelGGL((transpose_kernel<T, false>), dim3(bx, by), dim3(256), 0,
                               stream, static_cast<const T*>(src), rows, cols,
                               static_cast<T*>(dst));
        return hipGetLastError();
    });
}

hipError_t
AQZ_SHARDED(launch_xy_generic)(int dtype,
                  int method,
                  const void* src,
                  uint64_t src_frame_elems,
                  uint32_t w,
                  uint32_t h,
                  const LevelOut& out,
                  uint32_t n_frames,
                  hipStream_t stream)
{
    if (w == 0 || h == 0 || n_frames == 0)
        return hipErrorInvalidValue;
    if (out.w != (w + 1) / 2 || out.h != (h + 1) / 2)
        return hipErrorInvalidValue;
    const uint64_t total = uint64_t(out.w) * out.h * n_frames;
    const uint32_t grid = grid_for(total, 256, 8192);
    return with_dtype(dtype, [&](auto tag) -> hipError_t {
        using T = decltype(tag);
        return with_method(method, [&](auto mtag) -> hipError_t {
            constexpr int M = decltype(mtag)::value;
            hipLaunchKernelGGL((xy_generic_kernel<T, M>),
                               dim3(grid), dim3(256), 0, stream,
                               static_cast<const T*>(src), src_frame_elems, w,
                               h, static_cast<T*>(out.ptr), out.frame_elems,
                               out.w, out.h, total);
            return hipGetLastError();
        });
    });
}

hipError_t
AQZ_SHARDED(launch_zpair)(int dtype,
             int method,
             void* out,
             const void* earlier,
             const void* current,
             uint64_t n,
             hipStream_t stream)
{
    if (n == 0)
        return hipSuccess;
    const size_t b = dtype_bytes(dtype);
    if (!b)
        return hipErrorInvalidValue;
    // batch slots of odd-sized levels need not be 16-byte aligned
    const bool vec = ((reinterpret_cast<uintptr_t>(out) |
                       reinterpret_cast<uintptr_t>(earlier) |
                       reinterpret_cast<uintptr_t>(current)) %
                      16) == 0;
    const uint64_t items = vec ? (n * b + 15) / 16 : n;
    const uint32_t grid = grid_for(items, 256, 8192);
    return with_dtype(dtype, [&](auto tag) -> hipError_t {
        using T = decltype(tag);
        return with_method(method, [&](auto mtag) -> hipError_t {
            constexpr int M = decltype(mtag)::value;
            if (vec)
                hipLaunchKernelGGL((zpair_kernel<T, M, true>), dim3(grid),
                                   dim3(256), 0, stream, static_cast<T*>(out),
                                   static_cast<const T*>(earlier),
                                   static_cast<const T*>(current), n);
            else
                hipLaunchKernelGGL((zpair_kernel<T, M, false>), dim3(grid),
                                   dim3(256), 0, stream, static_cast<T*>(out),
                                   static_cast<const T*>(earlier),
                                   static_cast<const T*>(current), n);
            return hipGetLastError();
        });
    });
}

} // namespace aqz
