// volume_probe.hip — A/B of the volume Decimate access shape (measurement
// aid, not product code).
//
// BASELINE config V: 1024 x 1024 x 256 u16, 2 x 2 x 2 Decimate, 3 levels.
// Decimate keeps the top-left pixel of the earlier plane, so level 1 is
// src[2z][2r][2c] and level 2 src[4z][4r][4c]: a wave unit of 4 planes x 4
// rows x (64 * C) columns reads rows 0 and 2 of planes 0 and 2 only.  The
// library's volume_kernel runs one unit per wave with C = 8 (one 16-B load
// per row per lane): 4 KiB read per wave.  Variants here:
//   UPW  units per wave, every load of every unit issued before any store;
//   C    columns per lane (8: one 16-B load per row, 16: two);
//   ZF   unit order with the plane group fastest (else columns, rows, groups);
//   NT   nontemporal loads.
// Frames must tile exactly (W % (64 C) == 0, H % 4 == 0, planes % 4 == 0):
// the probe has no edge path.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

template<bool NT>
__device__ __forceinline__ u32x4
ld16(const uint16_t* p)
{
    const u32x4* q = reinterpret_cast<const u32x4*>(p);
    if constexpr (NT)
        return __builtin_nontemporal_load(q);
    else
        return *q;
}

// even u16 elements of a 16-B vector (elements 0, 2, 4, 6) -> 8 B
__device__ __forceinline__ uint64_t
even4(u32x4 v)
{
    const uint32_t a = (v.x & 0xFFFFu) | (v.y << 16);
    const uint32_t b = (v.z & 0xFFFFu) | (v.w << 16);
    return uint64_t(a) | (uint64_t(b) << 32);
}

// elements 0 and 4 of a 16-B vector -> 4 B
__device__ __forceinline__ uint32_t
every4(u32x4 v)
{
    return (v.x & 0xFFFFu) | (v.z << 16);
}

struct Geo
{
    const uint16_t* src;
    uint16_t* d1;
    uint16_t* d2;
    uint32_t W, H;
    uint32_t units_x, units_y, groups, total;
};

template<int UPW, int C, bool ZF, bool NT>
__global__ __launch_bounds__(256) void
vol_decimate(Geo g)
{
    constexpr int V = C / 8; // 16-B loads per row per lane
    const int lane = threadIdx.x & 63;
    const uint32_t wave = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t plane = uint64_t(g.W) * g.H;
    const uint32_t w1 = g.W / 2, h1 = g.H / 2, w2 = g.W / 4, h2 = g.H / 4;
    u32x4 v[UPW][2][2][V];
    uint32_t gz[UPW], uy[UPW], ux[UPW];
    bool ok[UPW];
#pragma unroll
    for (int i = 0; i < UPW; ++i) {
        const uint32_t u = wave * UPW + i;
        ok[i] = u < g.total;
        const uint32_t uu = ok[i] ? u : 0;
        if constexpr (ZF) {
            gz[i] = uu % g.groups;
            const uint32_t t = uu / g.groups;
            ux[i] = t % g.units_x;
            uy[i] = t / g.units_x;
        } else {
            ux[i] = uu % g.units_x;
            const uint32_t t = uu / g.units_x;
            uy[i] = t % g.units_y;
            gz[i] = t / g.units_y;
        }
        const uint32_t col0 = ux[i] * 64u * C + uint32_t(lane) * C;
#pragma unroll
        for (int zz = 0; zz < 2; ++zz)
#pragma unroll
            for (int rr = 0; rr < 2; ++rr) {
                const uint16_t* row = g.src + (uint64_t(gz[i]) * 4 + 2 * zz) * plane +
                                      uint64_t(uy[i] * 4 + 2 * rr) * g.W + col0;
#pragma unroll
                for (int k = 0; k < V; ++k)
                    v[i][zz][rr][k] = ld16<NT>(row + 8 * k);
            }
    }
#pragma unroll
    for (int i = 0; i < UPW; ++i) {
        if (!ok[i])
            continue;
        const uint32_t c1 = (ux[i] * 64u * C + uint32_t(lane) * C) / 2;
#pragma unroll
        for (int zz = 0; zz < 2; ++zz)
#pragma unroll
            for (int rr = 0; rr < 2; ++rr) {
                uint16_t* dst = g.d1 + (uint64_t(gz[i]) * 2 + zz) * (uint64_t(w1) * h1) +
                                uint64_t(uy[i] * 2 + rr) * w1 + c1;
                if constexpr (V == 1) {
                    __builtin_nontemporal_store(even4(v[i][zz][rr][0]),
                                                reinterpret_cast<uint64_t*>(dst));
                } else {
                    u32x4 q;
                    const uint64_t a = even4(v[i][zz][rr][0]), b = even4(v[i][zz][rr][1]);
                    q.x = uint32_t(a);
                    q.y = uint32_t(a >> 32);
                    q.z = uint32_t(b);
                    q.w = uint32_t(b >> 32);
                    __builtin_nontemporal_store(q, reinterpret_cast<u32x4*>(dst));
                }
            }
        const uint32_t c2 = (ux[i] * 64u * C + uint32_t(lane) * C) / 4;
        uint16_t* dst2 = g.d2 + uint64_t(gz[i]) * (uint64_t(w2) * h2) + uint64_t(uy[i]) * w2 + c2;
        if constexpr (V == 1) {
            __builtin_nontemporal_store(every4(v[i][0][0][0]), reinterpret_cast<uint32_t*>(dst2));
        } else {
            u32x2 q;
            q.x = every4(v[i][0][0][0]);
            q.y = every4(v[i][0][0][1]);
            __builtin_nontemporal_store(q, reinterpret_cast<u32x2*>(dst2));
        }
    }
}

template<int UPW, int C, bool ZF, bool NT>
hipError_t
launch(Geo g, hipStream_t s)
{
    const uint32_t waves = (g.total + UPW - 1) / UPW;
    hipLaunchKernelGGL((vol_decimate<UPW, C, ZF, NT>), dim3((waves + 3) / 4), dim3(256), 0, s, g);
    return hipGetLastError();
}

} // namespace

// variant: upw in {1,2,4,8}, cols in {8,16}, zfast, nt.  Returns a hipError_t.
extern "C" int
aqz_volume_probe(const void* src, void* d1, void* d2, uint32_t W, uint32_t H, uint32_t planes,
                 int upw, int cols, int zfast, int nt, void* stream)
{
    if (!src || !d1 || !d2 || W % (64u * uint32_t(cols)) || H % 4 || planes % 4)
        return int(hipErrorInvalidValue);
    Geo g{ static_cast<const uint16_t*>(src), static_cast<uint16_t*>(d1),
           static_cast<uint16_t*>(d2), W, H, 0, 0, 0, 0 };
    g.units_x = W / (64u * uint32_t(cols));
    g.units_y = H / 4;
    g.groups = planes / 4;
    g.total = g.units_x * g.units_y * g.groups;
    const auto s = static_cast<hipStream_t>(stream);
#define AQZ_V(U, CC)                                                                   \
    if (upw == U && cols == CC) {                                                      \
        if (zfast && nt)                                                               \
            return int(launch<U, CC, true, true>(g, s));                               \
        if (zfast)                                                                     \
            return int(launch<U, CC, true, false>(g, s));                              \
        if (nt)                                                                        \
            return int(launch<U, CC, false, true>(g, s));                              \
        return int(launch<U, CC, false, false>(g, s));                                 \
    }
    AQZ_V(1, 8)
    AQZ_V(2, 8)
    AQZ_V(4, 8)
    AQZ_V(8, 8)
    AQZ_V(1, 16)
    AQZ_V(2, 16)
    AQZ_V(4, 16)
#undef AQZ_V
    return int(hipErrorInvalidValue);
}
