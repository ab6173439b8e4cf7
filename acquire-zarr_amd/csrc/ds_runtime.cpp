// ds_runtime.cpp — implementation of the C ABI in include/aqz_downsampler.h.
//
// Host orchestration of the per-frame pyramid on one MI355X:
//   * the level planner (restates downsampler.cpp:8-37, 493-597);
//   * the add_frame state machine (restates downsampler.cpp:306-401): level
//     cascade, Z pairing against the stored earlier plane, odd-plane
//     pass-through, emit-without-overwrite (:599-605);
//   * take_frame (:403-414): the cached level frame is copied from HBM
//     straight into the caller's buffer.
// Runs of consecutive levels that only halve XY are fused into one cascade
// launch (up to 4 levels per launch), so the frame is read from HBM once.
//
// Level buffers: every level L >= 1 owns two device slots.  A frame emitted
// while the level's cache is empty becomes the cached frame (its slot is
// then left alone until take_frame); new results always go to the other
// slot, so an untaken frame is never overwritten — the reference's
// unordered_map::emplace rule.
#include "aqz_downsampler.h"
#include "abi_guard.hh"
#include "ds_kernels.hh"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <array>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace {

thread_local std::string g_last_error;

// Pyramids up to this many level bytes are read back eagerly (aqz_ds::eager).
// (A host memcpy of a larger pyramid would cost more than the round trips
// it saves)
constexpr size_t kEagerBytes = size_t(1) << 20;

void
set_global_error(const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
}

uint32_t
bit_width(uint32_t x)
{
    uint32_t n = 0;
    for (; x; x >>= 1)
        ++n;
    return n;
}

// Number of 2x divisions a dimension supports before it fits one chunk
// (downsampler.cpp:507-520): bit_width(ceil(size/chunk) - 1).
uint32_t
divisions(const aqz_dimension& d)
{
    const uint32_t n = (d.array_size_px + d.chunk_size_px - 1) / d.chunk_size_px;
    return n > 1 ? bit_width(n - 1) : 0;
}

// downsample_dimension, downsampler.cpp:8-37.
aqz_dimension
halve(const aqz_dimension& d)
{
    aqz_dimension o = d;
    o.array_size_px = (d.array_size_px + d.array_size_px % 2) / 2;
    const uint32_t n = (o.array_size_px + d.chunk_size_px - 1) / d.chunk_size_px;
    o.shard_size_chunks = std::min(n, d.shard_size_chunks);
    o.scale = d.scale * 2.0;
    return o;
}

bool
env_flag(const char* name)
{
    const char* v = std::getenv(name);
    return v && *v && std::strcmp(v, "0") != 0;
}

} // namespace

struct aqz_ds
{
    int device = 0;
    int dtype = 0;
    int method = 0;
    size_t bpp = 0;
    uint32_t n = 0;
    std::vector<aqz_level_desc> lv;
    std::vector<size_t> bytes;      // bytes of one frame per level
    std::vector<uint8_t> xy;        // level L halves XY (L >= 1)
    std::vector<uint8_t> zh;        // level L halves Z (L >= 1)
    std::vector<uint32_t> count;    // level_frame_count_
    std::vector<uint8_t> has_partial;
    // aqz_ds_add_frame_async_take with AQZ_TAKE_HOLD: the caller still holds
    // an untaken frame of the level, so new ones are dropped (the emplace
    // rule, downsampler.cpp:599-605) as if it were cached here
    std::vector<uint8_t> held;

    hipStream_t stream = nullptr;
    void* d_in = nullptr;                      // level-0 frame on device
    std::vector<std::pair<void*, void*>> slot; // two output slots per level
    std::vector<int> cached;                   // slot holding the untaken frame, -1 none
    std::vector<void*> d_partial;              // stored earlier plane (Z levels)
    hipEvent_t h2d_done = nullptr;
    // orders a caller's stream against `stream` around a batch run on it
    hipEvent_t join = nullptr;
    // optional pinned staging of host frames ($AQZ_PINNED_STAGING=1)
    bool staged = false;
    void* h_stage = nullptr;
    size_t device_bytes = 0;
    int last_batch_kind = -1;

    // Small pyramids (all levels together <= kEagerBytes): every newly cached
    // level frame is copied to pinned host memory right behind the kernels,
    // so the take_frame calls that follow cost one event wait and a memcpy
    // each instead of a device round trip each ($AQZ_EAGER_READBACK=0: off).
    bool eager = false;
    std::vector<uint8_t*> h_level;  // pinned copy per level
    std::vector<int> host_for;      // slot whose frame h_level holds, -1 none
    std::vector<uint8_t> no_eager;  // level taken tiled: the host copy would be wasted
    hipEvent_t levels_d2h = nullptr;

    // aqz_ds_take_frame_tiled: on-demand scratch (tiles, then slice flags)
    void* d_tiles = nullptr;
    size_t d_tiles_bytes = 0;
    // aqz_ds_run_device_batch_tiled: row-major copy of the last level of a
    // fused run that feeds the next run (pyramids deeper than 4 XY levels)
    void* d_chain = nullptr;
    size_t d_chain_bytes = 0;
    // recorded after every tiled batch: the next one (on any stream) waits on
    // it before it rewrites d_chain
    hipEvent_t chain_done = nullptr;
    // aqz_ds_run_device_batch_chunked: per-level frame offsets (elements),
    // staged in pinned memory and copied to the device on the batch's
    // stream; two halves used by alternate calls, each guarded by the event
    // recorded after the batch that read it
    uint64_t* d_lattice = nullptr;
    uint64_t* h_lattice = nullptr;
    size_t lattice_half = 0; // entries per half
    uint32_t lattice_calls = 0;
    hipEvent_t lattice_done[2] = { nullptr, nullptr };
    // aqz_ds_set_level_tiling: per level (tile_rows, tile_cols), two tiled
    // slots (tiles then slice flags) paired with `slot`, and which slot's
    // frame they currently hold (-1 none)
    std::vector<std::pair<uint32_t, uint32_t>> tiling;
    std::vector<std::pair<void*, void*>> tslot;
    std::vector<std::pair<uint8_t*, uint8_t*>> tflags; // pinned, kernel-written
    // per level and tiled slot: flag bytes each half can hold, and the flag
    // bytes per tile of the frame tiled there (tile_slices for the tile
    // kernel, cascade_tiled_slots for the one-pass tiled cascade)
    std::vector<std::array<size_t, 2>> tflag_cap;
    std::vector<std::array<uint32_t, 2>> tflag_slices;
    std::vector<int> tiled_for;
    // $AQZ_STREAM_TILE_PASS=1: eager tiling as a tile pass behind the
    // row-major cascade (the round-2 path), for A/B
    bool tile_pass = false;
    uint64_t stream_tiled_runs = 0; // runs the streaming path tiled in one launch
    // eager tiled readback (aqz_ds::eager): pinned copy of a level's tiles,
    // queued right behind its tile kernel, and which slot's frame it holds
    std::vector<uint8_t*> h_tiles;
    std::vector<int> htile_for;
    uint8_t* h_flags = nullptr; // pinned slice flags for on-demand tiling
    size_t h_flags_bytes = 0;

    // aqz_ds_set_input_transpose: input frames arrive in acquisition order
    // (rows = level-0 width) and are transposed into d_tin on the device
    bool transpose = false;
    void* d_tin = nullptr;
    // the last level-0 frame added (storage order), for aqz_ds_take_input_frame;
    // null once taken or after a batch
    const void* last_input = nullptr;

    // aqz_ds_run_host_batch pipeline, allocated on first use
    struct Pipe
    {
        uint32_t group = 0;                  // frames per group
        hipStream_t s_in = nullptr, s_work = nullptr, s_out = nullptr;
        void* d_in[2] = { nullptr, nullptr };
        std::vector<void*> d_out[2];         // per level, group-sized
        hipEvent_t in_done[2] = {}, work_done[2] = {}, out_done[2] = {};
    } pipe;

    // aqz_ds_add_frame_async: one worker thread (started on first use) runs
    // at most one pending add_frame; every other entry point settles it first
    struct Async
    {
        std::thread worker;
        std::mutex m;
        std::condition_variable cv;
        const void* frame = nullptr; // the pending job's frame, null when idle
        // the pending job's frame while the job may still read it (until its
        // upload is done); null once the caller may reuse it
        const void* input = nullptr;
        aqz_level_take* takes = nullptr; // aqz_ds_add_frame_async_take's takes
        bool stop = false;
        int rc = 0;                  // status of the last finished job
    } async;

    std::string err;

    int fail(hipError_t e, const char* what)
    {
        err = std::string(what) + ": " + hipGetErrorString(e);
        return AQZ_INTERNAL_ERROR;
    }
    int fail_arg(const std::string& what)
    {
        err = what;
        return AQZ_INVALID_ARGUMENT;
    }
    void* slot_ptr(uint32_t L, int k) const
    {
        return k == 0 ? slot[L].first : slot[L].second;
    }
    // where a new level-L frame is written: never the cached slot
    void* out_slot(uint32_t L) const { return slot_ptr(L, cached[L] == 0 ? 1 : 0); }
};

namespace aqz {

inline std::string*
abi_err_slot(aqz_ds* ds)
{
    return ds ? &ds->err : nullptr;
}

} // namespace aqz

namespace {

#define HIP_TRY(ds, expr, what)                                                \
    do {                                                                       \
        hipError_t e_ = (expr);                                                \
        if (e_ != hipSuccess)                                                  \
            return (ds)->fail(e_, what);                                       \
    } while (0)

// Where the frames a level emits go.
struct Sink
{
    // false: streaming add_frame — the frame may become the cached one
    bool batch = false;
    // batch mode: frame k of level L goes to out[L] + k*bytes[L]
    void* const* out = nullptr;
    std::vector<uint32_t>* emitted = nullptr;
};

uint64_t
elems(const aqz_ds* ds, uint32_t level)
{
    return uint64_t(ds->lv[level].width) * ds->lv[level].height;
}

// Tiled layout of level L at (tr, tc): tile bytes and slice-flag bytes.
struct TileGeom
{
    size_t n_tiles, tile_bytes, flag_bytes;
};

TileGeom
tile_geom(const aqz_ds* ds, uint32_t L, uint32_t tr, uint32_t tc)
{
    const aqz_level_desc& lv = ds->lv[L];
    const size_t ntx = (lv.width + tc - 1) / tc, nty = (lv.height + tr - 1) / tr;
    const size_t nt = ntx * nty;
    return { nt, nt * tr * tc * ds->bpp, nt * aqz::tile_slices(tr, tc) };
}

// One flag per tile: the OR of its `slices` flag bytes (pinned,
// kernel-written, tile-major).
void
reduce_slice_flags(const TileGeom& g, size_t slices, const uint8_t* flags,
                   uint8_t* tile_nonzero)
{
    for (size_t t = 0; t < g.n_tiles; ++t) {
        // most tiles hold data: stop at the first set flag
        const uint8_t* f = flags + t * slices;
        tile_nonzero[t] = std::any_of(f, f + slices, [](uint8_t b) { return b != 0; }) ? 1 : 0;
    }
}

// D2H of tiles already laid out on the device, then one flag per tile from
// its slice flags (pinned, written by the tile kernel).
int
tiles_to_host(aqz_ds* ds, const TileGeom& g, size_t slices, const void* d_tiles,
              const uint8_t* flags, void* dst, uint8_t* tile_nonzero)
{
    HIP_TRY(ds,
            hipMemcpyAsync(dst, d_tiles, g.tile_bytes, hipMemcpyDeviceToHost, ds->stream),
            "hipMemcpyAsync D2H");
    HIP_TRY(ds, hipStreamSynchronize(ds->stream), "hipStreamSynchronize");
    if (tile_nonzero)
        reduce_slice_flags(g, slices, flags, tile_nonzero);
    return AQZ_OK;
}

// Tile a device frame into the on-demand scratch buffers and copy it out.
int
tile_to_host(aqz_ds* ds, const void* d_frame, const aqz_level_desc& lv, uint32_t tile_rows,
             uint32_t tile_cols, const TileGeom& g, void* dst, uint8_t* tile_nonzero)
{
    if (ds->d_tiles_bytes < g.tile_bytes) {
        (void)hipFree(ds->d_tiles);
        ds->d_tiles = nullptr;
        ds->d_tiles_bytes = 0;
        HIP_TRY(ds, hipMalloc(&ds->d_tiles, g.tile_bytes), "hipMalloc tiles");
        ds->d_tiles_bytes = g.tile_bytes;
    }
    if (ds->h_flags_bytes < g.flag_bytes) {
        (void)hipHostFree(ds->h_flags);
        ds->h_flags = nullptr;
        ds->h_flags_bytes = 0;
        HIP_TRY(ds, hipHostMalloc(reinterpret_cast<void**>(&ds->h_flags), g.flag_bytes,
                                  hipHostMallocDefault), "hipHostMalloc flags");
        ds->h_flags_bytes = g.flag_bytes;
    }
    HIP_TRY(ds,
            aqz::launch_tile_frame_sliced(ds->dtype, d_frame, lv.width, lv.height, tile_rows,
                                          tile_cols, ds->d_tiles, ds->h_flags, ds->stream),
            "tile kernel");
    return tiles_to_host(ds, g, g.flag_bytes / g.n_tiles, ds->d_tiles, ds->h_flags, dst,
                         tile_nonzero);
}

// Working buffer for a level-L result: the caller's batch slot when the
// sink is a batch, else the level's free device slot.
void*
level_target(aqz_ds* ds, uint32_t L, const Sink& sink)
{
    if (sink.batch)
        return static_cast<uint8_t*>(sink.out[L]) +
               (*sink.emitted)[L] * ds->bytes[L];
    return ds->out_slot(L);
}

// emplace_downsampled_frame_ (downsampler.cpp:599-605).  `pretiled`: the
// one-pass tiled cascade has already written this frame's tiles and flags
// into the tiled slot paired with its slot.
int
emit(aqz_ds* ds, uint32_t level, const void* d_frame, const Sink& sink, bool pretiled = false)
{
    ++ds->count[level];
    void* want = level_target(ds, level, sink);
    if (want != d_frame) {
        HIP_TRY(ds,
                hipMemcpyAsync(want, d_frame, ds->bytes[level],
                               hipMemcpyDeviceToDevice, ds->stream),
                "hipMemcpyAsync D2D");
    }
    if (sink.batch) {
        ++(*sink.emitted)[level];
        return AQZ_OK;
    }
    // unordered_map::emplace keeps an untaken frame; the new one is dropped
    // (it stays in the free slot only as the next level's input).
    if (ds->cached[level] < 0 && !ds->held[level]) {
        const int k = (want == ds->slot[level].first) ? 0 : 1;
        ds->cached[level] = k;
        const auto [tr, tc] = ds->tiling[level];
        if (tr && pretiled) {
            ds->tiled_for[level] = k;
        } else if (tr) {
            // queue the chunk tiling right behind the pyramid (§8(f) row 2)
            void* tb = k == 0 ? ds->tslot[level].first : ds->tslot[level].second;
            uint8_t* fb = k == 0 ? ds->tflags[level].first : ds->tflags[level].second;
            HIP_TRY(ds,
                    aqz::launch_tile_frame_sliced(ds->dtype, want, ds->lv[level].width,
                                                  ds->lv[level].height, tr, tc, tb, fb,
                                                  ds->stream),
                    "tile kernel");
            ds->tiled_for[level] = k;
            ds->tflag_slices[level][k] = aqz::tile_slices(tr, tc);
        }
    }
    return AQZ_OK;
}

// One run of k pure-XY levels from L, every one of them tiled: the tiled
// cascade writes each level row-major into its free slot (the next run's
// input and take_frame's copy) and chunk-tiled, zero scan included, into the
// tiled slot paired with it — one launch instead of the cascade plus a tile
// pass per level.  *launched is false when the geometry needs the separate
// tile pass (nothing was queued but, at most, a flag clear).
int
launch_run_tiled(aqz_ds* ds, uint32_t L, uint32_t k, const void* cur,
                 const aqz::LevelOut* outs, bool* launched)
{
    *launched = false;
    if (ds->tile_pass)
        return AQZ_OK;
    const aqz_level_desc& a = ds->lv[L - 1];
    if (aqz::cascade_tiled_cols(ds->dtype, a.width) !=
        aqz::cascade_pick_cols(ds->dtype, cur, elems(ds, L - 1), a.width, a.height, outs, int(k)))
        return AQZ_OK;
    aqz::TiledOut t[aqz::kMaxFusedLevels];
    uint32_t slices[aqz::kMaxFusedLevels];
    int kk[aqz::kMaxFusedLevels];
    for (uint32_t j = 0; j < k; ++j) {
        const uint32_t l = L + j;
        const auto [tr, tc] = ds->tiling[l];
        if (!tr)
            return AQZ_OK;
        const int s = outs[j].ptr == ds->slot[l].first ? 0 : 1;
        const uint32_t slots = aqz::cascade_tiled_slots(ds->dtype, a.width, int(k), int(j + 1),
                                                        tr, tc, nullptr);
        if (!slots)
            return AQZ_OK; // one OR-ed flag per tile would need a clear of pinned memory
        slices[j] = slots;
        const TileGeom g = tile_geom(ds, l, tr, tc);
        const size_t need = g.n_tiles * slices[j];
        uint8_t*& fb = s == 0 ? ds->tflags[l].first : ds->tflags[l].second;
        if (ds->tflag_cap[l][s] < need) {
            // the half is free (its slot is not the cached one); earlier
            // kernels may still write it
            HIP_TRY(ds, hipStreamSynchronize(ds->stream), "hipStreamSynchronize");
            (void)hipHostFree(fb);
            fb = nullptr;
            ds->tflag_cap[l][s] = 0;
            HIP_TRY(ds, hipHostMalloc(reinterpret_cast<void**>(&fb), need, hipHostMallocDefault),
                    "hipHostMalloc flags");
            ds->tflag_cap[l][s] = need;
        }
        kk[j] = s;
        t[j] = { s == 0 ? ds->tslot[l].first : ds->tslot[l].second, tr, tc, fb };
    }
    const hipError_t e = aqz::launch_cascade_tiled(ds->dtype, ds->method, cur, elems(ds, L - 1),
                                                   a.width, a.height, outs, t, int(k), 1,
                                                   ds->stream);
    if (e == hipErrorInvalidValue)
        return AQZ_OK;
    HIP_TRY(ds, e, "tiled cascade kernel");
    for (uint32_t j = 0; j < k; ++j)
        ds->tflag_slices[L + j][kk[j]] = slices[j];
    ++ds->stream_tiled_runs;
    *launched = true;
    return AQZ_OK;
}

// XY-reduce `src` (level L-1 geometry) into `dst` (level L geometry).
int
reduce_xy(aqz_ds* ds, uint32_t L, const void* src, void* dst)
{
    const aqz_level_desc& a = ds->lv[L - 1];
    aqz::LevelOut o{ dst, elems(ds, L), ds->lv[L].width, ds->lv[L].height };
    hipError_t e;
    if (aqz::cascade_supported(ds->dtype, src, elems(ds, L - 1), a.width, a.height, &o, 1))
        e = aqz::launch_cascade(ds->dtype, ds->method, src, elems(ds, L - 1),
                                a.width, a.height, &o, 1, 1, ds->stream);
    else
        e = aqz::launch_xy_generic(ds->dtype, ds->method, src, elems(ds, L - 1),
                                   a.width, a.height, o, 1, ds->stream);
    HIP_TRY(ds, e, "xy level kernel");
    return AQZ_OK;
}

// One frame through the level cascade: Downsampler::add_frame
// (downsampler.cpp:306-401) with device buffers.
int
process_frame(aqz_ds* ds, const void* d_frame, const Sink& sink)
{
    ++ds->count[0];
    const void* cur = d_frame;
    uint32_t L = 1;
    while (L < ds->n) {
        if (ds->xy[L] && !ds->zh[L]) {
            // Run of pure-XY levels: they always emit, fuse up to 4.
            uint32_t k = 1;
            while (L + k < ds->n && k < aqz::kMaxFusedLevels && ds->xy[L + k] &&
                   !ds->zh[L + k])
                ++k;
            aqz::LevelOut outs[aqz::kMaxFusedLevels];
            for (uint32_t j = 0; j < k; ++j)
                outs[j] = { level_target(ds, L + j, sink), elems(ds, L + j),
                            ds->lv[L + j].width, ds->lv[L + j].height };
            const aqz_level_desc& a = ds->lv[L - 1];
            bool pretiled = false;
            if (!sink.batch)
                if (int rc = launch_run_tiled(ds, L, k, cur, outs, &pretiled))
                    return rc;
            if (pretiled) {
                // levels and their tiles written by the tiled cascade
            } else if (aqz::cascade_supported(ds->dtype, cur, elems(ds, L - 1), a.width,
                                              a.height, outs, int(k))) {
                HIP_TRY(ds,
                        aqz::launch_cascade(ds->dtype, ds->method, cur,
                                            elems(ds, L - 1), a.width, a.height,
                                            outs, int(k), 1, ds->stream),
                        "cascade kernel");
            } else {
                const void* s = cur;
                for (uint32_t j = 0; j < k; ++j) {
                    const aqz_level_desc& b = ds->lv[L + j - 1];
                    HIP_TRY(ds,
                            aqz::launch_xy_generic(ds->dtype, ds->method, s,
                                                   elems(ds, L + j - 1), b.width,
                                                   b.height, outs[j], 1,
                                                   ds->stream),
                            "xy level kernel");
                    s = outs[j].ptr;
                }
            }
            for (uint32_t j = 0; j < k; ++j) {
                int rc = emit(ds, L + j, outs[j].ptr, sink, pretiled);
                if (rc)
                    return rc;
            }
            cur = outs[k - 1].ptr;
            L += k;
            continue;
        }

        // General level: optional XY reduce, then optional Z pairing.
        const uint32_t prev_planes = ds->lv[L - 1].planes;
        bool average = ds->zh[L] != 0;
        if (prev_planes % 2 != 0 && ds->count[L - 1] % prev_planes == 0)
            average = false; // last plane of an odd stack passes through

        if (average && !ds->has_partial[L]) {
            // store this plane as the earlier half of the pair, then stop
            if (ds->xy[L]) {
                int rc = reduce_xy(ds, L, cur, ds->d_partial[L]);
                if (rc)
                    return rc;
            } else {
                HIP_TRY(ds,
                        hipMemcpyAsync(ds->d_partial[L], cur, ds->bytes[L],
                                       hipMemcpyDeviceToDevice, ds->stream),
                        "hipMemcpyAsync D2D");
            }
            ds->has_partial[L] = 1;
            break;
        }

        void* target = level_target(ds, L, sink);
        const void* next = cur;
        if (ds->xy[L]) {
            int rc = reduce_xy(ds, L, cur, target);
            if (rc)
                return rc;
            next = target;
        }
        if (average) {
            // average_two_frames(dst = earlier, src = current)
            HIP_TRY(ds,
                    aqz::launch_zpair(ds->dtype, ds->method, target,
                                      ds->d_partial[L], next, elems(ds, L),
                                      ds->stream),
                    "zpair kernel");
            ds->has_partial[L] = 0;
            next = target;
        }
        int rc = emit(ds, L, next, sink);
        if (rc)
            return rc;
        cur = target; // emit() left the level's frame in `target`
        ++L;
    }
    return AQZ_OK;
}

int
bind_device(aqz_ds* ds)
{
    HIP_TRY(ds, hipSetDevice(ds->device), "hipSetDevice");
    return AQZ_OK;
}

int
check_host_frame(aqz_ds* ds, const void* host_frame, size_t nbytes, const char* who)
{
    if (!host_frame || nbytes != ds->bytes[0])
        return ds->fail_arg(std::string(who) + ": expected " +
                            std::to_string(ds->bytes[0]) + " bytes, got " +
                            std::to_string(nbytes));
    return AQZ_OK;
}

// The pyramid of one level-0 frame already on the device.  With input
// transposition the frame is first transposed into storage order
// (transpose_frame, array.cpp:517-530), which is what the reference's
// downsampler receives.
int
process_input(aqz_ds* ds, const void* d_frame)
{
    if (ds->transpose) {
        // acquisition rows = storage width (array.dimensions.cpp:578-599)
        HIP_TRY(ds,
                aqz::launch_transpose(ds->dtype, d_frame, ds->lv[0].width,
                                      ds->lv[0].height, ds->d_tin, ds->stream),
                "transpose kernel");
        d_frame = ds->d_tin;
    }
    ds->last_input = d_frame;
    return process_frame(ds, d_frame, Sink{});
}

// Downsampler::add_frame for a host frame: upload it, queue the pyramid, and
// return once the upload has completed (the caller may then reuse its frame;
// the kernels are still queued).
// Queue the D2H of every newly cached level frame into its pinned copy,
// right behind the kernels that made it (aqz_ds::eager).
int
eager_readback(aqz_ds* ds)
{
    if (!ds->eager)
        return AQZ_OK;
    bool any = false;
    for (uint32_t L = 1; L < ds->n; ++L) {
        const int k = ds->cached[L];
        if (k < 0)
            continue;
        if (ds->no_eager[L]) {
            // taken tiled: copy the tiles out instead, so the D2H overlaps
            // whatever the caller does before take_frame_tiled
            if (ds->h_tiles[L] && ds->tiled_for[L] == k && ds->htile_for[L] != k) {
                const TileGeom g = tile_geom(ds, L, ds->tiling[L].first, ds->tiling[L].second);
                void* tb = k == 0 ? ds->tslot[L].first : ds->tslot[L].second;
                HIP_TRY(ds,
                        hipMemcpyAsync(ds->h_tiles[L], tb, g.tile_bytes, hipMemcpyDeviceToHost,
                                       ds->stream),
                        "hipMemcpyAsync D2H (eager tiles)");
                ds->htile_for[L] = k;
                any = true;
            }
            continue;
        }
        if (ds->host_for[L] == k)
            continue;
        HIP_TRY(ds,
                hipMemcpyAsync(ds->h_level[L], ds->slot_ptr(L, k), ds->bytes[L],
                               hipMemcpyDeviceToHost, ds->stream),
                "hipMemcpyAsync D2H (eager)");
        ds->host_for[L] = k;
        any = true;
    }
    if (any)
        HIP_TRY(ds, hipEventRecord(ds->levels_d2h, ds->stream), "hipEventRecord");
    return AQZ_OK;
}

int
add_host_frame(aqz_ds* ds, const void* host_frame)
{
    if (int rc = bind_device(ds))
        return rc;
    const size_t nbytes = ds->bytes[0];
    const void* src = host_frame;
    if (ds->staged) {
        // previous upload must be done before the staging buffer is reused
        HIP_TRY(ds, hipEventSynchronize(ds->h2d_done), "hipEventSynchronize");
        std::memcpy(ds->h_stage, host_frame, nbytes);
        src = ds->h_stage;
    }
    // Straight from the caller's (pageable) frame: the copy engine reads it
    // at full PCIe rate, no host staging memcpy (tools/e2e_probe.cpp).
    HIP_TRY(ds,
            hipMemcpyAsync(ds->d_in, src, nbytes, hipMemcpyHostToDevice, ds->stream),
            "hipMemcpyAsync H2D");
    // From here on the copy may still read the caller's frame: every way out
    // waits for it first, so that a failed add, too, releases the frame only
    // once nothing reads it (aqz_ds_wait_input's contract).
    if (const hipError_t e = hipEventRecord(ds->h2d_done, ds->stream); e != hipSuccess) {
        (void)hipStreamSynchronize(ds->stream);
        return ds->fail(e, "hipEventRecord");
    }
    int rc = process_input(ds, ds->d_in);
    if (rc == AQZ_OK)
        rc = eager_readback(ds);
    if (rc != AQZ_OK) {
        if (!ds->staged)
            (void)hipEventSynchronize(ds->h2d_done);
        return rc;
    }
    if (!ds->staged) {
        // the caller may reuse its frame as soon as we return
        HIP_TRY(ds, hipEventSynchronize(ds->h2d_done), "hipEventSynchronize");
    }
    return AQZ_OK;
}

// aqz_ds_take_frame's body (its caller has settled any pending add).
int
take_plain(aqz_ds* ds, uint32_t level, void* dst, size_t cap, size_t* nbytes, int* has_frame)
{
    *has_frame = 0;
    if (level == 0 || level >= ds->n)
        return AQZ_OK; // the reference's map lookup simply misses
    if (ds->cached[level] < 0)
        return AQZ_OK;
    *has_frame = 1;
    if (nbytes)
        *nbytes = ds->bytes[level];
    if (!dst)
        return AQZ_OK;
    if (cap < ds->bytes[level])
        return ds->fail_arg("take_frame: buffer too small");
    if (int rc = bind_device(ds))
        return rc;
    if (ds->eager && ds->host_for[level] == ds->cached[level]) {
        // already on its way to pinned memory (eager_readback)
        HIP_TRY(ds, hipEventSynchronize(ds->levels_d2h), "hipEventSynchronize");
        std::memcpy(dst, ds->h_level[level], ds->bytes[level]);
    } else {
        // HBM -> caller memory directly (stream-ordered after the kernels)
        HIP_TRY(ds,
                hipMemcpyAsync(dst, ds->slot_ptr(level, ds->cached[level]),
                               ds->bytes[level], hipMemcpyDeviceToHost, ds->stream),
                "hipMemcpyAsync D2H");
        HIP_TRY(ds, hipStreamSynchronize(ds->stream), "hipStreamSynchronize");
    }
    ds->cached[level] = -1;
    ds->tiled_for[level] = -1;
    ds->host_for[level] = -1;
    ds->htile_for[level] = -1;
    return AQZ_OK;
}

// aqz_ds_take_frame_tiled's body (its caller has settled any pending add).
int
take_tiled(aqz_ds* ds,
           uint32_t level,
           uint32_t tile_rows,
           uint32_t tile_cols,
           void* dst,
           size_t cap,
           uint8_t* tile_nonzero,
           size_t* nbytes,
           int* has_frame)
{
    *has_frame = 0;
    if (tile_rows == 0 || tile_cols == 0)
        return ds->fail_arg("take_frame_tiled: empty tile");
    if (level == 0 || level >= ds->n || ds->cached[level] < 0)
        return AQZ_OK;
    const TileGeom g = tile_geom(ds, level, tile_rows, tile_cols);
    *has_frame = 1;
    if (nbytes)
        *nbytes = g.tile_bytes;
    if (!dst)
        return AQZ_OK;
    if (cap < g.tile_bytes)
        return ds->fail_arg("take_frame_tiled: buffer too small");
    if (int rc = bind_device(ds))
        return rc;
    const int k = ds->cached[level];
    if (ds->tiling[level] == std::make_pair(tile_rows, tile_cols) &&
        ds->tiled_for[level] == k && ds->htile_for[level] == k) {
        // tiled and copied out when the frame was emitted (eager readback)
        HIP_TRY(ds, hipEventSynchronize(ds->levels_d2h), "hipEventSynchronize");
        std::memcpy(dst, ds->h_tiles[level], g.tile_bytes);
        if (tile_nonzero)
            reduce_slice_flags(g, ds->tflag_slices[level][k],
                               k == 0 ? ds->tflags[level].first : ds->tflags[level].second,
                               tile_nonzero);
    } else if (ds->tiling[level] == std::make_pair(tile_rows, tile_cols) &&
               ds->tiled_for[level] == k) {
        // tiled when the frame was emitted (aqz_ds_set_level_tiling)
        if (int rc = tiles_to_host(ds, g, ds->tflag_slices[level][k],
                                   k == 0 ? ds->tslot[level].first : ds->tslot[level].second,
                                   k == 0 ? ds->tflags[level].first : ds->tflags[level].second,
                                   dst, tile_nonzero))
            return rc;
    } else if (int rc = tile_to_host(ds, ds->slot_ptr(level, k), ds->lv[level], tile_rows,
                                     tile_cols, g, dst, tile_nonzero)) {
        return rc;
    }
    ds->cached[level] = -1;
    ds->tiled_for[level] = -1;
    ds->host_for[level] = -1;
    ds->htile_for[level] = -1;
    ds->no_eager[level] = 1; // this caller takes the level tiled
    return AQZ_OK;
}

// The takes of aqz_ds_add_frame_async_take, in the job right behind its add:
// each level's device-to-host copy then overlaps the caller's work too.
int
run_takes(aqz_ds* ds, aqz_level_take* takes)
{
    for (uint32_t L = 1; L < ds->n; ++L) {
        aqz_level_take& t = takes[L];
        t.has_frame = 0;
        t.nbytes = 0;
        if (t.mode != AQZ_TAKE_INTO)
            continue;
        const int rc = (t.tile_rows || t.tile_cols)
                         ? take_tiled(ds, L, t.tile_rows, t.tile_cols, t.dst, t.cap,
                                      t.tile_nonzero, &t.nbytes, &t.has_frame)
                         : take_plain(ds, L, t.dst, t.cap, &t.nbytes, &t.has_frame);
        if (rc)
            return rc;
    }
    return AQZ_OK;
}

void
async_worker(aqz_ds* ds)
{
    auto& a = ds->async;
    std::unique_lock<std::mutex> lk(a.m);
    for (;;) {
        a.cv.wait(lk, [&] { return a.stop || a.frame != nullptr; });
        if (!a.frame)
            return; // stop requested and nothing pending
        const void* frame = a.frame;
        aqz_level_take* takes = a.takes;
        lk.unlock();
        int rc;
        try {
            rc = add_host_frame(ds, frame);
            // add_host_frame returns once the upload no longer reads the
            // caller's frame (or on failure): release it before the takes
            {
                std::lock_guard<std::mutex> in(a.m);
                a.input = nullptr;
            }
            a.cv.notify_all();
            if (rc == AQZ_OK && takes)
                rc = run_takes(ds, takes);
        } catch (...) {
            rc = ABI_GUARD_FAIL(ds); // reported by the next settle()
        }
        lk.lock();
        a.rc = rc;
        a.frame = nullptr;
        a.input = nullptr;
        a.takes = nullptr;
        a.cv.notify_all();
    }
}

// Wait for a pending aqz_ds_add_frame_async; returns (and clears) its status.
int
settle(aqz_ds* ds)
{
    auto& a = ds->async;
    if (!a.worker.joinable())
        return AQZ_OK;
    std::unique_lock<std::mutex> lk(a.m);
    a.cv.wait(lk, [&] { return a.frame == nullptr; });
    const int rc = a.rc;
    a.rc = AQZ_OK;
    return rc;
}

void
release(aqz_ds* ds)
{
    if (!ds)
        return;
    if (ds->async.worker.joinable()) {
        (void)settle(ds);
        {
            std::lock_guard<std::mutex> lk(ds->async.m);
            ds->async.stop = true;
        }
        ds->async.cv.notify_all();
        ds->async.worker.join();
    }
    // Best-effort teardown: errors here have nowhere to go.
    (void)hipSetDevice(ds->device);
    if (ds->stream)
        (void)hipStreamSynchronize(ds->stream);
    (void)hipFree(ds->d_in);
    for (auto& s : ds->slot) {
        (void)hipFree(s.first);
        (void)hipFree(s.second);
    }
    for (void* p : ds->d_partial)
        (void)hipFree(p);
    (void)hipHostFree(ds->h_stage);
    (void)hipFree(ds->d_tiles);
    for (hipEvent_t e : ds->lattice_done)
        if (e) {
            (void)hipEventSynchronize(e);
            (void)hipEventDestroy(e);
        }
    (void)hipFree(ds->d_lattice);
    (void)hipHostFree(ds->h_lattice);
    if (ds->chain_done) {
        (void)hipEventSynchronize(ds->chain_done);
        (void)hipEventDestroy(ds->chain_done);
    }
    (void)hipFree(ds->d_chain);
    for (auto& t : ds->tslot) {
        (void)hipFree(t.first);
        (void)hipFree(t.second);
    }
    for (auto& t : ds->tflags) {
        (void)hipHostFree(t.first);
        (void)hipHostFree(t.second);
    }
    (void)hipHostFree(ds->h_flags);
    for (uint8_t* h : ds->h_level)
        (void)hipHostFree(h);
    for (uint8_t* h : ds->h_tiles)
        (void)hipHostFree(h);
    if (ds->levels_d2h)
        (void)hipEventDestroy(ds->levels_d2h);
    (void)hipFree(ds->d_tin);
    if (ds->h2d_done)
        (void)hipEventDestroy(ds->h2d_done);
    if (ds->join)
        (void)hipEventDestroy(ds->join);
    for (int b = 0; b < 2; ++b) {
        (void)hipFree(ds->pipe.d_in[b]);
        for (void* p : ds->pipe.d_out[b])
            (void)hipFree(p);
        for (hipEvent_t e : { ds->pipe.in_done[b], ds->pipe.work_done[b],
                              ds->pipe.out_done[b] })
            if (e)
                (void)hipEventDestroy(e);
    }
    for (hipStream_t st : { ds->pipe.s_in, ds->pipe.s_work, ds->pipe.s_out })
        if (st)
            (void)hipStreamDestroy(st);
    if (ds->stream)
        (void)hipStreamDestroy(ds->stream);
    delete ds;
}

} // namespace

extern "C" {

// array.dimensions.cpp:168-178 (bytes_per_chunk_, number_of_chunks_in_memory_)
// and :232-314 (chunk_lattice_index, tile_group_offset, chunk_internal_offset).
int
aqz_chunk_frame_offsets(const aqz_dimension* dims,
                        uint32_t ndims,
                        uint32_t bytes_per_px,
                        uint64_t first_frame,
                        uint32_t n_frames,
                        uint64_t* frame_offset_bytes,
                        uint64_t* chunk_bytes,
                        uint64_t* layer_bytes)
{
    try {
        if (!dims || ndims < 3 || bytes_per_px == 0 || (n_frames && !frame_offset_bytes)) {
            aqz::set_last_error("chunk_frame_offsets: invalid argument");
            return AQZ_INVALID_ARGUMENT;
        }
        for (uint32_t i = 0; i < ndims; ++i)
            if (dims[i].chunk_size_px == 0 || (i > 0 && dims[i].array_size_px == 0)) {
                aqz::set_last_error("chunk_frame_offsets: zero chunk size, or a zero-size "
                                    "dimension other than the append dimension");
                return AQZ_INVALID_ARGUMENT;
            }
        const int nd = int(ndims);
        uint64_t per_chunk = bytes_per_px, chunks_in_layer = 1;
        for (int i = 0; i < nd; ++i) {
            per_chunk *= dims[i].chunk_size_px;
            if (i > 0)
                chunks_in_layer *= (uint64_t(dims[i].array_size_px) + dims[i].chunk_size_px - 1) /
                                   dims[i].chunk_size_px;
        }
        // lattice strides of every dim (chunks), frames per chunk layer
        std::vector<uint64_t> strides(nd, 1);
        for (int i = nd - 1; i > 0; --i)
            strides[i - 1] =
              strides[i] * ((uint64_t(dims[i].array_size_px) + dims[i].chunk_size_px - 1) /
                            dims[i].chunk_size_px);
        uint64_t layer_frames = dims[0].chunk_size_px;
        for (int i = 1; i + 2 < nd; ++i)
            layer_frames *= dims[i].array_size_px;
        const uint64_t tile_bytes =
          uint64_t(bytes_per_px) * dims[nd - 1].chunk_size_px * dims[nd - 2].chunk_size_px;
        auto lattice_index = [&](uint64_t fid, int d) -> uint64_t {
            uint64_t mod = 1, div = 1;
            for (int i = d; i < nd - 2; ++i) {
                mod *= dims[i].array_size_px;
                div *= (i == d ? dims[i].chunk_size_px : dims[i].array_size_px);
            }
            return (fid % mod) / div;
        };
        auto internal = [&](uint64_t fid) -> uint64_t {
            std::vector<uint64_t> astr(nd - 2, 1), cstr(nd - 2, 1);
            uint64_t off = 0;
            for (int i = nd - 3; i > 0; --i) {
                const uint64_t idx =
                  (fid / astr[i]) % dims[i].array_size_px % dims[i].chunk_size_px;
                astr[i - 1] = astr[i] * dims[i].array_size_px;
                cstr[i - 1] = cstr[i] * dims[i].chunk_size_px;
                off += idx * cstr[i];
            }
            off += ((fid / astr[0]) % dims[0].chunk_size_px) * cstr[0];
            return off * tile_bytes;
        };
        const uint64_t layer0 = first_frame / layer_frames;
        for (uint32_t k = 0; k < n_frames; ++k) {
            const uint64_t fid = first_frame + k;
            uint64_t group = 0;
            for (int i = nd - 3; i > 0; --i)
                group += lattice_index(fid, i) * strides[i];
            frame_offset_bytes[k] = (fid / layer_frames - layer0) * chunks_in_layer * per_chunk +
                                    group * per_chunk + internal(fid);
        }
        if (chunk_bytes)
            *chunk_bytes = per_chunk;
        if (layer_bytes)
            *layer_bytes = chunks_in_layer * per_chunk;
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(nullptr);
    }
}

int
aqz_plan_levels(const aqz_dimension* dims,
                uint32_t ndims,
                uint32_t max_levels,
                aqz_dimension* out,
                uint32_t out_cap_levels,
                uint32_t* n_levels)
{
    try {
        if (!dims || !n_levels || ndims < 3 || ndims > AQZ_MAX_DIMS) {
            set_global_error("plan_levels: need 3..%d dimensions", AQZ_MAX_DIMS);
            return AQZ_INVALID_ARGUMENT;
        }
        for (uint32_t i = 0; i < ndims; ++i) {
            if (dims[i].chunk_size_px == 0) {
                set_global_error("plan_levels: dimension %u has chunk size 0", i);
                return AQZ_INVALID_ARGUMENT;
            }
        }
        const aqz_dimension& x = dims[ndims - 1];
        const aqz_dimension& y = dims[ndims - 2];
        const aqz_dimension& z = dims[ndims - 3];
        uint32_t levels = std::min(divisions(x), divisions(y));
        if (z.type == AQZ_DIM_SPACE)
            levels = std::max(levels, divisions(z));
        if (max_levels > 0)
            levels = std::min(levels, max_levels);
        *n_levels = levels + 1;
        if (!out)
            return AQZ_OK;
        if (out_cap_levels < levels + 1) {
            set_global_error("plan_levels: room for %u levels, need %u",
                             out_cap_levels, levels + 1);
            return AQZ_OVERFLOW;
        }
        std::copy(dims, dims + ndims, out);
        for (uint32_t l = 1; l <= levels; ++l) {
            const aqz_dimension* p = out + size_t(l - 1) * ndims;
            aqz_dimension* c = out + size_t(l) * ndims;
            std::copy(p, p + ndims - 3, c);
            const aqz_dimension& pz = p[ndims - 3];
            c[ndims - 3] = (pz.type == AQZ_DIM_SPACE && pz.array_size_px > pz.chunk_size_px)
                             ? halve(pz)
                             : pz;
            const aqz_dimension& py = p[ndims - 2];
            const aqz_dimension& px = p[ndims - 1];
            const bool shrink_xy = std::min(py.array_size_px, px.array_size_px) >
                                   std::max(py.chunk_size_px, px.chunk_size_px);
            c[ndims - 2] = shrink_xy ? halve(py) : py;
            c[ndims - 1] = shrink_xy ? halve(px) : px;
        }
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(nullptr);
    }
}

int
aqz_ds_create(const aqz_level_desc* levels,
              uint32_t n_levels,
              int dtype,
              int method,
              int device,
              aqz_ds** out)
{
    try {
        if (!out) {
            set_global_error("create: null output handle");
            return AQZ_INVALID_ARGUMENT;
        }
        *out = nullptr;
        if (!levels || n_levels == 0 || n_levels > AQZ_MAX_LEVELS) {
            set_global_error("create: need 1..%d levels", AQZ_MAX_LEVELS);
            return AQZ_INVALID_ARGUMENT;
        }
        if (!aqz::dtype_valid(dtype)) {
            set_global_error("Invalid data type: %d", dtype);
            return AQZ_INVALID_ARGUMENT;
        }
        if (!aqz::method_valid(method)) {
            set_global_error("Invalid downsampling method: %d", method);
            return AQZ_INVALID_ARGUMENT;
        }
        for (uint32_t l = 0; l < n_levels; ++l) {
            if (levels[l].width == 0 || levels[l].height == 0) {
                set_global_error("create: level %u has an empty frame", l);
                return AQZ_INVALID_ARGUMENT;
            }
            if (l > 0) {
                const aqz_level_desc& a = levels[l - 1];
                const aqz_level_desc& b = levels[l];
                const bool same = b.width == a.width && b.height == a.height;
                const bool half = b.width == (a.width + 1) / 2 &&
                                  b.height == (a.height + 1) / 2;
                // scale_image always halves both; anything else fails the
                // reference's dimension EXPECTs (downsampler.cpp:348-356).
                if (!same && !half) {
                    set_global_error("create: level %u is neither a copy nor a 2x "
                                     "reduction of level %u", l, l - 1);
                    return AQZ_INVALID_ARGUMENT;
                }
            }
        }

        int n_devices = 0;
        if (hipGetDeviceCount(&n_devices) != hipSuccess)
            n_devices = 0;
        if (device < 0) {
            const char* env = std::getenv("AQZ_GPU_DEVICE");
            if (env && std::strcmp(env, "spread") == 0) {
                // each new handle on the next GPU: the arrays of a stream (or
                // several streams in one process) spread their pyramids over
                // the node; their frames are independent, so no collective
                static std::atomic<uint32_t> next{ 0 };
                device = n_devices > 0 ? int(next++ % uint32_t(n_devices)) : 0;
            } else if (env && *env) {
                device = std::atoi(env);
            } else if (hipGetDevice(&device) != hipSuccess) {
                device = 0;
            }
        }
        if (n_devices > 0 && (device < 0 || device >= n_devices)) {
            set_global_error("create: no HIP device %d (%d visible)", device, n_devices);
            return AQZ_INVALID_ARGUMENT;
        }

        auto* ds = new aqz_ds();
        ds->device = device;
        ds->dtype = dtype;
        ds->method = method;
        ds->bpp = aqz::dtype_bytes(dtype);
        ds->n = n_levels;
        ds->lv.assign(levels, levels + n_levels);
        ds->bytes.resize(n_levels);
        ds->xy.assign(n_levels, 0);
        ds->zh.assign(n_levels, 0);
        ds->count.assign(n_levels, 0);
        ds->has_partial.assign(n_levels, 0);
        ds->slot.assign(n_levels, { nullptr, nullptr });
        ds->cached.assign(n_levels, -1);
        ds->d_partial.assign(n_levels, nullptr);
        ds->staged = env_flag("AQZ_PINNED_STAGING");
        ds->tiling.assign(n_levels, { 0, 0 });
        ds->tslot.assign(n_levels, { nullptr, nullptr });
        ds->held.assign(n_levels, 0);
        ds->tflags.assign(n_levels, { nullptr, nullptr });
        ds->tflag_cap.assign(n_levels, { 0, 0 });
        ds->tflag_slices.assign(n_levels, { 1, 1 });
        ds->tile_pass = env_flag("AQZ_STREAM_TILE_PASS");
        ds->tiled_for.assign(n_levels, -1);
        ds->h_tiles.assign(n_levels, nullptr);
        ds->htile_for.assign(n_levels, -1);
        ds->h_level.assign(n_levels, nullptr);
        ds->host_for.assign(n_levels, -1);
        ds->no_eager.assign(n_levels, 0);
        for (uint32_t l = 0; l < n_levels; ++l) {
            ds->bytes[l] = size_t(levels[l].width) * levels[l].height * ds->bpp;
            if (l > 0) {
                ds->xy[l] = levels[l].width < levels[l - 1].width ||
                            levels[l].height < levels[l - 1].height;
                ds->zh[l] = levels[l].planes < levels[l - 1].planes;
            }
        }

        auto fail = [&](hipError_t e, const char* what) {
            const int code = e == hipErrorOutOfMemory ? AQZ_OUT_OF_MEMORY
                                                      : AQZ_INTERNAL_ERROR;
            set_global_error("%s: %s", what, hipGetErrorString(e));
            release(ds);
            return code;
        };
        hipError_t e = hipSetDevice(device);
        if (e != hipSuccess)
            return fail(e, "hipSetDevice");
        if ((e = hipStreamCreateWithFlags(&ds->stream, hipStreamNonBlocking)) != hipSuccess)
            return fail(e, "hipStreamCreate");
        if ((e = hipEventCreateWithFlags(&ds->h2d_done, hipEventDisableTiming)) != hipSuccess)
            return fail(e, "hipEventCreate");
        if ((e = hipEventCreateWithFlags(&ds->join, hipEventDisableTiming)) != hipSuccess)
            return fail(e, "hipEventCreate");
        if ((e = hipMalloc(&ds->d_in, ds->bytes[0])) != hipSuccess)
            return fail(e, "hipMalloc level 0");
        size_t level_total = 0;
        for (uint32_t l = 1; l < n_levels; ++l)
            level_total += ds->bytes[l];
        const char* eager_env = std::getenv("AQZ_EAGER_READBACK");
        ds->eager = n_levels > 1 && level_total <= kEagerBytes &&
                    !(eager_env && std::strcmp(eager_env, "0") == 0);
        if (ds->eager) {
            if ((e = hipEventCreateWithFlags(&ds->levels_d2h, hipEventDisableTiming)) !=
                hipSuccess)
                return fail(e, "hipEventCreate");
            for (uint32_t l = 1; l < n_levels; ++l)
                if ((e = hipHostMalloc(reinterpret_cast<void**>(&ds->h_level[l]), ds->bytes[l],
                                       hipHostMallocDefault)) != hipSuccess)
                    return fail(e, "hipHostMalloc level copy");
        }
        if (ds->staged &&
            (e = hipHostMalloc(&ds->h_stage, ds->bytes[0], hipHostMallocDefault)) != hipSuccess)
            return fail(e, "hipHostMalloc staging");
        ds->device_bytes = ds->bytes[0];
        for (uint32_t l = 1; l < n_levels; ++l) {
            if ((e = hipMalloc(&ds->slot[l].first, ds->bytes[l])) != hipSuccess)
                return fail(e, "hipMalloc level");
            if ((e = hipMalloc(&ds->slot[l].second, ds->bytes[l])) != hipSuccess)
                return fail(e, "hipMalloc level");
            ds->device_bytes += 2 * ds->bytes[l];
            if (ds->zh[l]) {
                if ((e = hipMalloc(&ds->d_partial[l], ds->bytes[l])) != hipSuccess)
                    return fail(e, "hipMalloc partial");
                ds->device_bytes += ds->bytes[l];
            }
        }
        *out = ds;
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(nullptr);
    }
}

void
aqz_ds_destroy(aqz_ds* ds)
{
    try {
        release(ds);
    } catch (...) {
        (void)ABI_GUARD_FAIL(nullptr);
    }
}

int
aqz_ds_add_frame(aqz_ds* ds, const void* host_frame, size_t nbytes)
{
    try {
        if (!ds)
            return AQZ_INVALID_ARGUMENT;
        if (int rc = settle(ds))
            return rc;
        if (int rc = check_host_frame(ds, host_frame, nbytes, "add_frame"))
            return rc;
        std::fill(ds->held.begin(), ds->held.end(), 0);
        return add_host_frame(ds, host_frame);
    } catch (...) {
        return ABI_GUARD_FAIL(ds);
    }
}

int
aqz_ds_add_frame_async(aqz_ds* ds, const void* host_frame, size_t nbytes)
{
    try {
        if (!ds)
            return AQZ_INVALID_ARGUMENT;
        if (int rc = settle(ds))
            return rc;
        if (int rc = check_host_frame(ds, host_frame, nbytes, "add_frame_async"))
            return rc;
        std::fill(ds->held.begin(), ds->held.end(), 0);
        auto& a = ds->async;
        if (!a.worker.joinable())
            a.worker = std::thread(async_worker, ds);
        {
            std::lock_guard<std::mutex> lk(a.m);
            a.frame = host_frame;
            a.input = host_frame;
        }
        a.cv.notify_all();
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(ds);
    }
}

int
aqz_ds_add_frame_async_take(aqz_ds* ds,
                            const void* host_frame,
                            size_t nbytes,
                            aqz_level_take* takes)
{
    try {
        if (!ds || !takes)
            return AQZ_INVALID_ARGUMENT;
        if (int rc = settle(ds))
            return rc;
        if (int rc = check_host_frame(ds, host_frame, nbytes, "add_frame_async_take"))
            return rc;
        for (uint32_t L = 1; L < ds->n; ++L) {
            const aqz_level_take& t = takes[L];
            if (t.mode < AQZ_TAKE_NONE || t.mode > AQZ_TAKE_HOLD ||
                ((t.tile_rows == 0) != (t.tile_cols == 0)))
                return ds->fail_arg("add_frame_async_take: level " + std::to_string(L) +
                                    ": bad mode or tile shape");
            if (t.mode == AQZ_TAKE_HOLD && ds->cached[L] >= 0)
                return ds->fail_arg("add_frame_async_take: level " + std::to_string(L) +
                                    " is held by the caller but also cached here");
            // every take buffer is checked before the job is queued, so the
            // background takes cannot fail half way and leave a level taken
            // (uncached here) that the caller never learns about
            if (t.mode == AQZ_TAKE_INTO) {
                const size_t need = t.tile_rows
                                      ? tile_geom(ds, L, t.tile_rows, t.tile_cols).tile_bytes
                                      : ds->bytes[L];
                if (!t.dst || t.cap < need)
                    return ds->fail_arg("add_frame_async_take: level " + std::to_string(L) +
                                        ": take buffer missing or smaller than " +
                                        std::to_string(need) + " bytes");
            }
        }
        for (uint32_t L = 1; L < ds->n; ++L)
            ds->held[L] = takes[L].mode == AQZ_TAKE_HOLD;
        auto& a = ds->async;
        if (!a.worker.joinable())
            a.worker = std::thread(async_worker, ds);
        {
            std::lock_guard<std::mutex> lk(a.m);
            a.frame = host_frame;
            a.input = host_frame;
            a.takes = takes;
        }
        a.cv.notify_all();
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(ds);
    }
}

int
aqz_ds_wait(aqz_ds* ds)
{
    try {
        if (!ds)
            return AQZ_INVALID_ARGUMENT;
        return settle(ds);
    } catch (...) {
        return ABI_GUARD_FAIL(ds);
    }
}

int
aqz_ds_wait_input(aqz_ds* ds)
{
    try {
        if (!ds)
            return AQZ_INVALID_ARGUMENT;
        auto& a = ds->async;
        if (!a.worker.joinable())
            return AQZ_OK;
        std::unique_lock<std::mutex> lk(a.m);
        a.cv.wait(lk, [&] { return a.input == nullptr; });
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(ds);
    }
}

int
aqz_ds_input_pending(aqz_ds* ds, int* pending)
{
    try {
        if (!ds || !pending)
            return AQZ_INVALID_ARGUMENT;
        *pending = 0;
        auto& a = ds->async;
        if (a.worker.joinable()) {
            std::lock_guard<std::mutex> lk(a.m);
            *pending = a.input != nullptr;
        }
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(ds);
    }
}

int
aqz_ds_poll(aqz_ds* ds, int* done)
{
    try {
        if (!ds || !done)
            return AQZ_INVALID_ARGUMENT;
        *done = 1;
        auto& a = ds->async;
        if (a.worker.joinable()) {
            std::lock_guard<std::mutex> lk(a.m);
            *done = a.frame == nullptr;
        }
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(ds);
    }
}

int
aqz_ds_add_device_frame(aqz_ds* ds, const void* device_frame, size_t nbytes)
{
    try {
        if (!ds)
            return AQZ_INVALID_ARGUMENT;
        if (int rc = settle(ds))
            return rc;
        if (!device_frame || nbytes != ds->bytes[0])
            return ds->fail_arg("add_device_frame: expected " +
                                std::to_string(ds->bytes[0]) + " bytes, got " +
                                std::to_string(nbytes));
        std::fill(ds->held.begin(), ds->held.end(), 0);
        if (int rc = bind_device(ds))
            return rc;
        if (int rc = process_input(ds, device_frame))
            return rc;
        return eager_readback(ds);
    } catch (...) {
        return ABI_GUARD_FAIL(ds);
    }
}

int
aqz_ds_take_frame(aqz_ds* ds,
                  uint32_t level,
                  void* dst,
                  size_t cap,
                  size_t* nbytes,
                  int* has_frame)
{
    try {
        if (!ds || !has_frame)
            return AQZ_INVALID_ARGUMENT;
        *has_frame = 0;
        if (int rc = settle(ds))
            return rc;
        return take_plain(ds, level, dst, cap, nbytes, has_frame);
    } catch (...) {
        return ABI_GUARD_FAIL(ds);
    }
}

int
aqz_ds_set_level_tiling(aqz_ds* ds, uint32_t level, uint32_t tile_rows, uint32_t tile_cols)
{
    try {
        if (!ds)
            return AQZ_INVALID_ARGUMENT;
        if (int rc = settle(ds))
            return rc;
        if (level == 0 || level >= ds->n)
            return ds->fail_arg("set_level_tiling: bad level " + std::to_string(level));
        if ((tile_rows == 0) != (tile_cols == 0))
            return ds->fail_arg("set_level_tiling: tile rows/cols must both be 0 or >0");
        if (int rc = bind_device(ds))
            return rc;
        HIP_TRY(ds, hipStreamSynchronize(ds->stream), "hipStreamSynchronize");
        auto& t = ds->tslot[level];
        (void)hipFree(t.first);
        (void)hipFree(t.second);
        t = { nullptr, nullptr };
        auto& tf = ds->tflags[level];
        (void)hipHostFree(tf.first);
        (void)hipHostFree(tf.second);
        tf = { nullptr, nullptr };
        ds->tflag_cap[level] = { 0, 0 };
        (void)hipHostFree(ds->h_tiles[level]);
        ds->h_tiles[level] = nullptr;
        ds->htile_for[level] = -1;
        ds->tiling[level] = { 0, 0 };
        ds->tiled_for[level] = -1;
        ds->no_eager[level] = tile_rows != 0;
        if (tile_rows == 0)
            return AQZ_OK;
        const TileGeom g = tile_geom(ds, level, tile_rows, tile_cols);
        HIP_TRY(ds, hipMalloc(&t.first, g.tile_bytes), "hipMalloc tiles");
        HIP_TRY(ds, hipMalloc(&t.second, g.tile_bytes), "hipMalloc tiles");
        // slice flags live in pinned host memory the kernel writes directly, so
        // take_frame_tiled needs no separate flag copy
        HIP_TRY(ds, hipHostMalloc(reinterpret_cast<void**>(&tf.first), g.flag_bytes,
                                  hipHostMallocDefault), "hipHostMalloc flags");
        HIP_TRY(ds, hipHostMalloc(reinterpret_cast<void**>(&tf.second), g.flag_bytes,
                                  hipHostMallocDefault), "hipHostMalloc flags");
        ds->tflag_cap[level] = { g.flag_bytes, g.flag_bytes };
        if (ds->eager)
            HIP_TRY(ds, hipHostMalloc(reinterpret_cast<void**>(&ds->h_tiles[level]),
                                      g.tile_bytes, hipHostMallocDefault),
                    "hipHostMalloc tile copy");
        ds->tiling[level] = { tile_rows, tile_cols };
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(ds);
    }
}

int
aqz_ds_take_frame_tiled(aqz_ds* ds,
                        uint32_t level,
                        uint32_t tile_rows,
                        uint32_t tile_cols,
                        void* dst,
                        size_t cap,
                        uint8_t* tile_nonzero,
                        size_t* nbytes,
                        int* has_frame)
{
    try {
        if (!ds || !has_frame)
            return AQZ_INVALID_ARGUMENT;
        *has_frame = 0;
        if (int rc = settle(ds))
            return rc;
        return take_tiled(ds, level, tile_rows, tile_cols, dst, cap, tile_nonzero, nbytes,
                          has_frame);
    } catch (...) {
        return ABI_GUARD_FAIL(ds);
    }
}

int
aqz_ds_set_input_transpose(aqz_ds* ds, int transpose)
{
    try {
        if (!ds)
            return AQZ_INVALID_ARGUMENT;
        if (int rc = settle(ds))
            return rc;
        if (int rc = bind_device(ds))
            return rc;
        if (transpose && !ds->d_tin) {
            HIP_TRY(ds, hipStreamSynchronize(ds->stream), "hipStreamSynchronize");
            HIP_TRY(ds, hipMalloc(&ds->d_tin, ds->bytes[0]), "hipMalloc transposed input");
            ds->device_bytes += ds->bytes[0];
        }
        ds->transpose = transpose != 0;
        ds->last_input = nullptr;
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(ds);
    }
}

int
aqz_ds_take_input_frame(aqz_ds* ds,
                        uint32_t tile_rows,
                        uint32_t tile_cols,
                        void* dst,
                        size_t cap,
                        uint8_t* tile_nonzero,
                        size_t* nbytes,
                        int* has_frame)
{
    try {
        if (!ds || !has_frame)
            return AQZ_INVALID_ARGUMENT;
        *has_frame = 0;
        if (int rc = settle(ds))
            return rc;
        if ((tile_rows == 0) != (tile_cols == 0))
            return ds->fail_arg("take_input_frame: tile_rows and tile_cols must both be 0 "
                                "or both be nonzero");
        if (!ds->last_input)
            return AQZ_OK;
        const bool tiled = tile_rows != 0;
        const TileGeom g = tiled ? tile_geom(ds, 0, tile_rows, tile_cols)
                                 : TileGeom{ 1, ds->bytes[0], 0 };
        *has_frame = 1;
        if (nbytes)
            *nbytes = g.tile_bytes;
        if (!dst)
            return AQZ_OK;
        if (cap < g.tile_bytes)
            return ds->fail_arg("take_input_frame: buffer too small");
        if (int rc = bind_device(ds))
            return rc;
        if (tiled) {
            if (int rc = tile_to_host(ds, ds->last_input, ds->lv[0], tile_rows, tile_cols, g,
                                      dst, tile_nonzero))
                return rc;
        } else {
            HIP_TRY(ds,
                    hipMemcpyAsync(dst, ds->last_input, g.tile_bytes, hipMemcpyDeviceToHost,
                                   ds->stream),
                    "hipMemcpyAsync D2H");
            HIP_TRY(ds, hipStreamSynchronize(ds->stream), "hipStreamSynchronize");
        }
        ds->last_input = nullptr;
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(ds);
    }
}

int
aqz_transpose_frame_device(int dtype,
                           const void* device_src,
                           uint32_t rows,
                           uint32_t cols,
                           void* device_dst,
                           void* hip_stream)
{
    try {
        if (!aqz::dtype_valid(dtype) || !device_src || !device_dst || rows == 0 || cols == 0) {
            set_global_error("transpose_frame_device: invalid argument");
            return AQZ_INVALID_ARGUMENT;
        }
        const hipError_t e = aqz::launch_transpose(dtype, device_src, rows, cols, device_dst,
                                                   static_cast<hipStream_t>(hip_stream));
        if (e != hipSuccess) {
            set_global_error("transpose_frame_device: %s", hipGetErrorString(e));
            return e == hipErrorInvalidValue ? AQZ_INVALID_ARGUMENT : AQZ_INTERNAL_ERROR;
        }
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(nullptr);
    }
}

int
aqz_tile_frame_device(int dtype,
                      const void* device_frame,
                      uint32_t width,
                      uint32_t height,
                      uint32_t tile_rows,
                      uint32_t tile_cols,
                      void* device_tiles,
                      uint32_t* device_nonzero,
                      void* hip_stream)
{
    try {
        if (!aqz::dtype_valid(dtype) || !device_frame || !device_tiles ||
            !device_nonzero) {
            set_global_error("tile_frame_device: invalid argument");
            return AQZ_INVALID_ARGUMENT;
        }
        const hipError_t e = aqz::launch_tile_frame(
          dtype, device_frame, width, height, tile_rows, tile_cols, device_tiles,
          device_nonzero, static_cast<hipStream_t>(hip_stream));
        if (e != hipSuccess) {
            set_global_error("tile_frame_device: %s", hipGetErrorString(e));
            return e == hipErrorInvalidValue ? AQZ_INVALID_ARGUMENT : AQZ_INTERNAL_ERROR;
        }
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(nullptr);
    }
}

uint32_t
aqz_tile_slices(uint32_t tile_rows, uint32_t tile_cols)
{
    return aqz::tile_slices(tile_rows, tile_cols);
}

int
aqz_tile_frame_device_sliced(int dtype,
                             const void* device_frame,
                             uint32_t width,
                             uint32_t height,
                             uint32_t tile_rows,
                             uint32_t tile_cols,
                             void* device_tiles,
                             uint8_t* device_slice_flags,
                             void* hip_stream)
{
    try {
        if (!aqz::dtype_valid(dtype) || !device_frame || !device_tiles || !device_slice_flags) {
            set_global_error("tile_frame_device_sliced: invalid argument");
            return AQZ_INVALID_ARGUMENT;
        }
        const hipError_t e = aqz::launch_tile_frame_sliced(
          dtype, device_frame, width, height, tile_rows, tile_cols, device_tiles,
          device_slice_flags, static_cast<hipStream_t>(hip_stream));
        if (e != hipSuccess) {
            set_global_error("tile_frame_device_sliced: %s", hipGetErrorString(e));
            return e == hipErrorInvalidValue ? AQZ_INVALID_ARGUMENT : AQZ_INTERNAL_ERROR;
        }
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(nullptr);
    }
}

int
aqz_ds_run_device_batch(aqz_ds* ds,
                        const void* device_frames,
                        uint32_t n_frames,
                        void* const* device_out_levels,
                        uint32_t* out_counts,
                        void* hip_stream)
{
    try {
        if (!ds)
            return AQZ_INVALID_ARGUMENT;
        if (int rc = settle(ds))
            return rc;
        if (ds->transpose)
            return ds->fail_arg("ds_run_device_batch: input transposition applies to the per-frame path "
                                "(add_frame / add_device_frame) only");
        ds->last_input = nullptr;
        if (!device_frames || !device_out_levels)
            return ds->fail_arg("run_device_batch: null buffer");
        for (uint32_t l = 1; l < ds->n; ++l)
            if (!device_out_levels[l])
                return ds->fail_arg("run_device_batch: null output for level " +
                                    std::to_string(l));
        if (int rc = bind_device(ds))
            return rc;
        // The batch runs on the caller's stream.  The fused paths touch only
        // the caller's buffers; the per-frame fallback reads and writes the
        // handle's device state (the stored Z plane, level slots) that earlier
        // add_frame calls left queued on ds->stream, and later add_frame calls
        // must see what it wrote.  So the fallback joins the two streams both
        // ways (joining on every batch put a cross-stream wait in front of
        // each fused launch), and the guard restores ds->stream on
        // every exit, exceptions included.
        struct StreamSwap
        {
            aqz_ds* ds;
            hipStream_t saved, user;
            bool joined = false;
            void enter() { ds->stream = user ? user : saved; }
            hipError_t join()
            {
                if (!user || user == saved)
                    return hipSuccess;
                hipError_t e = hipEventRecord(ds->join, saved);
                if (e == hipSuccess)
                    e = hipStreamWaitEvent(user, ds->join, 0);
                joined = e == hipSuccess;
                return e;
            }
            ~StreamSwap()
            {
                if (joined && hipEventRecord(ds->join, ds->stream) == hipSuccess)
                    (void)hipStreamWaitEvent(saved, ds->join, 0);
                ds->stream = saved;
            }
        } swap{ ds, ds->stream, static_cast<hipStream_t>(hip_stream) };
        swap.enter();

        std::vector<uint32_t> emitted(ds->n, 0);
        int rc = AQZ_OK;

        bool pure_xy = ds->n > 1;
        bool pure_xyz = ds->n > 1;
        for (uint32_t l = 1; l < ds->n; ++l) {
            pure_xy = pure_xy && ds->xy[l] && !ds->zh[l];
            // every level halves XY and Z, no odd stack (no pass-through plane)
            // and no stored earlier plane: planes pair up consecutively
            pure_xyz = pure_xyz && ds->xy[l] && ds->zh[l] &&
                       ds->lv[l - 1].planes % 2 == 0 && !ds->has_partial[l];
        }
        pure_xyz = pure_xyz && n_frames > 0 && (n_frames % (1u << (ds->n - 1))) == 0;

        // Plan runs of up to `maxk` levels per launch.  A 2-D batch always stays
        // batched: a run the fused cascade cannot take (width or alignment) runs
        // as one batched single-level generic launch per level.  A volume batch
        // is all-or-nothing (its fallback is the per-frame state machine).
        struct Run
        {
            uint32_t L, k;
            bool fused;
        };
        auto plan_runs = [&](uint32_t maxk, bool volume) {
            std::vector<Run> runs;
            const void* src = device_frames;
            for (uint32_t L = 1; L < ds->n;) {
                const uint32_t k = std::min<uint32_t>(ds->n - L, maxk);
                aqz::LevelOut o[aqz::kMaxFusedLevels];
                for (uint32_t j = 0; j < k; ++j)
                    o[j] = { device_out_levels[L + j], elems(ds, L + j),
                             ds->lv[L + j].width, ds->lv[L + j].height };
                const aqz_level_desc& a = ds->lv[L - 1];
                const bool ok =
                  volume ? aqz::volume_supported(ds->dtype, src, a.width, a.height, o, int(k))
                         : aqz::cascade_supported(ds->dtype, src, elems(ds, L - 1), a.width,
                                                  a.height, o, int(k));
                if (!ok && volume)
                    return std::vector<Run>{};
                runs.push_back({ L, k, ok });
                src = o[k - 1].ptr;
                L += k;
            }
            return runs;
        };

        std::vector<Run> runs;
        bool volume = false;
        if (pure_xy && n_frames > 0) {
            runs = plan_runs(aqz::kMaxFusedLevels, false);
        } else if (pure_xyz) {
            runs = plan_runs(aqz::kMaxVolumeLevels, true);
            volume = true;
        }

        if (!runs.empty()) {
            // Whole batch in batched launches; every frame / plane group independent.
            const void* src = device_frames;
            uint32_t planes = n_frames;
            bool all_fused = true;
            for (const Run& run : runs) {
                aqz::LevelOut o[aqz::kMaxFusedLevels];
                for (uint32_t j = 0; j < run.k; ++j)
                    o[j] = { device_out_levels[run.L + j], elems(ds, run.L + j),
                             ds->lv[run.L + j].width, ds->lv[run.L + j].height };
                const aqz_level_desc& a = ds->lv[run.L - 1];
                hipError_t e = hipSuccess;
                if (volume) {
                    e = aqz::launch_volume(ds->dtype, ds->method, src, elems(ds, run.L - 1),
                                           a.width, a.height, o, int(run.k), planes, ds->stream);
                } else if (run.fused) {
                    e = aqz::launch_cascade(ds->dtype, ds->method, src, elems(ds, run.L - 1),
                                            a.width, a.height, o, int(run.k), n_frames,
                                            ds->stream);
                } else {
                    all_fused = false;
                    const void* s = src;
                    for (uint32_t j = 0; j < run.k && e == hipSuccess; ++j) {
                        const aqz_level_desc& in = ds->lv[run.L + j - 1];
                        e = aqz::launch_xy_generic(ds->dtype, ds->method, s,
                                                   elems(ds, run.L + j - 1), in.width, in.height,
                                                   o[j], n_frames, ds->stream);
                        s = o[j].ptr;
                    }
                }
                if (e != hipSuccess) {
                    rc = ds->fail(e, volume ? "batch volume" : "batch cascade");
                    break;
                }
                src = o[run.k - 1].ptr;
                if (volume)
                    planes >>= run.k;
            }
            // a failed launch leaves the counts (and the odd-stack state they
            // carry) where they were
            if (rc == AQZ_OK) {
                for (uint32_t l = 0; l < ds->n; ++l) {
                    emitted[l] = volume ? (n_frames >> l) : n_frames;
                    ds->count[l] += emitted[l];
                }
            }
            ds->last_batch_kind = volume ? 2 : (all_fused ? 1 : 3);
        } else {
            ds->last_batch_kind = 0;
            if (hipError_t e = swap.join(); e != hipSuccess)
                return ds->fail(e, "run_device_batch: stream join");
            Sink sink;
            sink.batch = true;
            sink.out = device_out_levels;
            sink.emitted = &emitted;
            const uint8_t* base = static_cast<const uint8_t*>(device_frames);
            for (uint32_t i = 0; i < n_frames && rc == AQZ_OK; ++i)
                rc = process_frame(ds, base + size_t(i) * ds->bytes[0], sink);
            emitted[0] = n_frames;
        }
        if (out_counts)
            std::copy(emitted.begin(), emitted.end(), out_counts);
        return rc;
    } catch (...) {
        return ABI_GUARD_FAIL(ds);
    }
}

} // extern "C"

namespace {

// Per-level frame offsets of a chunk-lattice batch into the device (elements),
// through one half of the pinned staging; returns the device pointers.
int
stage_lattice(aqz_ds* ds, const aqz_chunk_lattice* lat, uint32_t n_frames, hipStream_t stream,
              std::vector<const uint64_t*>* dev, int* half_out)
{
    const size_t need = size_t(ds->n) * n_frames;
    if (ds->lattice_half < need) {
        for (hipEvent_t e : ds->lattice_done)
            if (e)
                HIP_TRY(ds, hipEventSynchronize(e), "hipEventSynchronize lattice");
        (void)hipFree(ds->d_lattice);
        (void)hipHostFree(ds->h_lattice);
        ds->d_lattice = nullptr;
        ds->h_lattice = nullptr;
        ds->lattice_half = 0;
        HIP_TRY(ds, hipMalloc(reinterpret_cast<void**>(&ds->d_lattice), 2 * need * 8),
                "hipMalloc lattice");
        HIP_TRY(ds, hipHostMalloc(reinterpret_cast<void**>(&ds->h_lattice), 2 * need * 8),
                "hipHostMalloc lattice");
        ds->lattice_half = need;
        for (hipEvent_t& e : ds->lattice_done)
            if (!e)
                HIP_TRY(ds, hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
    }
    const int half = int(ds->lattice_calls++ & 1);
    // the batch two calls back read this half: it must have finished
    HIP_TRY(ds, hipEventSynchronize(ds->lattice_done[half]), "hipEventSynchronize lattice");
    uint64_t* h = ds->h_lattice + size_t(half) * ds->lattice_half;
    uint64_t* d = ds->d_lattice + size_t(half) * ds->lattice_half;
    dev->assign(ds->n, nullptr);
    for (uint32_t l = 1; l < ds->n; ++l)
        for (uint32_t k = 0; k < n_frames; ++k)
            h[size_t(l) * n_frames + k] = lat[l].frame_offset_bytes[k] / ds->bpp;
    HIP_TRY(ds, hipMemcpyAsync(d, h, need * 8, hipMemcpyHostToDevice, stream), "lattice upload");
    for (uint32_t l = 1; l < ds->n; ++l)
        (*dev)[l] = d + size_t(l) * n_frames;
    *half_out = half;
    return AQZ_OK;
}

// aqz_ds_run_device_batch_tiled (lat == nullptr: tiles of a frame back to
// back, frames back to back) and aqz_ds_run_device_batch_chunked (every tile
// into its chunk of the lattice).
int
run_tiled(aqz_ds* ds,
          const char* who,
          const void* device_frames,
          uint32_t n_frames,
          const uint32_t* tile_rows,
          const uint32_t* tile_cols,
          void* const* device_out_levels,
          const aqz_chunk_lattice* lat,
          uint8_t* const* device_tile_nonzero,
          uint32_t* out_counts,
          void* hip_stream)
{
    const std::string w(who);
    if (int rc = settle(ds))
        return rc;
    if (ds->transpose)
        return ds->fail_arg(w + ": input transposition applies to the per-frame path only");
    ds->last_input = nullptr;
    if (!device_frames || (!lat && (!device_out_levels || !tile_rows || !tile_cols)))
        return ds->fail_arg(w + ": null argument");
    if (ds->n < 2)
        return ds->fail_arg(w + ": the pyramid has no level to tile");
    for (uint32_t l = 1; l < ds->n; ++l) {
        if (!ds->xy[l] || ds->zh[l])
            return ds->fail_arg(w + ": pure-XY (2-D) pyramids only; level " + std::to_string(l) +
                                " does not halve XY alone");
        const uint32_t tr = lat ? lat[l].tile_rows : tile_rows[l];
        const uint32_t tc = lat ? lat[l].tile_cols : tile_cols[l];
        const void* out = lat ? lat[l].device_base : device_out_levels[l];
        if (!out || !tr || !tc)
            return ds->fail_arg(w + ": level " + std::to_string(l) +
                                " needs an output and a nonzero tile shape");
        if (lat) {
            // every tile of every frame inside the lattice buffer: a bad
            // offset must be an argument error here, not a device fault
            const aqz_chunk_lattice& c = lat[l];
            const uint64_t ntiles = uint64_t((ds->lv[l].width + tc - 1) / tc) *
                                    ((ds->lv[l].height + tr - 1) / tr);
            const uint64_t tile_bytes = uint64_t(tr) * tc * ds->bpp;
            if (!c.frame_offset_bytes || c.chunk_stride_bytes % ds->bpp ||
                c.chunk_stride_bytes < tile_bytes)
                return ds->fail_arg(w + ": level " + std::to_string(l) +
                                    ": chunk stride must hold a tile and be a multiple of the "
                                    "pixel size, and frame offsets are required");
            const uint64_t extent = (ntiles - 1) * c.chunk_stride_bytes + tile_bytes;
            for (uint32_t k = 0; k < n_frames; ++k) {
                const uint64_t off = c.frame_offset_bytes[k];
                if (off % ds->bpp || off > c.capacity_bytes || c.capacity_bytes - off < extent)
                    return ds->fail_arg(w + ": level " + std::to_string(l) + " frame " +
                                        std::to_string(k) + ": offset " + std::to_string(off) +
                                        " puts its tiles outside the lattice buffer");
            }
        }
    }
    if (int rc = bind_device(ds))
        return rc;
    hipStream_t stream = hip_stream ? static_cast<hipStream_t>(hip_stream) : ds->stream;
    std::vector<const uint64_t*> d_off;
    int half = -1;
    if (lat)
        if (int rc = stage_lattice(ds, lat, n_frames, stream, &d_off, &half))
            return rc;
    // From here on the staged half's upload is queued on `stream`: whatever
    // the exit, record the event that guards the pinned half, so a later call
    // never rewrites it while that copy may still read it.
    struct LatticeGuard
    {
        aqz_ds* ds;
        int half;
        hipStream_t stream;
        ~LatticeGuard()
        {
            if (half >= 0)
                (void)hipEventRecord(ds->lattice_done[half], stream);
        }
    } lattice_guard{ ds, half, stream };
    // Runs of up to kMaxFusedLevels levels; a run that feeds another also
    // writes its last level row-major into one half of d_chain (the runs
    // alternate halves, so a run never reads the half it writes).  The
    // first chained level is the largest: 1/256 of the base after 4 levels.
    const uint32_t first_feed = aqz::kMaxFusedLevels;
    const bool chained = first_feed + 1 < ds->n;
    // A previous batch may still be reading or writing d_chain on another
    // stream: order this one behind it.  Only pyramids deeper than one fused
    // run touch d_chain, so only they wait and record.  Once the wait is
    // queued, chain_done is recorded on every way out (ChainGuard), so a
    // failure after some runs were queued still fences them.
    if (chained) {
        if (ds->chain_done)
            HIP_TRY(ds, hipStreamWaitEvent(stream, ds->chain_done, 0), "hipStreamWaitEvent chain");
        else
            HIP_TRY(ds, hipEventCreateWithFlags(&ds->chain_done, hipEventDisableTiming), "event");
    }
    struct ChainGuard
    {
        aqz_ds* ds;
        hipStream_t stream;
        bool on;
        ~ChainGuard()
        {
            if (on)
                (void)hipEventRecord(ds->chain_done, stream);
        }
    } chain_guard{ ds, stream, chained };
    if (chained) {
        const size_t chain_half = size_t(n_frames) * ds->bytes[first_feed];
        if (ds->d_chain_bytes < 2 * chain_half) {
            HIP_TRY(ds, hipStreamSynchronize(stream), "hipStreamSynchronize");
            (void)hipFree(ds->d_chain);
            ds->d_chain = nullptr;
            ds->d_chain_bytes = 0;
            HIP_TRY(ds, hipMalloc(&ds->d_chain, 2 * chain_half), "hipMalloc chain");
            ds->d_chain_bytes = 2 * chain_half;
        }
    }
    const void* src = device_frames;
    for (uint32_t L = 1, run = 0; L < ds->n; ++run) {
        const uint32_t k = std::min<uint32_t>(ds->n - L, aqz::kMaxFusedLevels);
        const bool feeds = L + k < ds->n;
        aqz::LevelOut o[aqz::kMaxFusedLevels];
        aqz::TiledOut t[aqz::kMaxFusedLevels];
        for (uint32_t j = 0; j < k; ++j) {
            const uint32_t l = L + j;
            o[j] = { nullptr, elems(ds, l), ds->lv[l].width, ds->lv[l].height };
            uint8_t* nz = device_tile_nonzero ? device_tile_nonzero[l] : nullptr;
            if (lat)
                t[j] = { lat[l].device_base, lat[l].tile_rows, lat[l].tile_cols, nz, d_off[l],
                         lat[l].chunk_stride_bytes / ds->bpp };
            else
                t[j] = { device_out_levels[l], tile_rows[l], tile_cols[l], nz };
        }
        void* chain = static_cast<uint8_t*>(ds->d_chain) + (run & 1) * (ds->d_chain_bytes / 2);
        if (feeds)
            o[k - 1].ptr = chain;
        const aqz_level_desc& a = ds->lv[L - 1];
        if (!aqz::cascade_supported(ds->dtype, src, elems(ds, L - 1), a.width, a.height, o,
                                    int(k)))
            return ds->fail_arg(w + ": level " + std::to_string(L - 1) +
                                " is narrower than one vector load (" + std::to_string(a.width) +
                                " px)");
        const hipError_t e = aqz::launch_cascade_tiled(ds->dtype, ds->method, src,
                                                       elems(ds, L - 1), a.width, a.height, o, t,
                                                       int(k), n_frames, stream);
        if (e != hipSuccess)
            return e == hipErrorInvalidValue ? ds->fail_arg(w + ": unsupported geometry")
                                             : ds->fail(e, "batch tiled cascade");
        src = chain;
        L += k;
    }
    for (uint32_t l = 0; l < ds->n; ++l) {
        ds->count[l] += n_frames;
        if (out_counts)
            out_counts[l] = n_frames;
    }
    ds->last_batch_kind = 4;
    return AQZ_OK;
}

} // namespace

extern "C" {

int
aqz_ds_run_device_batch_tiled(aqz_ds* ds,
                              const void* device_frames,
                              uint32_t n_frames,
                              const uint32_t* tile_rows,
                              const uint32_t* tile_cols,
                              void* const* device_out_levels,
                              uint8_t* const* device_tile_nonzero,
                              uint32_t* out_counts,
                              void* hip_stream)
{
    try {
        if (!ds)
            return AQZ_INVALID_ARGUMENT;
        return run_tiled(ds, "run_device_batch_tiled", device_frames, n_frames, tile_rows,
                         tile_cols, device_out_levels, nullptr, device_tile_nonzero, out_counts,
                         hip_stream);
    } catch (...) {
        return ABI_GUARD_FAIL(ds);
    }
}

int
aqz_ds_run_device_batch_chunked(aqz_ds* ds,
                                const void* device_frames,
                                uint32_t n_frames,
                                const aqz_chunk_lattice* lattices,
                                uint8_t* const* device_tile_nonzero,
                                uint32_t* out_counts,
                                void* hip_stream)
{
    try {
        if (!ds)
            return AQZ_INVALID_ARGUMENT;
        if (!lattices)
            return ds->fail_arg("run_device_batch_chunked: null lattices");
        return run_tiled(ds, "run_device_batch_chunked", device_frames, n_frames, nullptr,
                         nullptr, nullptr, lattices, device_tile_nonzero, out_counts, hip_stream);
    } catch (...) {
        return ABI_GUARD_FAIL(ds);
    }
}

uint32_t
aqz_ds_tiled_flag_slots(const aqz_ds* ds, uint32_t level, uint32_t tile_rows, uint32_t tile_cols)
{
    if (!ds || level == 0 || level >= ds->n || tile_rows == 0 || tile_cols == 0)
        return 0;
    // the fused run holding `level`: levels 1-4, 5-8, ... (kMaxFusedLevels)
    const uint32_t start = 1 + ((level - 1) / aqz::kMaxFusedLevels) * aqz::kMaxFusedLevels;
    const uint32_t k = std::min<uint32_t>(ds->n - start, aqz::kMaxFusedLevels);
    const uint32_t s = aqz::cascade_tiled_slots(ds->dtype, ds->lv[start - 1].width, int(k),
                                                int(level - start + 1), tile_rows, tile_cols,
                                                nullptr);
    return s ? s : 1;
}

namespace {

// Frames per pipeline group: about 64 MiB of input per group, and a whole
// number of plane groups when the pyramid pairs planes (so fused volume
// launches see aligned groups).
uint32_t
pipe_group(const aqz_ds* ds, uint32_t n_frames)
{
    uint32_t g = uint32_t(std::max<size_t>(1, (size_t(64) << 20) / ds->bytes[0]));
    uint32_t align = 1;
    for (uint32_t l = 1; l < ds->n; ++l)
        if (ds->zh[l])
            align <<= 1;
    g = std::max(align, (g / align) * align);
    return std::min(g, std::max(align, n_frames));
}

int
ensure_pipe(aqz_ds* ds, uint32_t group)
{
    auto& p = ds->pipe;
    if (p.group >= group)
        return AQZ_OK;
    for (int b = 0; b < 2; ++b) {
        (void)hipFree(p.d_in[b]);
        p.d_in[b] = nullptr;
        for (void* q : p.d_out[b])
            (void)hipFree(q);
        p.d_out[b].assign(ds->n, nullptr);
    }
    if (!p.s_in) {
        HIP_TRY(ds, hipStreamCreateWithFlags(&p.s_in, hipStreamNonBlocking), "stream");
        HIP_TRY(ds, hipStreamCreateWithFlags(&p.s_work, hipStreamNonBlocking), "stream");
        HIP_TRY(ds, hipStreamCreateWithFlags(&p.s_out, hipStreamNonBlocking), "stream");
        for (int b = 0; b < 2; ++b) {
            HIP_TRY(ds, hipEventCreateWithFlags(&p.in_done[b], hipEventDisableTiming), "event");
            HIP_TRY(ds, hipEventCreateWithFlags(&p.work_done[b], hipEventDisableTiming), "event");
            HIP_TRY(ds, hipEventCreateWithFlags(&p.out_done[b], hipEventDisableTiming), "event");
            // start "done" so the first waits pass
            HIP_TRY(ds, hipEventRecord(p.work_done[b], p.s_work), "event");
            HIP_TRY(ds, hipEventRecord(p.out_done[b], p.s_out), "event");
        }
    }
    for (int b = 0; b < 2; ++b) {
        HIP_TRY(ds, hipMalloc(&p.d_in[b], size_t(group) * ds->bytes[0]), "hipMalloc pipe");
        for (uint32_t l = 1; l < ds->n; ++l)
            HIP_TRY(ds, hipMalloc(&p.d_out[b][l], size_t(group) * ds->bytes[l]),
                    "hipMalloc pipe");
    }
    p.group = group;
    return AQZ_OK;
}

} // namespace

int
aqz_ds_run_host_batch(aqz_ds* ds,
                      const void* host_frames,
                      uint32_t n_frames,
                      void* const* host_out_levels,
                      uint32_t* out_counts)
{
    try {
        if (!ds)
            return AQZ_INVALID_ARGUMENT;
        if (int rc = settle(ds))
            return rc;
        if (ds->transpose)
            return ds->fail_arg("ds_run_host_batch: input transposition applies to the per-frame path "
                                "(add_frame / add_device_frame) only");
        ds->last_input = nullptr;
        if (!host_frames || !host_out_levels)
            return ds->fail_arg("run_host_batch: null buffer");
        for (uint32_t l = 1; l < ds->n; ++l)
            if (!host_out_levels[l])
                return ds->fail_arg("run_host_batch: null output for level " +
                                    std::to_string(l));
        if (int rc = bind_device(ds))
            return rc;
        const uint32_t group = pipe_group(ds, n_frames);
        if (int rc = ensure_pipe(ds, group))
            return rc;
        auto& p = ds->pipe;
        std::vector<uint32_t> total(ds->n, 0);
        const uint8_t* src = static_cast<const uint8_t*>(host_frames);
        int rc = AQZ_OK;
        uint32_t k = 0;
        // Any failure below still drains all three streams before returning, so
        // no copy is left reading or writing the caller's buffers.
        auto drain = [&](int code) {
            (void)hipStreamSynchronize(p.s_in);
            (void)hipStreamSynchronize(p.s_work);
            (void)hipStreamSynchronize(p.s_out);
            return code;
        };
    #define HIP_TRY_DRAIN(ds, expr, what)                                          \
        do {                                                                       \
            hipError_t e_ = (expr);                                                \
            if (e_ != hipSuccess)                                                  \
                return drain((ds)->fail(e_, what));                                \
        } while (0)
        for (uint32_t f0 = 0; f0 < n_frames && rc == AQZ_OK; f0 += group, ++k) {
            const int b = int(k & 1);
            const uint32_t g = std::min(group, n_frames - f0);
            // upload: buffer b is free once group k-2's kernels are done with it
            HIP_TRY_DRAIN(ds, hipStreamWaitEvent(p.s_in, p.work_done[b], 0), "wait");
            HIP_TRY_DRAIN(ds,
                    hipMemcpyAsync(p.d_in[b], src + size_t(f0) * ds->bytes[0],
                                   size_t(g) * ds->bytes[0], hipMemcpyHostToDevice,
                                   p.s_in),
                    "hipMemcpyAsync H2D");
            HIP_TRY_DRAIN(ds, hipEventRecord(p.in_done[b], p.s_in), "event");
            // kernels: after the upload, and after group k-2's download of d_out[b]
            HIP_TRY_DRAIN(ds, hipStreamWaitEvent(p.s_work, p.in_done[b], 0), "wait");
            HIP_TRY_DRAIN(ds, hipStreamWaitEvent(p.s_work, p.out_done[b], 0), "wait");
            std::vector<uint32_t> counts(ds->n, 0);
            rc = aqz_ds_run_device_batch(ds, p.d_in[b], g, p.d_out[b].data(),
                                         counts.data(), p.s_work);
            if (rc)
                return drain(rc);
            HIP_TRY_DRAIN(ds, hipEventRecord(p.work_done[b], p.s_work), "event");
            // download every frame this group emitted, appended per level
            HIP_TRY_DRAIN(ds, hipStreamWaitEvent(p.s_out, p.work_done[b], 0), "wait");
            for (uint32_t l = 1; l < ds->n; ++l) {
                if (!counts[l])
                    continue;
                uint8_t* dst = static_cast<uint8_t*>(host_out_levels[l]) +
                               size_t(total[l]) * ds->bytes[l];
                HIP_TRY_DRAIN(ds,
                        hipMemcpyAsync(dst, p.d_out[b][l], size_t(counts[l]) * ds->bytes[l],
                                       hipMemcpyDeviceToHost, p.s_out),
                        "hipMemcpyAsync D2H");
                total[l] += counts[l];
            }
            HIP_TRY_DRAIN(ds, hipEventRecord(p.out_done[b], p.s_out), "event");
        }
        drain(AQZ_OK);
        total[0] = n_frames;
        if (out_counts)
            std::copy(total.begin(), total.end(), out_counts);
        return rc;
    #undef HIP_TRY_DRAIN
    } catch (...) {
        return ABI_GUARD_FAIL(ds);
    }
}

int
aqz_ds_last_batch_kind(const aqz_ds* ds)
{
    return ds ? ds->last_batch_kind : -1;
}

uint64_t
aqz_ds_stream_tiled_runs(const aqz_ds* ds)
{
    return ds ? ds->stream_tiled_runs : 0;
}

size_t
aqz_ds_level_bytes(const aqz_ds* ds, uint32_t level)
{
    return (ds && level < ds->n) ? ds->bytes[level] : 0;
}

uint32_t
aqz_ds_level_count(const aqz_ds* ds)
{
    return ds ? ds->n : 0;
}

int
aqz_ds_device(const aqz_ds* ds)
{
    return ds ? ds->device : -1;
}

size_t
aqz_ds_device_memory_usage(const aqz_ds* ds)
{
    return ds ? ds->device_bytes : 0;
}

const char*
aqz_ds_last_error(const aqz_ds* ds)
{
    return ds ? ds->err.c_str() : "null handle";
}

const char*
aqz_last_error(void)
{
    return g_last_error.c_str();
}

const char*
aqz_method_name(int method)
{
    // Downsampler::downsampling_method, downsampler.cpp:422-437
    switch (method) {
        case AQZ_METHOD_DECIMATE:
            return "decimate";
        case AQZ_METHOD_MEAN:
            return "local_mean";
        case AQZ_METHOD_MIN:
            return "local_min";
        case AQZ_METHOD_MAX:
            return "local_max";
        default:
            return nullptr;
    }
}

const char*
aqz_method_metadata_json(int method)
{
    // Downsampler::get_metadata, downsampler.cpp:440-485: the OME
    // `multiscales[0].metadata` object (nlohmann::json serialises keys in
    // sorted order).
    switch (method) {
        case AQZ_METHOD_MEAN:
            return "{\"description\":\"The fields in the metadata describe how "
                   "to reproduce this multiscaling in scikit-image. The method "
                   "and its parameters are given here.\",\"kwargs\":{\"cval\":"
                   "\"0\",\"factors\":\"(2, 2)\"},\"method\":\"skimage."
                   "transform.downscale_local_mean\",\"version\":\"0.25.2\"}";
        case AQZ_METHOD_DECIMATE:
            return "{\"args\":[\"(slice(0, None, 2), slice(0, None, 2))\"],"
                   "\"description\":\"Subsampling by taking every 2nd "
                   "pixel/voxel (top-left corner of each 2x2 block). "
                   "Equivalent to numpy array slicing with stride 2.\","
                   "\"method\":\"np.ndarray.__getitem__\",\"version\":"
                   "\"2.2.6\"}";
        case AQZ_METHOD_MIN:
            return "{\"description\":\"Minimum pooling over 2x2 blocks. "
                   "Equivalent to reshaping into blocks and taking numpy.min "
                   "along block dimensions.\",\"kwargs\":{\"func\":\"np.min\"},"
                   "\"method\":\"skimage.measure.block_reduce\",\"version\":"
                   "\"0.25.2\"}";
        case AQZ_METHOD_MAX:
            return "{\"description\":\"Maximum pooling over 2x2 blocks. "
                   "Equivalent to reshaping into blocks and taking numpy.max "
                   "along block dimensions.\",\"kwargs\":{\"func\":\"np.max\"},"
                   "\"method\":\"skimage.measure.block_reduce\",\"version\":"
                   "\"0.25.2\"}";
        default:
            return nullptr;
    }
}

const char*
aqz_version(void)
{
    // AQZ_BUILD_ID: the source revision and time the Makefile built this
    // library from, so a bench line names the binary it ran
#ifndef AQZ_BUILD_ID
#define AQZ_BUILD_ID "unknown build"
#endif
    return "aqz-mi355x 0.2.0 (gfx950; " AQZ_BUILD_ID ")";
}

} // extern "C"

namespace aqz {

// aqz_last_error() text for the other C-ABI translation units
// (codec_runtime.cpp)
void
set_last_error(const std::string& msg)
{
    g_last_error = msg;
}

} // namespace aqz
