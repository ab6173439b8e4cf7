// ds_node.cpp — frame sharding over the GPUs of one node.
//
// An aqz_node is one aqz_ds handle per entry of `devices` (entries may repeat
// an ordinal: two handles on one GPU).  Frames are independent work units
// once the Z pairing is respected, so a host batch is cut into contiguous
// blocks of whole SHARD UNITS, one block per handle, and every handle runs
// the pipelined host batch (aqz_ds_run_host_batch: its own streams, its own
// PCIe link) on its block in its own host thread.  Each block writes its
// levels straight to the place its frames hold in the batch's outputs, so
// the caller gets every level in frame-id order — the order
// Array::write_frame insists on (array.cpp:179-189) — with no re-sequencing
// pass and no collective.
//
// Shard unit: the fewest level-0 frames after which add_frame's state
// (downsampler.cpp:306-401: partial Z planes, level_frame_count_ modulo an
// odd plane count) is back where a fresh handle starts, so a fresh handle
// fed a block from a unit boundary emits exactly what one handle fed the
// whole stream would.
//   * no level halves Z: 1 frame;
//   * h levels halve Z and the stack's planes P divide by 2^h: 2^h planes
//     (every intermediate plane count is even, so no plane passes through);
//   * otherwise: the whole stack, P planes.
// aqz_shard_unit checks the unit by running add_frame's control flow
// (counts only) over one unit from a fresh state.
//
// Streaming (aqz_node_add_frame / _take_frame / _flush): frame k goes to
// handle (k / unit) % D as an add_frame_async that takes every level in its
// background job, so up to D frames (one per handle) are in flight; levels
// are queued in submission order and handed out in the order one
// Downsampler emits them.
//
// Device-resident batch (aqz_node_run_device_batch, BASELINE config F: frame
// batches sharded across GPUs over xGMI): the batch and its level outputs
// live on one GPU.  The same contiguous blocks of whole shard units are
// dealt; a handle on the batch's own GPU runs its block in place, on the
// caller's stream; a handle on another GPU pulls its block over xGMI into
// node-owned staging on its own GPU (hipMemcpyPeerAsync: the GPUs' DMA
// engines over the point-to-point link, no kernel of ours and no host hop),
// runs the fused batch there and pushes each level back to the block's place
// in the outputs.  Each remote block moves in sub-batches through two staging
// slots on three streams (pull, pyramid, push), so a sub-batch's pull, the
// previous one's pyramid and the one before's push overlap; every block
// starts behind an event on the caller's stream and the caller's stream
// waits for every block's last push, so the call is as asynchronous as
// aqz_ds_run_device_batch.  One process drives every GPU: no RCCL
// communicator is involved, and nothing is reduced — the frames only move.
#include "aqz_downsampler.h"
#include "abi_guard.hh"
#include "ds_kernels.hh"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <string>
#include <thread>
#include <vector>

namespace {

// A handle's staging for device batches whose frames live on another GPU:
// two slots (input block + every level's output), three streams and the
// events that order slot reuse across sub-batches and calls.
struct PeerStage
{
    int device = -1;
    hipStream_t pull = nullptr, run = nullptr, push = nullptr;
    hipEvent_t pulled[2]{}, ran[2]{}, pushed[2]{}, done = nullptr;
    uint8_t* stage = nullptr; // 2 slots of slot_bytes
    size_t slot_bytes = 0;
    uint32_t next_slot = 0;
    std::vector<int> peers_on; // source ordinals this device has peer access to
};

} // namespace

struct aqz_node
{
    std::vector<aqz_ds*> ds;
    std::vector<aqz_level_desc> lv;
    std::vector<size_t> bytes;      // one frame per level
    // streaming takes per level: (tile_rows, tile_cols), (0, 0) row-major,
    // and the bytes of one taken frame (tiled: with the zero tile overhang)
    std::vector<std::pair<uint32_t, uint32_t>> tiling;
    std::vector<size_t> take_bytes;
    uint32_t unit = 1;              // level-0 frames per shard unit
    std::vector<uint32_t> per_unit; // frames each level emits per unit
    uint64_t frames = 0;            // level-0 frames taken so far (batches and stream)
    std::string err;

    // Streaming (aqz_node_add_frame): one add in flight per handle, each
    // taking every level into node-owned buffers in its background job
    // (aqz_ds_add_frame_async_take); adds are published in submission order.
    struct Add
    {
        uint32_t handle = 0;
        uint64_t frame = 0; // the stream's frame index (aqz_node_inputs_released)
        bool settled = false;
        std::vector<aqz_level_take> takes;
        std::vector<std::vector<uint8_t>> bufs;
    };
    std::deque<Add> adds;                             // submission order
    std::vector<Add*> in_flight;                      // per handle, or null
    std::vector<std::deque<std::vector<uint8_t>>> ready; // per level, in order
    std::vector<std::vector<uint8_t>> pool;           // spare take buffers

    // Device batches (aqz_node_run_device_batch): per handle, staging used
    // when the batch lives on another GPU; per source ordinal, the event
    // that marks the batch ready on the caller's stream.
    std::vector<PeerStage> peers;
    std::vector<hipEvent_t> ready_ev;
};

namespace aqz {

inline std::string*
abi_err_slot(aqz_node* n)
{
    return n ? &n->err : nullptr;
}

} // namespace aqz

namespace {

// add_frame's control flow with the pixels left out (downsampler.cpp:
// 306-401, emplace :599-605): which levels emit a frame.  `count` and
// `partial` carry the state between frames.
void
count_frame(const std::vector<aqz_level_desc>& lv,
            std::vector<uint64_t>& count,
            std::vector<uint8_t>& partial,
            std::vector<uint32_t>& emitted)
{
    ++count[0];
    for (size_t L = 1; L < lv.size(); ++L) {
        const uint32_t prev_planes = lv[L - 1].planes, next_planes = lv[L].planes;
        bool average = next_planes < prev_planes;
        if (prev_planes % 2 != 0 && count[L - 1] % prev_planes == 0)
            average = false;
        if (average && !partial[L]) {
            partial[L] = 1;
            return;
        }
        partial[L] = 0;
        ++count[L];
        ++emitted[L];
    }
}

int
fail(aqz_node* n, int rc, const std::string& what)
{
    n->err = what;
    return rc;
}

// The caller thread's current HIP device is restored on every exit: the
// handles bind their own ordinals, and a caller driving several GPUs from
// one thread must not find its later work moved to another one.
struct DeviceGuard
{
    int saved = -1;
    DeviceGuard()
    {
        if (hipGetDevice(&saved) != hipSuccess)
            saved = -1;
    }
    ~DeviceGuard()
    {
        if (saved >= 0)
            (void)hipSetDevice(saved);
    }
};

int
hip_fail(aqz_node* n, hipError_t e, const std::string& what)
{
    return fail(n, e == hipErrorOutOfMemory ? AQZ_OUT_OF_MEMORY : AQZ_INTERNAL_ERROR,
                what + ": " + hipGetErrorString(e));
}

void
release_peer(PeerStage& p)
{
    if (p.device < 0)
        return;
    (void)hipSetDevice(p.device);
    for (hipStream_t s : { p.pull, p.run, p.push })
        if (s)
            (void)hipStreamSynchronize(s);
    for (int k = 0; k < 2; ++k)
        for (hipEvent_t e : { p.pulled[k], p.ran[k], p.pushed[k] })
            if (e)
                (void)hipEventDestroy(e);
    if (p.done)
        (void)hipEventDestroy(p.done);
    for (hipStream_t s : { p.pull, p.run, p.push })
        if (s)
            (void)hipStreamDestroy(s);
    if (p.stage)
        (void)hipFree(p.stage);
    p = PeerStage{};
}

// Staging of handle h on its device, with two slots of at least `slot`
// bytes (grown, never shrunk; growth waits for the slots' last use).
int
peer_stage(aqz_node* n, uint32_t h, int src_device, size_t slot)
{
    PeerStage& p = n->peers[h];
    const int dev = aqz_ds_device(n->ds[h]);
    hipError_t e = hipSetDevice(dev);
    if (e != hipSuccess)
        return hip_fail(n, e, "node device batch: hipSetDevice");
    if (p.device < 0) {
        p.device = dev;
        for (hipStream_t* s : { &p.pull, &p.run, &p.push })
            if ((e = hipStreamCreateWithFlags(s, hipStreamNonBlocking)) != hipSuccess)
                return hip_fail(n, e, "node device batch: stream");
        for (int k = 0; k < 2; ++k)
            for (hipEvent_t* ev : { &p.pulled[k], &p.ran[k], &p.pushed[k] })
                if ((e = hipEventCreateWithFlags(ev, hipEventDisableTiming)) != hipSuccess)
                    return hip_fail(n, e, "node device batch: event");
        if ((e = hipEventCreateWithFlags(&p.done, hipEventDisableTiming)) != hipSuccess)
            return hip_fail(n, e, "node device batch: event");
    }
    // direct xGMI access to the batch's GPU where the pair has it (the copies
    // work either way; this keeps them off any host bounce), for every source
    // ordinal a call names, not only the first one
    if (dev != src_device &&
        std::find(p.peers_on.begin(), p.peers_on.end(), src_device) == p.peers_on.end()) {
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, dev, src_device) == hipSuccess && can) {
            e = hipDeviceEnablePeerAccess(src_device, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
                return hip_fail(n, e, "node device batch: peer access");
            (void)hipGetLastError(); // clear "already enabled"
        }
        p.peers_on.push_back(src_device);
    }
    if (p.slot_bytes < slot) {
        for (hipStream_t s : { p.pull, p.run, p.push })
            if ((e = hipStreamSynchronize(s)) != hipSuccess)
                return hip_fail(n, e, "node device batch: drain before growing staging");
        if (p.stage)
            (void)hipFree(p.stage);
        p.stage = nullptr;
        p.slot_bytes = 0;
        void* mem = nullptr;
        if ((e = hipMalloc(&mem, 2 * slot)) != hipSuccess)
            return hip_fail(n, e,
                            "node device batch: staging of " + std::to_string(2 * slot) +
                              " bytes on device " + std::to_string(dev));
        p.stage = static_cast<uint8_t*>(mem);
        p.slot_bytes = slot;
    }
    return AQZ_OK;
}

// Wait for handle h's add in flight; its takes become publishable.
int
settle_handle(aqz_node* n, uint32_t h)
{
    aqz_node::Add* a = n->in_flight[h];
    if (!a)
        return AQZ_OK;
    n->in_flight[h] = nullptr;
    const int rc = aqz_ds_wait(n->ds[h]);
    a->settled = true;
    if (rc)
        return fail(n, rc, "node add on handle " + std::to_string(h) + ": " +
                             aqz_ds_last_error(n->ds[h]));
    return AQZ_OK;
}

// Move the takes of every settled add at the front of the submission order
// to the per-level queues: each level's frames come out in the order a
// single Downsampler would have emitted them.
void
publish(aqz_node* n)
{
    while (!n->adds.empty() && n->adds.front().settled) {
        aqz_node::Add& a = n->adds.front();
        for (size_t L = 1; L < a.takes.size(); ++L) {
            if (a.takes[L].has_frame)
                n->ready[L].push_back(std::move(a.bufs[L]));
            else if (!a.bufs[L].empty())
                n->pool.push_back(std::move(a.bufs[L]));
        }
        n->adds.pop_front();
    }
}

// Settle, without waiting, the adds at the front of the submission order
// whose background job has finished: their levels can be handed out now
// rather than when their handle is next used.  Stops at the first add still
// running, since later adds publish only after it anyway.
int
settle_finished(aqz_node* n)
{
    for (auto& a : n->adds) {
        if (a.settled)
            continue;
        if (n->in_flight[a.handle] != &a)
            break;
        int done = 0;
        if (int rc = aqz_ds_poll(n->ds[a.handle], &done))
            return fail(n, rc, "node take: poll failed");
        if (!done)
            break;
        if (int rc = settle_handle(n, a.handle))
            return rc;
    }
    return AQZ_OK;
}

int
flush_all(aqz_node* n)
{
    int rc = AQZ_OK;
    // in submission order, so a failure reports the earliest failed add
    for (auto& a : n->adds)
        if (!a.settled && n->in_flight[a.handle] == &a) {
            const int r = settle_handle(n, a.handle);
            if (r && !rc)
                rc = r;
        }
    publish(n);
    return rc;
}

} // namespace

extern "C" {

int
aqz_shard_unit(const aqz_level_desc* levels,
               uint32_t n_levels,
               uint32_t* unit,
               uint32_t* frames_per_unit)
{
    try {
        if (!levels || n_levels == 0 || n_levels > AQZ_MAX_LEVELS || !unit) {
            aqz::set_last_error("shard_unit: bad arguments");
            return AQZ_INVALID_ARGUMENT;
        }
        uint32_t halvings = 0;
        for (uint32_t L = 1; L < n_levels; ++L)
            halvings += levels[L].planes < levels[L - 1].planes;
        const uint32_t planes = levels[0].planes;
        uint32_t u = 1;
        if (halvings > 0)
            u = (halvings < 32 && planes % (1u << halvings) == 0) ? (1u << halvings) : planes;
        if (u == 0) {
            aqz::set_last_error("shard_unit: Z halves but level 0 has no planes");
            return AQZ_INVALID_ARGUMENT;
        }
        // one unit from a fresh state must leave it fresh again: no stored
        // plane, and every count the odd-stack pass-through reads (level L's
        // when L has an odd plane count and L+1 halves Z) at a multiple of
        // that plane count
        std::vector<aqz_level_desc> lv(levels, levels + n_levels);
        std::vector<uint64_t> count(n_levels, 0);
        std::vector<uint8_t> partial(n_levels, 0);
        std::vector<uint32_t> emitted(n_levels, 0);
        for (uint32_t f = 0; f < u; ++f)
            count_frame(lv, count, partial, emitted);
        emitted[0] = u;
        for (uint32_t L = 0; L < n_levels; ++L) {
            bool fresh = !partial[L];
            if (L + 1 < n_levels && levels[L].planes % 2 != 0 &&
                levels[L + 1].planes < levels[L].planes)
                fresh = fresh && count[L] % levels[L].planes == 0;
            if (!fresh) {
                aqz::set_last_error("shard_unit: no shard unit restores the Z-pairing state");
                return AQZ_INVALID_ARGUMENT;
            }
        }
        *unit = u;
        if (frames_per_unit)
            std::copy(emitted.begin(), emitted.end(), frames_per_unit);
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(nullptr);
    }
}

int
aqz_node_create(const aqz_level_desc* levels,
                uint32_t n_levels,
                int dtype,
                int method,
                const int* devices,
                uint32_t n_devices,
                aqz_node** out)
{
    try {
        if (!out) {
            aqz::set_last_error("node_create: null output handle");
            return AQZ_INVALID_ARGUMENT;
        }
        *out = nullptr;
        if (!devices || n_devices == 0 || n_devices > 64) {
            aqz::set_last_error("node_create: need 1..64 device entries");
            return AQZ_INVALID_ARGUMENT;
        }
        // the reference's order: dtype, then method (downsampler.cpp:293-303)
        if (!aqz::dtype_valid(dtype)) {
            aqz::set_last_error("Invalid data type: " + std::to_string(dtype));
            return AQZ_INVALID_ARGUMENT;
        }
        if (!aqz::method_valid(method)) {
            aqz::set_last_error("Invalid downsampling method: " + std::to_string(method));
            return AQZ_INVALID_ARGUMENT;
        }
        uint32_t unit = 0;
        std::vector<uint32_t> per_unit(n_levels, 0);
        if (levels && n_levels > 0 && n_levels <= AQZ_MAX_LEVELS)
            if (int rc = aqz_shard_unit(levels, n_levels, &unit, per_unit.data()))
                return rc;
        DeviceGuard guard;
        auto* n = new aqz_node();
        for (uint32_t d = 0; d < n_devices; ++d) {
            aqz_ds* h = nullptr;
            // aqz_ds_create validates levels, dtype, method and the ordinal
            if (int rc = aqz_ds_create(levels, n_levels, dtype, method, devices[d], &h)) {
                aqz_node_destroy(n);
                return rc;
            }
            n->ds.push_back(h);
        }
        n->lv.assign(levels, levels + n_levels);
        for (uint32_t L = 0; L < n_levels; ++L)
            n->bytes.push_back(aqz_ds_level_bytes(n->ds[0], L));
        n->tiling.assign(n_levels, { 0u, 0u });
        n->take_bytes = n->bytes;
        n->unit = unit;
        n->per_unit = per_unit;
        n->in_flight.assign(n_devices, nullptr);
        n->ready.resize(n_levels);
        n->peers.resize(n_devices);
        *out = n;
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(nullptr);
    }
}

void
aqz_node_destroy(aqz_node* n)
{
    if (!n)
        return;
    DeviceGuard guard;
    // staging drains its streams before it is freed
    for (PeerStage& p : n->peers)
        release_peer(p);
    for (size_t d = 0; d < n->ready_ev.size(); ++d)
        if (n->ready_ev[d]) {
            (void)hipSetDevice(int(d));
            (void)hipEventDestroy(n->ready_ev[d]);
        }
    // aqz_ds_destroy settles a handle's add in flight before freeing it, so
    // no background take still writes into this node's buffers
    for (aqz_ds* h : n->ds)
        aqz_ds_destroy(h);
    delete n;
}

int
aqz_node_add_frame(aqz_node* n, const void* host_frame, size_t nbytes)
{
    try {
        if (!n)
            return AQZ_INVALID_ARGUMENT;
        DeviceGuard guard;
        if (!host_frame || nbytes != n->bytes[0])
            return fail(n, AQZ_INVALID_ARGUMENT,
                        "node_add_frame: frame of " + std::to_string(nbytes) + " bytes, expected " +
                          std::to_string(n->bytes[0]));
        const uint32_t D = uint32_t(n->ds.size());
        const uint32_t h = uint32_t((n->frames / n->unit) % D);
        // the handle's previous add (D units ago, or the previous frame of
        // this unit) must be done before its take buffers are reused
        if (int rc = settle_handle(n, h))
            return rc;
        publish(n);
        const uint32_t nl = uint32_t(n->lv.size());
        n->adds.emplace_back();
        aqz_node::Add& a = n->adds.back();
        a.handle = h;
        a.frame = n->frames;
        a.takes.assign(nl, aqz_level_take{});
        a.bufs.resize(nl);
        for (uint32_t L = 1; L < nl; ++L) {
            auto& b = a.bufs[L];
            if (!n->pool.empty()) {
                b = std::move(n->pool.back());
                n->pool.pop_back();
            }
            b.resize(n->take_bytes[L]);
            a.takes[L].mode = AQZ_TAKE_INTO;
            a.takes[L].tile_rows = n->tiling[L].first;
            a.takes[L].tile_cols = n->tiling[L].second;
            a.takes[L].dst = b.data();
            a.takes[L].cap = b.size();
        }
        const int rc = aqz_ds_add_frame_async_take(n->ds[h], host_frame, nbytes, a.takes.data());
        if (rc) {
            n->adds.pop_back();
            return fail(n, rc, std::string("node_add_frame: ") + aqz_ds_last_error(n->ds[h]));
        }
        n->in_flight[h] = &a;
        ++n->frames;
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(n);
    }
}

int
aqz_node_take_frame(aqz_node* n,
                    uint32_t level,
                    void* dst,
                    size_t cap,
                    size_t* nbytes,
                    int* has_frame)
{
    try {
        if (!n || !has_frame)
            return AQZ_INVALID_ARGUMENT;
        *has_frame = 0;
        if (nbytes)
            *nbytes = 0;
        if (level == 0 || level >= n->lv.size())
            return AQZ_OK;
        DeviceGuard guard;
        if (int rc = settle_finished(n))
            return rc;
        publish(n);
        auto& q = n->ready[level];
        if (q.empty())
            return AQZ_OK;
        if (nbytes)
            *nbytes = q.front().size();
        *has_frame = 1;
        if (!dst)
            return AQZ_OK; // size query: the frame stays queued
        if (cap < q.front().size())
            return fail(n, AQZ_INVALID_ARGUMENT, "node_take_frame: buffer too small");
        std::memcpy(dst, q.front().data(), q.front().size());
        n->pool.push_back(std::move(q.front()));
        q.pop_front();
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(n);
    }
}

int
aqz_node_flush(aqz_node* n)
{
    try {
        if (!n)
            return AQZ_INVALID_ARGUMENT;
        DeviceGuard guard;
        return flush_all(n);
    } catch (...) {
        return ABI_GUARD_FAIL(n);
    }
}

int
aqz_node_set_level_tiling(aqz_node* n, uint32_t level, uint32_t tile_rows, uint32_t tile_cols)
{
    try {
        if (!n)
            return AQZ_INVALID_ARGUMENT;
        if (level == 0 || level >= n->lv.size() || (tile_rows == 0) != (tile_cols == 0))
            return fail(n, AQZ_INVALID_ARGUMENT, "node_set_level_tiling: bad level or tile shape");
        if (n->frames != 0)
            return fail(n, AQZ_INVALID_ARGUMENT,
                        "node_set_level_tiling: frames were already added");
        DeviceGuard guard;
        // every handle tiles the level on its GPU right behind the pyramid
        for (aqz_ds* h : n->ds)
            if (int rc = aqz_ds_set_level_tiling(h, level, tile_rows, tile_cols))
                return fail(n, rc, std::string("node_set_level_tiling: ") + aqz_ds_last_error(h));
        n->tiling[level] = { tile_rows, tile_cols };
        const aqz_level_desc& d = n->lv[level];
        n->take_bytes[level] =
          tile_rows == 0 ? n->bytes[level]
                         : size_t((d.width + tile_cols - 1) / tile_cols) *
                             ((d.height + tile_rows - 1) / tile_rows) * tile_rows * tile_cols *
                             (n->bytes[level] / (size_t(d.width) * d.height));
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(n);
    }
}

int
aqz_node_wait_input(aqz_node* n)
{
    try {
        if (!n)
            return AQZ_INVALID_ARGUMENT;
        for (uint32_t h = 0; h < n->ds.size(); ++h)
            if (n->in_flight[h])
                if (int rc = aqz_ds_wait_input(n->ds[h]))
                    return fail(n, rc, "node_wait_input: handle " + std::to_string(h));
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(n);
    }
}

uint32_t
aqz_node_handle_count(const aqz_node* n)
{
    return n ? uint32_t(n->ds.size()) : 0;
}

aqz_ds*
aqz_node_handle(aqz_node* n, uint32_t i)
{
    return n && i < n->ds.size() ? n->ds[i] : nullptr;
}

int
aqz_node_run_host_batch(aqz_node* n,
                        const void* host_frames,
                        uint32_t n_frames,
                        void* const* host_out_levels,
                        uint32_t* out_counts)
{
    try {
        if (!n)
            return AQZ_INVALID_ARGUMENT;
        DeviceGuard guard;
        const uint32_t nl = uint32_t(n->lv.size());
        if (!host_frames || !host_out_levels)
            return fail(n, AQZ_INVALID_ARGUMENT, "node_run_host_batch: null buffer");
        for (uint32_t L = 1; L < nl; ++L)
            if (!host_out_levels[L])
                return fail(n, AQZ_INVALID_ARGUMENT,
                            "node_run_host_batch: null output for level " + std::to_string(L));
        if (n->frames % n->unit != 0)
            return fail(n, AQZ_INVALID_ARGUMENT,
                        "node_run_host_batch: the stream stands inside a shard unit (" +
                          std::to_string(n->frames % n->unit) + " of " +
                          std::to_string(n->unit) + " frames)");
        if (int rc = flush_all(n))
            return rc;
        if (n_frames % n->unit != 0)
            return fail(n, AQZ_INVALID_ARGUMENT,
                        "node_run_host_batch: " + std::to_string(n_frames) +
                          " frames is not a whole number of shard units of " +
                          std::to_string(n->unit) + " (Z pairs must stay on one GPU)");
        // contiguous blocks of whole units, the first (units % D) handles one
        // unit more
        const uint32_t units = n_frames / n->unit;
        const uint32_t D = uint32_t(n->ds.size());
        std::vector<uint32_t> first(D + 1, 0);
        for (uint32_t d = 0; d < D; ++d)
            first[d + 1] = first[d] + units / D + (d < units % D ? 1 : 0);
        std::vector<int> rc(D, AQZ_OK);
        std::vector<std::vector<uint32_t>> counts(D, std::vector<uint32_t>(nl, 0));
        std::vector<std::thread> workers;
        // joins whatever started, also when a thread fails to start or the
        // caller's share throws, so no joinable thread is ever destroyed
        struct JoinAll
        {
            std::vector<std::thread>& t;
            ~JoinAll()
            {
                for (auto& w : t)
                    if (w.joinable())
                        w.join();
            }
        } join_all{ workers };
        auto run = [&](uint32_t d) {
            const uint32_t u0 = first[d], nu = first[d + 1] - first[d];
            if (nu == 0)
                return;
            std::vector<void*> outs(nl, nullptr);
            for (uint32_t L = 1; L < nl; ++L)
                outs[L] = static_cast<uint8_t*>(host_out_levels[L]) +
                          size_t(u0) * n->per_unit[L] * n->bytes[L];
            rc[d] = aqz_ds_run_host_batch(
              n->ds[d],
              static_cast<const uint8_t*>(host_frames) + size_t(u0) * n->unit * n->bytes[0],
              nu * n->unit, outs.data(), counts[d].data());
        };
        for (uint32_t d = 1; d < D; ++d)
            workers.emplace_back(run, d);
        run(0);
        for (auto& t : workers)
            t.join();
        for (uint32_t d = 0; d < D; ++d)
            if (rc[d])
                return fail(n, rc[d], "node_run_host_batch: handle " + std::to_string(d) +
                                        ": " + aqz_ds_last_error(n->ds[d]));
        for (uint32_t d = 0; d < D; ++d)
            for (uint32_t L = 1; L < nl; ++L)
                if (counts[d][L] != (first[d + 1] - first[d]) * n->per_unit[L])
                    return fail(n, AQZ_INTERNAL_ERROR,
                                "node_run_host_batch: handle " + std::to_string(d) +
                                  " emitted an unexpected frame count at level " +
                                  std::to_string(L));
        if (out_counts) {
            out_counts[0] = n_frames;
            for (uint32_t L = 1; L < nl; ++L)
                out_counts[L] = units * n->per_unit[L];
        }
        n->frames += n_frames;
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(n);
    }
}

int
aqz_node_run_device_batch(aqz_node* n,
                          const void* device_frames,
                          int src_device,
                          uint32_t n_frames,
                          void* const* device_out_levels,
                          uint32_t* out_counts,
                          void* hip_stream,
                          uint32_t flags)
{
    try {
        if (!n)
            return AQZ_INVALID_ARGUMENT;
        DeviceGuard guard;
        const uint32_t nl = uint32_t(n->lv.size());
        if (!device_frames || !device_out_levels)
            return fail(n, AQZ_INVALID_ARGUMENT, "node_run_device_batch: null buffer");
        for (uint32_t L = 1; L < nl; ++L)
            if (!device_out_levels[L])
                return fail(n, AQZ_INVALID_ARGUMENT,
                            "node_run_device_batch: null output for level " + std::to_string(L));
        if (flags & ~uint32_t(AQZ_NODE_STAGE_ALL))
            return fail(n, AQZ_INVALID_ARGUMENT, "node_run_device_batch: unknown flags");
        int n_dev = 0;
        if (hipGetDeviceCount(&n_dev) != hipSuccess || src_device < 0 || src_device >= n_dev)
            return fail(n, AQZ_INVALID_ARGUMENT,
                        "node_run_device_batch: no HIP device " + std::to_string(src_device));
        if (n->frames % n->unit != 0)
            return fail(n, AQZ_INVALID_ARGUMENT,
                        "node_run_device_batch: the stream stands inside a shard unit (" +
                          std::to_string(n->frames % n->unit) + " of " +
                          std::to_string(n->unit) + " frames)");
        if (n_frames % n->unit != 0)
            return fail(n, AQZ_INVALID_ARGUMENT,
                        "node_run_device_batch: " + std::to_string(n_frames) +
                          " frames is not a whole number of shard units of " +
                          std::to_string(n->unit) + " (Z pairs must stay on one GPU)");
        if (int rc = flush_all(n))
            return rc;
        const uint32_t units = n_frames / n->unit;
        const uint32_t D = uint32_t(n->ds.size());
        std::vector<uint32_t> first(D + 1, 0);
        for (uint32_t d = 0; d < D; ++d)
            first[d + 1] = first[d] + units / D + (d < units % D ? 1 : 0);

        // bytes of one shard unit: its input frames, and each level's output
        size_t unit_out = 0;
        std::vector<size_t> unit_bytes(nl, 0);
        unit_bytes[0] = size_t(n->unit) * n->bytes[0];
        for (uint32_t L = 1; L < nl; ++L) {
            unit_bytes[L] = size_t(n->per_unit[L]) * n->bytes[L];
            unit_out += unit_bytes[L];
        }
        // sub-batch of a remote block: the units that fit the staging budget
        // ($AQZ_NODE_STAGE_MB per slot, default 256 MiB), at least one
        size_t budget = size_t(256) << 20;
        if (const char* env = std::getenv("AQZ_NODE_STAGE_MB"))
            if (long v = std::atol(env); v > 0)
                budget = size_t(v) << 20;
        const uint32_t sub_units =
          uint32_t(std::max<size_t>(1, budget / (unit_bytes[0] + unit_out)));

        hipError_t e = hipSetDevice(src_device);
        if (e != hipSuccess)
            return hip_fail(n, e, "node_run_device_batch: hipSetDevice");
        hipStream_t caller = static_cast<hipStream_t>(hip_stream);
        if (n->ready_ev.size() < size_t(n_dev))
            n->ready_ev.resize(n_dev, nullptr);
        hipEvent_t& ready = n->ready_ev[src_device];
        if (!ready && (e = hipEventCreateWithFlags(&ready, hipEventDisableTiming)) != hipSuccess)
            return hip_fail(n, e, "node_run_device_batch: event");
        if ((e = hipEventRecord(ready, caller)) != hipSuccess)
            return hip_fail(n, e, "node_run_device_batch: event record");

        // Everything queued so far drains before an error returns: blocks
        // still read the caller's batch and write its outputs on the
        // handles' streams, and the caller may free them on an error.
        auto deal = [&]() -> int {
            const uint8_t* in = static_cast<const uint8_t*>(device_frames);
            std::vector<hipEvent_t> joins;
            int rc = AQZ_OK;
            for (uint32_t d = 0; d < D && rc == AQZ_OK; ++d) {
                const uint32_t u0 = first[d], nu = first[d + 1] - first[d];
                if (nu == 0)
                    continue;
                aqz_ds* h = n->ds[d];
                const int dev = aqz_ds_device(h);
                std::vector<void*> outs(nl, nullptr);
                for (uint32_t L = 1; L < nl; ++L)
                    outs[L] = static_cast<uint8_t*>(device_out_levels[L]) + size_t(u0) * unit_bytes[L];
                std::vector<uint32_t> cnt(nl, 0);
                if (dev == src_device && !(flags & AQZ_NODE_STAGE_ALL)) {
                    // in place, on the caller's stream
                    rc = aqz_ds_run_device_batch(h, in + size_t(u0) * unit_bytes[0], nu * n->unit,
                                                 outs.data(), cnt.data(), caller);
                    if (rc)
                        return fail(n, rc, "node_run_device_batch: handle " + std::to_string(d) +
                                             ": " + aqz_ds_last_error(h));
                    for (uint32_t L = 1; L < nl; ++L)
                        if (cnt[L] != nu * n->per_unit[L])
                            return fail(n, AQZ_INTERNAL_ERROR,
                                        "node_run_device_batch: handle " + std::to_string(d) +
                                          " emitted an unexpected frame count at level " +
                                          std::to_string(L));
                    continue;
                }
                const uint32_t g_max = std::min(sub_units, nu);
                if ((rc = peer_stage(n, d, src_device, size_t(g_max) * (unit_bytes[0] + unit_out))))
                    break;
                PeerStage& p = n->peers[d];
                if ((e = hipStreamWaitEvent(p.pull, ready, 0)) != hipSuccess)
                    return hip_fail(n, e, "node_run_device_batch: wait for the batch");
                for (uint32_t j = 0; j < nu; j += g_max) {
                    const uint32_t g = std::min(g_max, nu - j);
                    const uint32_t s = p.next_slot;
                    p.next_slot ^= 1u;
                    uint8_t* slot = p.stage + size_t(s) * p.slot_bytes;
                    std::vector<void*> souts(nl, nullptr);
                    size_t off = size_t(g) * unit_bytes[0];
                    for (uint32_t L = 1; L < nl; ++L) {
                        souts[L] = slot + off;
                        off += size_t(g) * unit_bytes[L];
                    }
                    // pull: once the slot's previous pyramid has read its input
                    if ((e = hipStreamWaitEvent(p.pull, p.ran[s], 0)) != hipSuccess ||
                        (e = hipMemcpyPeerAsync(slot, dev, in + size_t(u0 + j) * unit_bytes[0],
                                                src_device, size_t(g) * unit_bytes[0], p.pull)) !=
                          hipSuccess ||
                        (e = hipEventRecord(p.pulled[s], p.pull)) != hipSuccess)
                        return hip_fail(n, e, "node_run_device_batch: pull over xGMI");
                    // pyramid: once pulled and the slot's previous push has left
                    if ((e = hipStreamWaitEvent(p.run, p.pulled[s], 0)) != hipSuccess ||
                        (e = hipStreamWaitEvent(p.run, p.pushed[s], 0)) != hipSuccess)
                        return hip_fail(n, e, "node_run_device_batch: stream order");
                    rc = aqz_ds_run_device_batch(h, slot, g * n->unit, souts.data(), cnt.data(),
                                                 p.run);
                    if (rc)
                        return fail(n, rc, "node_run_device_batch: handle " + std::to_string(d) +
                                             ": " + aqz_ds_last_error(h));
                    for (uint32_t L = 1; L < nl; ++L)
                        if (cnt[L] != g * n->per_unit[L])
                            return fail(n, AQZ_INTERNAL_ERROR,
                                        "node_run_device_batch: handle " + std::to_string(d) +
                                          " emitted an unexpected frame count at level " +
                                          std::to_string(L));
                    if ((e = hipSetDevice(dev)) != hipSuccess ||
                        (e = hipEventRecord(p.ran[s], p.run)) != hipSuccess ||
                        (e = hipStreamWaitEvent(p.push, p.ran[s], 0)) != hipSuccess)
                        return hip_fail(n, e, "node_run_device_batch: stream order");
                    // push: each level to the block's place in the outputs
                    for (uint32_t L = 1; L < nl; ++L)
                        if ((e = hipMemcpyPeerAsync(static_cast<uint8_t*>(outs[L]) +
                                                      size_t(j) * unit_bytes[L],
                                                    src_device, souts[L], dev,
                                                    size_t(g) * unit_bytes[L], p.push)) != hipSuccess)
                            return hip_fail(n, e, "node_run_device_batch: push over xGMI");
                    if ((e = hipEventRecord(p.pushed[s], p.push)) != hipSuccess)
                        return hip_fail(n, e, "node_run_device_batch: event record");
                }
                if ((e = hipEventRecord(p.done, p.push)) != hipSuccess)
                    return hip_fail(n, e, "node_run_device_batch: event record");
                joins.push_back(p.done);
            }
            if (rc)
                return rc;
            // the caller's stream owns the outputs again once every push is done
            if ((e = hipSetDevice(src_device)) != hipSuccess)
                return hip_fail(n, e, "node_run_device_batch: hipSetDevice");
            for (hipEvent_t ev : joins)
                if ((e = hipStreamWaitEvent(caller, ev, 0)) != hipSuccess)
                    return hip_fail(n, e, "node_run_device_batch: join");
            return AQZ_OK;
        };
        if (const int rc = deal(); rc != AQZ_OK) {
            for (PeerStage& p : n->peers)
                if (p.device >= 0) {
                    (void)hipSetDevice(p.device);
                    for (hipStream_t st : { p.pull, p.run, p.push })
                        (void)hipStreamSynchronize(st);
                }
            (void)hipSetDevice(src_device);
            (void)hipStreamSynchronize(caller);
            return rc;
        }
        if (out_counts) {
            out_counts[0] = n_frames;
            for (uint32_t L = 1; L < nl; ++L)
                out_counts[L] = units * n->per_unit[L];
        }
        n->frames += n_frames;
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(n);
    }
}

int
aqz_node_inputs_released(aqz_node* n, uint64_t* released)
{
    try {
        if (!n || !released)
            return AQZ_INVALID_ARGUMENT;
        // adds are in submission order; only a handle's add in flight can
        // still read its frame, and the earliest such one bounds the prefix
        uint64_t r = n->frames;
        for (const auto& a : n->adds) {
            if (a.settled || n->in_flight[a.handle] != &a)
                continue;
            int pending = 0;
            if (int rc = aqz_ds_input_pending(n->ds[a.handle], &pending))
                return fail(n, rc, "node_inputs_released: handle " + std::to_string(a.handle));
            if (pending) {
                r = a.frame;
                break;
            }
        }
        *released = r;
        return AQZ_OK;
    } catch (...) {
        return ABI_GUARD_FAIL(n);
    }
}

const char*
aqz_node_last_error(const aqz_node* n)
{
    return n ? n->err.c_str() : "";
}

} // extern "C"
