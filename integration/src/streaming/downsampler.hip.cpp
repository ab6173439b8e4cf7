// downsampler.hip.cpp — zarr::Downsampler on MI355X (acquire-zarr v0.8.1).
//
// Goes into the reference tree as src/streaming/downsampler.hip.cpp and is
// compiled only when AQZ_DOWNSAMPLER=hip (cmake/hip.cmake, which also defines
// AQZ_DOWNSAMPLER_HIP and links libaqz_downsampler).  It defines the
// per-frame half of the class over the C ABI in include/aqz_downsampler.h:
//
//   Downsampler(config, method)  downsampler.cpp:249-304  -> aqz_ds_create
//   ~Downsampler()               (implicit)               -> aqz_ds_destroy
//   add_frame(frame)             downsampler.cpp:306-401  -> aqz_ds_add_frame
//   take_frame(level, out)       downsampler.cpp:403-414  -> aqz_ds_take_frame
//   add_frame_async(frame)       new -> aqz_ds_add_frame_async_take
//   wait()                       new                      -> aqz_ds_wait
//   release_frame(frame)         new                      -> wait(), or (node mode)
//                                                            keeps the buffer
//   take_frame_tiled(level, t)   new -> aqz_ds_take_frame_tiled
//   level_is_tiled(level)        new
//   flush()                      new                      -> (node mode) aqz_node_flush
//
// take_frame on a level the add's background job already took tiled untiles
// that copy on the host; add_frame and add_frame_async settle a previous
// pending add first, so the levels it took are held before anything else
// happens.
//
// Node mode ($AQZ_GPU_DEVICES with two or more HIP ordinals, e.g. "0,1,2,3"):
// one aqz_node deals the stream's frames over those GPUs, so
// several frames' pyramids and level copies run at once, each GPU over its
// own PCIe link.  add_frame_async hands the frame to the next GPU and wait()
// returns once it is uploaded (aqz_node_wait_input), not when its levels are
// done.  release_frame() — what the patched MultiscaleArray calls once level
// 0 is written — does not wait at all: it keeps the frame's buffer while the
// GPU may still read it and swaps a spare of the same size into the caller's
// vector (the frame queue's, which FrameQueue::pop fills by swap and push
// refills by resize + memcpy, frame.queue.cpp:20-74, and which
// process_frame_queue_ never reads after write_frame, zarr.stream.cpp:
// 1671-1685).  So uploads to different GPUs overlap, and the buffers recycle
// as aqz_node_inputs_released reports their uploads done: at most one per
// GPU plus one spare, no copy.  take_frame / take_frame_tiled hand out, in
// emission order, the next level frame that is ready.  The patched MultiscaleArray takes every ready
// frame per level after each add and calls flush() before it closes its
// arrays, so each level receives exactly the frames, in the order, that the
// reference's add_frame + take_frame loop produces (multiscale.array.cpp:
// 291-325).  Z planes still waiting for their pair at close are dropped, as
// the reference drops them.  A caller that skips takes gets no emplace drop
// in this mode: the node takes every frame.
//
// The rest of the class stays in the reference's downsampler.cpp, compiled
// unchanged: acquire-zarr-hip.patch only puts the CPU constructor, add_frame,
// take_frame, emplace_downsampled_frame_ and the scalar kernels they use
// (downsampler.cpp:39-414, 599-605) under #ifndef AQZ_DOWNSAMPLER_HIP.  So
// make_writer_configurations_ (the level geometry MultiscaleArray builds its
// arrays from), writer_configurations, downsampling_method and get_metadata
// (the OME metadata) are the reference's own code, and the level geometry
// handed to the GPU is read back from those configurations.
//
// Error behaviour is the reference's: every failure throws std::runtime_error
// (EXPECT, macros.hh), which MultiscaleArray::create_downsampler_ logs and
// turns into a failed ZarrStream_create (multiscale.array.cpp:172-189), and
// which the frame-queue consumer turns into a stream error
// (zarr.stream.cpp:1705-1720).

#include "downsampler.hh"
#include "macros.hh"
#include "zarr.common.hh"

#include "aqz_downsampler.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace {

// $AQZ_GPU_DEVICES as HIP ordinals ("0,1,2"); fewer than two: no node.
std::vector<int>
node_devices()
{
    std::vector<int> devs;
    const char* env = std::getenv("AQZ_GPU_DEVICES");
    if (!env) {
        return devs;
    }
    const std::string s(env);
    size_t pos = 0;
    while (pos <= s.size()) {
        const size_t end = std::min(s.find(',', pos), s.size());
        const std::string item = s.substr(pos, end - pos);
        if (!item.empty()) {
            size_t used = 0;
            int d = -1;
            try {
                d = std::stoi(item, &used);
            } catch (const std::exception&) {
                used = 0;
            }
            EXPECT(used == item.size() && d >= 0,
                   "GPU downsampler: bad entry in AQZ_GPU_DEVICES: '",
                   item,
                   "'");
            devs.push_back(d);
        }
        pos = end + 1;
    }
    if (devs.size() < 2) {
        devs.clear();
    }
    return devs;
}

// The reference validates the dtype before the method, with these messages
// (downsampler.cpp:295-302).
void
check_dtype_and_method(ZarrDataType dtype, ZarrDownsamplingMethod method)
{
    if (static_cast<int>(dtype) < 0 || dtype >= ZarrDataTypeCount) {
        throw std::runtime_error("Invalid data type: " + std::to_string(dtype));
    }
    EXPECT(method < ZarrDownsamplingMethodCount,
           "Invalid downsampling method: ",
           static_cast<int>(method));
}

} // namespace

zarr::Downsampler::Downsampler(std::shared_ptr<ArrayConfig> config,
                               ZarrDownsamplingMethod method)
{
    make_writer_configurations_(config); // reference code, downsampler.cpp
    check_dtype_and_method(config->dtype, method);
    method_ = method;

    // Per-level geometry exactly as add_frame reads it (downsampler.cpp:
    // 309-338): width/height are the storage-order last two dimensions,
    // planes is dimension ndims-3 (the phantom singleton for 2-D arrays).
    const size_t n = n_levels_();
    std::vector<aqz_level_desc> levels(n);
    for (size_t level = 0; level < n; ++level) {
        const auto& dims = writer_configurations_.at(int(level))->dimensions;
        levels[level].width = dims->width_dim().array_size_px;
        levels[level].height = dims->height_dim().array_size_px;
        levels[level].planes = dims->at(dims->ndims() - 3).array_size_px;
    }

    tiles_.assign(n, { 0u, 0u });
    takes_.assign(n, aqz_level_take{});
    taken_.assign(n, {});
    holding_.assign(n, 0);

    if (const std::vector<int> devs = node_devices(); !devs.empty()) {
        aqz_node* node = nullptr;
        const int rc = aqz_node_create(levels.data(),
                                       static_cast<uint32_t>(n),
                                       static_cast<int>(config->dtype),
                                       static_cast<int>(method),
                                       devs.data(),
                                       static_cast<uint32_t>(devs.size()),
                                       &node);
        EXPECT(rc == AQZ_OK, "GPU downsampler: ", aqz_last_error());
        node_ = node;
    } else {
        aqz_ds* handle = nullptr;
        const int rc = aqz_ds_create(levels.data(),
                                     static_cast<uint32_t>(n),
                                     static_cast<int>(config->dtype),
                                     static_cast<int>(method),
                                     -1, // $AQZ_GPU_DEVICE, else the current device
                                     &handle);
        EXPECT(rc == AQZ_OK, "GPU downsampler: ", aqz_last_error());
        gpu_ = handle;
    }

    // Levels >= 1 are tiled on the GPU right behind the pyramid, in their
    // own chunk shape (downsample_dimension keeps chunk sizes), so that
    // MultiscaleArray can hand each tile to its chunk in one copy
    // (array.tiled.cpp).  A transposed storage order keeps the row-major
    // path: Array chunks the transpose of what it is given.
    if (config->dimensions->needs_xy_transposition()) {
        return;
    }
    try {
        for (size_t level = 1; level < n; ++level) {
            const auto& dims = writer_configurations_.at(int(level))->dimensions;
            const uint32_t tile_rows = dims->height_dim().chunk_size_px;
            const uint32_t tile_cols = dims->width_dim().chunk_size_px;
            if (tile_rows == 0 || tile_cols == 0) {
                continue;
            }
            if (node_) {
                EXPECT(aqz_node_set_level_tiling(
                         node_, uint32_t(level), tile_rows, tile_cols) == AQZ_OK,
                       "GPU downsampler: ",
                       aqz_node_last_error(node_));
            } else {
                EXPECT(aqz_ds_set_level_tiling(
                         gpu_, uint32_t(level), tile_rows, tile_cols) == AQZ_OK,
                       "GPU downsampler: ",
                       aqz_ds_last_error(gpu_));
            }
            tiles_[level] = { tile_rows, tile_cols };
        }
    } catch (...) {
        // no destructor runs for a throwing constructor
        aqz_node_destroy(node_);
        aqz_ds_destroy(gpu_);
        node_ = nullptr;
        gpu_ = nullptr;
        throw;
    }
}

zarr::Downsampler::~Downsampler()
{
    // each handle settles its add in flight first, so no upload still reads
    // a buffer in node_inputs_ when the members go
    aqz_node_destroy(node_);
    aqz_ds_destroy(gpu_); // settles a pending add_frame_async first
}

void
zarr::Downsampler::add_frame(std::vector<uint8_t>& frame)
{
    if (node_) {
        add_frame_async(frame);
        wait(); // the frame is uploaded; its levels come when ready
        return;
    }
    // a pending add_frame_async first: its takes mark the levels they took
    // as held, which decides where this frame's levels may go
    if (pending_) {
        wait();
    }
    for (const uint8_t h : holding_) {
        if (h) {
            // frames taken ahead are still unconsumed: their levels must drop
            // this frame's results, as a cached frame would
            add_frame_async(frame);
            wait();
            return;
        }
    }
    const int rc = aqz_ds_add_frame(gpu_, frame.data(), frame.size());
    EXPECT(rc == AQZ_OK, "GPU downsampler: ", aqz_ds_last_error(gpu_));
}

void
zarr::Downsampler::add_frame_async(std::vector<uint8_t>& frame)
{
    if (node_) {
        // the previous frame may still be uploading to its GPU; this one
        // goes to the next GPU in the deal
        if (node_caller_frame_) {
            wait(); // an earlier add_frame_async nobody released
        }
        const int rc = aqz_node_add_frame(node_, frame.data(), frame.size());
        EXPECT(rc == AQZ_OK, "GPU downsampler: ", aqz_node_last_error(node_));
        node_caller_frame_ = frame.data();
        ++node_added_;
        pending_ = true;
        return;
    }
    // A previous add_frame_async may still be running its takes into takes_
    // and taken_: settle it (which also marks the levels it took as held)
    // before either is touched.
    if (pending_) {
        wait();
    }
    // The takes write_multiscale_frames_ makes right after the add
    // (multiscale.array.cpp:298-325) run in the same background job, so the
    // levels' device-to-host copies overlap level 0's chunking too.  A level
    // whose earlier frame is still unconsumed here is held instead.
    for (size_t level = 1; level < takes_.size(); ++level) {
        aqz_level_take& t = takes_[level];
        t = aqz_level_take{};
        if (holding_[level]) {
            t.mode = AQZ_TAKE_HOLD;
            continue;
        }
        const auto [tile_rows, tile_cols] = tiles_[level];
        size_t bytes = aqz_ds_level_bytes(gpu_, uint32_t(level));
        if (tile_rows != 0) {
            const auto& dims = writer_configurations_.at(int(level))->dimensions;
            const size_t w = dims->width_dim().array_size_px;
            const size_t h = dims->height_dim().array_size_px;
            bytes = ((w + tile_cols - 1) / tile_cols) * ((h + tile_rows - 1) / tile_rows) *
                    tile_rows * tile_cols * (bytes / (w * h));
        }
        // a vector the caller swapped back keeps its capacity: no new
        // allocation once both have reached the level's size
        taken_[level].resize(bytes);
        t.mode = AQZ_TAKE_INTO;
        t.tile_rows = tile_rows;
        t.tile_cols = tile_cols;
        t.dst = taken_[level].data();
        t.cap = taken_[level].size();
    }
    const int rc =
      aqz_ds_add_frame_async_take(gpu_, frame.data(), frame.size(), takes_.data());
    EXPECT(rc == AQZ_OK, "GPU downsampler: ", aqz_ds_last_error(gpu_));
    pending_ = true;
}

void
zarr::Downsampler::wait()
{
    if (node_) {
        // the caller's frame of the last add is uploaded: the caller may
        // reuse it (buffers release_frame kept need no wait)
        pending_ = false;
        if (!node_caller_frame_) {
            return;
        }
        node_caller_frame_ = nullptr;
        const int rc = aqz_node_wait_input(node_);
        EXPECT(rc == AQZ_OK, "GPU downsampler: ", aqz_node_last_error(node_));
        return;
    }
    const int rc = aqz_ds_wait(gpu_);
    const bool had_takes = pending_;
    pending_ = false;
    EXPECT(rc == AQZ_OK, "GPU downsampler: ", aqz_ds_last_error(gpu_));
    if (!had_takes) {
        return;
    }
    for (size_t level = 1; level < takes_.size(); ++level) {
        if (takes_[level].mode == AQZ_TAKE_INTO && takes_[level].has_frame) {
            holding_[level] = 1;
        }
    }
}

void
zarr::Downsampler::release_frame(std::vector<uint8_t>& frame)
{
    if (!node_ || !node_caller_frame_ || frame.data() != node_caller_frame_ ||
        frame.empty()) {
        wait(); // one GPU: the add's takes are settled here, as before
        return;
    }
    // Buffers whose uploads are done become spares (in stream order: the
    // node reports a prefix of its frames).
    uint64_t released = 0;
    const int rc = aqz_node_inputs_released(node_, &released);
    EXPECT(rc == AQZ_OK, "GPU downsampler: ", aqz_node_last_error(node_));
    while (!node_inputs_.empty() && node_inputs_.front().first < released) {
        node_spares_.push_back(std::move(node_inputs_.front().second));
        node_inputs_.pop_front();
    }
    // Keep the caller's buffer (a vector swap moves no bytes: the node goes
    // on reading the same memory) and give the caller a spare of its size.
    ByteVector spare;
    if (!node_spares_.empty()) {
        spare = std::move(node_spares_.back());
        node_spares_.pop_back();
    }
    ByteVector kept;
    kept.swap(frame);
    spare.resize(kept.size());
    frame.swap(spare);
    node_inputs_.emplace_back(node_added_ - 1, std::move(kept));
    node_caller_frame_ = nullptr;
    pending_ = false;
}

bool
zarr::Downsampler::hand_over_(int level, std::vector<uint8_t>& out)
{
    if (level < 1 || static_cast<size_t>(level) >= holding_.size() || !holding_[level]) {
        return false;
    }
    if (pending_) {
        wait();
    }
    out.swap(taken_[level]); // handed over by swap, as downsampler.cpp:403-414
    holding_[level] = 0;
    return true;
}

void
zarr::Downsampler::untile_(int level,
                           const std::vector<uint8_t>& tiled,
                           std::vector<uint8_t>& out) const
{
    // `tiled` holds a level frame chunk-tiled (tile t = ty * n_tiles_x + tx,
    // tile_rows x tile_cols, row-major, zero overhang); take_frame hands it
    // out row-major, as the reference's cached frame would be.
    const auto [tile_rows, tile_cols] = tiles_[level];
    const auto& dims = writer_configurations_.at(level)->dimensions;
    const size_t w = dims->width_dim().array_size_px;
    const size_t h = dims->height_dim().array_size_px;
    const size_t bpp = zarr::bytes_of_type(writer_configurations_.at(level)->dtype);
    const size_t ntx = (w + tile_cols - 1) / tile_cols;
    const uint8_t* tiles = tiled.data();
    out.resize(w * h * bpp);
    for (size_t y = 0; y < h; ++y) {
        const size_t ty = y / tile_rows, r = y % tile_rows;
        for (size_t tx = 0; tx < ntx; ++tx) {
            const size_t x0 = tx * tile_cols;
            const size_t n = std::min<size_t>(tile_cols, w - x0);
            const size_t t = ty * ntx + tx;
            std::memcpy(out.data() + (y * w + x0) * bpp,
                        tiles + ((t * tile_rows + r) * tile_cols) * bpp,
                        n * bpp);
        }
    }
}

void
zarr::Downsampler::untile_held_(int level, std::vector<uint8_t>& out)
{
    untile_(level, taken_[level], out);
    holding_[level] = 0;
}

bool
zarr::Downsampler::node_take_(int level, std::vector<uint8_t>& out)
{
    // the next ready frame of the level, in emission order (tiled if the
    // level is): size query, then the copy
    size_t nbytes = 0;
    int has_frame = 0;
    int rc = aqz_node_take_frame(
      node_, static_cast<uint32_t>(level), nullptr, 0, &nbytes, &has_frame);
    EXPECT(rc == AQZ_OK, "GPU downsampler: ", aqz_node_last_error(node_));
    if (!has_frame) {
        return false;
    }
    out.resize(nbytes);
    rc = aqz_node_take_frame(node_,
                             static_cast<uint32_t>(level),
                             out.data(),
                             out.size(),
                             &nbytes,
                             &has_frame);
    EXPECT(rc == AQZ_OK, "GPU downsampler: ", aqz_node_last_error(node_));
    return has_frame != 0;
}

void
zarr::Downsampler::flush()
{
    if (node_) {
        const int rc = aqz_node_flush(node_);
        EXPECT(rc == AQZ_OK, "GPU downsampler: ", aqz_node_last_error(node_));
        return;
    }
    wait();
}

bool
zarr::Downsampler::take_frame(int level, std::vector<uint8_t>& frame_data)
{
    // The reference returns false for any level it holds no frame for,
    // including out-of-range ones (downsampler.cpp:403-414).
    if (level < 1 || static_cast<size_t>(level) >= n_levels_()) {
        return false;
    }
    if (node_) {
        if (!level_is_tiled(level)) {
            return node_take_(level, frame_data);
        }
        std::vector<uint8_t> tiled;
        if (!node_take_(level, tiled)) {
            return false;
        }
        untile_(level, tiled, frame_data);
        return true;
    }
    if (pending_) {
        wait();
    }
    if (holding_[level]) {
        // taken in the add's background job; a tiled level took it tiled
        if (level_is_tiled(level)) {
            untile_held_(level, frame_data);
            return true;
        }
        return hand_over_(level, frame_data);
    }
    // Size query first: the frame stays cached until it is copied out.
    size_t nbytes = 0;
    int has_frame = 0;
    int rc = aqz_ds_take_frame(
      gpu_, static_cast<uint32_t>(level), nullptr, 0, &nbytes, &has_frame);
    EXPECT(rc == AQZ_OK, "GPU downsampler: ", aqz_ds_last_error(gpu_));
    if (!has_frame) {
        return false;
    }
    // The reference hands its cached vector over by swap, so the caller's
    // buffer ends up exactly the level frame's size.
    frame_data.resize(nbytes);
    rc = aqz_ds_take_frame(gpu_,
                           static_cast<uint32_t>(level),
                           frame_data.data(),
                           frame_data.size(),
                           &nbytes,
                           &has_frame);
    EXPECT(rc == AQZ_OK, "GPU downsampler: ", aqz_ds_last_error(gpu_));
    return has_frame != 0;
}

bool
zarr::Downsampler::level_is_tiled(int level) const
{
    return level >= 1 && static_cast<size_t>(level) < tiles_.size() &&
           tiles_[level].first != 0;
}

bool
zarr::Downsampler::take_frame_tiled(int level, std::vector<uint8_t>& tiles)
{
    if (!level_is_tiled(level)) {
        return false;
    }
    if (node_) {
        return node_take_(level, tiles);
    }
    if (pending_) {
        wait();
    }
    if (hand_over_(level, tiles)) {
        return true; // taken, tiled, in the add's background job
    }
    const auto [tile_rows, tile_cols] = tiles_[level];
    size_t nbytes = 0;
    int has_frame = 0;
    int rc = aqz_ds_take_frame_tiled(gpu_,
                                     static_cast<uint32_t>(level),
                                     tile_rows,
                                     tile_cols,
                                     nullptr,
                                     0,
                                     nullptr,
                                     &nbytes,
                                     &has_frame);
    EXPECT(rc == AQZ_OK, "GPU downsampler: ", aqz_ds_last_error(gpu_));
    if (!has_frame) {
        return false;
    }
    // The chunk zero scan stays with Chunk::write_tile_rows, which stops at
    // the first nonzero byte; the tiles alone travel.
    tiles.resize(nbytes);
    rc = aqz_ds_take_frame_tiled(gpu_,
                                 static_cast<uint32_t>(level),
                                 tile_rows,
                                 tile_cols,
                                 tiles.data(),
                                 tiles.size(),
                                 nullptr,
                                 &nbytes,
                                 &has_frame);
    EXPECT(rc == AQZ_OK, "GPU downsampler: ", aqz_ds_last_error(gpu_));
    return has_frame != 0;
}
