// array.tiled.cpp — chunk-tiled level frames into zarr::Array (MI355X backend).
//
// Goes into the reference tree as src/streaming/array.tiled.cpp, compiled
// only when AQZ_DOWNSAMPLER=hip (cmake/hip.cmake).  SURVEY §8(f) row 2: the
// GPU emits each pyramid level in the order Array::write_frame_to_chunks_
// (array.cpp:507-622) walks it — tile t = ty * n_tiles_x + tx, chunk_y x
// chunk_x pixels row-major, zero where the tile overhangs the frame — so every
// tile lands in its chunk slot as ONE contiguous copy instead of one memcpy
// per row.  The zero overhang is what the reference leaves in the slot (chunk
// buffers start zeroed, chunk.cpp:8-15, and each flush frees the slot), so the
// chunk bytes and their has_data flag come out identical.
//
// acquire-zarr-hip.patch adds the declarations (array.hh) and three hooks in
// array.cpp: Array::write_frame counts a tiled frame's payload as one frame
// (for the size check and for the Ok/PartialWrite result), and
// write_frame_to_chunks_ hands a tiled frame to write_tiles_to_chunks_.  The
// placement itself is zarr::tiled::write_tiles_to_chunks (array.tiled.hh).
// Everything else — size, bounds and frame-order checks, flushing, banding,
// rollover — is the reference's own Array::write_frame.

#include "array.tiled.hh"

#ifndef AQZ_TILED_STANDALONE // the harness links the placement only
#include "array.hh"
#include "macros.hh"
#include "zarr.common.hh"
#endif

#include <algorithm>

zarr::tiled::TileGrid
zarr::tiled::tile_grid(const ArrayDimensions& dims)
{
    TileGrid g{};
    g.frame_cols = dims.width_dim().array_size_px;
    g.frame_rows = dims.height_dim().array_size_px;
    g.tile_cols = dims.width_dim().chunk_size_px;
    g.tile_rows = dims.height_dim().chunk_size_px;
    if (g.tile_cols && g.tile_rows) {
        g.n_tiles_x = (g.frame_cols + g.tile_cols - 1) / g.tile_cols;
        g.n_tiles_y = (g.frame_rows + g.tile_rows - 1) / g.tile_rows;
    }
    return g;
}

size_t
zarr::tiled::tiled_frame_bytes(const ArrayDimensions& dims, size_t bytes_per_px)
{
    const TileGrid g = tile_grid(dims);
    return static_cast<size_t>(g.n_tiles_x) * g.n_tiles_y * g.tile_rows *
           g.tile_cols * bytes_per_px;
}

size_t
zarr::tiled::write_tiles_to_chunks(const ArrayDimensions& dims,
                                   size_t bytes_per_px,
                                   uint64_t frames_written,
                                   const uint8_t* tiles,
                                   std::vector<std::shared_ptr<Chunk>>& chunks,
                                   std::vector<std::mutex>& chunk_mutexes)
{
    const TileGrid g = tile_grid(dims);
    if (g.tile_cols == 0 || g.tile_rows == 0) {
        return 0;
    }
    const size_t tile_bytes =
      static_cast<size_t>(g.tile_rows) * g.tile_cols * bytes_per_px;
    const size_t bytes_per_chunk = dims.bytes_per_chunk();

    // Same chunk lattice position and in-chunk slot as write_frame_to_chunks_:
    // the frame index is the number of frames already written, in storage
    // order.
    const auto frame_id = dims.transpose_frame_id(frames_written);
    const auto group_offset = dims.tile_group_offset(frame_id);
    const auto chunk_offset = dims.chunk_internal_offset(frame_id);

    const int n_tiles = static_cast<int>(g.n_tiles_x * g.n_tiles_y);
    size_t bytes_written = 0;

#pragma omp parallel for reduction(+ : bytes_written)
    for (int t = 0; t < n_tiles; ++t) {
        auto& chunk = chunks[t + group_offset];
        {
            std::unique_lock lock(chunk_mutexes[t + group_offset]);
            if (chunk == nullptr) {
                chunk = std::make_shared<Chunk>(bytes_per_chunk, bytes_per_px);
            }
        }
        // the whole tile, overhang zeros included, as one row of tile_bytes:
        // the overhang lands on bytes the reference leaves at their initial
        // zero (chunk.cpp:8-15), and zeros never set has_data
        chunk->write_tile_rows(chunk_offset,
                               tiles + static_cast<size_t>(t) * tile_bytes,
                               tile_bytes,
                               tile_bytes,
                               tile_bytes,
                               1);

        // Report the frame pixels the tile carries, as the reference does.
        const uint32_t tx = t % g.n_tiles_x, ty = t / g.n_tiles_x;
        const uint32_t cols = std::min(g.tile_cols, g.frame_cols - tx * g.tile_cols);
        const uint32_t rows = std::min(g.tile_rows, g.frame_rows - ty * g.tile_rows);
        bytes_written += static_cast<size_t>(cols) * rows * bytes_per_px;
    }

    return bytes_written;
}

#ifndef AQZ_TILED_STANDALONE // the harness links the placement only
size_t
zarr::Array::tiled_frame_bytes_() const
{
    return tiled::tiled_frame_bytes(*config_->dimensions,
                                    bytes_of_type(config_->dtype));
}

zarr::WriteResult
zarr::Array::write_tiled_frame(std::vector<uint8_t>& tiles,
                               size_t& bytes_written,
                               uint64_t frame_id)
{
    bytes_written = 0;
    // The tile order is the storage order; a transposed array chunks the
    // transpose of its input (array.cpp:515-534) and takes write_frame.
    if (config_->dimensions->needs_xy_transposition() ||
        tiles.size() != tiled_frame_bytes_()) {
        LOG_ERROR("Tiled frame size mismatch: expected ",
                  tiled_frame_bytes_(),
                  ", got ",
                  tiles.size(),
                  ". Skipping");
        return WriteResult::FrameSizeMismatch;
    }

    tiled_ = true;
    struct Reset
    {
        bool& flag;
        ~Reset() { flag = false; }
    } reset{ tiled_ };
    return write_frame(tiles, bytes_written, frame_id);
}

size_t
zarr::Array::write_tiles_to_chunks_(const std::vector<uint8_t>& tiles)
{
    return tiled::write_tiles_to_chunks(*config_->dimensions,
                                        bytes_of_type(config_->dtype),
                                        frames_written_(),
                                        tiles.data(),
                                        chunks_,
                                        chunk_mutexes_);
}
#endif
