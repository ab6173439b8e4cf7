// array.tiled.hh — chunk-tiled frames into the chunk lattice (MI355X backend).
//
// The placement behind Array::write_tiled_frame (array.tiled.cpp), as free
// functions over the reference's own ArrayDimensions and Chunk, so that it
// can also run outside zarr::Array (tests/integration/tiled_writer_harness.cpp
// drives it with the reference's chunk.cpp and array.dimensions.cpp).
#pragma once

#include "array.dimensions.hh"
#include "chunk.hh"

#include <cstddef>
#include <cstdint>
#include <memory>
#include <mutex>
#include <vector>

namespace zarr::tiled {

struct TileGrid
{
    uint32_t frame_cols = 0, frame_rows = 0, tile_cols = 0, tile_rows = 0;
    uint32_t n_tiles_x = 0, n_tiles_y = 0;
};

// The storage-order XY tile grid of one frame (array.cpp:547-563).
TileGrid
tile_grid(const ArrayDimensions& dims);

// Bytes of one chunk-tiled frame: every tile whole, overhang included.
size_t
tiled_frame_bytes(const ArrayDimensions& dims, size_t bytes_per_px);

// Writes the tiled frame `tiles` (tiled_frame_bytes long) as frame number
// `frames_written` (acquisition order) into `chunks` — the same chunk and
// in-chunk slot Array::write_frame_to_chunks_ uses (array.cpp:563-617), one
// copy per tile — creating missing chunks as the reference does.  Returns
// the frame pixel bytes the tiles carry (overhang excluded), which is what
// write_frame_to_chunks_ returns for the same frame.
size_t
write_tiles_to_chunks(const ArrayDimensions& dims,
                      size_t bytes_per_px,
                      uint64_t frames_written,
                      const uint8_t* tiles,
                      std::vector<std::shared_ptr<Chunk>>& chunks,
                      std::vector<std::mutex>& chunk_mutexes);

} // namespace zarr::tiled
