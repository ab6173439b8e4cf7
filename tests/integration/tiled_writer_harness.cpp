// tiled_writer_harness.cpp — executes the drop-in's tiled chunk writer
// (integration/src/streaming/array.tiled.cpp, zarr::tiled::write_tiles_to_chunks)
// on the reference's own ArrayDimensions (array.dimensions.cpp) and Chunk
// (chunk.cpp), compiled from /root/reference by tests/test_integration.py.
//
// TEST INFRASTRUCTURE ONLY.  It plays the part of zarr::Array around the
// placement: one chunk layer of number_of_chunks_in_memory() chunks
// (array.cpp's chunks_), frames numbered by frames written, and the layer
// handed out and cleared every frames_per_chunk_layer() frames, as a flush
// does (array.cpp:180-221).
//
// stdin:  ndims bytes_per_px dtype n_frames
//         ndims lines "type array_size chunk_size shard_size" (storage order)
// argv[1] the n_frames chunk-tiled frames back to back (tiled_frame_bytes each)
// argv[2] output: per layer, every chunk slot as [u8 state][bytes_per_chunk]
//         (state 0 = never created, 1 = created without data, 2 = has_data)
// stdout: "frame <k> <bytes written>" per frame, then "tiled_frame_bytes <n>"
#include "array.dimensions.hh"
#include "array.tiled.hh"
#include "chunk.hh"

#include <cstdio>
#include <fstream>
#include <iostream>
#include <iterator>
#include <memory>
#include <mutex>
#include <vector>

int
main(int argc, char** argv)
{
    if (argc != 3) {
        std::cerr << "usage: tiled_writer_harness <tiles> <chunks-out> < spec\n";
        return 2;
    }
    size_t ndims = 0, bpp = 0, n_frames = 0;
    int dtype = 0;
    std::cin >> ndims >> bpp >> dtype >> n_frames;
    std::vector<ZarrDimension> dims;
    for (size_t i = 0; i < ndims; ++i) {
        int type = 0;
        uint32_t a = 0, c = 0, s = 0;
        std::cin >> type >> a >> c >> s;
        dims.emplace_back("d" + std::to_string(i),
                          static_cast<ZarrDimensionType>(type), a, c, s);
    }
    try {
        ArrayDimensions ad(std::move(dims), static_cast<ZarrDataType>(dtype));
        const size_t frame_tiles = zarr::tiled::tiled_frame_bytes(ad, bpp);
        std::ifstream in(argv[1], std::ios::binary);
        std::vector<uint8_t> all((std::istreambuf_iterator<char>(in)),
                                 std::istreambuf_iterator<char>());
        if (all.size() != frame_tiles * n_frames) {
            std::cerr << "tiles file holds " << all.size() << " bytes, want "
                      << frame_tiles * n_frames << "\n";
            return 3;
        }
        const size_t n_chunks = ad.number_of_chunks_in_memory();
        const size_t per_layer = ad.frames_per_chunk_layer();
        std::vector<std::shared_ptr<zarr::Chunk>> chunks(n_chunks);
        std::vector<std::mutex> mutexes(n_chunks);
        std::ofstream out(argv[2], std::ios::binary);
        const std::vector<uint8_t> zeros(ad.bytes_per_chunk(), 0);
        auto dump = [&]() {
            for (auto& ch : chunks) {
                const uint8_t state = !ch ? 0 : (ch->has_data() ? 2 : 1);
                out.put(static_cast<char>(state));
                const auto& buf = ch ? ch->buffer() : zeros;
                out.write(reinterpret_cast<const char*>(buf.data()), buf.size());
                ch.reset();
            }
        };
        for (size_t k = 0; k < n_frames; ++k) {
            const size_t n = zarr::tiled::write_tiles_to_chunks(
              ad, bpp, k, all.data() + k * frame_tiles, chunks, mutexes);
            std::printf("frame %zu %zu\n", k, n);
            if ((k + 1) % per_layer == 0) {
                dump();
            }
        }
        if (n_frames % per_layer) {
            dump();
        }
        std::printf("tiled_frame_bytes %zu\n", frame_tiles);
    } catch (const std::exception& e) {
        std::cerr << "error: " << e.what() << "\n";
        return 1;
    }
    return 0;
}
