// tools/write_frame_probe.cpp — caller-side timing of the MI355X downsampler
// inside a restatement of acquire-zarr's per-frame write path (SURVEY §8(f)
// rows 1-2).  Not product code: it plays the part of the caller,
// `MultiscaleArray::write_frame` (multiscale.array.cpp:57-74,291-325), which
// chunks level 0 through `Array::write_frame_to_chunks_` (array.cpp:507-622,
// an OpenMP loop of `Chunk::write_tile_rows`, chunk.cpp:17-58) and then feeds
// the downsampler and chunks every level it returns.  Compression and sinks
// are left out: they sit after this path and are the same in every mode.
//
// Modes (ms per frame, one 4096^2 u16 stream, 5 levels, 256^2 chunks that
// are 16 frames deep):
//   sync       the reference call order on the drop-in ABI: host-tile level 0,
//              aqz_ds_add_frame, aqz_ds_take_frame per level, host-tile it
//   async      aqz_ds_add_frame_async first, host-tile level 0 while the frame
//              crosses PCIe, then eager-tiled level takes (one memcpy per tile)
//   gpu_tiled  everything tiled on the GPU: add_frame_async, then
//              aqz_ds_take_input_frame (level 0, tiled) and the tiled levels
//   transposed storage order (Y<->X swapped), reference: transpose_frame's
//              per-pixel loop (array.cpp:488-504) then `sync`
//   transposed_gpu the same on the GPU: aqz_ds_set_input_transpose + gpu_tiled
//   async_take the patched MultiscaleArray's order with the level takes in the
//              add's background job (aqz_ds_add_frame_async_take): add, host-
//              tile level 0, wait, place the tiles
// and the parts, each alone: host_tile (level 0 on the OpenMP threads),
// h2d_pageable (add_frame_async + aqz_ds_wait_input: the upload of a
// pageable frame), gpu_side (add_frame_async, wait, tiled takes: everything
// but the host tiling); and, inside `async`, the host tiling's own time while
// the upload runs beside it (async_phases: tile, then the wait that is left,
// then the takes).  bench.py runs this binary for its e2e.caller_cpp entry.
//
// Build: make -C acquire-zarr_amd probe   (hipcc -fopenmp, links the library)
#include "aqz_downsampler.h"

#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

using clk = std::chrono::steady_clock;

void
check(int rc, const char* what, aqz_ds* ds)
{
    if (rc != AQZ_OK) {
        std::fprintf(stderr, "%s failed (%d): %s\n", what, rc,
                     ds ? aqz_ds_last_error(ds) : aqz_last_error());
        std::exit(2);
    }
}

// One level's chunk lattice for one frame group: n_tiles chunk buffers, each
// `depth` frames of tile_rows x tile_cols pixels (the reference's Chunk).
struct Lattice
{
    uint32_t width, height, tile_rows, tile_cols, depth;
    size_t bpp, tile_bytes, n_tiles_x, n_tiles;
    std::vector<std::vector<uint8_t>> chunk;
    std::vector<uint8_t> has_data;

    Lattice(uint32_t w, uint32_t h, uint32_t tr, uint32_t tc, uint32_t d, size_t b)
      : width(w), height(h), tile_rows(tr), tile_cols(tc), depth(d), bpp(b)
    {
        tile_bytes = size_t(tr) * tc * bpp;
        n_tiles_x = (w + tc - 1) / tc;
        n_tiles = n_tiles_x * ((h + tr - 1) / tr);
        chunk.assign(n_tiles, std::vector<uint8_t>(tile_bytes * depth, 0));
        has_data.assign(n_tiles, 0);
    }

    // write_frame_to_chunks_ + write_tile_rows: row copies plus the zero
    // scan, tiles in parallel (array.cpp:575)
    void host_tile(const uint8_t* frame, uint64_t frame_id)
    {
        const size_t off = (frame_id % depth) * tile_bytes;
        const size_t src_stride = size_t(width) * bpp;
        const size_t dst_stride = size_t(tile_cols) * bpp;
#pragma omp parallel for schedule(static)
        for (long t = 0; t < long(n_tiles); ++t) {
            const uint32_t ty = uint32_t(t / n_tiles_x), tx = uint32_t(t % n_tiles_x);
            const uint32_t row0 = ty * tile_rows;
            const uint32_t n_rows = std::min(tile_rows, height - row0);
            const uint32_t col0 = tx * tile_cols;
            const size_t copy = size_t(std::min(col0 + tile_cols, width) - col0) * bpp;
            const uint8_t* s = frame + (size_t(row0) * width + col0) * bpp;
            uint8_t* d = chunk[t].data() + off;
            bool any = has_data[t];
            for (uint32_t r = 0; r < n_rows; ++r) {
                const uint8_t* sr = s + r * src_stride;
                std::memcpy(d + r * dst_stride, sr, copy);
                if (!any)
                    any = std::any_of(sr, sr + copy, [](uint8_t b) { return b != 0; });
            }
            has_data[t] = any;
        }
    }

    // the GPU-tiled form: one contiguous copy per tile, flags precomputed
    void place_tiles(const uint8_t* tiles, const uint8_t* nonzero, uint64_t frame_id)
    {
        const size_t off = (frame_id % depth) * tile_bytes;
#pragma omp parallel for schedule(static)
        for (long t = 0; t < long(n_tiles); ++t) {
            std::memcpy(chunk[t].data() + off, tiles + t * tile_bytes, tile_bytes);
            has_data[t] |= nonzero[t];
        }
    }
};

// transpose_frame (array.cpp:488-504) as the reference runs it: one
// bytes_per_pixel memcpy per pixel, single thread
void
transpose_frame_cpu(const uint8_t* src, uint8_t* dst, uint32_t rows, uint32_t cols, size_t bpp)
{
    for (uint32_t row = 0; row < rows; ++row)
        for (uint32_t col = 0; col < cols; ++col)
            std::memcpy(dst + (size_t(col) * rows + row) * bpp,
                        src + (size_t(row) * cols + col) * bpp, bpp);
}

} // namespace

int
main(int argc, char** argv)
{
    const uint32_t W = 4096, H = 4096, NL = 5, TILE = 256, DEPTH = 16;
    const int frames = argc > 1 ? std::atoi(argv[1]) : 48;
    const int transposed_frames = argc > 2 ? std::atoi(argv[2]) : 4;
    const size_t bpp = 2;
    const int dtype = 1; // ZarrDataType_uint16

    std::vector<aqz_level_desc> lv(NL);
    for (uint32_t l = 0, w = W, h = H; l < NL; ++l, w = (w + 1) / 2, h = (h + 1) / 2)
        lv[l] = { w, h, 1 };

    // 8 distinct frames, a quarter of each zero (exercises the zero scan)
    const size_t fbytes = size_t(W) * H * bpp;
    std::vector<std::vector<uint8_t>> host(8, std::vector<uint8_t>(fbytes));
    uint32_t x = 12345;
    for (auto& f : host) {
        auto* p = reinterpret_cast<uint16_t*>(f.data());
        for (size_t i = 0; i < size_t(W) * H; ++i) {
            x = x * 1664525u + 1013904223u;
            p[i] = uint16_t(x >> 16);
        }
        for (uint32_t r = 0; r < H / 2; ++r)
            std::memset(f.data() + size_t(r) * W * bpp, 0, W / 2 * bpp);
    }

    std::vector<Lattice> lat;
    for (uint32_t l = 0; l < NL; ++l)
        lat.emplace_back(lv[l].width, lv[l].height, std::min(TILE, lv[l].height),
                         std::min(TILE, lv[l].width), DEPTH, bpp);
    std::vector<std::vector<uint8_t>> level_buf(NL), tile_buf(NL), flag_buf(NL);
    for (uint32_t l = 0; l < NL; ++l) {
        level_buf[l].resize(size_t(lv[l].width) * lv[l].height * bpp);
        tile_buf[l].resize(lat[l].n_tiles * lat[l].tile_bytes);
        flag_buf[l].resize(lat[l].n_tiles);
    }
    std::vector<uint8_t> transposed(fbytes);

    aqz_ds* ds = nullptr;
    check(aqz_ds_create(lv.data(), NL, dtype, /*mean*/ 1, -1, &ds), "create", nullptr);
    for (uint32_t l = 1; l < NL; ++l)
        check(aqz_ds_set_level_tiling(ds, l, lat[l].tile_rows, lat[l].tile_cols), "tiling", ds);

    auto take_levels_host = [&](uint64_t id) {
        for (uint32_t l = 1; l < NL; ++l) {
            size_t n = 0;
            int has = 0;
            check(aqz_ds_take_frame(ds, l, level_buf[l].data(), level_buf[l].size(), &n, &has),
                  "take_frame", ds);
            if (has)
                lat[l].host_tile(level_buf[l].data(), id);
        }
    };
    auto take_levels_tiled = [&](uint64_t id) {
        for (uint32_t l = 1; l < NL; ++l) {
            size_t n = 0;
            int has = 0;
            check(aqz_ds_take_frame_tiled(ds, l, lat[l].tile_rows, lat[l].tile_cols,
                                          tile_buf[l].data(), tile_buf[l].size(),
                                          flag_buf[l].data(), &n, &has),
                  "take_frame_tiled", ds);
            if (has)
                lat[l].place_tiles(tile_buf[l].data(), flag_buf[l].data(), id);
        }
    };
    auto take_input_tiled = [&](uint64_t id) {
        size_t n = 0;
        int has = 0;
        check(aqz_ds_take_input_frame(ds, TILE, TILE, tile_buf[0].data(), tile_buf[0].size(),
                                      flag_buf[0].data(), &n, &has),
              "take_input_frame", ds);
        if (has)
            lat[0].place_tiles(tile_buf[0].data(), flag_buf[0].data(), id);
    };

    // async_take: every level taken tiled in the add's background job
    std::vector<aqz_level_take> takes(NL);
    for (uint32_t l = 1; l < NL; ++l) {
        takes[l].mode = AQZ_TAKE_INTO;
        takes[l].tile_rows = lat[l].tile_rows;
        takes[l].tile_cols = lat[l].tile_cols;
        takes[l].dst = tile_buf[l].data();
        takes[l].cap = tile_buf[l].size();
        takes[l].tile_nonzero = flag_buf[l].data();
    }
    auto place_taken = [&](uint64_t id) {
        for (uint32_t l = 1; l < NL; ++l)
            if (takes[l].has_frame)
                lat[l].place_tiles(tile_buf[l].data(), flag_buf[l].data(), id);
    };

    auto run = [&](const char* name, int n, auto&& step) {
        for (int i = 0; i < 2; ++i) // warm-up: first-touch of every buffer
            step(host[i % 8].data(), uint64_t(i));
        const auto t0 = clk::now();
        for (int i = 0; i < n; ++i)
            step(host[i % 8].data(), uint64_t(i));
        const double ms =
          std::chrono::duration<double, std::milli>(clk::now() - t0).count() / n;
        std::printf("%s\"%s\": %.3f", std::strcmp(name, "sync") ? ", " : "", name, ms);
        std::fflush(stdout);
        return ms;
    };

    std::printf("{\"workload\": \"write_frame 4096x4096 u16, 5 levels, 256^2 chunks x %u "
                "frames\", \"omp_threads\": %d, \"ms_per_frame\": {",
                DEPTH, omp_get_max_threads());
    run("sync", frames, [&](const uint8_t* f, uint64_t id) {
        lat[0].host_tile(f, id);
        check(aqz_ds_add_frame(ds, f, fbytes), "add_frame", ds);
        take_levels_host(id);
    });
    double ph_tile = 0, ph_wait = 0, ph_take = 0;
    int ph_n = 0;
    run("async", frames, [&](const uint8_t* f, uint64_t id) {
        const auto t0 = clk::now();
        check(aqz_ds_add_frame_async(ds, f, fbytes), "add_frame_async", ds);
        lat[0].host_tile(f, id); // overlaps the upload and the pyramid
        const auto t1 = clk::now();
        check(aqz_ds_wait(ds), "wait", ds);
        const auto t2 = clk::now();
        take_levels_tiled(id);
        const auto t3 = clk::now();
        ph_tile += std::chrono::duration<double, std::milli>(t1 - t0).count();
        ph_wait += std::chrono::duration<double, std::milli>(t2 - t1).count();
        ph_take += std::chrono::duration<double, std::milli>(t3 - t2).count();
        ++ph_n;
    });
    run("async_take", frames, [&](const uint8_t* f, uint64_t id) {
        check(aqz_ds_add_frame_async_take(ds, f, fbytes, takes.data()), "add_frame_async_take",
              ds);
        lat[0].host_tile(f, id);
        check(aqz_ds_wait(ds), "wait", ds);
        place_taken(id);
    });
    // the same overlapped order with one OpenMP thread fewer: the library's
    // upload thread then has a core of the box's share to itself
    const int nthreads = omp_get_max_threads();
    if (nthreads > 1) {
        omp_set_num_threads(nthreads - 1);
        run("async_one_thread_fewer", frames, [&](const uint8_t* f, uint64_t id) {
            check(aqz_ds_add_frame_async(ds, f, fbytes), "add_frame_async", ds);
            lat[0].host_tile(f, id);
            check(aqz_ds_wait(ds), "wait", ds);
            take_levels_tiled(id);
        });
        run("host_tile_one_thread_fewer", frames,
            [&](const uint8_t* f, uint64_t id) { lat[0].host_tile(f, id); });
        omp_set_num_threads(nthreads);
    }
    run("host_tile", frames, [&](const uint8_t* f, uint64_t id) { lat[0].host_tile(f, id); });
    run("h2d_pageable", frames, [&](const uint8_t* f, uint64_t) {
        check(aqz_ds_add_frame_async(ds, f, fbytes), "add_frame_async", ds);
        check(aqz_ds_wait_input(ds), "wait_input", ds);
        check(aqz_ds_wait(ds), "wait", ds);
    });
    run("gpu_side", frames, [&](const uint8_t* f, uint64_t id) {
        check(aqz_ds_add_frame_async(ds, f, fbytes), "add_frame_async", ds);
        take_levels_tiled(id);
    });
    run("gpu_tiled", frames, [&](const uint8_t* f, uint64_t id) {
        check(aqz_ds_add_frame_async(ds, f, fbytes), "add_frame_async", ds);
        take_input_tiled(id);
        take_levels_tiled(id);
    });
    // transposed storage order: the acquisition frame is H rows x W cols
    run("transposed", transposed_frames, [&](const uint8_t* f, uint64_t id) {
        transpose_frame_cpu(f, transposed.data(), H, W, bpp);
        lat[0].host_tile(transposed.data(), id);
        check(aqz_ds_add_frame(ds, transposed.data(), fbytes), "add_frame", ds);
        take_levels_host(id);
    });
    check(aqz_ds_set_input_transpose(ds, 1), "set_input_transpose", ds);
    run("transposed_gpu", frames, [&](const uint8_t* f, uint64_t id) {
        check(aqz_ds_add_frame_async(ds, f, fbytes), "add_frame_async", ds);
        take_input_tiled(id);
        take_levels_tiled(id);
    });
    std::printf("}, \"async_phases_ms\": {\"add_and_host_tile\": %.3f, \"wait_after_tile\": %.3f, "
                "\"takes\": %.3f}}\n",
                ph_tile / (ph_n ? ph_n : 1), ph_wait / (ph_n ? ph_n : 1),
                ph_take / (ph_n ? ph_n : 1));
    aqz_ds_destroy(ds);
    return 0;
}
