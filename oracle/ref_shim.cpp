/*
 * ref_shim.cpp — C ABI over the REFERENCE's own zarr::Downsampler and
 * ArrayDimensions (TEST INFRASTRUCTURE ONLY).
 *
 * oracle/Makefile's `ref` target compiles, UNMODIFIED and from where they lie
 * under /root/reference, acquire-zarr v0.8.1's
 *   src/streaming/downsampler.cpp        (the hot path, :8-605)
 *   src/streaming/array.dimensions.cpp   (geometry + chunk addressing)
 *   src/streaming/zarr.common.cpp        (bytes_of_type & co.)
 *   src/logger/logger.cpp
 * against the image's genuine nlohmann/json 3.1.1 (/opt/conda/include/json.hpp)
 * and links them with this file into oracle/_ref/libref_downsampler.so.
 * Nothing here restates the algorithm: every call goes to the reference's
 * code.  tests/, bench.py's cpu_baseline leg and tests/golden/
 * make_reference_vectors.py load it through oracle/ref.py; the product
 * (acquire-zarr_amd/) never does.
 *
 * Exceptions thrown by the reference (EXPECT, std::runtime_error) are caught
 * here and reported as -1 plus the message, so the Python side can assert on
 * the reference's own error behaviour.
 */
#include "downsampler.hh"

#include <cstring>
#include <memory>
#include <string>
#include <vector>

namespace {

struct RefDim
{
    int32_t type;
    uint32_t array_size_px;
    uint32_t chunk_size_px;
    uint32_t shard_size_chunks;
    double scale;
};

struct RefDs
{
    std::unique_ptr<zarr::Downsampler> ds;
    std::shared_ptr<ArrayDimensions> dims;
    std::vector<uint8_t> frame; // caller-filled input (ref_ds_frame_buffer)
    std::vector<uint8_t> taken;
    ZarrDataType dtype;
};

void
put_err(char* err, size_t cap, const std::string& msg)
{
    if (err && cap) {
        const size_t n = std::min(cap - 1, msg.size());
        std::memcpy(err, msg.data(), n);
        err[n] = '\0';
    }
}

std::vector<ZarrDimension>
make_dims(const RefDim* d, uint32_t n)
{
    static const char* names[] = { "d0", "d1", "d2", "d3", "d4", "d5", "d6", "d7" };
    std::vector<ZarrDimension> v;
    v.reserve(n);
    for (uint32_t i = 0; i < n; ++i) {
        v.emplace_back(i < 8 ? names[i] : "dn",
                       static_cast<ZarrDimensionType>(d[i].type),
                       d[i].array_size_px,
                       d[i].chunk_size_px,
                       d[i].shard_size_chunks,
                       "",
                       d[i].scale);
    }
    return v;
}

size_t
put_string(const std::string& s, char* out, size_t cap)
{
    if (out && cap) {
        const size_t n = std::min(cap - 1, s.size());
        std::memcpy(out, s.data(), n);
        out[n] = '\0';
    }
    return s.size();
}

} // namespace

extern "C"
{
    /* zarr::Downsampler(config, method) (downsampler.cpp:249-304) on an
     * ArrayConfig("", "/0", …, dims, dtype, method, LOD 0, max_levels). */
    void* ref_ds_create(const RefDim* dims,
                        uint32_t ndims,
                        int dtype,
                        int method,
                        uint32_t max_levels,
                        char* err,
                        size_t errcap)
    {
        try {
            auto h = std::make_unique<RefDs>();
            h->dtype = static_cast<ZarrDataType>(dtype);
            h->dims = std::make_shared<ArrayDimensions>(make_dims(dims, ndims), h->dtype);
            auto config = std::make_shared<zarr::ArrayConfig>(
              "",
              "/0",
              std::nullopt,
              std::nullopt,
              h->dims,
              h->dtype,
              static_cast<ZarrDownsamplingMethod>(method),
              0,
              max_levels);
            h->ds = std::make_unique<zarr::Downsampler>(
              config, static_cast<ZarrDownsamplingMethod>(method));
            return h.release();
        } catch (const std::exception& e) {
            put_err(err, errcap, e.what());
        } catch (...) {
            put_err(err, errcap, "unknown exception");
        }
        return nullptr;
    }

    void ref_ds_destroy(void* h) { delete static_cast<RefDs*>(h); }

    /* writer_configurations().size() */
    uint32_t ref_ds_n_levels(void* h)
    {
        return static_cast<uint32_t>(static_cast<RefDs*>(h)->ds->writer_configurations().size());
    }

    /* writer_configurations().at(level)->dimensions, in storage order */
    int ref_ds_level_dims(void* h, uint32_t level, RefDim* out, uint32_t cap)
    {
        const auto& cfgs = static_cast<RefDs*>(h)->ds->writer_configurations();
        const auto it = cfgs.find(static_cast<int>(level));
        if (it == cfgs.end())
            return -1;
        const auto& d = *it->second->dimensions;
        if (d.ndims() > cap)
            return -1;
        for (size_t i = 0; i < d.ndims(); ++i) {
            const auto& z = d.at(i);
            out[i] = RefDim{ static_cast<int32_t>(z.type),
                             z.array_size_px,
                             z.chunk_size_px,
                             z.shard_size_chunks,
                             z.scale };
        }
        return static_cast<int>(d.ndims());
    }

    /* A frame buffer owned by the handle: fill it, then ref_ds_add_buffered
     * hands it to add_frame without a copy outside the reference's own. */
    void* ref_ds_frame_buffer(void* h, size_t nbytes)
    {
        auto* r = static_cast<RefDs*>(h);
        r->frame.resize(nbytes);
        return r->frame.data();
    }

    /* Downsampler::add_frame (downsampler.cpp:306-401) */
    int ref_ds_add_buffered(void* h, char* err, size_t errcap)
    {
        try {
            auto* r = static_cast<RefDs*>(h);
            r->ds->add_frame(r->frame);
            return 0;
        } catch (const std::exception& e) {
            put_err(err, errcap, e.what());
        } catch (...) {
            put_err(err, errcap, "unknown exception");
        }
        return -1;
    }

    int ref_ds_add_frame(void* h, const void* src, size_t nbytes, char* err, size_t errcap)
    {
        auto* r = static_cast<RefDs*>(h);
        r->frame.assign(static_cast<const uint8_t*>(src),
                        static_cast<const uint8_t*>(src) + nbytes);
        return ref_ds_add_buffered(h, err, errcap);
    }

    /* Downsampler::take_frame (downsampler.cpp:403-414): 1 and the bytes when
     * a frame was cached (copied out, at most cap bytes), 0 when not. */
    int ref_ds_take_frame(void* h, int level, void* dst, size_t cap, size_t* nbytes)
    {
        auto* r = static_cast<RefDs*>(h);
        r->taken.clear();
        if (!r->ds->take_frame(level, r->taken)) {
            if (nbytes)
                *nbytes = 0;
            return 0;
        }
        if (nbytes)
            *nbytes = r->taken.size();
        if (dst)
            std::memcpy(dst, r->taken.data(), std::min(cap, r->taken.size()));
        return 1;
    }

    /* downsampling_method() (downsampler.cpp:422-438) */
    size_t ref_ds_method_string(void* h, char* out, size_t cap)
    {
        return put_string(static_cast<RefDs*>(h)->ds->downsampling_method(), out, cap);
    }

    /* get_metadata().dump() (downsampler.cpp:440-485) */
    size_t ref_ds_metadata_json(void* h, char* out, size_t cap)
    {
        return put_string(static_cast<RefDs*>(h)->ds->get_metadata().dump(), out, cap);
    }

    /* ArrayDimensions::chunk_lattice_index / tile_group_offset /
     * chunk_internal_offset (array.dimensions.cpp:232-314); all-ones when the
     * reference throws (an invalid dimension index). */
    uint32_t ref_chunk_lattice_index(const RefDim* dims,
                                     uint32_t ndims,
                                     uint64_t frame_id,
                                     uint32_t dim_index,
                                     int dtype)
    {
        try {
            ArrayDimensions d(make_dims(dims, ndims), static_cast<ZarrDataType>(dtype));
            return d.chunk_lattice_index(frame_id, dim_index);
        } catch (...) {
            return ~0u;
        }
    }

    uint64_t ref_tile_group_offset(const RefDim* dims, uint32_t ndims, uint64_t frame_id, int dtype)
    {
        try {
            ArrayDimensions d(make_dims(dims, ndims), static_cast<ZarrDataType>(dtype));
            return d.tile_group_offset(frame_id);
        } catch (...) {
            return ~0ull;
        }
    }

    uint64_t ref_chunk_internal_offset(const RefDim* dims,
                                       uint32_t ndims,
                                       uint64_t frame_id,
                                       int dtype)
    {
        try {
            ArrayDimensions d(make_dims(dims, ndims), static_cast<ZarrDataType>(dtype));
            return d.chunk_internal_offset(frame_id);
        } catch (...) {
            return ~0ull;
        }
    }
}
