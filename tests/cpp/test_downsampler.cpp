// Known-answer tests of aqz::Downsampler (GPU path through the C ABI).
//
// Each case restates one test of the reference suite
// acquire-zarr v0.8.1 tests/unit-tests/downsampler.cpp (cited per case):
// same configurations, same inputs, same expected values.  Runs on a GPU.
#include "downsampler.hh"
#include "test_macros.hh"

#include <algorithm>
#include <cstring>
#include <vector>

using namespace aqz;

namespace {

using Dims = std::vector<ZarrDimension>;

std::shared_ptr<ArrayConfig>
config_for(Dims dims, ZarrDataType dtype, uint32_t max_levels = 0)
{
    auto ad = std::make_shared<ArrayDimensions>(std::move(dims), dtype);
    return std::make_shared<ArrayConfig>("", "/0", std::nullopt, ad, dtype,
                                         ZarrDownsamplingMethod_Mean, 0,
                                         max_levels);
}

template<typename T>
std::vector<uint8_t>
filled(size_t w, size_t h, T value)
{
    std::vector<uint8_t> bytes(w * h * sizeof(T));
    for (size_t i = 0; i < w * h; ++i)
        std::memcpy(bytes.data() + i * sizeof(T), &value, sizeof(T));
    return bytes;
}

template<typename T>
T
pixel(const std::vector<uint8_t>& bytes, size_t i)
{
    T v;
    std::memcpy(&v, bytes.data() + i * sizeof(T), sizeof(T));
    return v;
}

template<typename T>
void
require_all(const std::vector<uint8_t>& bytes, size_t n, T expected)
{
    REQUIRE_EQ(size_t, bytes.size(), n * sizeof(T));
    for (size_t i = 0; i < n; ++i)
        REQUIRE_EQ(T, pixel<T>(bytes, i), expected);
}

Dims
dims_2d(uint32_t yx, uint32_t chunk)
{
    return { { "t", ZarrDimensionType_Time, 0, 5, 1 },
             { "y", ZarrDimensionType_Space, yx, chunk, 1 },
             { "x", ZarrDimensionType_Space, yx, chunk, 1 } };
}

Dims
dims_3d_20()
{
    return { { "t", ZarrDimensionType_Time, 0, 5, 1 },
             { "c", ZarrDimensionType_Channel, 3, 1, 3 },
             { "z", ZarrDimensionType_Space, 20, 5, 1 },
             { "y", ZarrDimensionType_Space, 20, 5, 1 },
             { "x", ZarrDimensionType_Space, 20, 5, 1 } };
}

// downsampler.cpp:25-74
void
basic_downsampling()
{
    Downsampler ds(config_for(dims_2d(10, 5), ZarrDataType_uint8),
                   ZarrDownsamplingMethod_Mean);
    REQUIRE_EQ(size_t, ds.writer_configurations().size(), 2);
    REQUIRE(ds.writer_configurations().count(1) == 1, "level 1 config");

    auto img = filled<uint8_t>(10, 10, 100);
    ds.add_frame(img);
    std::vector<uint8_t> out;
    REQUIRE(ds.take_frame(1, out), "level 1 frame");
    require_all<uint8_t>(out, 25, 100);
    REQUIRE(!ds.take_frame(1, out), "take_frame must not be idempotent");
}

// downsampler.cpp:76-152
void
volume_downsampling()
{
    Downsampler ds(config_for(dims_3d_20(), ZarrDataType_uint16),
                   ZarrDownsamplingMethod_Mean);
    std::vector<uint8_t> out;
    const uint16_t values[4] = { 100, 200, 300, 400 };

    auto f0 = filled<uint16_t>(20, 20, values[0]);
    ds.add_frame(f0);
    REQUIRE(!ds.take_frame(1, out), "level 1 waits for its pair");

    auto f1 = filled<uint16_t>(20, 20, values[1]);
    ds.add_frame(f1);
    REQUIRE(ds.take_frame(1, out), "level 1 after the pair");
    require_all<uint16_t>(out, 100, 150);
    REQUIRE(!ds.take_frame(2, out), "level 2 waits");

    auto f2 = filled<uint16_t>(20, 20, values[2]);
    ds.add_frame(f2);
    REQUIRE(!ds.take_frame(1, out), "level 1 waits after the 3rd plane");
    REQUIRE(!ds.take_frame(2, out), "level 2 waits after the 3rd plane");

    auto f3 = filled<uint16_t>(20, 20, values[3]);
    ds.add_frame(f3);
    REQUIRE(ds.take_frame(2, out), "level 2 after 4 planes");
    require_all<uint16_t>(out, 25, 250);
}

// downsampler.cpp:154-254
template<typename T>
void
one_type(ZarrDataType dt)
{
    Downsampler ds(config_for(dims_2d(10, 5), dt), ZarrDownsamplingMethod_Mean);
    auto img = filled<T>(10, 10, T(100));
    ds.add_frame(img);
    std::vector<uint8_t> out;
    REQUIRE(ds.take_frame(1, out), "frame for dtype ", int(dt));
    REQUIRE_EQ(size_t, out.size(), 25 * sizeof(T));
    require_all<T>(out, 25, T(100));
}

void
all_data_types()
{
    one_type<uint8_t>(ZarrDataType_uint8);
    one_type<uint16_t>(ZarrDataType_uint16);
    one_type<uint32_t>(ZarrDataType_uint32);
    one_type<uint64_t>(ZarrDataType_uint64);
    one_type<int8_t>(ZarrDataType_int8);
    one_type<int16_t>(ZarrDataType_int16);
    one_type<int32_t>(ZarrDataType_int32);
    one_type<int64_t>(ZarrDataType_int64);
    one_type<float>(ZarrDataType_float32);
    one_type<double>(ZarrDataType_float64);
}

// downsampler.cpp:256-314
void
writer_configurations()
{
    const Dims d = { { "t", ZarrDimensionType_Time, 100, 10, 1 },
                     { "c", ZarrDimensionType_Channel, 3, 3, 1 },
                     { "z", ZarrDimensionType_Space, 128, 8, 1 },
                     { "y", ZarrDimensionType_Space, 512, 64, 1 },
                     { "x", ZarrDimensionType_Space, 512, 64, 1 } };
    Downsampler ds(config_for(d, ZarrDataType_uint16), ZarrDownsamplingMethod_Mean);
    const auto& cfgs = ds.writer_configurations();
    REQUIRE_EQ(size_t, cfgs.size(), 5);
    for (const auto& [level, cfg] : cfgs) {
        if (level == 0)
            continue;
        const auto& ld = *cfg->dimensions;
        REQUIRE_EQ(uint32_t, ld.at(0).array_size_px, 100);
        REQUIRE_EQ(uint32_t, ld.at(1).array_size_px, 3);
        for (int i = 2; i < 5; ++i) {
            const uint32_t want =
              std::max(d[i].chunk_size_px, d[i].array_size_px / (1u << level));
            REQUIRE_EQ(uint32_t, ld.at(i).array_size_px, want);
        }
    }
}

// downsampler.cpp:316-409
void
anisotropic_writer_configurations()
{
    const Dims d = { { "t", ZarrDimensionType_Time, 100, 10, 1 },
                     { "c", ZarrDimensionType_Channel, 3, 3, 1 },
                     { "z", ZarrDimensionType_Space, 1000, 128, 1 },
                     { "y", ZarrDimensionType_Space, 2000, 512, 1 },
                     { "x", ZarrDimensionType_Space, 2000, 256, 1 } };
    Downsampler ds(config_for(d, ZarrDataType_uint16), ZarrDownsamplingMethod_Mean);
    const auto& cfgs = ds.writer_configurations();
    REQUIRE_EQ(size_t, cfgs.size(), 4);
    // {level, z size, z chunk, y size, y chunk, x size, x chunk}
    const uint32_t want[3][7] = { { 1, 500, 128, 1000, 512, 1000, 256 },
                                  { 2, 250, 128, 500, 512, 500, 256 },
                                  { 3, 125, 128, 500, 512, 500, 256 } };
    for (const auto& row : want) {
        const auto& ld = *cfgs.at(int(row[0]))->dimensions;
        REQUIRE_EQ(uint32_t, ld.at(0).array_size_px, 100);
        REQUIRE_EQ(uint32_t, ld.at(1).array_size_px, 3);
        for (int k = 0; k < 3; ++k) {
            REQUIRE_EQ(uint32_t, ld.at(2 + k).array_size_px, row[1 + 2 * k]);
            REQUIRE_EQ(uint32_t, ld.at(2 + k).chunk_size_px, row[2 + 2 * k]);
        }
    }
}

// downsampler.cpp:411-445
void
odd_edges()
{
    Downsampler ds(config_for(dims_2d(11, 5), ZarrDataType_uint8),
                   ZarrDownsamplingMethod_Mean);
    std::vector<uint8_t> img(11 * 11, 100);
    ds.add_frame(img);
    std::vector<uint8_t> out;
    REQUIRE(ds.take_frame(1, out), "odd-size frame");
    REQUIRE_EQ(size_t, out.size(), 36);
    require_all<uint8_t>(out, 36, 100);
}

// downsampler.cpp:447-528: every 2x2 block is [100 200; 150 250]
void
min_max_mean_blocks()
{
    std::vector<uint8_t> img(100);
    for (size_t y = 0; y < 10; ++y)
        for (size_t x = 0; x < 10; ++x)
            img[y * 10 + x] = (y % 2 == 0) ? (x % 2 == 0 ? 100 : 200)
                                           : (x % 2 == 0 ? 150 : 250);
    const struct
    {
        ZarrDownsamplingMethod m;
        uint8_t want;
    } cases[] = { { ZarrDownsamplingMethod_Mean, 175 },
                  { ZarrDownsamplingMethod_Min, 100 },
                  { ZarrDownsamplingMethod_Max, 250 },
                  { ZarrDownsamplingMethod_Decimate, 100 } };
    for (const auto& c : cases) {
        Downsampler ds(config_for(dims_2d(10, 5), ZarrDataType_uint8), c.m);
        ds.add_frame(img);
        std::vector<uint8_t> out;
        REQUIRE(ds.take_frame(1, out), "method ", int(c.m));
        require_all<uint8_t>(out, 25, c.want);
    }
}

// downsampler.cpp:530-624
void
volume_min_max()
{
    const struct
    {
        ZarrDownsamplingMethod m;
        uint16_t want;
    } pair_cases[] = { { ZarrDownsamplingMethod_Min, 100 },
                       { ZarrDownsamplingMethod_Max, 200 } };
    for (const auto& c : pair_cases) {
        Downsampler ds(config_for(dims_3d_20(), ZarrDataType_uint16), c.m);
        auto a = filled<uint16_t>(20, 20, 100);
        auto b = filled<uint16_t>(20, 20, 200);
        ds.add_frame(a);
        ds.add_frame(b);
        std::vector<uint8_t> out;
        REQUIRE(ds.take_frame(1, out), "pair for method ", int(c.m));
        require_all<uint16_t>(out, 100, c.want);
    }
    Downsampler ds(config_for(dims_3d_20(), ZarrDataType_uint16),
                   ZarrDownsamplingMethod_Max);
    for (uint16_t v : { 100, 200, 300, 400 }) {
        auto f = filled<uint16_t>(20, 20, v);
        ds.add_frame(f);
    }
    std::vector<uint8_t> out;
    REQUIRE(ds.take_frame(2, out), "level 2 max");
    require_all<uint16_t>(out, 25, 400);
}

// downsampler.cpp:626-729: gradient 100 + 20x + 50y
void
gradient_blocks()
{
    std::vector<uint8_t> img(8 * 8 * 2);
    auto px = [](size_t x, size_t y) { return uint16_t(100 + x * 20 + y * 50); };
    for (size_t y = 0; y < 8; ++y)
        for (size_t x = 0; x < 8; ++x) {
            const uint16_t v = px(x, y);
            std::memcpy(img.data() + (y * 8 + x) * 2, &v, 2);
        }
    for (auto m : { ZarrDownsamplingMethod_Mean, ZarrDownsamplingMethod_Min,
                    ZarrDownsamplingMethod_Max }) {
        Downsampler ds(config_for(dims_2d(8, 4), ZarrDataType_uint16), m);
        ds.add_frame(img);
        std::vector<uint8_t> out;
        REQUIRE(ds.take_frame(1, out), "gradient method ", int(m));
        for (size_t y = 0; y < 4; ++y)
            for (size_t x = 0; x < 4; ++x) {
                const uint16_t a = px(2 * x, 2 * y), b = px(2 * x + 1, 2 * y);
                const uint16_t c = px(2 * x, 2 * y + 1), d = px(2 * x + 1, 2 * y + 1);
                uint16_t want;
                if (m == ZarrDownsamplingMethod_Mean)
                    want = uint16_t((a + b + c + d) / 4);
                else if (m == ZarrDownsamplingMethod_Min)
                    want = std::min(std::min(a, b), std::min(c, d));
                else
                    want = std::max(std::max(a, b), std::max(c, d));
                REQUIRE_EQ(uint16_t, pixel<uint16_t>(out, y * 4 + x), want);
            }
    }
}

// downsampler.cpp:730-785
void
max_levels()
{
    const Dims d = { { "t", ZarrDimensionType_Time, 100, 10, 1 },
                     { "y", ZarrDimensionType_Space, 512, 64, 1 },
                     { "x", ZarrDimensionType_Space, 512, 64, 1 } };
    Downsampler capped(config_for(d, ZarrDataType_uint16, 2),
                       ZarrDownsamplingMethod_Mean);
    const auto& c = capped.writer_configurations();
    REQUIRE_EQ(size_t, c.size(), 3);
    REQUIRE(c.count(0) && c.count(1) && c.count(2) && !c.count(3), "levels 0-2");

    Downsampler open(config_for(d, ZarrDataType_uint16, 0),
                     ZarrDownsamplingMethod_Mean);
    REQUIRE(open.writer_configurations().size() > 3, "no limit => more levels");
}

// Constructor error behaviour (downsampler.cpp:249-304, 493-504).
void
constructor_errors()
{
    auto cfg = config_for(dims_2d(10, 5), ZarrDataType_uint8);
    bool threw = false;
    try {
        Downsampler ds(cfg, ZarrDownsamplingMethod(7));
    } catch (const std::runtime_error&) {
        threw = true;
    }
    REQUIRE(threw, "invalid method must throw");

    auto bad = config_for(dims_2d(10, 5), ZarrDataType_uint8);
    bad->node_key = "/1";
    threw = false;
    try {
        Downsampler ds(bad, ZarrDownsamplingMethod_Mean);
    } catch (const std::runtime_error&) {
        threw = true;
    }
    REQUIRE(threw, "node key must end in /0");

    Downsampler ds(cfg, ZarrDownsamplingMethod_Mean);
    std::vector<uint8_t> wrong(99);
    threw = false;
    try {
        ds.add_frame(wrong);
    } catch (const std::runtime_error&) {
        threw = true;
    }
    REQUIRE(threw, "wrong frame size must throw");
    REQUIRE(ds.downsampling_method() == "local_mean", "method name");
    REQUIRE(ds.get_metadata().find("downscale_local_mean") != std::string::npos,
            "metadata");
}

} // namespace

int
main()
{
    try {
        RUN(basic_downsampling);
        RUN(volume_downsampling);
        RUN(all_data_types);
        RUN(writer_configurations);
        RUN(anisotropic_writer_configurations);
        RUN(odd_edges);
        RUN(min_max_mean_blocks);
        RUN(volume_min_max);
        RUN(gradient_blocks);
        RUN(max_levels);
        RUN(constructor_errors);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "FAILED: %s\n", e.what());
        return 1;
    }
    std::printf("test_downsampler: all passed\n");
    return 0;
}
