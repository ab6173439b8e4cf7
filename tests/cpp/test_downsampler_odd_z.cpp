// Odd-Z known-answer tests of aqz::Downsampler (GPU path through the C ABI),
// restating acquire-zarr v0.8.1 tests/unit-tests/downsampler-odd-z.cpp:
//   * z = 15 planes, u8, 64x48: 7 pairs emit on every 2nd plane and the 15th
//     plane passes through alone (:88-132), three stacks in a row (:163-165);
//   * T2 x C2 x Z3 channel sequence must not bleed across stacks (:19-86,
//     acquire-zarr#226).
#include "downsampler.hh"
#include "test_macros.hh"

#include <vector>

using namespace aqz;

namespace {

void
fifteen_plane_stacks()
{
    auto dims = std::make_shared<ArrayDimensions>(
      std::vector<ZarrDimension>{ { "t", ZarrDimensionType_Time, 0, 1, 1 },
                                  { "z", ZarrDimensionType_Space, 15, 3, 1 },
                                  { "y", ZarrDimensionType_Space, 48, 16, 1 },
                                  { "x", ZarrDimensionType_Space, 64, 16, 1 } },
      ZarrDataType_uint8);
    auto cfg = std::make_shared<ArrayConfig>("", "/0", std::nullopt, dims,
                                             ZarrDataType_uint8,
                                             ZarrDownsamplingMethod_Mean, 0);
    Downsampler ds(cfg, ZarrDownsamplingMethod_Mean);
    const auto& cfgs = ds.writer_configurations();
    REQUIRE(cfgs.size() > 1, "at least 2 levels");
    REQUIRE_EQ(uint32_t, cfgs.at(1)->dimensions->at(1).array_size_px, 8);

    for (uint8_t value : { uint8_t(63), uint8_t(127), uint8_t(255) }) {
        std::vector<uint8_t> plane(64 * 48, value);
        int pairs = 0;
        for (int z = 0; z < 15; ++z) {
            ds.add_frame(plane);
            if (z % 2 == 1) {
                std::vector<uint8_t> out;
                REQUIRE(ds.take_frame(1, out), "pair ready at plane ", z);
                ++pairs;
                for (uint8_t v : out)
                    REQUIRE_EQ(int, v, value);
            }
        }
        REQUIRE_EQ(int, pairs, 7);
        std::vector<uint8_t> last;
        REQUIRE(ds.take_frame(1, last), "odd last plane passes through");
        for (uint8_t v : last)
            REQUIRE_EQ(int, v, value);
    }
}

void
no_bleed_between_stacks()
{
    auto dims = std::make_shared<ArrayDimensions>(
      std::vector<ZarrDimension>{ { "t", ZarrDimensionType_Time, 0, 1, 1 },
                                  { "c", ZarrDimensionType_Channel, 2, 1, 2 },
                                  { "z", ZarrDimensionType_Space, 3, 1, 1 },
                                  { "y", ZarrDimensionType_Space, 8, 4, 1 },
                                  { "x", ZarrDimensionType_Space, 8, 4, 1 } },
      ZarrDataType_uint16);
    auto cfg = std::make_shared<ArrayConfig>("", "/0", std::nullopt, dims,
                                             ZarrDataType_uint16,
                                             ZarrDownsamplingMethod_Mean, 0);
    Downsampler ds(cfg, ZarrDownsamplingMethod_Mean);

    std::vector<uint16_t> seen;
    for (int t = 0; t < 2; ++t) {
        for (uint16_t value : { uint16_t(100), uint16_t(200) }) {
            for (int z = 0; z < 3; ++z) {
                std::vector<uint8_t> plane(8 * 8 * 2);
                for (size_t i = 0; i < 64; ++i) {
                    plane[2 * i] = uint8_t(value & 0xff);
                    plane[2 * i + 1] = uint8_t(value >> 8);
                }
                ds.add_frame(plane);
                std::vector<uint8_t> out;
                if (ds.take_frame(1, out)) {
                    const uint16_t first = uint16_t(out[0] | (out[1] << 8));
                    for (size_t i = 0; i < out.size() / 2; ++i)
                        REQUIRE_EQ(int, out[2 * i] | (out[2 * i + 1] << 8), first);
                    seen.push_back(first);
                }
            }
        }
    }
    const std::vector<uint16_t> want = { 100, 100, 200, 200, 100, 100, 200, 200 };
    REQUIRE_EQ(size_t, seen.size(), want.size());
    for (size_t i = 0; i < want.size(); ++i)
        REQUIRE_EQ(int, seen[i], want[i]);
    std::vector<uint8_t> leftover;
    REQUIRE(!ds.take_frame(1, leftover), "no leftover level-1 frame");
}

} // namespace

int
main()
{
    try {
        RUN(fifteen_plane_stacks);
        RUN(no_bleed_between_stacks);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "FAILED: %s\n", e.what());
        return 1;
    }
    std::printf("test_downsampler_odd_z: all passed\n");
    return 0;
}
