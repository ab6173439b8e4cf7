// downsampler.hh — C++ host side of the MI355X downsampler, mirroring the
// reference's internal interface `zarr::Downsampler`
// (acquire-zarr v0.8.1 src/streaming/downsampler.hh:11-64) over the C ABI in
// include/aqz_downsampler.h.
//
// Same names, argument meaning and error behaviour as the reference:
//   Downsampler(config, method)         throws std::runtime_error on a bad
//                                        node key / LOD / dtype / method
//   add_frame(std::vector<uint8_t>&)    throws on a size mismatch or a
//                                        device error
//   take_frame(level, vector&) -> bool  hands the cached frame over, not
//                                        idempotent
//   writer_configurations()             level -> ArrayConfig
//   downsampling_method(), get_metadata()
// `get_metadata()` returns the JSON text (the reference returns an
// nlohmann::json object; nlohmann is not part of this build).
//
// The small value types below (ZarrDimension, ArrayDimensions, ArrayConfig)
// carry only what the pyramid reads from their reference counterparts
// (array.dimensions.hh:12-43,45-281; array.base.hh:15-57).
#pragma once

#include "aqz_downsampler.h"

#include <cstdint>
#include <memory>
#include <optional>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

namespace aqz {

// Numeric values equal the reference's zarr.types.h enums.
enum ZarrDataType : int
{
    ZarrDataType_uint8 = AQZ_DTYPE_UINT8,
    ZarrDataType_uint16 = AQZ_DTYPE_UINT16,
    ZarrDataType_uint32 = AQZ_DTYPE_UINT32,
    ZarrDataType_uint64 = AQZ_DTYPE_UINT64,
    ZarrDataType_int8 = AQZ_DTYPE_INT8,
    ZarrDataType_int16 = AQZ_DTYPE_INT16,
    ZarrDataType_int32 = AQZ_DTYPE_INT32,
    ZarrDataType_int64 = AQZ_DTYPE_INT64,
    ZarrDataType_float32 = AQZ_DTYPE_FLOAT32,
    ZarrDataType_float64 = AQZ_DTYPE_FLOAT64,
    ZarrDataTypeCount = AQZ_DTYPE_COUNT
};

enum ZarrDownsamplingMethod : int
{
    ZarrDownsamplingMethod_Decimate = AQZ_METHOD_DECIMATE,
    ZarrDownsamplingMethod_Mean = AQZ_METHOD_MEAN,
    ZarrDownsamplingMethod_Min = AQZ_METHOD_MIN,
    ZarrDownsamplingMethod_Max = AQZ_METHOD_MAX,
    ZarrDownsamplingMethodCount = AQZ_METHOD_COUNT
};

enum ZarrDimensionType : int
{
    ZarrDimensionType_Space = AQZ_DIM_SPACE,
    ZarrDimensionType_Channel = AQZ_DIM_CHANNEL,
    ZarrDimensionType_Time = AQZ_DIM_TIME,
    ZarrDimensionType_Other = AQZ_DIM_OTHER
};

size_t bytes_of_type(ZarrDataType dtype);

struct ZarrDimension
{
    ZarrDimension() = default;
    ZarrDimension(std::string_view name,
                  ZarrDimensionType type,
                  uint32_t array_size_px,
                  uint32_t chunk_size_px,
                  uint32_t shard_size_chunks,
                  std::string_view unit = "",
                  double scale = 1.0);

    std::string name;
    ZarrDimensionType type{ ZarrDimensionType_Space };
    std::optional<std::string> unit;
    double scale{ 1.0 };
    uint32_t array_size_px{ 0 };
    uint32_t chunk_size_px{ 0 };
    uint32_t shard_size_chunks{ 0 };
};

// Storage-order dimensions.  A 2-D array gets the reference's phantom
// singleton dimension in front (array.dimensions.cpp:149-152); the last two
// dimensions must be spatial (:156-163).
class ArrayDimensions
{
  public:
    ArrayDimensions(std::vector<ZarrDimension>&& dims, ZarrDataType dtype);

    size_t ndims() const { return dims_.size(); }
    const ZarrDimension& at(size_t i) const { return dims_.at(i); }
    const ZarrDimension& operator[](size_t i) const { return dims_[i]; }
    const ZarrDimension& height_dim() const { return dims_[dims_.size() - 2]; }
    const ZarrDimension& width_dim() const { return dims_.back(); }
    ZarrDataType dtype() const { return dtype_; }

  private:
    std::vector<ZarrDimension> dims_;
    ZarrDataType dtype_;
};

struct ArrayConfig
{
    ArrayConfig() = default;
    ArrayConfig(std::string_view store_root,
                std::string_view node_key,
                std::optional<std::string> bucket_name,
                std::shared_ptr<ArrayDimensions> dimensions,
                ZarrDataType dtype,
                std::optional<ZarrDownsamplingMethod> downsampling_method,
                uint16_t level_of_detail,
                uint32_t max_levels = 0);

    std::string store_root;
    std::string node_key;
    std::optional<std::string> bucket_name;
    std::shared_ptr<ArrayDimensions> dimensions;
    ZarrDataType dtype{ ZarrDataType_uint8 };
    std::optional<ZarrDownsamplingMethod> downsampling_method;
    uint16_t level_of_detail{ 0 };
    uint32_t max_levels{ 0 };
};

class Downsampler
{
  public:
    // `device` = HIP ordinal, -1 = $AQZ_GPU_DEVICE or the current device.
    Downsampler(std::shared_ptr<ArrayConfig> config,
                ZarrDownsamplingMethod method,
                int device = -1);
    ~Downsampler();

    Downsampler(const Downsampler&) = delete;
    Downsampler& operator=(const Downsampler&) = delete;

    void add_frame(std::vector<uint8_t>& frame);
    bool take_frame(int level, std::vector<uint8_t>& frame_data);

    const std::unordered_map<int, std::shared_ptr<ArrayConfig>>&
    writer_configurations() const;

    std::string downsampling_method() const;
    std::string get_metadata() const;

    // Not in the reference: bytes of device memory this instance holds.
    size_t device_memory_usage() const;

  private:
    ZarrDownsamplingMethod method_;
    std::unordered_map<int, std::shared_ptr<ArrayConfig>> writer_configurations_;
    aqz_ds* handle_ = nullptr;

    void make_writer_configurations_(const std::shared_ptr<ArrayConfig>& config);
};

} // namespace aqz
