// downsampler.cpp — aqz::Downsampler over the C ABI (see downsampler.hh).
#include "downsampler.hh"

#include <regex>
#include <stdexcept>

namespace aqz {

namespace {

[[noreturn]] void
throw_status(int code, const std::string& what)
{
    throw std::runtime_error(what + " (status " + std::to_string(code) + ")");
}

aqz_dimension
to_c(const ZarrDimension& d)
{
    return aqz_dimension{ d.type, d.array_size_px, d.chunk_size_px,
                          d.shard_size_chunks, d.scale };
}

} // namespace

size_t
bytes_of_type(ZarrDataType dtype)
{
    switch (dtype) {
        case ZarrDataType_uint8:
        case ZarrDataType_int8:
            return 1;
        case ZarrDataType_uint16:
        case ZarrDataType_int16:
            return 2;
        case ZarrDataType_uint32:
        case ZarrDataType_int32:
        case ZarrDataType_float32:
            return 4;
        case ZarrDataType_uint64:
        case ZarrDataType_int64:
        case ZarrDataType_float64:
            return 8;
        default:
            throw std::invalid_argument("Invalid data type: " +
                                        std::to_string(int(dtype)));
    }
}

ZarrDimension::ZarrDimension(std::string_view name,
                             ZarrDimensionType type,
                             uint32_t array_size_px,
                             uint32_t chunk_size_px,
                             uint32_t shard_size_chunks,
                             std::string_view unit,
                             double scale)
  : name(name)
  , type(type)
  , scale(scale)
  , array_size_px(array_size_px)
  , chunk_size_px(chunk_size_px)
  , shard_size_chunks(shard_size_chunks)
{
    if (!unit.empty())
        this->unit = std::string(unit);
}

ArrayDimensions::ArrayDimensions(std::vector<ZarrDimension>&& dims,
                                 ZarrDataType dtype)
  : dims_(std::move(dims))
  , dtype_(dtype)
{
    if (dims_.size() < 2)
        throw std::runtime_error("Array must have at least two dimensions.");
    if (dims_.size() == 2)
        dims_.insert(dims_.begin(),
                     ZarrDimension("_singleton", ZarrDimensionType_Other, 1, 1, 1));
    const size_t n = dims_.size();
    if (dims_[n - 2].type != ZarrDimensionType_Space)
        throw std::runtime_error("Second-to-last dimension must be spatial");
    if (dims_[n - 1].type != ZarrDimensionType_Space)
        throw std::runtime_error("Last dimension must be spatial");
}

ArrayConfig::ArrayConfig(std::string_view store_root,
                         std::string_view node_key,
                         std::optional<std::string> bucket_name,
                         std::shared_ptr<ArrayDimensions> dimensions,
                         ZarrDataType dtype,
                         std::optional<ZarrDownsamplingMethod> downsampling_method,
                         uint16_t level_of_detail,
                         uint32_t max_levels)
  : store_root(store_root)
  , node_key(node_key)
  , bucket_name(std::move(bucket_name))
  , dimensions(std::move(dimensions))
  , dtype(dtype)
  , downsampling_method(downsampling_method)
  , level_of_detail(level_of_detail)
  , max_levels(max_levels)
{
    if (downsampling_method &&
        (*downsampling_method < 0 ||
         *downsampling_method >= ZarrDownsamplingMethodCount))
        throw std::runtime_error("Invalid downsampling method: " +
                                 std::to_string(int(*downsampling_method)));
}

Downsampler::Downsampler(std::shared_ptr<ArrayConfig> config,
                         ZarrDownsamplingMethod method,
                         int device)
  : method_(method)
{
    make_writer_configurations_(config);

    if (config->dtype < 0 || config->dtype >= ZarrDataTypeCount)
        throw std::runtime_error("Invalid data type: " +
                                 std::to_string(int(config->dtype)));
    if (method < 0 || method >= ZarrDownsamplingMethodCount)
        throw std::runtime_error("Invalid downsampling method: " +
                                 std::to_string(int(method)));

    std::vector<aqz_level_desc> lv(writer_configurations_.size());
    for (const auto& [level, cfg] : writer_configurations_) {
        const auto& d = *cfg->dimensions;
        lv[level] = aqz_level_desc{ d.width_dim().array_size_px,
                                    d.height_dim().array_size_px,
                                    d.at(d.ndims() - 3).array_size_px };
    }
    const int rc = aqz_ds_create(lv.data(), uint32_t(lv.size()), config->dtype,
                                 method, device, &handle_);
    if (rc != AQZ_OK)
        throw_status(rc, std::string("Failed to create downsampler: ") +
                           aqz_last_error());
}

Downsampler::~Downsampler()
{
    aqz_ds_destroy(handle_);
}

void
Downsampler::make_writer_configurations_(const std::shared_ptr<ArrayConfig>& config)
{
    // Validation as downsampler.cpp:495-504
    if (!config)
        throw std::runtime_error("Null pointer: config");
    const std::string& key = config->node_key;
    if (key.size() < 2 || key.compare(key.size() - 2, 2, "/0") != 0)
        throw std::runtime_error("Invalid node key: '" + key + "'");
    if (config->level_of_detail != 0)
        throw std::runtime_error("Invalid level of detail: " +
                                 std::to_string(config->level_of_detail));

    const auto& base = *config->dimensions;
    const size_t nd = base.ndims();
    std::vector<aqz_dimension> dims(nd);
    for (size_t i = 0; i < nd; ++i)
        dims[i] = to_c(base.at(i));

    uint32_t n_levels = 0;
    int rc = aqz_plan_levels(dims.data(), uint32_t(nd), config->max_levels,
                             nullptr, 0, &n_levels);
    if (rc != AQZ_OK)
        throw_status(rc, aqz_last_error());
    std::vector<aqz_dimension> planned(size_t(n_levels) * nd);
    rc = aqz_plan_levels(dims.data(), uint32_t(nd), config->max_levels,
                         planned.data(), n_levels, &n_levels);
    if (rc != AQZ_OK)
        throw_status(rc, aqz_last_error());

    writer_configurations_.emplace(0, config);
    for (uint32_t level = 1; level < n_levels; ++level) {
        const auto& prev = writer_configurations_.at(int(level) - 1);
        std::vector<ZarrDimension> level_dims(nd);
        for (size_t i = 0; i < nd; ++i) {
            const aqz_dimension& c = planned[size_t(level) * nd + i];
            ZarrDimension d = prev->dimensions->at(i); // name, unit
            d.type = ZarrDimensionType(c.type);
            d.array_size_px = c.array_size_px;
            d.chunk_size_px = c.chunk_size_px;
            d.shard_size_chunks = c.shard_size_chunks;
            d.scale = c.scale;
            level_dims[i] = std::move(d);
        }
        // Same parent node, next level of detail (downsampler.cpp:579-584).
        auto cfg = std::make_shared<ArrayConfig>(
          prev->store_root,
          std::regex_replace(prev->node_key, std::regex("(\\d+)$"),
                             std::to_string(prev->level_of_detail + 1)),
          prev->bucket_name,
          std::make_shared<ArrayDimensions>(std::move(level_dims), prev->dtype),
          prev->dtype,
          prev->downsampling_method,
          uint16_t(prev->level_of_detail + 1));
        writer_configurations_.emplace(cfg->level_of_detail, cfg);
    }
}

void
Downsampler::add_frame(std::vector<uint8_t>& frame)
{
    const int rc = aqz_ds_add_frame(handle_, frame.data(), frame.size());
    if (rc != AQZ_OK)
        throw_status(rc, aqz_ds_last_error(handle_));
}

bool
Downsampler::take_frame(int level, std::vector<uint8_t>& frame_data)
{
    if (level < 0)
        return false;
    size_t nbytes = 0;
    int has = 0;
    int rc = aqz_ds_take_frame(handle_, uint32_t(level), nullptr, 0, &nbytes, &has);
    if (rc != AQZ_OK)
        throw_status(rc, aqz_ds_last_error(handle_));
    if (!has)
        return false;
    std::vector<uint8_t> out(nbytes);
    rc = aqz_ds_take_frame(handle_, uint32_t(level), out.data(), out.size(),
                           &nbytes, &has);
    if (rc != AQZ_OK)
        throw_status(rc, aqz_ds_last_error(handle_));
    frame_data.swap(out);
    return true;
}

const std::unordered_map<int, std::shared_ptr<ArrayConfig>>&
Downsampler::writer_configurations() const
{
    return writer_configurations_;
}

std::string
Downsampler::downsampling_method() const
{
    const char* name = aqz_method_name(method_);
    if (!name)
        throw std::runtime_error("Invalid downsampling method: " +
                                 std::to_string(int(method_)));
    return name;
}

std::string
Downsampler::get_metadata() const
{
    const char* json = aqz_method_metadata_json(method_);
    if (!json)
        throw std::runtime_error("Invalid downsampling method: " +
                                 std::to_string(int(method_)));
    return json;
}

size_t
Downsampler::device_memory_usage() const
{
    return aqz_ds_device_memory_usage(handle_);
}

} // namespace aqz
