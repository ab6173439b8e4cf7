// COMPILE-ONLY STAND-IN for nlohmann/json.hpp (absent from this image).
//
// Used by tests/test_integration.py alone, to syntax- and link-check the
// acquire-zarr HIP integration (integration/) against the reference's own
// headers: downsampler.hh and the array headers include <nlohmann/json.hpp>.
// Every operation is a no-op, so nothing built with it computes JSON — it is
// never an oracle, never linked into the product and never run.
#pragma once

#include <cmath> // the real header brings <cmath> in; array.cpp relies on it
#include <cstddef>
#include <initializer_list>
#include <string>

namespace nlohmann {
class json
{
  public:
    json() = default;
    json(std::nullptr_t) {}
    json(std::initializer_list<json>) {}
    template<typename T>
    json(const T&)
    {
    }

    template<typename T>
    json& operator=(const T&)
    {
        return *this;
    }

    json& operator[](const char*) { return *this; }
    json& operator[](const std::string&) { return *this; }
    json& operator[](int) { return *this; }
    json& operator[](std::size_t) { return *this; }
    const json& operator[](const char*) const { return *this; }

    template<typename T>
    void push_back(const T&)
    {
    }
    void push_back(std::initializer_list<json>) {}

    static json object() { return {}; }
    static json object(std::initializer_list<json>) { return {}; }
    static json array() { return {}; }
    static json array(std::initializer_list<json>) { return {}; }
};
} // namespace nlohmann
