// abi_guard.hh — no C++ exception crosses the C ABI.
//
// The reference's public C functions return a ZarrStatusCode and never throw
// (acquire.zarr.cpp:639-645, 679-684).  Every int-returning entry point of
// include/aqz_downsampler.h and include/aqz_codec.h wraps its body in
// try { ... } catch (...) { return ABI_GUARD_FAIL(handle); }, which maps the
// in-flight exception to a status (std::bad_alloc -> AQZ_OUT_OF_MEMORY,
// anything else -> AQZ_INTERNAL_ERROR) and records its text for
// aqz_ds_last_error / aqz_last_error.
#pragma once

#include "aqz_downsampler.h"

#include <cstddef>
#include <exception>
#include <new>
#include <string>

namespace aqz {

void set_last_error(const std::string& msg);

// Call only from inside a catch handler.
inline int
exception_status(std::string* err) noexcept
{
    int rc = AQZ_INTERNAL_ERROR;
    const char* what = "unknown C++ exception";
    try {
        throw;
    } catch (const std::bad_alloc&) {
        rc = AQZ_OUT_OF_MEMORY;
        what = "out of host memory";
    } catch (const std::exception& e) {
        what = e.what();
    } catch (...) {
    }
    try {
        if (err)
            *err = what;
        set_last_error(what);
    } catch (...) {
    }
    return rc;
}

inline std::string*
abi_err_slot(std::nullptr_t)
{
    return nullptr;
}

} // namespace aqz

#define ABI_GUARD_FAIL(h) aqz::exception_status(aqz::abi_err_slot(h))
