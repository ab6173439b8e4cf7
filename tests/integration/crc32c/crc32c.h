// Compile-only stand-in for google/crc32c's public header (the library is
// not in this image).  TEST INFRASTRUCTURE: lets tests/test_integration.py
// run -fsyntax-only over the patched array.cpp; nothing built with it is
// linked or run.  Declares the one entry point array.cpp / shard.cpp call.
#pragma once
#include <cstddef>
#include <cstdint>

namespace crc32c {
uint32_t
Crc32c(const uint8_t* data, size_t count);
uint32_t
Crc32c(const char* data, size_t count);
} // namespace crc32c
