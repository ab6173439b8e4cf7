// Minimal check helpers for the C++ parity tests (a failed check throws, the
// test's main() returns 1) — the same pass/fail contract as the reference's
// tests/unit-tests/unit.test.macros.hh, written independently.
#pragma once

#include <cstdio>
#include <sstream>
#include <stdexcept>
#include <string>

namespace aqz_test {

template<typename... Args>
std::string
cat(Args&&... args)
{
    std::ostringstream os;
    (os << ... << args);
    return os.str();
}

inline void
check(bool ok, const std::string& what, const char* file, int line)
{
    if (!ok)
        throw std::runtime_error(cat(file, ":", line, ": ", what));
}

} // namespace aqz_test

#define REQUIRE(cond, ...)                                                     \
    ::aqz_test::check((cond), ::aqz_test::cat(#cond, " — ", __VA_ARGS__),      \
                      __FILE__, __LINE__)

#define REQUIRE_EQ(T, a, b)                                                    \
    do {                                                                       \
        const T a_ = static_cast<T>(a);                                        \
        const T b_ = static_cast<T>(b);                                        \
        ::aqz_test::check(a_ == b_,                                            \
                          ::aqz_test::cat(#a, " == ", #b, " (", +a_, " vs ",    \
                                          +b_, ")"),                           \
                          __FILE__, __LINE__);                                 \
    } while (0)

#define RUN(fn)                                                                \
    do {                                                                       \
        fn();                                                                  \
        std::printf("  ok  %s\n", #fn);                                        \
    } while (0)
