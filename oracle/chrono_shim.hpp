// Test infrastructure only (oracle/_ref build). libstdc++ 11 lacks C++20 chrono
// stream output, which the reference uses only in log lines (BVH.hpp:441,785,
// Integrators.cpp:127). This prints the raw tick count; it changes no result.
#pragma once
#include <chrono>
#include <ostream>
namespace std::chrono {
template <class C, class T, class R, class P>
std::basic_ostream<C, T>& operator<<(std::basic_ostream<C, T>& os, const duration<R, P>& d) {
    return os << d.count();
}
}  // namespace std::chrono
