/*
 * srcdsp_dropin_common.h -- shared pieces of the C++ drop-in headers
 * (the headers in include/srcdsp), which keep SrcDsp's class templates, namespaces and
 * step() signatures and forward every call to libsrcdsp_hip.so's C ABI.
 *
 * Build a reference user's code against them by replacing the include path of
 * the SrcDsp tree with include/srcdsp and linking libsrcdsp_hip.so.
 *
 * Errors: where the reference asserts, these wrappers assert too; with NDEBUG
 * (where the reference has undefined behaviour) they throw std::runtime_error.
 */
#ifndef SRCDSP_DROPIN_COMMON_H
#define SRCDSP_DROPIN_COMMON_H

#include <cassert>
#include <complex>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "../srcdsp_hip.h"

namespace dsptl {

/// A device-resident buffer (HIP device pointer + element count) for the
/// device overloads of step(); the host std::vector overloads stage through
/// pinned memory and are PCIe-bound.
template <class T>
struct DeviceSpan {
    T *data;
    size_t size;
};

namespace srcdsp_detail {

inline void check(int rc, const char *what) {
    if (rc != SRCDSP_OK) {
        std::string msg = std::string(what) + ": " + srcdsp_last_error();
        assert(!"libsrcdsp_hip call failed" && what);
        throw std::runtime_error(msg);
    }
}

/// An output buffer shorter than the call writes: the reference writes past
/// its end (undefined behaviour, e.g. mixers.h:172-175); here it asserts, and
/// with NDEBUG throws std::length_error before any byte is staged or launched.
inline void check_size(bool ok, const char *what) {
    assert(ok && "output buffer smaller than the call writes");
    if (!ok) throw std::length_error(std::string(what) + ": output buffer smaller than the input");
}

/// Vector shapes a call needs but the C ABI cannot check (one length for all
/// channels, no output sizes): asserts, and with NDEBUG throws
/// std::length_error before anything is copied or launched.
inline void check_shape(bool ok, const char *what) {
    assert(ok && "buffer shapes do not match the call");
    if (!ok) throw std::length_error(what);
}

template <class T> struct kind;  // sample / coefficient type codes
template <> struct kind<std::complex<float>> { static constexpr int v = 0; };
template <> struct kind<std::complex<int16_t>> { static constexpr int v = 1; };
template <> struct kind<std::complex<int32_t>> { static constexpr int v = 2; };
template <> struct kind<float> { static constexpr int v = 3; };
template <> struct kind<int16_t> { static constexpr int v = 4; };
template <> struct kind<int32_t> { static constexpr int v = 5; };

constexpr int code4(int a, int b, int c, int d) { return ((a * 8 + b) * 8 + c) * 8 + d; }

template <class In, class Out, class Internal, class Coef>
constexpr int code_of() {
    return code4(kind<In>::v, kind<Out>::v, kind<Internal>::v, kind<Coef>::v);
}

/// The reference operators are value types (implicit copy constructor and
/// assignment over their member vectors): a copy here is a new handle with
/// the same coefficients AND the source's current streaming state (history,
/// phase, registers), made through the C ABI's *_clone entry.
template <class H>
inline H clone_handle(H h, int (*clone)(H, H *), const char *what) {
    if (!h) return nullptr;
    H c = nullptr;
    check(clone(h, &c), what);
    return c;
}

}  // namespace srcdsp_detail
}  // namespace dsptl

#endif
