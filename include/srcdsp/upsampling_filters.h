/*
 * Drop-in for SrcDsp's upsampling_filters.h:
 * dsptl::FilterUpsamplingFir<InType, OutType, InternalType, CoefType, L>
 * (reference upsampling_filters.h:36-326), executed by libsrcdsp_hip.so.
 * Instantiations the reference compiles (integer only, dsp_complex.h:87):
 *   <complex<int16_t>, complex<int16_t>, complex<int32_t>, int32_t | int16_t>
 *   <int16_t, int16_t, int32_t, int32_t>
 */
#ifndef SRCDSP_DROPIN_UPSAMPLING_FILTERS_H
#define SRCDSP_DROPIN_UPSAMPLING_FILTERS_H

#include <algorithm>

#include "srcdsp_dropin_common.h"

namespace dsptl {
namespace srcdsp_detail {
template <class In, class Out, class Internal, class Coef>
constexpr int up_variant() {
    using C16 = std::complex<int16_t>;
    using I32 = std::complex<int32_t>;
    return code_of<In, Out, Internal, Coef>() == code_of<C16, C16, I32, int32_t>()              ? 0
           : code_of<In, Out, Internal, Coef>() == code_of<C16, C16, I32, int16_t>()            ? 1
           : code_of<In, Out, Internal, Coef>() == code_of<int16_t, int16_t, int32_t, int32_t>() ? 2
                                                                                                 : -1;
}
}  // namespace srcdsp_detail

template <class InType, class OutType, class InternalType, class CoefType, unsigned L>
class FilterUpsamplingFir {
    static constexpr int kVariant = srcdsp_detail::up_variant<InType, OutType, InternalType, CoefType>();
    static_assert(kVariant >= 0, "FilterUpsamplingFir: limitScale needs integer types (dsp_complex.h:87)");

public:
    /// upsampling_filters.h:86-94
    FilterUpsamplingFir(const std::vector<CoefType> &firCoeff = std::vector<CoefType>()) : h_(nullptr) {
        if (!firCoeff.empty()) setCoefficients(firCoeff);
    }
    ~FilterUpsamplingFir() { srcdsp_up_destroy(h_); }
    /// copies (upsampling_filters.h:36-87 is a value type): taps and the history ring
    FilterUpsamplingFir(const FilterUpsamplingFir &o)
        : h_(srcdsp_detail::clone_handle(o.h_, srcdsp_up_clone, "FilterUpsamplingFir(copy)")) {}
    FilterUpsamplingFir(FilterUpsamplingFir &&o) noexcept : h_(o.h_) { o.h_ = nullptr; }
    FilterUpsamplingFir &operator=(FilterUpsamplingFir o) noexcept {
        std::swap(h_, o.h_);
        return *this;
    }

    /// upsampling_filters.h:107-126
    void setCoefficients(const std::vector<CoefType> &firCoeff) {
        assert(!firCoeff.empty());
        assert(firCoeff.size() % L == 0);
        if (!h_)
            srcdsp_detail::check(srcdsp_up_create(&h_, kVariant, L, firCoeff.data(), (int)firCoeff.size()),
                                 "FilterUpsamplingFir");
        else
            srcdsp_detail::check(srcdsp_up_set_coeffs(h_, firCoeff.data(), (int)firCoeff.size()),
                                 "setCoefficients");
    }
    /// upsampling_filters.h:149-233
    void step(const std::vector<InType> &signal, std::vector<OutType> &filteredSignal, bool flush = false) {
        if (!flush) assert(signal.size() * L == filteredSignal.size());
        srcdsp_detail::check(srcdsp_up_step_host(h_, signal.data(), signal.size(), filteredSignal.data(),
                                                 filteredSignal.size(), flush ? 1 : 0, 0),
                             "FilterUpsamplingFir::step");
    }
    /// upsampling_filters.h:240-323 (output shift 0)
    void step(const std::vector<InType> &signal, typename std::vector<OutType>::iterator filteredSignal,
              bool flush = false) {
        std::vector<OutType> tmp(L * (signal.size() + (flush ? getLength() / L : 0)));
        srcdsp_detail::check(srcdsp_up_step_host(h_, signal.data(), signal.size(), tmp.data(), tmp.size(),
                                                 flush ? 1 : 0, 1),
                             "FilterUpsamplingFir::step(iterator)");
        std::copy(tmp.begin(), tmp.end(), filteredSignal);
    }
    void step(const DeviceSpan<const InType> &signal, DeviceSpan<OutType> out, bool flush = false,
              bool iteratorShift = false, void *stream = nullptr) {
        srcdsp_detail::check(srcdsp_up_step(h_, signal.data, signal.size, out.data, out.size, flush ? 1 : 0,
                                            iteratorShift ? 1 : 0, stream),
                             "FilterUpsamplingFir::step(device)");
    }
    /// upsampling_filters.h:50-55
    void reset() { srcdsp_detail::check(srcdsp_up_reset(h_), "FilterUpsamplingFir::reset"); }
    /// upsampling_filters.h:57-67
    int getLength() const { int a = 0; srcdsp_up_get_length(h_, &a, nullptr, nullptr); return a; }
    int getImpLength() const { int b = 0; srcdsp_up_get_length(h_, nullptr, &b, nullptr); return b; }
    int getUpsamplingRatio() const { return L; }

private:
    srcdsp_up_t h_;
};

}  // namespace dsptl
#endif
