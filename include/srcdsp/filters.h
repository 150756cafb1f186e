/*
 * Drop-in for SrcDsp's filters.h: ::FilterFir<InType, OutType, InternalType,
 * CoefType> in the GLOBAL namespace (reference filters.h:42-169), executed by
 * libsrcdsp_hip.so.  Instantiations the reference compiles:
 *   <complex<float>, complex<float>, complex<float>, float>
 *   <float, complex<float>, float, float>
 *   <complex<int16_t>, complex<int16_t>, complex<int32_t>, int32_t>
 */
#ifndef SRCDSP_DROPIN_FILTERS_H
#define SRCDSP_DROPIN_FILTERS_H

#include "srcdsp_dropin_common.h"

#ifndef SRCDSP_DEFAULT_FLAGS
#define SRCDSP_DEFAULT_FLAGS 0u
#endif

namespace dsptl {
namespace srcdsp_detail {
template <class In, class Out, class Internal, class Coef>
constexpr int fir_variant() {
    using C32 = std::complex<float>;
    using C16 = std::complex<int16_t>;
    using I32 = std::complex<int32_t>;
    return code_of<In, Out, Internal, Coef>() == code_of<C32, C32, C32, float>()        ? 0
           : code_of<In, Out, Internal, Coef>() == code_of<float, C32, float, float>()  ? 1
           : code_of<In, Out, Internal, Coef>() == code_of<C16, C16, I32, int32_t>()   ? 2
                                                                                        : -1;
}
}  // namespace srcdsp_detail
}  // namespace dsptl

template <class InType, class OutType, class InternalType, class CoefType>
class FilterFir {
    static constexpr int kVariant = dsptl::srcdsp_detail::fir_variant<InType, OutType, InternalType, CoefType>();
    static_assert(kVariant >= 0, "FilterFir: this type combination does not compile in the reference "
                                 "(filters.h:164 returns complex<int16_t>)");

public:
    FilterFir() : h_(nullptr) {}  // filters.h:49
    FilterFir(const std::vector<CoefType> &firCoeff, unsigned flags = SRCDSP_DEFAULT_FLAGS)
        : h_(nullptr), flags_(flags) {
        setCoeffs(firCoeff);
    }
    ~FilterFir() { srcdsp_fir_destroy(h_); }
    /// copies (filters.h:42-70 is a value type): taps, shift, history
    FilterFir(const FilterFir &o) : h_(dsptl::srcdsp_detail::clone_handle(o.h_, srcdsp_fir_clone, "FilterFir(copy)")), flags_(o.flags_) {}
    FilterFir(FilterFir &&o) noexcept : h_(o.h_), flags_(o.flags_) { o.h_ = nullptr; }
    FilterFir &operator=(FilterFir o) noexcept {
        std::swap(h_, o.h_);
        std::swap(flags_, o.flags_);
        return *this;
    }

    /// filters.h:131-169 ; filteredSignal.size() == signal.size()
    void step(const std::vector<InType> &signal, std::vector<OutType> &filteredSignal) {
        assert(signal.size() == filteredSignal.size());
        dsptl::srcdsp_detail::check(
            srcdsp_fir_step_host(h_, signal.data(), signal.size(), filteredSignal.data(), filteredSignal.size()),
            "FilterFir::step");
    }
    void step(const dsptl::DeviceSpan<const InType> &signal, dsptl::DeviceSpan<OutType> filteredSignal,
              void *stream = nullptr) {
        dsptl::srcdsp_detail::check(
            srcdsp_fir_step(h_, signal.data, signal.size, filteredSignal.data, filteredSignal.size, stream),
            "FilterFir::step(device)");
    }
    /// filters.h:107-113
    void reset() { dsptl::srcdsp_detail::check(srcdsp_fir_reset(h_), "FilterFir::reset"); }
    /// filters.h:86-97
    void setCoeffs(const std::vector<CoefType> &firCoeff) {
        if (!h_)
            dsptl::srcdsp_detail::check(
                srcdsp_fir_create(&h_, kVariant, firCoeff.data(), (int)firCoeff.size(), flags_), "FilterFir");
        else
            dsptl::srcdsp_detail::check(srcdsp_fir_set_coeffs(h_, firCoeff.data(), (int)firCoeff.size()),
                                        "FilterFir::setCoeffs");
    }

private:
    srcdsp_fir_t h_;
    unsigned flags_ = SRCDSP_DEFAULT_FLAGS;
};

#endif
