/*
 * Drop-in for SrcDsp's dnsampling_filters.h / dsptl_dnsampling_filters.h:
 * dsptl::FilterDnsamplingFir<InType, OutType, InternalType, CoefType, M>
 * (reference: dnsampling_filters.h:49-172, dsptl_dnsampling_filters.h:47-220),
 * executed by libsrcdsp_hip.so on MI355X.
 *
 * Supported instantiations = those the reference compiles:
 *   <complex<float>,   complex<float>,   complex<float>,   float>
 *   <complex<int16_t>, complex<int16_t>, complex<int32_t>, int32_t | int16_t>
 *   <complex<int32_t>, complex<int16_t>, complex<int32_t>, int32_t>
 * Others fail to compile, as in the reference.
 *
 * Float contract: SRCDSP_DEFAULT_FLAGS (default 0 = sequential FMA per output,
 * bit-exact to the reference built with -mfma); define it to
 * SRCDSP_FLAG_FP_STRICT for bit-exactness with the -O2 x86-64 build.
 */
#ifndef SRCDSP_DROPIN_DNSAMPLING_FILTERS_H
#define SRCDSP_DROPIN_DNSAMPLING_FILTERS_H

#include "srcdsp_dropin_common.h"

#ifndef SRCDSP_DEFAULT_FLAGS
#define SRCDSP_DEFAULT_FLAGS 0u
#endif

namespace dsptl {
namespace srcdsp_detail {
template <class In, class Out, class Internal, class Coef>
constexpr int decim_variant() {
    using C32 = std::complex<float>;
    using C16 = std::complex<int16_t>;
    using I32 = std::complex<int32_t>;
    return code_of<In, Out, Internal, Coef>() == code_of<C32, C32, C32, float>()       ? 0
           : code_of<In, Out, Internal, Coef>() == code_of<C16, C16, I32, int32_t>()  ? 1
           : code_of<In, Out, Internal, Coef>() == code_of<C16, C16, I32, int16_t>()  ? 2
           : code_of<In, Out, Internal, Coef>() == code_of<I32, C16, I32, int32_t>()  ? 3
                                                                                       : -1;
}
}  // namespace srcdsp_detail

template <class InType, class OutType, class InternalType, class CoefType, unsigned M>
class FilterDnsamplingFir {
    static constexpr int kVariant = srcdsp_detail::decim_variant<InType, OutType, InternalType, CoefType>();
    static_assert(kVariant >= 0,
                  "FilterDnsamplingFir: this type combination does not compile in the reference "
                  "(limitScale16 returns complex<int16_t>, dsptl_dnsampling_filters.h:215)");
    static_assert(M >= 1, "decimation ratio");

public:
    /// dsptl_dnsampling_filters.h:81-83 -- uninitialised until setCoeffs()
    FilterDnsamplingFir() : h_(nullptr) {}
    /// dnsampling_filters.h:84-97 (a converting constructor, as the reference's :52)
    FilterDnsamplingFir(const std::vector<CoefType> &firCoeff, unsigned flags = SRCDSP_DEFAULT_FLAGS)
        : h_(nullptr), flags_(flags) {
        srcdsp_detail::check(
            srcdsp_decim_create(&h_, kVariant, M, firCoeff.data(), (int)firCoeff.size(), flags_),
            "FilterDnsamplingFir");
    }
    ~FilterDnsamplingFir() { srcdsp_decim_destroy(h_); }
    /// copies (dnsampling_filters.h:47-79 is a value type): coefficients,
    /// shifts and the current history, so a copy continues the stream
    FilterDnsamplingFir(const FilterDnsamplingFir &o)
        : h_(srcdsp_detail::clone_handle(o.h_, srcdsp_decim_clone, "FilterDnsamplingFir(copy)")), flags_(o.flags_) {}
    FilterDnsamplingFir(FilterDnsamplingFir &&o) noexcept : h_(o.h_), flags_(o.flags_) { o.h_ = nullptr; }
    FilterDnsamplingFir &operator=(FilterDnsamplingFir o) noexcept {  // copy-and-swap
        std::swap(h_, o.h_);
        std::swap(flags_, o.flags_);
        return *this;
    }

    /// dsptl_dnsampling_filters.h:114-134 (asserts N % M == 0)
    void setCoeffs(const std::vector<CoefType> &firCoeff) {
        assert(firCoeff.size() % M == 0);
        if (!h_)
            srcdsp_detail::check(
                srcdsp_decim_create(&h_, kVariant, M, firCoeff.data(), (int)firCoeff.size(), flags_),
                "setCoeffs");
        else
            srcdsp_detail::check(srcdsp_decim_set_coeffs(h_, firCoeff.data(), (int)firCoeff.size(), 1),
                                 "setCoeffs");
    }
    /// dnsampling_filters.h:129-172: filteredSignal pre-sized to input.size()/M
    void step(const std::vector<InType> &input, std::vector<OutType> &filteredSignal) {
        assert(filteredSignal.size() * M == input.size());
        srcdsp_detail::check(srcdsp_decim_step_host(h_, input.data(), input.size(), filteredSignal.data(),
                                                    filteredSignal.size()),
                             "FilterDnsamplingFir::step");
    }
    /// device-resident overload (asynchronous on `stream`, a hipStream_t)
    void step(const DeviceSpan<const InType> &input, DeviceSpan<OutType> filteredSignal, void *stream = nullptr) {
        srcdsp_detail::check(srcdsp_decim_step(h_, input.data, input.size, filteredSignal.data,
                                               filteredSignal.size, stream),
                             "FilterDnsamplingFir::step(device)");
    }
    /// dnsampling_filters.h:56-60
    void reset() { srcdsp_detail::check(srcdsp_decim_reset(h_), "reset"); }
    /// dnsampling_filters.h:63
    void setLeftShiftBy2(int leftShiftBy2) {
        srcdsp_detail::check(srcdsp_decim_set_left_shift(h_, leftShiftBy2), "setLeftShiftBy2");
    }
    srcdsp_decim_t handle() const { return h_; }

private:
    srcdsp_decim_t h_;
    unsigned flags_ = SRCDSP_DEFAULT_FLAGS;
};

}  // namespace dsptl
#endif
