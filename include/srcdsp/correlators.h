/*
 * Drop-in for SrcDsp's correlators.h:
 * dsptl::FixedPatternCorrelator<int16_t, int32_t, N, S>
 * (reference correlators.h:54-316), executed by libsrcdsp_hip.so.
 *
 * CREATE_DEBUG_FILES (correlators.h:29,107-111,128-132,253-257): defined
 * before this header, the constructor opens debug_corr_energy.dat,
 * debug_corr_values.dat and debug_corr_threshold.dat in the working directory
 * and every processed sample appends sqrt(energy), sqrt(corr) and
 * 2.5 sqrt(energy) with the reference's stream formatting; step() then runs
 * srcdsp_corr_step(_host)_trace, which returns those per-sample registers.
 * As in the reference, the object is then movable but not copyable.
 */
#ifndef SRCDSP_DROPIN_CORRELATORS_H
#define SRCDSP_DROPIN_CORRELATORS_H

#include <array>
#include <sstream>
#ifdef CREATE_DEBUG_FILES
#include <cmath>
#include <fstream>
#endif

#include "srcdsp_dropin_common.h"

namespace dsptl {

template <class InType = int16_t, class CompType = int32_t, size_t N = 32, size_t S = 4>
class FixedPatternCorrelator {
    static_assert(std::is_same<InType, int16_t>::value && std::is_same<CompType, int32_t>::value,
                  "FixedPatternCorrelator is provided for <int16_t, int32_t, N, S>");

public:
    /// correlators.h:59-81 (InputEnergy is never written by the reference; 0 here)
    struct CorrState {
        static const int Nelements = 3;
        float InputEnergy;
        uint32_t coeffsEnergy;
        int coeffScaling;
        uint32_t energyValue[Nelements];
        uint32_t corrValue[Nelements];
        double thresholdFactor;
        std::string prettyString() {
            std::ostringstream os;
            os << "Input Energy: " << InputEnergy << '\n';
            os << "Coeffs Energy: " << coeffsEnergy << '\n';
            os << "Coeff Scaling: " << coeffScaling << '\n';
            os << "Threshold Factor: " << thresholdFactor << '\n';
            for (int i = 0; i < Nelements; ++i) os << "Energy Value " << i << ": " << energyValue[i] << '\n';
            for (int i = 0; i < Nelements; ++i) os << "CorrValue " << i << ": " << corrValue[i] << '\n';
            return os.str();
        }
    };

    /// correlators.h:119-132
    FixedPatternCorrelator() : h_(nullptr) {
        srcdsp_detail::check(srcdsp_corr_create(&h_, (unsigned)N, (unsigned)S), "FixedPatternCorrelator");
#ifdef CREATE_DEBUG_FILES
        fenergy.open("debug_corr_energy.dat");
        fcorr.open("debug_corr_values.dat");
        fthreshold.open("debug_corr_threshold.dat");
#endif
    }
    ~FixedPatternCorrelator() { srcdsp_corr_destroy(h_); }
#ifndef CREATE_DEBUG_FILES
    /// copies (correlators.h:54-118 is a value type): pattern, thresholds,
    /// history ring, registers and bitSamples
    FixedPatternCorrelator(const FixedPatternCorrelator &o)
        : h_(srcdsp_detail::clone_handle(o.h_, srcdsp_corr_clone, "FixedPatternCorrelator(copy)")) {}
    FixedPatternCorrelator(FixedPatternCorrelator &&o) noexcept : h_(o.h_) { o.h_ = nullptr; }
    FixedPatternCorrelator &operator=(FixedPatternCorrelator o) noexcept {
        std::swap(h_, o.h_);
        return *this;
    }
#else
    // the reference's std::ofstream members make it move-only
    FixedPatternCorrelator(const FixedPatternCorrelator &) = delete;
    FixedPatternCorrelator &operator=(const FixedPatternCorrelator &) = delete;
    FixedPatternCorrelator(FixedPatternCorrelator &&o) noexcept
        : h_(o.h_), fenergy(std::move(o.fenergy)), fcorr(std::move(o.fcorr)), fthreshold(std::move(o.fthreshold)) {
        o.h_ = nullptr;
    }
    // the reference's implicit move assignment (its ofstream members are
    // move-assignable): take o's handle and streams, o keeps ours to destroy
    FixedPatternCorrelator &operator=(FixedPatternCorrelator &&o) noexcept {
        std::swap(h_, o.h_);
        fenergy = std::move(o.fenergy);
        fcorr = std::move(o.fcorr);
        fthreshold = std::move(o.fthreshold);
        return *this;
    }
#endif

    /// correlators.h:209-303
    bool step(const std::vector<std::complex<InType>> &in, int &corrIndex) {
        int found = 0, idx = corrIndex;
#ifdef CREATE_DEBUG_FILES
        std::vector<uint32_t> c(in.size()), e(in.size());
        size_t cnt = 0;
        srcdsp_detail::check(srcdsp_corr_step_host_trace(h_, in.data(), in.size(), &found, &idx, c.data(), e.data(),
                                                         &cnt),
                             "step");
        debug_write(c, e, cnt);
#else
        srcdsp_detail::check(srcdsp_corr_step_host(h_, in.data(), in.size(), &found, &idx), "step");
#endif
        if (found) corrIndex = idx;
        return found != 0;
    }
    bool step(const DeviceSpan<const std::complex<InType>> &in, int &corrIndex, void *stream = nullptr) {
        int found = 0, idx = corrIndex;
#ifdef CREATE_DEBUG_FILES
        std::vector<uint32_t> c(in.size), e(in.size);
        size_t cnt = 0;
        srcdsp_detail::check(srcdsp_corr_step_trace(h_, in.data, in.size, &found, &idx, c.data(), e.data(), &cnt,
                                                    stream),
                             "step(device)");
        debug_write(c, e, cnt);
#else
        srcdsp_detail::check(srcdsp_corr_step(h_, in.data, in.size, &found, &idx, stream), "step(device)");
#endif
        if (found) corrIndex = idx;
        return found != 0;
    }
    /// correlators.h:167-194
    void setPattern(const std::array<std::complex<CompType>, N> &in, double thresholdCoeff = 0.8) {
        std::vector<int32_t> p(2 * N);
        for (size_t i = 0; i < N; ++i) {
            p[2 * i] = in[i].real();
            p[2 * i + 1] = in[i].imag();
        }
        srcdsp_detail::check(srcdsp_corr_set_pattern(h_, p.data(), thresholdCoeff), "setPattern");
    }
    /// correlators.h:146-159
    void reset() { srcdsp_detail::check(srcdsp_corr_reset(h_), "reset"); }
    /// correlators.h:311-316
    std::vector<std::complex<InType>> getRefBitSamples() {
        std::vector<std::complex<InType>> b(N);
        srcdsp_detail::check(srcdsp_corr_get_bit_samples(h_, reinterpret_cast<int16_t *>(b.data())),
                             "getRefBitSamples");
        return b;
    }
    /// correlators.h:90
    CorrState getStatus() {
        CorrState s{};
        srcdsp_detail::check(srcdsp_corr_get_status(h_, s.energyValue, s.corrValue, &s.coeffsEnergy,
                                                    &s.coeffScaling, &s.thresholdFactor),
                             "getStatus");
        return s;
    }

private:
    srcdsp_corr_t h_;
#ifdef CREATE_DEBUG_FILES
    // correlators.h:108-110 and :254-256: one line per processed sample
    std::ofstream fenergy;
    std::ofstream fcorr;
    std::ofstream fthreshold;
    void debug_write(const std::vector<uint32_t> &c, const std::vector<uint32_t> &e, size_t cnt) {
        for (size_t k = 0; k < cnt; ++k) {
            fenergy << std::sqrt((double)e[k]) << '\n';
            fcorr << std::sqrt((double)c[k]) << '\n';
            fthreshold << std::sqrt((double)e[k]) * 2.5 << '\n';
        }
    }
#endif
};

}  // namespace dsptl
#endif
