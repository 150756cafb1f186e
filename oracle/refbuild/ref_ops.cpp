// Reference-build harness TU for filters.h, upsampling_filters.h, mixers.h and
// correlators.h.  Canonical include order.  Test infrastructure
// only: instantiates the unmodified reference templates and forwards calls.
#include <cmath>
#include <cassert>
#include <complex>
#include <cstdint>
#include <vector>
#include <array>
#include "filters.h"
#include "upsampling_filters.h"
#include "mixers.h"
#include "correlators.h"
#include "ref_api.h"
#include <cstring>

#define REF_EXPORT __attribute__((visibility("default")))

namespace {
typedef std::complex<float> cf32;
typedef std::complex<int16_t> ci16;
typedef std::complex<int32_t> ci32;

/* ------------------------------ FilterFir ------------------------------ */
struct FirBase {
    virtual ~FirBase() {}
    virtual void step(const void *in, long n, void *out) = 0;
    virtual void reset() = 0;
    virtual void setCoeffs(const void *, int) = 0;
};
template <class In, class Out, class Internal, class Coef> struct FirBox : FirBase {
    FilterFir<In, Out, Internal, Coef> f;
    explicit FirBox(const std::vector<Coef> &c) : f(c) {}
    void step(const void *in, long n, void *out) override {
        std::vector<In> vin(static_cast<const In *>(in), static_cast<const In *>(in) + n);
        std::vector<Out> vout(n);
        f.step(vin, vout);
        std::memcpy(out, vout.data(), n * sizeof(Out));
    }
    void reset() override { f.reset(); }
    void setCoeffs(const void *c, int n) override {
        f.setCoeffs(std::vector<Coef>(static_cast<const Coef *>(c), static_cast<const Coef *>(c) + n));
    }
};
template <class In, class Out, class Internal, class Coef>
FirBase *mkFir(const void *c, int n) {
    return new FirBox<In, Out, Internal, Coef>(
        std::vector<Coef>(static_cast<const Coef *>(c), static_cast<const Coef *>(c) + n));
}

/* ------------------------- FilterUpsamplingFir ------------------------- */
struct UpBase {
    virtual ~UpBase() {}
    virtual void step(const void *in, long n, void *out, bool flush, bool iter) = 0;
    virtual void reset() = 0;
    virtual int length() = 0;
    virtual int impLength() = 0;
};
template <class In, class Out, class Internal, class Coef, unsigned L> struct UpBox : UpBase {
    dsptl::FilterUpsamplingFir<In, Out, Internal, Coef, L> f;
    explicit UpBox(const std::vector<Coef> &c) : f(c) {}
    void step(const void *in, long n, void *out, bool flush, bool iter) override {
        std::vector<In> vin(static_cast<const In *>(in), static_cast<const In *>(in) + n);
        size_t nout = static_cast<size_t>(n) * L + (flush ? L * (f.getLength() / L) : 0);
        std::vector<Out> vout(nout);
        if (iter)
            f.step(vin, vout.begin(), flush);
        else
            f.step(vin, vout, flush);
        std::memcpy(out, vout.data(), nout * sizeof(Out));
    }
    void reset() override { f.reset(); }
    int length() override { return f.getLength(); }
    int impLength() override { return f.getImpLength(); }
};
template <class In, class Out, class Internal, class Coef>
UpBase *mkUp(unsigned L, const void *c, int n) {
    std::vector<Coef> v(static_cast<const Coef *>(c), static_cast<const Coef *>(c) + n);
    switch (L) {
    case 2: return new UpBox<In, Out, Internal, Coef, 2>(v);
    case 3: return new UpBox<In, Out, Internal, Coef, 3>(v);
    case 4: return new UpBox<In, Out, Internal, Coef, 4>(v);
    case 8: return new UpBox<In, Out, Internal, Coef, 8>(v);
    default: return nullptr;
    }
}

/* -------------------------------- Mixer -------------------------------- */
struct MixBase {
    virtual ~MixBase() {}
    virtual void step(const int16_t *in, long n, int16_t *out) = 0;
    virtual void reset(float) = 0;
    virtual void setFrequency(float) = 0;
    virtual void adjustFrequency(float) = 0;
    virtual void state(int *, int *, float *) = 0;
    virtual void table(int16_t *) = 0;
};
// Derived only to read the protected phase/frequency/table members.
template <unsigned N>
struct MixProbe : dsptl::Mixer<ci16, ci16, int16_t, N> {
    typedef dsptl::_Mixer<ci16, ci16, int16_t, N> B;
    int phi() const { return B::phi; }
    int freq() const { return B::freq; }
    float nominal() const { return B::nominalFreq; }
    const std::vector<int16_t> &tab() const { return B::ptable; }
};
template <unsigned N> struct MixBox : MixBase {
    MixProbe<N> m;
    void step(const int16_t *in, long n, int16_t *out) override {
        std::vector<ci16> vin(reinterpret_cast<const ci16 *>(in), reinterpret_cast<const ci16 *>(in) + n);
        std::vector<ci16> vout(n);
        m.step(vin, vout);
        std::memcpy(out, vout.data(), n * sizeof(ci16));
    }
    void reset(float f) override { m.reset(f); }
    void setFrequency(float f) override { m.setFrequency(f); }
    void adjustFrequency(float f) override { m.adjustFrequency(f); }
    void state(int *p, int *f, float *nom) override { *p = m.phi(); *f = m.freq(); *nom = m.nominal(); }
    void table(int16_t *t) override { std::memcpy(t, m.tab().data(), N * sizeof(int16_t)); }
};

/* ------------------------ FixedPatternCorrelator ----------------------- */
struct CorrBase {
    virtual ~CorrBase() {}
    virtual void setPattern(const int32_t *, double) = 0;
    virtual void reset() = 0;
    virtual int step(const int16_t *, long, int *) = 0;
    virtual void bitSamples(int16_t *) = 0;
    virtual void status(uint32_t *, uint32_t *, uint32_t *, int *, double *) = 0;
};
template <size_t N, size_t S> struct CorrBox : CorrBase {
    dsptl::FixedPatternCorrelator<int16_t, int32_t, N, S> c;
    void setPattern(const int32_t *p, double th) override {
        std::array<ci32, N> a;
        for (size_t i = 0; i < N; ++i) a[i] = ci32(p[2 * i], p[2 * i + 1]);
        c.setPattern(a, th);
    }
    void reset() override { c.reset(); }
    int step(const int16_t *in, long n, int *idx) override {
        std::vector<ci16> v(reinterpret_cast<const ci16 *>(in), reinterpret_cast<const ci16 *>(in) + n);
        return c.step(v, *idx) ? 1 : 0;
    }
    void bitSamples(int16_t *out) override {
        std::vector<ci16> b = c.getRefBitSamples();
        std::memcpy(out, b.data(), b.size() * sizeof(ci16));
    }
    void status(uint32_t *e3, uint32_t *c3, uint32_t *ce, int *cs, double *tf) override {
        auto st = c.getStatus();
        for (int i = 0; i < 3; ++i) { e3[i] = st.energyValue[i]; c3[i] = st.corrValue[i]; }
        *ce = st.coeffsEnergy; *cs = st.coeffScaling; *tf = st.thresholdFactor;
    }
};
} // namespace

extern "C" {
REF_EXPORT void *ref_fir_create(int variant, const void *c, int n) {
    switch (variant) {
    case 0: return mkFir<cf32, cf32, cf32, float>(c, n);
    case 1: return mkFir<float, cf32, float, float>(c, n);
    case 2: return mkFir<ci16, ci16, ci32, int32_t>(c, n);
    default: return nullptr;
    }
}
REF_EXPORT void ref_fir_set_coeffs(void *h, const void *c, int n) { static_cast<FirBase *>(h)->setCoeffs(c, n); }
REF_EXPORT void ref_fir_reset(void *h) { static_cast<FirBase *>(h)->reset(); }
REF_EXPORT void ref_fir_step(void *h, const void *in, long n, void *out) { static_cast<FirBase *>(h)->step(in, n, out); }
REF_EXPORT void ref_fir_destroy(void *h) { delete static_cast<FirBase *>(h); }

REF_EXPORT void *ref_up_create(int variant, unsigned L, const void *c, int n) {
    switch (variant) {
    case 0: return mkUp<ci16, ci16, ci32, int32_t>(L, c, n);
    case 1: return mkUp<ci16, ci16, ci32, int16_t>(L, c, n);
    case 2: return mkUp<int16_t, int16_t, int32_t, int32_t>(L, c, n);
    default: return nullptr;
    }
}
REF_EXPORT void ref_up_reset(void *h) { static_cast<UpBase *>(h)->reset(); }
REF_EXPORT int ref_up_get_length(void *h) { return static_cast<UpBase *>(h)->length(); }
REF_EXPORT int ref_up_get_imp_length(void *h) { return static_cast<UpBase *>(h)->impLength(); }
REF_EXPORT void ref_up_step(void *h, const void *in, long n, void *out, int flush) {
    static_cast<UpBase *>(h)->step(in, n, out, flush != 0, false);
}
REF_EXPORT void ref_up_step_iter(void *h, const void *in, long n, void *out, int flush) {
    static_cast<UpBase *>(h)->step(in, n, out, flush != 0, true);
}
REF_EXPORT void ref_up_destroy(void *h) { delete static_cast<UpBase *>(h); }

REF_EXPORT void *ref_mixer_create(unsigned N) {
    switch (N) {
    case 256: return new MixBox<256>();
    case 1024: return new MixBox<1024>();
    case 4096: return new MixBox<4096>();
    default: return nullptr;
    }
}
REF_EXPORT void ref_mixer_reset(void *h, float f) { static_cast<MixBase *>(h)->reset(f); }
REF_EXPORT void ref_mixer_set_frequency(void *h, float f) { static_cast<MixBase *>(h)->setFrequency(f); }
REF_EXPORT void ref_mixer_adjust_frequency(void *h, float f) { static_cast<MixBase *>(h)->adjustFrequency(f); }
REF_EXPORT void ref_mixer_step(void *h, const int16_t *in, long n, int16_t *out) {
    static_cast<MixBase *>(h)->step(in, n, out);
}
REF_EXPORT void ref_mixer_state(void *h, int *phi, int *freq, float *nom) {
    static_cast<MixBase *>(h)->state(phi, freq, nom);
}
REF_EXPORT void ref_mixer_table(void *h, int16_t *t) { static_cast<MixBase *>(h)->table(t); }
REF_EXPORT void ref_mixer_destroy(void *h) { delete static_cast<MixBase *>(h); }

REF_EXPORT void *ref_corr_create(unsigned N, unsigned S) {
    if (N == 32 && S == 4) return new CorrBox<32, 4>();
    if (N == 1024 && S == 1) return new CorrBox<1024, 1>();
    if (N == 16 && S == 1) return new CorrBox<16, 1>();
    if (N == 64 && S == 2) return new CorrBox<64, 2>();
    if (N == 128 && S == 1) return new CorrBox<128, 1>();
    return nullptr;
}
REF_EXPORT void ref_corr_set_pattern(void *h, const int32_t *p, double th) { static_cast<CorrBase *>(h)->setPattern(p, th); }
REF_EXPORT void ref_corr_reset(void *h) { static_cast<CorrBase *>(h)->reset(); }
REF_EXPORT int ref_corr_step(void *h, const int16_t *in, long n, int *idx) {
    return static_cast<CorrBase *>(h)->step(in, n, idx);
}
REF_EXPORT void ref_corr_bit_samples(void *h, int16_t *out) { static_cast<CorrBase *>(h)->bitSamples(out); }
REF_EXPORT void ref_corr_status(void *h, uint32_t *e3, uint32_t *c3, uint32_t *ce, int *cs, double *tf) {
    static_cast<CorrBase *>(h)->status(e3, c3, ce, cs, tf);
}
REF_EXPORT void ref_corr_destroy(void *h) { delete static_cast<CorrBase *>(h); }
}
