// Reference-build harness TU for buffers.h (FifoWithTimeTrack) and
// dsptl_files.h (binary I/Q capture format).  Test infrastructure only:
// instantiates the unmodified reference templates and forwards calls.
#include <cmath>
#include <cassert>
#include <complex>
#include <cstdint>
#include <vector>
#include <array>
#include <fstream>
#include "buffers.h"
#include "dsptl_files.h"
#include "ref_api.h"
#include <cstring>

#define REF_EXPORT __attribute__((visibility("default")))

namespace {
typedef std::complex<int16_t> ci16;

struct FifoBase {
    virtual ~FifoBase() {}
    virtual void write(const void *in, long n, unsigned sec, double frac) = 0;
    virtual int read(void *out, long n, uint64_t *start) = 0;
    virtual size_t count() = 0;
    virtual void reset() = 0;
    virtual void abs_time(uint64_t tp, double frac, unsigned *sec, double *fs) = 0;
};

template <class T, size_t N>
struct FifoBox : FifoBase {
    dsptl::FifoWithTimeTrack<T, N> f;
    explicit FifoBox(double fs) : f(fs) {}
    void write(const void *in, long n, unsigned sec, double frac) override {
        std::vector<T> v((const T *)in, (const T *)in + n);
        f.write(v, sec, frac);
    }
    int read(void *out, long n, uint64_t *start) override {
        std::vector<T> v((size_t)n);
        bool err = f.read(v, *start);
        std::memcpy(out, v.data(), sizeof(T) * (size_t)n);
        return err ? 1 : 0;
    }
    size_t count() override { return f.count(); }
    void reset() override { f.reset(); }
    void abs_time(uint64_t tp, double frac, unsigned *sec, double *fs) override {
        std::pair<unsigned, double> r = f.getAbsoluteTime(tp, frac);
        *sec = r.first;
        *fs = r.second;
    }
};
}  // namespace

extern "C" {
/* kind 0: <double, 15> (buffers_test.cpp), 1: <complex<int16_t>, 64>,
 *      2: <complex<int16_t>, 1000> */
REF_EXPORT void *ref_fifo_create(int kind, double sampling_frequency) {
    switch (kind) {
    case 0: return new FifoBox<double, 15>(sampling_frequency);
    case 1: return new FifoBox<ci16, 64>(sampling_frequency);
    default: return new FifoBox<ci16, 1000>(sampling_frequency);
    }
}
REF_EXPORT void ref_fifo_write(void *h, const void *in, long n, unsigned sec, double frac) {
    ((FifoBase *)h)->write(in, n, sec, frac);
}
REF_EXPORT int ref_fifo_read(void *h, void *out, long n, uint64_t *start) {
    return ((FifoBase *)h)->read(out, n, start);
}
REF_EXPORT unsigned long ref_fifo_count(void *h) { return (unsigned long)((FifoBase *)h)->count(); }
REF_EXPORT void ref_fifo_reset(void *h) { ((FifoBase *)h)->reset(); }
REF_EXPORT void ref_fifo_abs_time(void *h, uint64_t tp, double frac, unsigned *sec, double *fs) {
    ((FifoBase *)h)->abs_time(tp, frac, sec, fs);
}
REF_EXPORT void ref_fifo_destroy(void *h) { delete (FifoBase *)h; }

/* dsptl_files.h:101-109 saveBinarySamples / :250-262 readBinarySamples.
 * type 0: int16_t components, 1: float components. */
REF_EXPORT void ref_iq_save(const char *path, int type, const void *in, long n) {
    std::ofstream os(path, std::ios::binary);
    if (type == 0) {
        std::vector<ci16> v((const ci16 *)in, (const ci16 *)in + n);
        dsptl::saveBinarySamples(v, os);
    } else {
        std::vector<std::complex<float>> v((const std::complex<float> *)in, (const std::complex<float> *)in + n);
        dsptl::saveBinarySamples(v, os);
    }
}
/* returns the number of samples the reference appends (incl. its trailing
 * sample from the failed read at EOF); copies at most cap of them */
REF_EXPORT long ref_iq_read(const char *path, int type, void *out, long cap) {
    std::ifstream is(path, std::ios::binary);
    if (type == 0) {
        std::vector<ci16> v;
        dsptl::readBinarySamples(is, v);
        std::memcpy(out, v.data(), sizeof(ci16) * (size_t)std::min<long>(cap, (long)v.size()));
        return (long)v.size();
    }
    std::vector<std::complex<float>> v;
    dsptl::readBinarySamples(is, v);
    std::memcpy(out, v.data(), sizeof(std::complex<float>) * (size_t)std::min<long>(cap, (long)v.size()));
    return (long)v.size();
}
}
