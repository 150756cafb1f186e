// Drop-in test program: reference-style C++ (std::vector in/out, dsptl:: class
// templates, step()) compiled against include/srcdsp/ instead of the SrcDsp
// tree and linked with libsrcdsp_hip.so.  tests/test_dropin_cpp.py writes the
// inputs, runs this on the GPU box and compares every output with the oracle.
//
//   dropin_main <in.bin> <out.bin>
// in.bin / out.bin: records {int32 tag, int64 nbytes, payload}.
#include <complex>
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <map>
#include <vector>

#include "buffers.h"
#include "correlators.h"
#include "dnsampling_filters.h"
#include "dsptl_files.h"
#include "filters.h"
#include "mixers.h"
#include "upsampling_filters.h"

using cf32 = std::complex<float>;
using ci16 = std::complex<int16_t>;
using ci32 = std::complex<int32_t>;

static std::map<int, std::vector<char>> read_records(const char *path) {
    std::map<int, std::vector<char>> m;
    std::ifstream f(path, std::ios::binary);
    int32_t tag;
    int64_t nb;
    while (f.read((char *)&tag, 4) && f.read((char *)&nb, 8)) {
        std::vector<char> b(nb);
        f.read(b.data(), nb);
        m[tag] = std::move(b);
    }
    return m;
}

template <class T>
static std::vector<T> as(const std::vector<char> &b) {
    return std::vector<T>((const T *)b.data(), (const T *)(b.data() + b.size()));
}

struct Out {
    std::ofstream f;
    explicit Out(const char *p) : f(p, std::ios::binary) {}
    template <class T>
    void put(int32_t tag, const std::vector<T> &v) {
        int64_t nb = (int64_t)(v.size() * sizeof(T));
        f.write((const char *)&tag, 4);
        f.write((const char *)&nb, 8);
        f.write((const char *)v.data(), nb);
    }
};

int main(int argc, char **argv) {
    if (argc != 3) {
        std::fprintf(stderr, "usage: %s in.bin out.bin\n", argv[0]);
        return 2;
    }
    auto in = read_records(argv[1]);
    Out out(argv[2]);

    // 1. headline decimator, two chained calls
    {
        auto c = as<float>(in[1]);
        auto x = as<cf32>(in[2]);
        dsptl::FilterDnsamplingFir<cf32, cf32, cf32, float, 4> f(c);
        size_t h = (x.size() / 2) & ~size_t(3);
        std::vector<cf32> a(x.begin(), x.begin() + h), b(x.begin() + h, x.end());
        std::vector<cf32> ya(a.size() / 4), yb(b.size() / 4);
        f.step(a, ya);
        f.step(b, yb);
        ya.insert(ya.end(), yb.begin(), yb.end());
        out.put(101, ya);
    }
    // 2. fixed-point decimator (config 4 shape) and mixer -> decimator chain
    {
        auto cq = as<int32_t>(in[4]);
        auto x = as<ci16>(in[3]);
        dsptl::FilterDnsamplingFir<ci16, ci16, ci32, int32_t, 4> d(cq);
        std::vector<ci16> y(x.size() / 4);
        d.step(x, y);
        out.put(102, y);
        dsptl::Mixer<ci16, ci16, int16_t, 4096> m;
        m.reset(0.1f);
        dsptl::FilterDnsamplingFir<ci16, ci16, ci32, int32_t, 4> d2(cq);
        std::vector<ci16> mixed(x.size()), y2(x.size() / 4);
        m.step(x, mixed);
        d2.step(mixed, y2);
        out.put(103, mixed);
        out.put(104, y2);
    }
    // 3. FilterFir<float, complex<float>, float, float>, 31 taps (config 1 shape)
    {
        auto c = as<float>(in[5]);
        auto x = as<float>(in[6]);
        FilterFir<float, cf32, float, float> f(c);
        std::vector<cf32> y(x.size());
        f.step(x, y);
        out.put(105, y);
    }
    // 4. upsampler: vector overload then iterator overload with flush
    {
        auto c = as<int32_t>(in[7]);
        auto x = as<ci16>(in[3]);
        std::vector<ci16> xa(x.begin(), x.begin() + 1000), xb(x.begin() + 1000, x.begin() + 1500);
        dsptl::FilterUpsamplingFir<ci16, ci16, ci32, int32_t, 4> u(c);
        std::vector<ci16> ya(4 * xa.size());
        u.step(xa, ya);
        std::vector<ci16> yb(4 * (xb.size() + u.getLength() / 4));
        u.step(xb, yb.begin(), true);
        ya.insert(ya.end(), yb.begin(), yb.end());
        out.put(106, ya);
    }
    // 5. correlator <int16_t, int32_t, 32, 4>
    {
        auto p = as<int32_t>(in[8]);
        auto x = as<ci16>(in[9]);
        dsptl::FixedPatternCorrelator<int16_t, int32_t, 32, 4> corr;
        std::array<ci32, 32> pat;
        for (int i = 0; i < 32; ++i) pat[i] = ci32(p[2 * i], p[2 * i + 1]);
        corr.setPattern(pat);
        int idx = -7;
        bool found = corr.step(x, idx);
        auto st = corr.getStatus();
        std::vector<int32_t> r = {found ? 1 : 0, idx, (int32_t)st.corrValue[0], (int32_t)st.energyValue[0],
                                  st.coeffScaling};
        out.put(107, r);
        out.put(108, corr.getRefBitSamples());
    }
    // 6. FifoWithTimeTrack<double, 15>: the scenario of the reference's own
    //    buffers_test.cpp (its reads and counts)
    {
        dsptl::FifoWithTimeTrack<double, 15> fifo;
        std::vector<double> input, res;
        double value = 0;
        auto block = [&](size_t n) {
            input.assign(n, 0.0);
            for (auto &e : input) e = (value += 1);
        };
        for (int i = 0; i < 23; ++i) {
            block(14);
            fifo.write(input);
        }
        res.push_back((double)fifo.count());
        for (size_t n : {10, 5, 7}) {
            block(n);
            fifo.write(input);
            res.push_back((double)fifo.count());
        }
        fifo.reset();
        res.push_back((double)fifo.count());
        value = 0;
        const size_t reads[3][2] = {{3, 4}, {15, 3}, {4, 6}};
        const size_t adds[3] = {7, 10, 4};
        for (int k = 0; k < 3; ++k) {
            block(adds[k]);
            fifo.write(input);
            std::vector<double> o(reads[k][0]);
            uint64_t start = reads[k][1];
            bool err = fifo.read(o, start);
            res.push_back(err ? 1.0 : 0.0);
            res.push_back((double)start);
            res.insert(res.end(), o.begin(), o.end());
        }
        res.push_back((double)fifo.count());
        out.put(109, res);
    }
    // 7. binary I/Q capture round trip through the drop-in dsptl_files.h
    {
        auto x = as<ci16>(in[3]);
        {
            std::ofstream os(argv[2] + std::string(".iq"), std::ios::binary);
            dsptl::saveBinarySamples(x, os);
        }
        std::ifstream is(argv[2] + std::string(".iq"), std::ios::binary);
        std::vector<ci16> back(5, ci16(1, 1));  // replaced, not appended to
        dsptl::readBinarySamples(is, back);
        out.put(110, back);
    }
    // 8. value semantics, as the reference's implicit copies (dnsampling_filters.h:52,
    //    filters.h:49, upsampling_filters.h:42, correlators.h:85, mixers.h:134):
    //    copy-initialisation from the coefficient vector, a configured filter copied
    //    mid-stream continues from the original's history, a bank built as
    //    std::vector<Filter>(K, proto) (config 3's natural shape), copy assignment
    {
        using Dec = dsptl::FilterDnsamplingFir<cf32, cf32, cf32, float, 4>;
        auto c = as<float>(in[1]);
        auto x = as<cf32>(in[2]);
        Dec f = c;  // copy-initialisation: the converting constructor is implicit
        size_t h = (x.size() / 2) & ~size_t(3);
        std::vector<cf32> a(x.begin(), x.begin() + h), b(x.begin() + h, x.end());
        std::vector<cf32> ya(a.size() / 4), yb(b.size() / 4), yc(b.size() / 4);
        f.step(a, ya);
        Dec g(f);  // copy after one call: g owns f's history
        f.step(b, yb);
        g.step(b, yc);
        out.put(111, yb);
        out.put(112, yc);
        std::vector<Dec> bank(3, g);  // three copies of g's state (after both halves)
        std::vector<cf32> z(a.size() / 4);
        const int bank_tags[3] = {113, 123, 124};
        for (size_t i = 0; i < bank.size(); ++i) {
            bank[i].step(a, z);
            out.put(bank_tags[i], z);
        }
        Dec k(c);
        k = f;  // copy assignment: k takes f's state
        k.step(a, z);
        out.put(114, z);
        // the other operators: a copy continues exactly like the original
        auto cq = as<int32_t>(in[4]);
        auto xi = as<ci16>(in[3]);
        std::vector<ci16> xa(xi.begin(), xi.begin() + 1000), xb(xi.begin() + 1000, xi.begin() + 2000);
        dsptl::Mixer<ci16, ci16, int16_t, 4096> m;
        m.reset(0.1f);
        std::vector<ci16> ma(xa.size()), mb(xb.size()), mc(xb.size());
        m.step(xa, ma);
        auto m2 = m;
        m.step(xb, mb);
        m2.step(xb, mc);
        out.put(115, mb);
        out.put(116, mc);
        FilterFir<ci16, ci16, ci32, int32_t> fi = cq;
        std::vector<ci16> fa(xa.size()), fb(xb.size()), fc(xb.size());
        fi.step(xa, fa);
        auto fi2 = fi;
        fi.step(xb, fb);
        fi2.step(xb, fc);
        out.put(117, fb);
        out.put(118, fc);
        auto cu = as<int32_t>(in[7]);
        dsptl::FilterUpsamplingFir<ci16, ci16, ci32, int32_t, 4> u = cu;
        std::vector<ci16> ua(4 * xa.size()), ub(4 * xb.size()), uc(4 * xb.size());
        u.step(xa, ua);
        auto u2 = u;
        u.step(xb, ub);
        u2.step(xb, uc);
        out.put(119, ub);
        out.put(120, uc);
        auto p = as<int32_t>(in[8]);
        auto xc = as<ci16>(in[9]);
        dsptl::FixedPatternCorrelator<int16_t, int32_t, 32, 4> corr;
        std::array<ci32, 32> pat;
        for (int i = 0; i < 32; ++i) pat[i] = ci32(p[2 * i], p[2 * i + 1]);
        corr.setPattern(pat);
        std::vector<ci16> xc1(xc.begin(), xc.begin() + 2000), xc2(xc.begin() + 2000, xc.end());
        int i1 = -7, i2 = -7;
        corr.step(xc1, i1);  // no detection in the first part
        auto corr2 = corr;
        bool f1 = corr.step(xc2, i1), f2 = corr2.step(xc2, i2);
        std::vector<int32_t> r = {f1 ? 1 : 0, i1, f2 ? 1 : 0, i2};
        out.put(121, r);
        out.put(122, corr2.getRefBitSamples());
    }
    std::printf("dropin_main: ok\n");
    return 0;
}
