// One source, two builds: the reference's FixedPatternCorrelator
// (-I /root/reference, linked with its dsp_complex.cpp; made only in the build
// container by tests/golden/gen_corr_debug.py) and the drop-in
// (-I include/srcdsp, linked with libsrcdsp_hip.so; made on the GPU box by
// tests/test_dropin_cpp.py).  Both compiled with -DCREATE_DEBUG_FILES: the
// three debug_corr_*.dat files each writes in its working directory must be
// byte-identical (correlators.h:107-132, 253-257).
//
//   corr_debug_main <in.bin> <steps.txt>
// in.bin: int32 chunk, int32 pattern N x (re, im) int32, then int16 (re, im)
// samples to the end of the file.  Compile with -DCORR_N=.. -DCORR_S=..
// The samples are stepped in chunks of `chunk`, resuming two samples after
// each detection (corrIndex + 2), as the parity tests do; steps.txt gets one
// line per call: offset, length, found, corrIndex.
#include <cmath>
#include <cassert>
#include <complex>
#include <cstdint>
#include <vector>
#include <array>
#include "correlators.h"
#include <cstdio>
#include <fstream>

#ifndef CORR_N
#define CORR_N 32
#endif
#ifndef CORR_S
#define CORR_S 4
#endif

int main(int argc, char **argv) {
    if (argc != 3) {
        std::fprintf(stderr, "usage: %s in.bin steps.txt\n", argv[0]);
        return 2;
    }
    std::ifstream f(argv[1], std::ios::binary);
    int32_t chunk = 0;
    f.read((char *)&chunk, 4);
    std::array<std::complex<int32_t>, CORR_N> pattern;
    for (auto &p : pattern) {
        int32_t re = 0, im = 0;
        f.read((char *)&re, 4);
        f.read((char *)&im, 4);
        p = std::complex<int32_t>(re, im);
    }
    std::vector<std::complex<int16_t>> x;
    int16_t v[2];
    while (f.read((char *)v, 4)) x.emplace_back(v[0], v[1]);
    if (chunk <= 0) return 2;

    dsptl::FixedPatternCorrelator<int16_t, int32_t, CORR_N, CORR_S> corr;
    corr.setPattern(pattern);
    std::FILE *log = std::fopen(argv[2], "w");
    size_t pos = 0;
    while (pos < x.size()) {
        const size_t k = std::min<size_t>(chunk, x.size() - pos);
        std::vector<std::complex<int16_t>> in(x.begin() + pos, x.begin() + pos + k);
        int idx = -1;
        const bool found = corr.step(in, idx);
        std::fprintf(log, "%zu %zu %d %d\n", pos, k, found ? 1 : 0, found ? idx : -1);
        pos += found ? (size_t)(idx + 2) : k;
    }
    std::fclose(log);
    return 0;
}
