// corr_hit.h -- the detection test of dsptl::FixedPatternCorrelator::step
// (correlators.h:262-268) on the device, exactly:
//
//   corr[1] > corr[2] && corr[1] > corr[0]                        (:262)
//   sqrt((double)corr[1]) > sqrt((double)energy[1]) * 2.7          (:265-268)
//     && sqrt((double)energy[1]) > 300
//
// Shared by the product kernels (corr.hip) and the test-only probe
// (tests/hip/corr_hit_probe.hip), which evaluates it over crafted register
// values -- exact ties c*100 == 729*e, their neighbours, the uint32 maxima --
// against the host's IEEE double evaluation.
//
// Build switch (never set in the product build): SRCDSP_CORR_ALWAYS_EXACT
// makes corr_hit take the correctly rounded square roots for every peak (the
// fast sign test's band widened to infinity); the test suite runs a library
// built that way beside the product and requires identical detections.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srcdsp {

// s = m * 2^q is RN(sqrt(n)) iff (2m-1)^2 < n * 2^(2-2q) < (2m+1)^2 (no ties
// for integer n), checked in exact 128-bit integer arithmetic.
__device__ __forceinline__ bool rn_sqrt_ok(double s, uint32_t n) {
    if (s <= 0) return n == 0 && s == 0;
    unsigned long long b = (unsigned long long)__double_as_longlong(s);
    int E = (int)((b >> 52) & 0x7ff);
    unsigned long long m = (b & ((1ull << 52) - 1)) | (1ull << 52);
    int K = -2 * (E - 1075) + 2;  // n * 2^K
    if (K < 0 || K > 127 - 32) return false;
    unsigned __int128 T = (unsigned __int128)n << K;
    unsigned __int128 lo = (unsigned __int128)(2 * m - 1) * (2 * m - 1);
    unsigned __int128 hi = (unsigned __int128)(2 * m + 1) * (2 * m + 1);
    return lo < T && T < hi;
}

// neighbouring doubles of a positive finite value
__device__ __forceinline__ double dnext(double s, long long d) {
    return __longlong_as_double(__double_as_longlong(s) + d);
}

// the correctly rounded double square root of a uint32 (what libm's sqrt
// returns on the reference's host): the hardware estimate, corrected by the
// exact neighbour check
static __device__ double crsqrt_u32(uint32_t n) {
    if (n == 0) return 0.0;
    const double s = __builtin_sqrt((double)n);
    if (rn_sqrt_ok(s, n)) return s;
    for (long long d = 1; d <= 4; ++d) {
        if (rn_sqrt_ok(dnext(s, -d), n)) return dnext(s, -d);
        if (rn_sqrt_ok(dnext(s, d), n)) return dnext(s, d);
    }
    return s;  // unreachable: the hardware estimate is within a few ulp
}

// the threshold test with correctly rounded square roots; out of line: the
// scan tests 16 outputs per lane, and inlined 16 times this rarely taken path
// made up 40 % of the kernel's code
static __device__ __attribute__((noinline)) bool corr_hit_exact(uint32_t c1, uint32_t e1) {
    const double cm = crsqrt_u32(c1), em = crsqrt_u32(e1);
    return cm > em * 2.7;
}

// correlators.h:262-268 evaluated exactly.
// Fast path: with correctly rounded square roots, sqrt(c) > sqrt(e) * 2.7 in
// double holds exactly when c > 7.29 e up to a relative ~1e-15 (the roundings
// of the two square roots, of 2.7 and of the product), so outside a 1e-9
// relative band around c = 7.29 e the sign of c - 7.29 e (one fma) decides;
// inside it, the exact square roots do.  In noise about a third of all
// outputs are local peaks with energy above 300^2 and reach this test; the
// exact path for every one of them cost ~9 % of the fused scan's VALU work.
// sqrt(e) > 300 in double <=> e >= 90001 for integer e (300^2 = 90000 and the
// square root is correctly rounded and monotonic).
__device__ __forceinline__ bool corr_hit(uint32_t c2, uint32_t c1, uint32_t c0, uint32_t e1) {
    if (!(c1 > c2 && c1 > c0)) return false;
    if (e1 <= 90000u) return false;
#ifdef SRCDSP_CORR_ALWAYS_EXACT
    return corr_hit_exact(c1, e1);
#else
    const double dc = (double)c1, d = __builtin_fma(-7.29, (double)e1, dc);
    if (d > 1e-9 * dc) return true;
    if (d < -1e-9 * dc) return false;
    return corr_hit_exact(c1, e1);
#endif
}

}  // namespace srcdsp
