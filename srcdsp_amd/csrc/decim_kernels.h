// decim_kernels.h -- device kernels of the FIR core (FilterDnsamplingFir /
// FilterFir), shared by decim.hip (the product dispatch) and the tuning
// harness under scripts/tune.  See decim.hip for the semantics.
#pragma once
#include "ops.h"

namespace srcdsp {
typedef short short2_t_ __attribute__((ext_vector_type(2)));
typedef float f2_t __attribute__((ext_vector_type(2)));

// One packed fma step of a complex<float> accumulator by a real tap that sits
// in one half of an SGPR pair: acc = fma(c, x, acc) per component.  Inline asm
// so the tap loop issues in the order written (every accumulator's chain
// advances one tap before any advances the next): the scheduler otherwise
// groups up to ten dependent v_pk_fma_f32 of one chain back to back, each
// waiting for the previous one's result.  HI: the tap is the pair's odd
// element.  ZERO: acc starts from +0 (fma(c, x, +0), as the first step of
// the reference's accumulation from 0).
template <bool HI, bool ZERO>
__device__ __forceinline__ void pk_fma_tap(f2_t &acc, unsigned long long cp, f2_t x) {
    if constexpr (ZERO && HI)
        asm volatile("v_pk_fma_f32 %0, %1, %2, 0 op_sel:[1,0,0] op_sel_hi:[1,1,0]" : "=v"(acc) : "s"(cp), "v"(x));
    else if constexpr (ZERO)
        asm volatile("v_pk_fma_f32 %0, %1, %2, 0 op_sel_hi:[0,1,0]" : "=v"(acc) : "s"(cp), "v"(x));
    else if constexpr (HI)
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "s"(cp), "v"(x));
    else
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(acc) : "s"(cp), "v"(x));
}

// The strict contract's step acc = acc + c*x (separately rounded product,
// then sum, as the reference's -O2 x86-64 build computes it), split so a
// tap's R products can issue before its R sums: pk_mul_tap writes the
// product, pk_add_acc adds it.
template <bool HI>
__device__ __forceinline__ void pk_mul_tap(f2_t &p, unsigned long long cp, f2_t x) {
    if constexpr (HI)
        asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]" : "=v"(p) : "s"(cp), "v"(x));
    else
        asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(p) : "s"(cp), "v"(x));
}
__device__ __forceinline__ void pk_add_acc(f2_t &acc, f2_t p) {
    asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(acc) : "v"(p));
}

// One tap over R accumulators, skipped (by a branch inside the asm, so the
// compiler sees straight-line code) unless k < n as unsigned, i.e. 0 <= k < n.
// Used by the runtime-tap kernel's last chunk only.
template <int R, bool HI, bool FMA>
struct TapGuarded;

template <>
struct TapGuarded<1, false, true> {
    static __device__ __forceinline__ void run(f2_t (&a)[1], unsigned long long c, const f2_t (&x)[1], int k, int n) {
        asm volatile(
            "s_cmp_lt_u32 %[k], %[n]\n\t"
            "s_cbranch_scc0 1f\n\t"
            "v_pk_fma_f32 %[a0], %[c], %[x0], %[a0] op_sel_hi:[0,1,1]\n\t"
            "1:"
            : [a0] "+v"(a[0])
            : [k] "s"(k), [n] "s"(n), [c] "s"(c), [x0] "v"(x[0])
            : "scc");
    }
};
template <>
struct TapGuarded<1, false, false> {
    static __device__ __forceinline__ void run(f2_t (&a)[1], unsigned long long c, const f2_t (&x)[1], int k, int n) {
        f2_t t[1];
        asm volatile(
            "s_cmp_lt_u32 %[k], %[n]\n\t"
            "s_cbranch_scc0 1f\n\t"
            "v_pk_mul_f32 %[t0], %[c], %[x0] op_sel_hi:[0,1]\n\t"
            "v_pk_add_f32 %[a0], %[a0], %[t0]\n\t"
            "1:"
            : [a0] "+v"(a[0]), [t0] "=&v"(t[0])
            : [k] "s"(k), [n] "s"(n), [c] "s"(c), [x0] "v"(x[0])
            : "scc");
    }
};
template <>
struct TapGuarded<1, true, true> {
    static __device__ __forceinline__ void run(f2_t (&a)[1], unsigned long long c, const f2_t (&x)[1], int k, int n) {
        asm volatile(
            "s_cmp_lt_u32 %[k], %[n]\n\t"
            "s_cbranch_scc0 1f\n\t"
            "v_pk_fma_f32 %[a0], %[c], %[x0], %[a0] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
            "1:"
            : [a0] "+v"(a[0])
            : [k] "s"(k), [n] "s"(n), [c] "s"(c), [x0] "v"(x[0])
            : "scc");
    }
};
template <>
struct TapGuarded<1, true, false> {
    static __device__ __forceinline__ void run(f2_t (&a)[1], unsigned long long c, const f2_t (&x)[1], int k, int n) {
        f2_t t[1];
        asm volatile(
            "s_cmp_lt_u32 %[k], %[n]\n\t"
            "s_cbranch_scc0 1f\n\t"
            "v_pk_mul_f32 %[t0], %[c], %[x0] op_sel:[1,0] op_sel_hi:[1,1]\n\t"
            "v_pk_add_f32 %[a0], %[a0], %[t0]\n\t"
            "1:"
            : [a0] "+v"(a[0]), [t0] "=&v"(t[0])
            : [k] "s"(k), [n] "s"(n), [c] "s"(c), [x0] "v"(x[0])
            : "scc");
    }
};
template <>
struct TapGuarded<2, false, true> {
    static __device__ __forceinline__ void run(f2_t (&a)[2], unsigned long long c, const f2_t (&x)[2], int k, int n) {
        asm volatile(
            "s_cmp_lt_u32 %[k], %[n]\n\t"
            "s_cbranch_scc0 1f\n\t"
            "v_pk_fma_f32 %[a0], %[c], %[x0], %[a0] op_sel_hi:[0,1,1]\n\t"
            "v_pk_fma_f32 %[a1], %[c], %[x1], %[a1] op_sel_hi:[0,1,1]\n\t"
            "1:"
            : [a0] "+v"(a[0]), [a1] "+v"(a[1])
            : [k] "s"(k), [n] "s"(n), [c] "s"(c), [x0] "v"(x[0]), [x1] "v"(x[1])
            : "scc");
    }
};
template <>
struct TapGuarded<2, false, false> {
    static __device__ __forceinline__ void run(f2_t (&a)[2], unsigned long long c, const f2_t (&x)[2], int k, int n) {
        f2_t t[2];
        asm volatile(
            "s_cmp_lt_u32 %[k], %[n]\n\t"
            "s_cbranch_scc0 1f\n\t"
            "v_pk_mul_f32 %[t0], %[c], %[x0] op_sel_hi:[0,1]\n\t"
            "v_pk_mul_f32 %[t1], %[c], %[x1] op_sel_hi:[0,1]\n\t"
            "v_pk_add_f32 %[a0], %[a0], %[t0]\n\t"
            "v_pk_add_f32 %[a1], %[a1], %[t1]\n\t"
            "1:"
            : [a0] "+v"(a[0]), [a1] "+v"(a[1]), [t0] "=&v"(t[0]), [t1] "=&v"(t[1])
            : [k] "s"(k), [n] "s"(n), [c] "s"(c), [x0] "v"(x[0]), [x1] "v"(x[1])
            : "scc");
    }
};
template <>
struct TapGuarded<2, true, true> {
    static __device__ __forceinline__ void run(f2_t (&a)[2], unsigned long long c, const f2_t (&x)[2], int k, int n) {
        asm volatile(
            "s_cmp_lt_u32 %[k], %[n]\n\t"
            "s_cbranch_scc0 1f\n\t"
            "v_pk_fma_f32 %[a0], %[c], %[x0], %[a0] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
            "v_pk_fma_f32 %[a1], %[c], %[x1], %[a1] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
            "1:"
            : [a0] "+v"(a[0]), [a1] "+v"(a[1])
            : [k] "s"(k), [n] "s"(n), [c] "s"(c), [x0] "v"(x[0]), [x1] "v"(x[1])
            : "scc");
    }
};
template <>
struct TapGuarded<2, true, false> {
    static __device__ __forceinline__ void run(f2_t (&a)[2], unsigned long long c, const f2_t (&x)[2], int k, int n) {
        f2_t t[2];
        asm volatile(
            "s_cmp_lt_u32 %[k], %[n]\n\t"
            "s_cbranch_scc0 1f\n\t"
            "v_pk_mul_f32 %[t0], %[c], %[x0] op_sel:[1,0] op_sel_hi:[1,1]\n\t"
            "v_pk_mul_f32 %[t1], %[c], %[x1] op_sel:[1,0] op_sel_hi:[1,1]\n\t"
            "v_pk_add_f32 %[a0], %[a0], %[t0]\n\t"
            "v_pk_add_f32 %[a1], %[a1], %[t1]\n\t"
            "1:"
            : [a0] "+v"(a[0]), [a1] "+v"(a[1]), [t0] "=&v"(t[0]), [t1] "=&v"(t[1])
            : [k] "s"(k), [n] "s"(n), [c] "s"(c), [x0] "v"(x[0]), [x1] "v"(x[1])
            : "scc");
    }
};
template <>
struct TapGuarded<4, false, true> {
    static __device__ __forceinline__ void run(f2_t (&a)[4], unsigned long long c, const f2_t (&x)[4], int k, int n) {
        asm volatile(
            "s_cmp_lt_u32 %[k], %[n]\n\t"
            "s_cbranch_scc0 1f\n\t"
            "v_pk_fma_f32 %[a0], %[c], %[x0], %[a0] op_sel_hi:[0,1,1]\n\t"
            "v_pk_fma_f32 %[a1], %[c], %[x1], %[a1] op_sel_hi:[0,1,1]\n\t"
            "v_pk_fma_f32 %[a2], %[c], %[x2], %[a2] op_sel_hi:[0,1,1]\n\t"
            "v_pk_fma_f32 %[a3], %[c], %[x3], %[a3] op_sel_hi:[0,1,1]\n\t"
            "1:"
            : [a0] "+v"(a[0]), [a1] "+v"(a[1]), [a2] "+v"(a[2]), [a3] "+v"(a[3])
            : [k] "s"(k), [n] "s"(n), [c] "s"(c), [x0] "v"(x[0]), [x1] "v"(x[1]), [x2] "v"(x[2]), [x3] "v"(x[3])
            : "scc");
    }
};
template <>
struct TapGuarded<4, false, false> {
    static __device__ __forceinline__ void run(f2_t (&a)[4], unsigned long long c, const f2_t (&x)[4], int k, int n) {
        f2_t t[4];
        asm volatile(
            "s_cmp_lt_u32 %[k], %[n]\n\t"
            "s_cbranch_scc0 1f\n\t"
            "v_pk_mul_f32 %[t0], %[c], %[x0] op_sel_hi:[0,1]\n\t"
            "v_pk_mul_f32 %[t1], %[c], %[x1] op_sel_hi:[0,1]\n\t"
            "v_pk_mul_f32 %[t2], %[c], %[x2] op_sel_hi:[0,1]\n\t"
            "v_pk_mul_f32 %[t3], %[c], %[x3] op_sel_hi:[0,1]\n\t"
            "v_pk_add_f32 %[a0], %[a0], %[t0]\n\t"
            "v_pk_add_f32 %[a1], %[a1], %[t1]\n\t"
            "v_pk_add_f32 %[a2], %[a2], %[t2]\n\t"
            "v_pk_add_f32 %[a3], %[a3], %[t3]\n\t"
            "1:"
            : [a0] "+v"(a[0]), [a1] "+v"(a[1]), [a2] "+v"(a[2]), [a3] "+v"(a[3]), [t0] "=&v"(t[0]), [t1] "=&v"(t[1]), [t2] "=&v"(t[2]), [t3] "=&v"(t[3])
            : [k] "s"(k), [n] "s"(n), [c] "s"(c), [x0] "v"(x[0]), [x1] "v"(x[1]), [x2] "v"(x[2]), [x3] "v"(x[3])
            : "scc");
    }
};
template <>
struct TapGuarded<4, true, true> {
    static __device__ __forceinline__ void run(f2_t (&a)[4], unsigned long long c, const f2_t (&x)[4], int k, int n) {
        asm volatile(
            "s_cmp_lt_u32 %[k], %[n]\n\t"
            "s_cbranch_scc0 1f\n\t"
            "v_pk_fma_f32 %[a0], %[c], %[x0], %[a0] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
            "v_pk_fma_f32 %[a1], %[c], %[x1], %[a1] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
            "v_pk_fma_f32 %[a2], %[c], %[x2], %[a2] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
            "v_pk_fma_f32 %[a3], %[c], %[x3], %[a3] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
            "1:"
            : [a0] "+v"(a[0]), [a1] "+v"(a[1]), [a2] "+v"(a[2]), [a3] "+v"(a[3])
            : [k] "s"(k), [n] "s"(n), [c] "s"(c), [x0] "v"(x[0]), [x1] "v"(x[1]), [x2] "v"(x[2]), [x3] "v"(x[3])
            : "scc");
    }
};
template <>
struct TapGuarded<4, true, false> {
    static __device__ __forceinline__ void run(f2_t (&a)[4], unsigned long long c, const f2_t (&x)[4], int k, int n) {
        f2_t t[4];
        asm volatile(
            "s_cmp_lt_u32 %[k], %[n]\n\t"
            "s_cbranch_scc0 1f\n\t"
            "v_pk_mul_f32 %[t0], %[c], %[x0] op_sel:[1,0] op_sel_hi:[1,1]\n\t"
            "v_pk_mul_f32 %[t1], %[c], %[x1] op_sel:[1,0] op_sel_hi:[1,1]\n\t"
            "v_pk_mul_f32 %[t2], %[c], %[x2] op_sel:[1,0] op_sel_hi:[1,1]\n\t"
            "v_pk_mul_f32 %[t3], %[c], %[x3] op_sel:[1,0] op_sel_hi:[1,1]\n\t"
            "v_pk_add_f32 %[a0], %[a0], %[t0]\n\t"
            "v_pk_add_f32 %[a1], %[a1], %[t1]\n\t"
            "v_pk_add_f32 %[a2], %[a2], %[t2]\n\t"
            "v_pk_add_f32 %[a3], %[a3], %[t3]\n\t"
            "1:"
            : [a0] "+v"(a[0]), [a1] "+v"(a[1]), [a2] "+v"(a[2]), [a3] "+v"(a[3]), [t0] "=&v"(t[0]), [t1] "=&v"(t[1]), [t2] "=&v"(t[2]), [t3] "=&v"(t[3])
            : [k] "s"(k), [n] "s"(n), [c] "s"(c), [x0] "v"(x[0]), [x1] "v"(x[1]), [x2] "v"(x[2]), [x3] "v"(x[3])
            : "scc");
    }
};
template <>
struct TapGuarded<8, false, true> {
    static __device__ __forceinline__ void run(f2_t (&a)[8], unsigned long long c, const f2_t (&x)[8], int k, int n) {
        asm volatile(
            "s_cmp_lt_u32 %[k], %[n]\n\t"
            "s_cbranch_scc0 1f\n\t"
            "v_pk_fma_f32 %[a0], %[c], %[x0], %[a0] op_sel_hi:[0,1,1]\n\t"
            "v_pk_fma_f32 %[a1], %[c], %[x1], %[a1] op_sel_hi:[0,1,1]\n\t"
            "v_pk_fma_f32 %[a2], %[c], %[x2], %[a2] op_sel_hi:[0,1,1]\n\t"
            "v_pk_fma_f32 %[a3], %[c], %[x3], %[a3] op_sel_hi:[0,1,1]\n\t"
            "v_pk_fma_f32 %[a4], %[c], %[x4], %[a4] op_sel_hi:[0,1,1]\n\t"
            "v_pk_fma_f32 %[a5], %[c], %[x5], %[a5] op_sel_hi:[0,1,1]\n\t"
            "v_pk_fma_f32 %[a6], %[c], %[x6], %[a6] op_sel_hi:[0,1,1]\n\t"
            "v_pk_fma_f32 %[a7], %[c], %[x7], %[a7] op_sel_hi:[0,1,1]\n\t"
            "1:"
            : [a0] "+v"(a[0]), [a1] "+v"(a[1]), [a2] "+v"(a[2]), [a3] "+v"(a[3]), [a4] "+v"(a[4]), [a5] "+v"(a[5]), [a6] "+v"(a[6]), [a7] "+v"(a[7])
            : [k] "s"(k), [n] "s"(n), [c] "s"(c), [x0] "v"(x[0]), [x1] "v"(x[1]), [x2] "v"(x[2]), [x3] "v"(x[3]), [x4] "v"(x[4]), [x5] "v"(x[5]), [x6] "v"(x[6]), [x7] "v"(x[7])
            : "scc");
    }
};
template <>
struct TapGuarded<8, false, false> {
    static __device__ __forceinline__ void run(f2_t (&a)[8], unsigned long long c, const f2_t (&x)[8], int k, int n) {
        f2_t t[8];
        asm volatile(
            "s_cmp_lt_u32 %[k], %[n]\n\t"
            "s_cbranch_scc0 1f\n\t"
            "v_pk_mul_f32 %[t0], %[c], %[x0] op_sel_hi:[0,1]\n\t"
            "v_pk_mul_f32 %[t1], %[c], %[x1] op_sel_hi:[0,1]\n\t"
            "v_pk_mul_f32 %[t2], %[c], %[x2] op_sel_hi:[0,1]\n\t"
            "v_pk_mul_f32 %[t3], %[c], %[x3] op_sel_hi:[0,1]\n\t"
            "v_pk_mul_f32 %[t4], %[c], %[x4] op_sel_hi:[0,1]\n\t"
            "v_pk_mul_f32 %[t5], %[c], %[x5] op_sel_hi:[0,1]\n\t"
            "v_pk_mul_f32 %[t6], %[c], %[x6] op_sel_hi:[0,1]\n\t"
            "v_pk_mul_f32 %[t7], %[c], %[x7] op_sel_hi:[0,1]\n\t"
            "v_pk_add_f32 %[a0], %[a0], %[t0]\n\t"
            "v_pk_add_f32 %[a1], %[a1], %[t1]\n\t"
            "v_pk_add_f32 %[a2], %[a2], %[t2]\n\t"
            "v_pk_add_f32 %[a3], %[a3], %[t3]\n\t"
            "v_pk_add_f32 %[a4], %[a4], %[t4]\n\t"
            "v_pk_add_f32 %[a5], %[a5], %[t5]\n\t"
            "v_pk_add_f32 %[a6], %[a6], %[t6]\n\t"
            "v_pk_add_f32 %[a7], %[a7], %[t7]\n\t"
            "1:"
            : [a0] "+v"(a[0]), [a1] "+v"(a[1]), [a2] "+v"(a[2]), [a3] "+v"(a[3]), [a4] "+v"(a[4]), [a5] "+v"(a[5]), [a6] "+v"(a[6]), [a7] "+v"(a[7]), [t0] "=&v"(t[0]), [t1] "=&v"(t[1]), [t2] "=&v"(t[2]), [t3] "=&v"(t[3]), [t4] "=&v"(t[4]), [t5] "=&v"(t[5]), [t6] "=&v"(t[6]), [t7] "=&v"(t[7])
            : [k] "s"(k), [n] "s"(n), [c] "s"(c), [x0] "v"(x[0]), [x1] "v"(x[1]), [x2] "v"(x[2]), [x3] "v"(x[3]), [x4] "v"(x[4]), [x5] "v"(x[5]), [x6] "v"(x[6]), [x7] "v"(x[7])
            : "scc");
    }
};
template <>
struct TapGuarded<8, true, true> {
    static __device__ __forceinline__ void run(f2_t (&a)[8], unsigned long long c, const f2_t (&x)[8], int k, int n) {
        asm volatile(
            "s_cmp_lt_u32 %[k], %[n]\n\t"
            "s_cbranch_scc0 1f\n\t"
            "v_pk_fma_f32 %[a0], %[c], %[x0], %[a0] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
            "v_pk_fma_f32 %[a1], %[c], %[x1], %[a1] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
            "v_pk_fma_f32 %[a2], %[c], %[x2], %[a2] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
            "v_pk_fma_f32 %[a3], %[c], %[x3], %[a3] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
            "v_pk_fma_f32 %[a4], %[c], %[x4], %[a4] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
            "v_pk_fma_f32 %[a5], %[c], %[x5], %[a5] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
            "v_pk_fma_f32 %[a6], %[c], %[x6], %[a6] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
            "v_pk_fma_f32 %[a7], %[c], %[x7], %[a7] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
            "1:"
            : [a0] "+v"(a[0]), [a1] "+v"(a[1]), [a2] "+v"(a[2]), [a3] "+v"(a[3]), [a4] "+v"(a[4]), [a5] "+v"(a[5]), [a6] "+v"(a[6]), [a7] "+v"(a[7])
            : [k] "s"(k), [n] "s"(n), [c] "s"(c), [x0] "v"(x[0]), [x1] "v"(x[1]), [x2] "v"(x[2]), [x3] "v"(x[3]), [x4] "v"(x[4]), [x5] "v"(x[5]), [x6] "v"(x[6]), [x7] "v"(x[7])
            : "scc");
    }
};
template <>
struct TapGuarded<8, true, false> {
    static __device__ __forceinline__ void run(f2_t (&a)[8], unsigned long long c, const f2_t (&x)[8], int k, int n) {
        f2_t t[8];
        asm volatile(
            "s_cmp_lt_u32 %[k], %[n]\n\t"
            "s_cbranch_scc0 1f\n\t"
            "v_pk_mul_f32 %[t0], %[c], %[x0] op_sel:[1,0] op_sel_hi:[1,1]\n\t"
            "v_pk_mul_f32 %[t1], %[c], %[x1] op_sel:[1,0] op_sel_hi:[1,1]\n\t"
            "v_pk_mul_f32 %[t2], %[c], %[x2] op_sel:[1,0] op_sel_hi:[1,1]\n\t"
            "v_pk_mul_f32 %[t3], %[c], %[x3] op_sel:[1,0] op_sel_hi:[1,1]\n\t"
            "v_pk_mul_f32 %[t4], %[c], %[x4] op_sel:[1,0] op_sel_hi:[1,1]\n\t"
            "v_pk_mul_f32 %[t5], %[c], %[x5] op_sel:[1,0] op_sel_hi:[1,1]\n\t"
            "v_pk_mul_f32 %[t6], %[c], %[x6] op_sel:[1,0] op_sel_hi:[1,1]\n\t"
            "v_pk_mul_f32 %[t7], %[c], %[x7] op_sel:[1,0] op_sel_hi:[1,1]\n\t"
            "v_pk_add_f32 %[a0], %[a0], %[t0]\n\t"
            "v_pk_add_f32 %[a1], %[a1], %[t1]\n\t"
            "v_pk_add_f32 %[a2], %[a2], %[t2]\n\t"
            "v_pk_add_f32 %[a3], %[a3], %[t3]\n\t"
            "v_pk_add_f32 %[a4], %[a4], %[t4]\n\t"
            "v_pk_add_f32 %[a5], %[a5], %[t5]\n\t"
            "v_pk_add_f32 %[a6], %[a6], %[t6]\n\t"
            "v_pk_add_f32 %[a7], %[a7], %[t7]\n\t"
            "1:"
            : [a0] "+v"(a[0]), [a1] "+v"(a[1]), [a2] "+v"(a[2]), [a3] "+v"(a[3]), [a4] "+v"(a[4]), [a5] "+v"(a[5]), [a6] "+v"(a[6]), [a7] "+v"(a[7]), [t0] "=&v"(t[0]), [t1] "=&v"(t[1]), [t2] "=&v"(t[2]), [t3] "=&v"(t[3]), [t4] "=&v"(t[4]), [t5] "=&v"(t[5]), [t6] "=&v"(t[6]), [t7] "=&v"(t[7])
            : [k] "s"(k), [n] "s"(n), [c] "s"(c), [x0] "v"(x[0]), [x1] "v"(x[1]), [x2] "v"(x[2]), [x3] "v"(x[3]), [x4] "v"(x[4]), [x5] "v"(x[5]), [x6] "v"(x[6]), [x7] "v"(x[7])
            : "scc");
    }
};

// ------------------------------------------------------------ arithmetic
template <bool FMA>
__device__ __forceinline__ float mac(float c, float x, float y) {
    if constexpr (FMA) return __builtin_fmaf(c, x, y);
    else return y + x * c;  // -ffp-contract=off: rounded product, then rounded sum
}

__device__ __forceinline__ float q16f(float y, unsigned shift) {
    return (float)limit16(cvt_f2i_x86(y), shift);
}

// read one input sample of channel data / history; idx may be negative (history)
template <typename T>
__device__ __forceinline__ T fetch(const T *in, const T *hist, long idx, long n_in, int H) {
    if (idx >= 0) return idx < n_in ? in[idx] : T{};
    long h = idx + H;
    return h >= 0 ? hist[h] : T{};
}

// ---------------------------------------------------------------- history
// hist_out[k] = (hist_in ++ in)[H + n_in - H + k], k < H
template <typename T>
__device__ void write_history(const T *in, long n_in, const T *hist_in, T *hist_out, int H) {
    for (int k = threadIdx.x; k < H; k += blockDim.x) {
        long idx = n_in - H + k;
        hist_out[k] = idx >= 0 ? in[idx] : hist_in[H + idx];
    }
}

// ================================================================ generic
template <int KV, bool FMA>
__global__ void decim_generic(DecimLaunch a, unsigned M) {
    const int ch = blockIdx.y;
    const int N = a.ntaps, H = N - 1;
    const long n_out = a.n_out, n_in = a.n_in;
    if (blockIdx.x == 0) {
        if constexpr (KV == KV_CF32 || KV == KV_CI32_I32) {
            write_history((const uint2 *)a.in + ch * a.in_stride, n_in, (const uint2 *)a.hist_in[ch],
                          (uint2 *)a.hist_out[ch], H);
        } else {
            write_history((const uint32_t *)a.in + ch * a.in_stride, n_in, (const uint32_t *)a.hist_in[ch],
                          (uint32_t *)a.hist_out[ch], H);
        }
    }
    for (long o = (long)blockIdx.x * blockDim.x + threadIdx.x; o < n_out; o += (long)gridDim.x * blockDim.x) {
        const long j = o * (long)M;
        if constexpr (KV == KV_CF32) {
            const float2 *in = (const float2 *)a.in + ch * a.in_stride;
            const float2 *hist = (const float2 *)a.hist_in[ch];
            const float *c = (const float *)a.coef;
            float yr = 0.f, yi = 0.f;
            for (int k = 0; k < N; ++k) {
                float2 x = fetch(in, hist, j - k, n_in, H);
                yr = mac<FMA>(c[k], x.x, yr);
                yi = mac<FMA>(c[k], x.y, yi);
            }
            ((float2 *)a.out + ch * a.out_stride)[o] = make_float2(q16f(yr, a.shift), q16f(yi, a.shift));
        } else if constexpr (KV == KV_F32_REAL) {
            const float *in = (const float *)a.in + ch * a.in_stride;
            const float *hist = (const float *)a.hist_in[ch];
            const float *c = (const float *)a.coef;
            float y = 0.f;
            for (int k = 0; k < N; ++k) y = mac<FMA>(c[k], fetch(in, hist, j - k, n_in, H), y);
            ((float2 *)a.out + ch * a.out_stride)[o] = make_float2(q16f(y, a.shift), 0.f);
        } else if constexpr (KV == KV_CI32_I32) {
            const int2 *in = (const int2 *)a.in + ch * a.in_stride;
            const int2 *hist = (const int2 *)a.hist_in[ch];
            const int32_t *c = (const int32_t *)a.coef;
            uint32_t yr = 0, yi = 0;
            for (int k = 0; k < N; ++k) {
                int2 x = fetch(in, hist, j - k, n_in, H);
                yr += (uint32_t)c[k] * (uint32_t)x.x;
                yi += (uint32_t)c[k] * (uint32_t)x.y;
            }
            ((uint32_t *)a.out + ch * a.out_stride)[o] =
                pack16(limit16((int32_t)yr, a.shift), limit16((int32_t)yi, a.shift));
        } else {  // KV_CI16_I32, KV_CI16_I16
            const uint32_t *in = (const uint32_t *)a.in + ch * a.in_stride;
            const uint32_t *hist = (const uint32_t *)a.hist_in[ch];
            const int32_t *c = (const int32_t *)a.coef;
            uint32_t yr = 0, yi = 0;
            for (int k = 0; k < N; ++k) {
                uint32_t w = fetch(in, hist, j - k, n_in, H);
                uint32_t pr = (uint32_t)c[k] * (uint32_t)sext16(w);
                uint32_t pi = (uint32_t)c[k] * (uint32_t)sext16_hi(w);
                if constexpr (KV == KV_CI16_I16) {  // std::operator*(short, complex<short>): int16 wrap
                    pr = (uint32_t)sext16(pr);
                    pi = (uint32_t)sext16(pi);
                }
                yr += pr;
                yi += pi;
            }
            ((uint32_t *)a.out + ch * a.out_stride)[o] =
                pack16(limit16((int32_t)yr, a.shift), limit16((int32_t)yi, a.shift));
        }
    }
}


// ============================================================ ci16 tiles
// complex<int16_t> samples are 4 B, so a 4-sample polyphase group is one
// 16-B granule.  Lane chunk = R granules; an even R gets one pad granule per
// chunk (stride R+1 odd), an odd R is conflict-free as is.
template <int R>
struct Ci16Geo {
    static constexpr int PAD = (R % 2 == 0) ? 1 : 0;
};

// NCO mixer of mixers.h:169-188 on one packed sample
__device__ __forceinline__ uint32_t mix_sample(uint32_t w, const int16_t *tab, unsigned N, unsigned phi) {
    unsigned ic = phi + N / 4;  // (phi + N/4) % N with phi < N
    ic = ic >= N ? ic - N : ic;
    int32_t lr = tab[ic], li = tab[phi];
    int32_t ar = sext16(w), ai = sext16_hi(w);
    int32_t r = ar * lr - ai * li;   // |.| < 2^31: |T| <= 16383
    int32_t i = ai * lr + li * ar;
    return pack16(limit16(r, 14), limit16(i, 14));
}

}  // namespace srcdsp
namespace srcdsp {

// ------------------------------------------------------- persistent cf32
// LDS hand-off between the waves of one workgroup without a memory fence:
// waits for this wave's LDS traffic only, so outstanding global loads (the
// next tile's prefetch) and output stores stay in flight across the barrier.
#define SRCDSP_LDS_BARRIER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")

// Phase clock of decim_dot2_ci16 (tuning builds only, -DSRCDSP_PHASE_CLOCK,
// scripts/tune/phase_clock.py): every wave sums the shader cycles (s_memtime)
// it spends in each phase of its tile loop, and lane 0 adds the sums to
// phase_clock[] (vector atomics) at exit:
//   0 prologue (table build, history, first staging load), 1 wait at the
//   barrier before staging, 2 staging (mix + LDS writes), 3 wait at the
//   barrier after staging (+ next tile's load issue), 4 tap loop + quantise,
//   5 stores, 6 waves, 7 tiles.
// The stamps wait for outstanding LDS reads (lgkmcnt), so they perturb the
// schedule a little; they are a diagnosis, not a timing.
#ifdef SRCDSP_PHASE_CLOCK
static __device__ unsigned long long phase_clock[8];
#define SRCDSP_PH(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define SRCDSP_PH_ADD(k, d) ph_acc[k] += (d)
#else
#define SRCDSP_PH(v)
#define SRCDSP_PH_ADD(k, d)
#endif


}  // namespace srcdsp
namespace srcdsp {

// limitScale16 of a float accumulator when (coeffScaling - leftShift) & 31 == 0:
// trunc, clamp to +-32767, and 0 for |y| >= 2^31 or NaN (x86 cvttss2si gives
// INT_MIN there, which limitScale16 passes through and int16 truncates to 0).
// 4 VALU ops instead of the integer path's ~8; identical results.
__device__ __forceinline__ float q16f_shift0(float y) {
    // "+ 0.0f" turns the -0.0 that trunc gives for y in (-1, 0) into +0.0, as the
    // integer round trip of the reference does
    const float t = __builtin_fminf(__builtin_fmaxf(__builtin_truncf(y), -32767.0f), 32767.0f) + 0.0f;
    return __builtin_fabsf(y) < 2147483648.0f ? t : 0.0f;
}

// Persistent complex<float> decimator: the headline (a1, M = 4, R = 4) and the
// same schedule at M = 16 / 8 / 3 / 2 / 1 with R = 1 / 2 / 4 / 4 / 8 outputs
// per lane (lane chunks of M R = 16 / 16 / 12 / 8 / 8 input samples; M = 1 is
// the complex<float> FilterFir).
//
// Tiles.  A tile is BLOCK*R outputs; its input span (M*BLOCK*R samples + a
// 4*NQ sample halo, NQ = ceil(N/4)) is staged HBM -> VGPR -> LDS as 16-B
// granules (2 samples).  LDS granule of tile granule g:
//   L(g) = g + (g - 2NQ + KPAD*PR) / PR,  PR = M*R/2 granules per lane chunk,
// i.e. one pad granule in front of every lane chunk, so lane t's chunk starts
// at B_t = 2NQ + KPAD + (PR+1) t and the 16 lanes of a ds_read_b128 group hit
// 16 distinct 16-B bank slots.
// Memory schedule.  Persistent grid, tiles in grid-stride order (the chip
// sweeps one contiguous window of the input at a time); the NEXT tile's
// loads (buffer_load_dwordx4, non-temporal, one descriptor per tile: the
// range check zero-fills past the end) are issued into VGPRs before this
// tile's taps and land in LDS after its stores, in one loop iteration, so
// the wait for them leaves the stores in flight.
// Taps.  Each lane owns R consecutive outputs and walks the taps as 4
// polyphase register windows sliding one sample per 4 taps; taps are
// wave-uniform SGPR pairs issued tap-major through inline asm (pk_fma_tap:
// every accumulator chain advances one tap before any advances the next).
// FMA: one v_pk_fma_f32 per tap and output (bit-exact to the -mfma build);
// strict: R v_pk_mul_f32, then R v_pk_add_f32 (bit-exact to the -O2 build).
// Tap count.  NT > 0: compiled in (the tap loop unrolls completely).  NT = 0:
// a.ntaps at run time (<= kCfMaxTaps), the tap loop in chunks of S 4-tap
// steps whose window groups rotate through S register slots (2S a multiple
// of PR, so a chunk's LDS reads are one base plus immediates), the chunk's
// taps loaded one chunk ahead, taps past N skipped (never multiplied by 0:
// 0 * inf would differ); the LDS image is dynamic, sized by the host.
// Outputs.  Quantised (Q0: the shift-0 quantiser) and paired across lanes
// by v_permlane32_swap / v_permlane16_swap (store_wave_lines) so every store
// instruction writes 1 KiB of whole lines, non-temporal.
template <bool NTS>
__device__ __forceinline__ void store16(float4 *p, float4 v) {
    if constexpr (NTS) {
        typedef float f4_t __attribute__((ext_vector_type(4)));
        f4_t w = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(w, (f4_t *)p);
    } else {
        *p = v;
    }
}
// Whole-line stores of one wave's outputs without an LDS round trip.  Lane l
// holds R = 4 or 8 consecutive float2 outputs (wave output l*R + r), i.e.
// R/2 16-B units; storing them as they stand would make every store
// instruction half- or quarter-cover its 128-B lines.  A transpose of units
// across 32-lane halves (v_permlane32_swap) and, for R = 8, 16-lane rows
// (v_permlane16_swap) leaves in register j the units of lanes
// [64j/(R/2), 64(j+1)/(R/2)): each store instruction then writes 1 KiB of
// whole lines.  wo = the wave's first output; ln = lane in wave.
template <int R, bool NTS>
__device__ __forceinline__ void store_wave_lines(float2 *wo, const float2 (&o)[R], int ln) {
    static_assert(R == 4 || R == 8, "4 or 8 outputs per lane");
    constexpr int U = R / 2;  // 16-B units per lane
    unsigned u[U][4];
#pragma unroll
    for (int k = 0; k < U; ++k) {
        u[k][0] = __float_as_uint(o[2 * k].x);
        u[k][1] = __float_as_uint(o[2 * k].y);
        u[k][2] = __float_as_uint(o[2 * k + 1].x);
        u[k][3] = __float_as_uint(o[2 * k + 1].y);
    }
    // vdst rows of the upper half <-> vsrc rows of the lower half
#pragma unroll
    for (int k = 0; k < U / 2; ++k)
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            auto sw = __builtin_amdgcn_permlane32_swap(u[k][d], u[k + U / 2][d], false, false);
            u[k][d] = sw[0];
            u[k + U / 2][d] = sw[1];
        }
    if constexpr (U == 4) {  // odd 16-lane rows of vdst <-> even rows of vsrc
#pragma unroll
        for (int k = 0; k < U; k += 2)
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                auto sw = __builtin_amdgcn_permlane16_swap(u[k][d], u[k + 1][d], false, false);
                u[k][d] = sw[0];
                u[k + 1][d] = sw[1];
            }
    }
    // register j, lane ln: unit (ln / (64/U)) of lane (64/U) j + ln % (64/U)
    constexpr int LPJ = 64 / U;
    float2 *base = wo + (ln % LPJ) * R + 2 * (ln / LPJ);
#pragma unroll
    for (int j = 0; j < U; ++j)
        store16<NTS>((float4 *)(base + LPJ * R * j), make_float4(__uint_as_float(u[j][0]), __uint_as_float(u[j][1]),
                                                                __uint_as_float(u[j][2]), __uint_as_float(u[j][3])));
}
constexpr int kCfMaxTaps = 1024;

// runtime-tap kernel geometry: the window's register slots (the EH + 3 live
// groups, EH = M(R-1)/4) and the 4-tap steps per chunk (the smallest multiple
// of the slots that makes 2 U a multiple of the PR granules of a lane chunk,
// so a chunk's LDS reads are one base plus immediates), and the front slack of
// its LDS image (granules below the halo that the tail chunk's unconditional
// window reads may touch)
__host__ __device__ constexpr int cf32_rt_slots(int M, int R) { return (M * (R - 1)) / 4 + 3; }
__host__ __device__ constexpr int cf32_rt_steps(int M, int R) {
    int u = cf32_rt_slots(M, R);
    while ((2 * u) % (M * R / 2) != 0) u += cf32_rt_slots(M, R);
    return u;
}
__host__ __device__ constexpr int cf32_rt_front(int M, int R) {
    return 2 * cf32_rt_steps(M, R) + ceildiv(2 * cf32_rt_steps(M, R), M * R / 2) + 2;
}
// dynamic LDS granules of the runtime-tap kernel (decim_stream_cf32<0, ...>)
__host__ __device__ constexpr int cf32_lds_granules(int M, int R, int BLOCK, int ntaps) {
    return cf32_rt_front(M, R) + (M * BLOCK * R / 2 + 2 * ((ntaps + 3) / 4)) +
           ((M * BLOCK * R / 2 + 2 * ((ntaps + 3) / 4)) + ceildiv(2 * ((ntaps + 3) / 4), M * R / 2) * (M * R / 2)) /
               (M * R / 2) +
           1;
}

template <int NT, int R, int BLOCK, bool FMA, int MINW, bool Q0, int M>
__global__ __launch_bounds__(BLOCK, MINW) void decim_stream_cf32(DecimLaunch a) {
    static_assert((M * R) % 4 == 0 && M * R <= 16, "a lane chunk is 4, 8, 12 or 16 input samples");
    static_assert(R == 1 || R == 2 || R == 4 || R == 8, "whole-line stores assume 1, 2, 4 or 8 outputs per lane");
    constexpr bool RT = NT == 0;
    // the compiled-in tap loop unrolls completely over a window of 4 (NQ + M R / 4)
    // samples; at M = 4 beyond 128 taps and at M = 1 beyond 64 it no longer stays
    // in registers (1-2 KiB of scratch per lane), so those lengths take NT = 0
    static_assert(RT || (M == 1 ? NT <= 64 : (M > 4 || NT <= 128)),
                  "compile the tap count in only where the unrolled window stays in registers");
    constexpr int NQC = RT ? (kCfMaxTaps + 3) / 4 : (NT + 3) / 4;  // the register prefetch is sized for this halo
    constexpr int TO = BLOCK * R;
    constexpr int PR = M * R / 2;  // granules per lane chunk (M R samples)
    constexpr int PER = ceildiv(M * TO / 2 + 2 * NQC, BLOCK);
    const int N = RT ? a.ntaps : NT;
    const int NQ = RT ? (N + 3) / 4 : NQC;
    const int TG = M * TO / 2 + 2 * NQ;  // staged granules: M TO input samples + the halo
    const int KPAD = ceildiv(2 * NQ, PR);
    float4 *lds;
    if constexpr (RT) {
        extern __shared__ float4 lds_dyn[];
        lds = lds_dyn + cf32_rt_front(M, R);
    } else {
        constexpr int TGC = M * TO / 2 + 2 * NQC, KPC = ceildiv(2 * NQC, PR);
        __shared__ float4 lds_st[TGC + (TGC + KPC * PR) / PR + 1];
        lds = lds_st;
    }

    const int ch = blockIdx.y;
    const float2 *in = (const float2 *)a.in + ch * a.in_stride;
    const float2 *hist = (const float2 *)a.hist_in[ch];
    float2 *out = (float2 *)a.out + ch * a.out_stride;
    const long n_in = a.n_in;
    const int H = N - 1;
    const int t = threadIdx.x;
    const long nb = gridDim.x;
    const long b = xcd_tile(blockIdx.x, nb);
    // grid-stride tile order: tiles b, b + nb, b + 2 nb, ...
    if (b == 0 && a.ntiles > 0) write_history(in, n_in, hist, (float2 *)a.hist_out[ch], H);

    float4 v[PER];
    // tiles >= 1: one descriptor per tile, 32-bit lane offsets, range-checked
    auto stage_load = [&](float4 (&v)[PER], long tile) {
        const long b0 = M * tile * TO - 4 * NQ;  // >= 0 for tile >= 1
        const long remb = (n_in - b0) * 8;
        const unsigned nrec = (unsigned)(remb > 0xfffffff0L ? 0xfffffff0L : (remb < 0 ? 0 : remb));
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(in + b0), 0, nrec, 0x00020000);
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int g = t + i * BLOCK;
            if ((i + 1) * BLOCK <= M * TO / 2 || g < TG) {  // the tile body always exists; the halo tail may not
                // lane offset in the VGPR, the per-load step in soffset (an
                // SGPR constant): one offset VGPR for all PER loads; aux 2 = nt
                auto w = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * t, 16 * i * BLOCK, 2);
                v[i] = make_float4(__uint_as_float(w[0]), __uint_as_float(w[1]), __uint_as_float(w[2]),
                                   __uint_as_float(w[3]));
            }
        }
    };
    if (b < a.ntiles) {
        if (b == 0) {  // tile 0: the halo comes from the history
            const long b0 = -4 * NQ;
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int g = t + i * BLOCK;
                const long s = b0 + 2 * (long)g;
                if (g < TG) {
                    float2 lo = fetch(in, hist, s, n_in, H), hi = fetch(in, hist, s + 1, n_in, H);
                    v[i] = make_float4(lo.x, lo.y, hi.x, hi.y);
                }
            }
        } else {
            stage_load(v, b);
        }
    }
    const int Bt = 2 * NQ + KPAD + (PR + 1) * t;
    // the staged tile lands in LDS once every wave is done with the previous
    // tile's image
    // LDS granule of staged granule g = t + i BLOCK: g + (g - 2NQ + KPAD PR) / PR,
    // the quotient's lane part computed once (BLOCK a multiple of PR)
    const int lq = (t - 2 * NQ + KPAD * PR) / PR;  // >= 0
    auto stage_to_lds = [&]() {
        SRCDSP_LDS_BARRIER();
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int g = t + i * BLOCK;
            if ((i + 1) * BLOCK <= M * TO / 2 || g < TG) {
                if constexpr (BLOCK % PR == 0)
                    lds[g + lq + i * (BLOCK / PR)] = v[i];
                else
                    lds[g + (g - 2 * NQ + KPAD * PR) / PR] = v[i];
            }
        }
        SRCDSP_LDS_BARRIER();
    };
    // one tap step (4 taps k = 4q..4q+3) over the R accumulators; xs(r, p) is
    // sample M r - 4q - p of the lane frame; cp2(j) the tap pair j of the step
    auto tap_step = [&](f2_t (&acc)[R], int k0, auto first_tag, auto guard_tag, auto &&xs, auto &&cp2, int kn) {
        constexpr bool FIRST = decltype(first_tag)::value;  // k0 == 0: accumulators start from +0
        constexpr bool GUARD = decltype(guard_tag)::value;  // taps k0 + p >= kn skipped
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            if (GUARD && k0 + p >= kn) break;
            const unsigned long long cp = cp2(p >> 1);
            if constexpr (FMA) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const float2 x = xs(r, p);
                    const f2_t xv = {x.x, x.y};
                    if (FIRST && p == 0) pk_fma_tap<false, true>(acc[r], cp, xv);
                    else if (p & 1) pk_fma_tap<true, false>(acc[r], cp, xv);
                    else pk_fma_tap<false, false>(acc[r], cp, xv);
                }
            } else {
                f2_t pr[R];
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const float2 x = xs(r, p);
                    const f2_t xv = {x.x, x.y};
                    if (p & 1) pk_mul_tap<true>(pr[r], cp, xv);
                    else pk_mul_tap<false>(pr[r], cp, xv);
                }
#pragma unroll
                for (int r = 0; r < R; ++r) pk_add_acc(acc[r], pr[r]);
            }
        }
    };
    // one tile: taps over the LDS image, outputs stored
    // WHOLE: the tile's TO outputs all exist (every tile but a partial last one)
    auto do_tile = [&](long tile, auto whole_tag) {
        constexpr bool WHOLE = decltype(whole_tag)::value;
        ConstPtr<unsigned long long> tp2 = const_view<unsigned long long>(a.coef);
        asm volatile("" : "+s"(tp2));
        f2_t acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = f2_t{0.f, 0.f};
        auto rd = [&](int idx) { return lds[idx]; };
        if constexpr (!RT) {
            constexpr int GPC = M * R / 4;  // 4-sample groups per lane chunk
            float2 X[4 * (NQC + GPC)];
            auto load_group = [&](int e) {
                const float4 g0 = rd(Bt + 2 * e + floordiv(2 * e, PR));
                const float4 g1 = rd(Bt + 2 * e + 1 + floordiv(2 * e + 1, PR));
                X[4 * e + 4 * NQC + 0] = make_float2(g0.x, g0.y);
                X[4 * e + 4 * NQC + 1] = make_float2(g0.z, g0.w);
                X[4 * e + 4 * NQC + 2] = make_float2(g1.x, g1.y);
                X[4 * e + 4 * NQC + 3] = make_float2(g1.z, g1.w);
            };
#pragma unroll
            for (int e = -1; e < GPC; ++e) load_group(e);
#pragma unroll
            for (int q = 0; q < NQC; ++q) {
                if (q + 1 < NQC) load_group(-q - 2);
                if ((q & 3) == 0) asm volatile("" : "+s"(tp2));
                auto xs = [&](int r, int p) { return X[M * r - 4 * q - p + 4 * NQC]; };
                auto cp2 = [&](int j) { return tp2[2 * q + j]; };
                if (q == 0)
                    tap_step(acc, 4 * q, std::true_type{}, std::integral_constant<bool, (4 * NQC > NT)>{}, xs, cp2, NT);
                else if (q == NQC - 1)
                    tap_step(acc, 4 * q, std::false_type{}, std::integral_constant<bool, (4 * NQC > NT)>{}, xs, cp2, NT);
                else
                    tap_step(acc, 4 * q, std::false_type{}, std::false_type{}, xs, cp2, NT);
            }
        } else {
            // window groups e (samples 4e..4e+3 of the lane frame) in S rotating
            // register slots; a step q reads groups -q-1 .. EH-q and prefetches
            // -q-2; chunks of U steps (q0 a multiple of U)
            constexpr int EH = (M * (R - 1)) / 4;
            constexpr int S = cf32_rt_slots(M, R), U = cf32_rt_steps(M, R);
            static_assert(S == EH + 3 && U % S == 0 && (2 * U) % PR == 0, "window slots / chunk steps");
            float2 X[S][4];
            auto slot = [](int e) { return ((e % S) + S) % S; };
            // chunk base: LDS granule of group c - q0 is cb + 2c + floordiv(2c, PR)
            auto load_group = [&](int cb, int c) {
                const float4 g0 = rd(cb + 2 * c + floordiv(2 * c, PR));
                const float4 g1 = rd(cb + 2 * c + 1 + floordiv(2 * c + 1, PR));
                float2(&d)[4] = X[slot(c)];
                d[0] = make_float2(g0.x, g0.y);
                d[1] = make_float2(g0.z, g0.w);
                d[2] = make_float2(g1.x, g1.y);
                d[3] = make_float2(g1.z, g1.w);
            };
#pragma unroll
            for (int e = -1; e <= EH; ++e) load_group(Bt, e);
            // the chunk body: U steps from q0 (a multiple of U).  TAIL: the
            // last chunk, every tap through TapGuarded (k < N, a branch inside
            // the asm: the compiler sees the same straight line as a full
            // chunk); its window reads are unconditional (the image has front
            // slack for the reads past the halo)
            auto chunk = [&](int q0, auto tail_tag, auto jb_tag, auto je_tag) {
                constexpr bool TAIL = decltype(tail_tag)::value;
                constexpr int JB = decltype(jb_tag)::value, JE = decltype(je_tag)::value;  // steps [JB, JE)
                const int cb = Bt - 2 * q0 - 2 * q0 / PR;
                ConstPtr<unsigned long long> tc = tp2 + 2 * q0;
                asm volatile("" : "+s"(tc));
                const int kb = 4 * q0;
#pragma unroll
                for (int j = JB; j < JE; ++j) {
                    if (j > JB && (j & 3) == 0) asm volatile("" : "+s"(tc));  // taps in batches of 16 (one s_load_dwordx16)
                    load_group(cb, -j - 2);
#pragma unroll
                    for (int p = 0; p < 4; ++p) {
                        const unsigned long long cp = tc[2 * j + (p >> 1)];
                        f2_t xv[R];
#pragma unroll
                        for (int r = 0; r < R; ++r) {
                            const int s = M * r - 4 * j - p;  // sample of the frame, relative to -4 q0
                            const int e = floordiv(s, 4);
                            const float2 x = X[slot(e)][s - 4 * e];
                            xv[r] = f2_t{x.x, x.y};
                        }
                        if constexpr (TAIL) {
                            if (p & 1) TapGuarded<R, true, FMA>::run(acc, cp, xv, kb + 4 * j + p, N);
                            else TapGuarded<R, false, FMA>::run(acc, cp, xv, kb + 4 * j + p, N);
                        } else if constexpr (FMA) {
#pragma unroll
                            for (int r = 0; r < R; ++r) {
                                if (p & 1) pk_fma_tap<true, false>(acc[r], cp, xv[r]);
                                else pk_fma_tap<false, false>(acc[r], cp, xv[r]);
                            }
                        } else {
                            f2_t pr[R];
#pragma unroll
                            for (int r = 0; r < R; ++r) {
                                if (p & 1) pk_mul_tap<true>(pr[r], cp, xv[r]);
                                else pk_mul_tap<false>(pr[r], cp, xv[r]);
                            }
#pragma unroll
                            for (int r = 0; r < R; ++r) pk_add_acc(acc[r], pr[r]);
                        }
                    }
                    // one step at a time: the next step's group is already in
                    // flight; hoisting more reads only lengthens the live window
                    __builtin_amdgcn_sched_barrier(0);
                }
            };
            // full chunks while all their taps exist, then the last chunk,
            // guarded, in two halves: the second only when steps remain there
            // (the guarded steps' reads and branches are the runtime kernel's
            // overhead over a compiled tap count)
            using I0 = std::integral_constant<int, 0>;
            using IH = std::integral_constant<int, U / 2>;
            using IU = std::integral_constant<int, U>;
            int q0 = 0;
            for (; 4 * (q0 + U) <= N; q0 += U) chunk(q0, std::false_type{}, I0{}, IU{});
            if (q0 < NQ) {
                chunk(q0, std::true_type{}, I0{}, IH{});
                if (q0 + U / 2 < NQ) chunk(q0, std::true_type{}, IH{}, IU{});
            }
        }
        const long n0 = tile * TO + (long)t * R;
        const unsigned sh = a.shift;
        auto q = [&](float y) { return Q0 ? q16f_shift0(y) : q16f(y, sh); };
        if constexpr (WHOLE && R == 2) {  // 16 B per lane: whole lines as they stand
            store16<true>((float4 *)(out + n0), make_float4(q(acc[0].x), q(acc[0].y), q(acc[1].x), q(acc[1].y)));
        } else if constexpr (WHOLE && R == 1) {  // 8 B per lane, lane-contiguous
            out[n0] = make_float2(q(acc[0].x), q(acc[0].y));
        } else if constexpr (WHOLE) {
            float2 o[R];
#pragma unroll
            for (int r = 0; r < R; ++r) o[r] = make_float2(q(acc[r].x), q(acc[r].y));
            store_wave_lines<R, true>(out + tile * TO + (t & ~63) * R, o, t & 63);
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (n0 + r < a.n_out) out[n0 + r] = make_float2(q(acc[r].x), q(acc[r].y));
        }
    };
    // Every iteration of the loop prefetches (the workgroup's last tile is
    // peeled off after it), and only the launch's last tile can be partial, so
    // the loop body is one straight path with a fixed number of stores: the
    // compiler waits for the prefetch with a counted vmcnt and the stores stay
    // in flight across iterations.
    if (b < a.ntiles) {
        stage_to_lds();
        long tile = b;
        for (; tile + nb < a.ntiles; tile += nb) {
            stage_load(v, tile + nb);
            do_tile(tile, std::true_type{});
            stage_to_lds();
        }
        if ((tile + 1) * TO <= a.n_out)
            do_tile(tile, std::true_type{});
        else
            do_tile(tile, std::false_type{});
    }
}


}  // namespace srcdsp
namespace srcdsp {

// Persistent complex<int16_t> x int32-tap decimator (M = 4), optionally with
// the NCO mixer of mixers.h fused into the staging pass (config 4).
// Same skeleton as decim_stream2_cf32: a 4-sample polyphase group is one
// 16-B granule (4 packed words); one pad granule per lane chunk (R even) keeps
// the lanes' ds_read_b128 conflict-free; next tile prefetched into VGPRs.
// Products c*x with |c| < 2^23 (host-checked) are exact as v_mad_i32_i24 and
// the int32 accumulation wraps like the reference's complex<int32_t>.
template <int NT, int R, int BLOCK, bool MIX, int MINW>
__global__ __launch_bounds__(BLOCK, MINW) void decim_stream_ci16(DecimLaunch a) {
    static_assert(R % 2 == 0, "padded layout assumes an even lane chunk");
    constexpr int NQ = (NT + 3) / 4;
    constexpr int TO = BLOCK * R;
    constexpr int TG = TO + NQ;  // granules of 4 samples
    constexpr int PR = R;
    constexpr int KPAD = ceildiv(NQ, PR);
    constexpr int LG = TG + (TG + KPAD * PR) / PR + 1;
    constexpr int PER = ceildiv(TG, BLOCK);
    constexpr int TABMAX = MIX ? 4096 : 1;
    __shared__ uint4 lds[LG];
    __shared__ int16_t tab[TABMAX];

    const int ch = blockIdx.y;
    const uint32_t *in = (const uint32_t *)a.in + ch * a.in_stride;
    const uint32_t *hist = (const uint32_t *)a.hist_in[ch];
    uint32_t *out = (uint32_t *)a.out + ch * a.out_stride;
    const long n_in = a.n_in;
    const int H = NT - 1;
    const int t = threadIdx.x;
    const unsigned N = a.mix_N, fr = a.mix_freq;
    const long nb = gridDim.x;
    const long b = xcd_tile(blockIdx.x, nb);
    const long per = a.ntiles / nb, rem = a.ntiles % nb;
    const long t_begin = b * per + (b < rem ? b : rem);
    const long t_end = t_begin + per + (b < rem ? 1 : 0);

    if constexpr (MIX) {
        for (int i = t; i < (int)N; i += BLOCK) tab[i] = a.mix_table[i];
        __syncthreads();
    }
    auto adv = [&](unsigned p, unsigned d) { p += d; return p >= N ? p - N : p; };
    // 32-bit phase arithmetic only: (base + (k mod N) * fr) mod N with k, fr < 2^16
    auto phase_add = [&](unsigned base, unsigned k) { return (base + (k % N) * fr) % N; };
    auto mix = [&](uint32_t w, unsigned ph) { return mix_sample(w, tab, N, ph); };
    if (t_begin == 0 && t_end > 0) {  // new history = last H samples of (history ++ mixed input)
        uint32_t *ho = (uint32_t *)a.hist_out[ch];
        for (int k = t; k < H; k += BLOCK) {
            long idx = n_in - H + k;
            uint32_t w = idx >= 0 ? in[idx] : hist[H + idx];
            if constexpr (MIX)  // mix_phase_hist = phase of sample n_in - H (>= 0 whenever idx >= 0)
                if (idx >= 0) w = mix(w, idx < k ? phase_add(a.mix_phase0, (unsigned)idx)
                                                 : phase_add(a.mix_phase_hist, (unsigned)k));
            ho[k] = w;
        }
    }
    // per-lane phase offsets of the staged granules: sample b0 + 4g, g = t + i*BLOCK
    const unsigned d_lane = MIX ? phase_add(0, 4 * t) : 0;
    const unsigned d_i = MIX ? phase_add(0, 4 * BLOCK) : 0;
    // phase of a tile's first staged sample (b0 = 4*tile*TO - 4*NQ)
    auto tile_phase = [&](long tile) {
        return (a.mix_phase_tile0 + ((unsigned)(tile % N)) * a.mix_dtile) % N;
    };

    uint4 v[PER];
    auto mix4 = [&](uint4 &w, unsigned ph) {
        w.x = mix(w.x, ph); ph = adv(ph, fr);
        w.y = mix(w.y, ph); ph = adv(ph, fr);
        w.z = mix(w.z, ph); ph = adv(ph, fr);
        w.w = mix(w.w, ph);
    };
    auto stage_load = [&](long tile) {  // tile >= 1
        const long b0 = 4 * tile * TO - 4 * NQ;
        const long remb = (n_in - b0) * 4;
        const unsigned nrec = (unsigned)(remb > 0xfffffff0L ? 0xfffffff0L : (remb < 0 ? 0 : remb));
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(in + b0), 0, nrec, 0x00020000);
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int g = t + i * BLOCK;
            if (g < TG) {
                auto w = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * g, 0, 0);
                v[i] = make_uint4(w[0], w[1], w[2], w[3]);
            }
        }
    };
    // mix the staged words in registers before they go to LDS.  Past the input
    // end the range-checked loads returned 0, and mixing 0 gives 0, so no
    // per-lane bound checks are needed (tiles >= 1 have no negative indices).
    auto stage_mix = [&](long tile) {
        if constexpr (MIX) {
            unsigned ph = adv(tile_phase(tile), d_lane);
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                if (t + i * BLOCK < TG) mix4(v[i], ph);
                ph = adv(ph, d_i);
            }
        }
    };
    if (t_begin < t_end) {
        if (t_begin == 0) {  // tile 0: halo from the (already mixed) history
            const long b0 = -4 * NQ;
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int g = t + i * BLOCK;
                const long s = b0 + 4 * (long)g;
                if (g < TG) {
                    uint32_t w[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        w[j] = fetch(in, hist, s + j, n_in, H);
                        if constexpr (MIX)
                            if (s + j >= 0 && s + j < n_in) w[j] = mix(w[j], phase_add(a.mix_phase0, (unsigned)(s + j)));
                    }
                    v[i] = make_uint4(w[0], w[1], w[2], w[3]);
                }
            }
        } else {
            stage_load(t_begin);
        }
    }
    const int Bt = NQ + KPAD + (PR + 1) * t;
    for (long tile = t_begin; tile < t_end; ++tile) {
        SRCDSP_LDS_BARRIER();
        // mixing here (after the barrier, once the prefetch has landed) keeps
        // the compiler from hoisting it into the FMA loop (register spills)
        if (tile != 0) stage_mix(tile);
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int g = t + i * BLOCK;
            if (g < TG) lds[g + (g - NQ + KPAD * PR) / PR] = v[i];
        }
        SRCDSP_LDS_BARRIER();
        if (tile + 1 < t_end) stage_load(tile + 1);

        ConstPtr<int32_t> tp = const_view<int32_t>(a.coef);
        asm volatile("" : "+s"(tp));
        int32_t Xr[4 * (NQ + R)], Xi[4 * (NQ + R)];
        int32_t yr[R], yi[R];
#pragma unroll
        for (int r = 0; r < R; ++r) yr[r] = yi[r] = 0;
        auto load_group = [&](int e) {
            const uint4 g = lds[Bt + e + floordiv(e, PR)];
            const int o = 4 * e + 4 * NQ;
            Xr[o + 0] = sext16(g.x); Xi[o + 0] = sext16_hi(g.x);
            Xr[o + 1] = sext16(g.y); Xi[o + 1] = sext16_hi(g.y);
            Xr[o + 2] = sext16(g.z); Xi[o + 2] = sext16_hi(g.z);
            Xr[o + 3] = sext16(g.w); Xi[o + 3] = sext16_hi(g.w);
        };
#pragma unroll
        for (int e = -1; e < R; ++e) load_group(e);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            if (q + 1 < NQ) load_group(-q - 2);
            if ((q & 3) == 0) asm volatile("" : "+s"(tp));
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const int k = 4 * q + p;
                if (k < NT) {
                    const int32_t c = tp[k];
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const int o = 4 * (r - q) - p + 4 * NQ;
                        yr[r] += __mul24(c, Xr[o]);
                        yi[r] += __mul24(c, Xi[o]);
                    }
                }
            }
        }
        const long n0 = tile * TO + (long)t * R;
        const unsigned sh = a.shift;
        if (n0 + R <= a.n_out && R == 4) {
            *(uint4 *)(out + n0) = make_uint4(pack16(limit16(yr[0], sh), limit16(yi[0], sh)),
                                              pack16(limit16(yr[1], sh), limit16(yi[1], sh)),
                                              pack16(limit16(yr[2], sh), limit16(yi[2], sh)),
                                              pack16(limit16(yr[3], sh), limit16(yi[3], sh)));
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (n0 + r < a.n_out) out[n0 + r] = pack16(limit16(yr[r], sh), limit16(yi[r], sh));
        }
    }
}

// ------------------------------------------------- ci16 x int16-range taps
// Persistent complex<int16_t> decimator (M = 4) on v_dot2_i32_i16: each dot2
// is TWO taps of one component.  The staged samples are split into a real
// and an imaginary plane of packed int16 pairs (x[2e], x[2e+1]); with the taps
// paired as P_j = (lo c[2j], hi c[2j-1]) (c[-1] = c[NT] = 0) output r of a
// lane (input sample 4r of its chunk) is
//   y_r = sum_{j=0}^{J-1} dot2(D[2r - j], P_j),  D[d] = plane dword d,
// so a lane's 4 outputs slide ONE register window down the plane by one dword
// per tap pair: 8 dot2 per pair, one ds_read_b128 per plane every 4 pairs.
// Products int16 x int16 and the int32 accumulation wrap exactly as the
// reference's complex<int32_t> arithmetic (host checks |c| <= 32767).
// Fused mixer (MIX): the LDS table holds (lo T[(k+N/4)%N], hi T[k]) = (lr, li);
// re = dot2(x, (lr, -li)), im = dot2(swap(x), (lr, li)).
// LDS: the planes are stored column-major.  Plane granule G (8 samples of one
// component, 16 B) of plane pl sits in slot  pl*2NC + (G&1)*NC + (G>>1)
// (NC = 4 mod 8).  A lane's window reads (granule 2t + HG + c, c compile-time)
// are then one per-lane base t plus an immediate offset -- no per-read
// address arithmetic -- and the 16 lanes of a ds_read_b128 group hit 16
// consecutive slots; the staging writes (staged granule g -> 8-B half g&1 of
// plane granule g>>1) put 16 consecutive lanes on 16 distinct 8-B bank slots
// because 2NC = 8 (mod 16).  No padding.  (The XOR-swizzled layout this
// replaces needed ~6 VALU ops per read: ~200 per wave tile.)
template <int NC>
__device__ __forceinline__ int dot2_slot(int G, int pl) {
    static_assert(NC % 8 == 4, "2 NC = 8 (mod 16): conflict-free staging writes");
    return pl * 2 * NC + (G & 1) * NC + (G >> 1);
}
// outputs per lane of decim_dot2_ci16 at decimation M: a lane chunk is 16
// input samples (2 plane granules) at every M
__host__ __device__ constexpr int dot2_r(int M) { return 16 / M; }
// run-time tap count (decim_dot2_ci16<0, ...>): N <= kDot2MaxTaps; tap pairs
// padded with zero pairs to whole 4-pair steps (exact: integer products of a
// zero pair add 0), and the halo of that padded count plus one plane granule
// pair (the window granule read one step ahead of the last step)
constexpr int kDot2MaxTaps = 1024;
__host__ __device__ constexpr int dot2_rt_pairs(int ntaps) { return 4 * ceildiv(ntaps / 2 + 1, 4); }
__host__ __device__ constexpr int dot2_rt_halo(int ntaps) {
    return 16 * ceildiv(2 * (dot2_rt_pairs(ntaps) - 1), 16) + 16;
}
// device tap-pair array length: zero pairs of slack past the padded count for
// the chunk of up to 24 pairs requested one chunk ahead
constexpr int dot2_pair_slack = 32;  // >= the largest chunk (24 pairs at M = 1)
__host__ __device__ constexpr int dot2_pair_alloc(int ntaps) { return dot2_rt_pairs(ntaps) + dot2_pair_slack; }
__device__ __forceinline__ int32_t clamp_s14(int32_t v) {
    const int32_t a = v >> 14;  // |v| < 2^30: never INT_MIN
    return a > 32767 ? 32767 : (a < -32767 ? -32767 : a);
}
__device__ __forceinline__ uint32_t lo16_pair(uint32_t a, uint32_t b) {  // (lo a, lo b)
    return __builtin_amdgcn_perm(b, a, 0x05040100u);
}
__device__ __forceinline__ uint32_t hi16_pair(uint32_t a, uint32_t b) {  // (hi a, hi b)
    return __builtin_amdgcn_perm(b, a, 0x07060302u);
}
__device__ __forceinline__ int32_t sdot2(uint32_t a, uint32_t b, int32_t c) {
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t_, a), __builtin_bit_cast(short2_t_, b), c, false);
}
// dot2 into a fresh accumulator: the VOP3 form with an inline 0 (the compiler
// otherwise materialises the 0 with a v_mov for the accumulating VOP2 form)
__device__ __forceinline__ int32_t sdot2_0(uint32_t a, uint32_t b) {
    int32_t r;
    asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// limitScale16 of a complex<int32_t> accumulator pair for a shift in 1..31
// (never INT_MIN after the shift): saturating pack, then -32768 -> -32767
__device__ __forceinline__ uint32_t limit16_pair_sh(int32_t re, int32_t im, unsigned shift) {
    const short2_t_ p = __builtin_amdgcn_cvt_pk_i16(re >> (shift & 31u), im >> (shift & 31u));
    const short2_t_ lo = {-32767, -32767};
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(p, lo));
}
// two mixer outputs (int32, >> 14 pending) -> one packed int16 pair clamped to
// +-32767 (limitScale16; |v >> 14| < 2^17 so INT_MIN never occurs):
// saturating v_cvt_pk_i16_i32, then v_pk_max_i16 with -32767
__device__ __forceinline__ uint32_t clamp_pair_s14(int32_t a, int32_t b) {
    const short2_t_ p = __builtin_amdgcn_cvt_pk_i16(a >> 14, b >> 14);
    const short2_t_ lo = {-32767, -32767};
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(p, lo));
}

// mixers.h:169-188 on one packed sample with the (lr, li) table word
__device__ __forceinline__ void mix_dot2(uint32_t w, uint32_t C, int32_t &re, int32_t &im) {
    const uint32_t A = __builtin_bit_cast(uint32_t, __builtin_bit_cast(short2_t_, C) * (short2_t_){1, -1});
    const uint32_t ws = __builtin_amdgcn_alignbit(w, w, 16);
    re = clamp_s14(sdot2(w, A, 0));
    im = clamp_s14(sdot2(ws, C, 0));
}

// Tiled decimator for any tap count (<= kDtMaxTaps) at M in {2, 4, 8}
// (dnsampling_filters.h:129-172 off the headline's 127/128-tap M=4 shape),
// complex<float> (KV_CF32; P = 1: fma chain, 0: mul+add) or complex<int16_t>
// with int32 (KV_CI16_I32; P = 0: |c| < 2^23 as v_mad_i32_i24, 1: full 32-bit
// products) or int16 taps (KV_CI16_I16, P = 2: products wrapped to int16).
// A lane owns R = 16/M consecutive outputs, i.e. one 16-sample block b = lane
// of the tile's input image; output r, tap k reads sample r*M - k of the
// lane's block frame.  Taps run in chunks of 16 (one SGPR s_load each); chunk
// c touches blocks b-c ("cur") and b-c-1 ("nxt"), so three 16-sample register
// windows rotate over the chunks (the next chunk's window is read from LDS
// while this one's MACs run).  Each output is one sequential chain in
// ascending k; taps past N are skipped, never multiplied by zero (0 * inf
// would differ).  ci16 samples are split into int32 (re, im) while staging,
// so the image has the cf32 layout: LDS blocks are 8 granules + one pad
// granule and the lanes' ds_read_b128 are conflict-free.  One tile per
// workgroup; the image holds ceil(N/16) halo blocks before the tile.
__device__ __forceinline__ float4 nt_load4(const float4 *p) {
    typedef float f4_t __attribute__((ext_vector_type(4)));
    const f4_t w = __builtin_nontemporal_load((const f4_t *)p);
    return make_float4(w[0], w[1], w[2], w[3]);
}
constexpr int kDtBlock = 256, kDtMaxTaps = 1024;
// samples per lane block: a multiple of M and of 4 (an even number of 16-B
// granules, so the padded block stride RM/2 + 1 is odd: conflict-free reads)
__host__ __device__ constexpr int dt_rm(int M) { return M <= 2 || M == 4 ? 8 : (M == 3 || M == 6 ? 12 : (M == 5 ? 20 : 16)); }
__host__ __device__ constexpr int dt_bs(int M) { return dt_rm(M) / 2 + 1; }  // LDS granules per block

template <int KV, int M, int P>
__global__ __launch_bounds__(kDtBlock) void decim_tile(DecimLaunch a) {
    constexpr int RM = dt_rm(M), BS = dt_bs(M);
    static_assert(RM % M == 0 && RM % 4 == 0, "block geometry");
    static_assert(KV == KV_CF32 || KV == KV_CI16_I32 || KV == KV_CI16_I16, "sample kinds");
    constexpr bool CF = KV == KV_CF32;
    typedef typename std::conditional<CF, float2, int2>::type X2;
    typedef typename std::conditional<CF, float2, uint32_t>::type SIn;
    constexpr int R = RM / M, TO = kDtBlock * R;
    extern __shared__ float4 dimg[];
    const int ch = blockIdx.y;
    const SIn *in = (const SIn *)a.in + ch * a.in_stride;
    const SIn *hist = (const SIn *)a.hist_in[ch];
    const long n_in = a.n_in;
    const int N = a.ntaps, H = N - 1;
    const int NCH = (N + RM - 1) / RM;  // tap chunks = halo blocks
    const int t = threadIdx.x;
    const long tile = blockIdx.x;
    if (tile == 0) write_history(in, n_in, hist, (SIn *)a.hist_out[ch], H);
    // image block i holds samples s0 + 16 i .. s0 + 16 i + 15, as (re, im) pairs
    const long s0 = tile * (long)TO * M - (long)NCH * RM;
    const int NG = (NCH + kDtBlock) * (RM / 2);  // 2-sample granules
    auto put = [&](int g, float4 v) { dimg[(g / (RM / 2)) * BS + g % (RM / 2)] = v; };
    auto split = [&](uint32_t w0, uint32_t w1) {
        return make_float4(__int_as_float(sext16(w0)), __int_as_float(sext16_hi(w0)), __int_as_float(sext16(w1)),
                           __int_as_float(sext16_hi(w1)));
    };
    // the tile's own span (every tile but the launch's last lies inside the
    // input): all RM/2 granule loads of a lane issued before any lands in LDS
    const int G0 = NCH * (RM / 2);
    const bool body_in = (tile + 1) * (long)TO * M <= n_in;
    if (body_in) {
        float4 v[RM / 2];
#pragma unroll
        for (int i = 0; i < RM / 2; ++i) {
            const long s = s0 + 2L * (G0 + t + i * kDtBlock);
            // complex<float>: non-temporal, the body is read once (the halo
            // re-read is an L2 hit): 4 % at M = 2/4 x 63 taps; complex<int16_t>
            // measured 0-5 % slower with it (profiles/tuning/r02_tile_nt_ab.txt)
            if constexpr (CF) {
                v[i] = nt_load4((const float4 *)(in + s));
            } else {
                const uint2 w = *(const uint2 *)(in + s);
                v[i] = split(w.x, w.y);
            }
        }
#pragma unroll
        for (int i = 0; i < RM / 2; ++i) put(G0 + t + i * kDtBlock, v[i]);
    }
    for (int g = t; g < (body_in ? G0 : NG); g += kDtBlock) {
        const long s = s0 + 2L * g;
        float4 v;
        if constexpr (CF) {
            if (s >= 0 && s + 1 < n_in) {
                v = *(const float4 *)(in + s);
            } else {
                const float2 lo = fetch(in, hist, s, n_in, H), hi = fetch(in, hist, s + 1, n_in, H);
                v = make_float4(lo.x, lo.y, hi.x, hi.y);
            }
        } else {
            uint32_t w0, w1;
            if (s >= 0 && s + 1 < n_in) {
                const uint2 w = *(const uint2 *)(in + s);
                w0 = w.x;
                w1 = w.y;
            } else {
                w0 = fetch(in, hist, s, n_in, H);
                w1 = fetch(in, hist, s + 1, n_in, H);
            }
            v = split(w0, w1);
        }
        put(g, v);
    }
    __syncthreads();
    X2 W0[RM], W1[RM], W2[RM];
    auto load = [&](X2 (&w)[RM], int blk) {
#pragma unroll
        for (int i = 0; i < RM / 2; ++i) {
            const float4 v = dimg[blk * BS + i];
            if constexpr (CF) {
                w[2 * i] = make_float2(v.x, v.y);
                w[2 * i + 1] = make_float2(v.z, v.w);
            } else {
                w[2 * i] = make_int2(__float_as_int(v.x), __float_as_int(v.y));
                w[2 * i + 1] = make_int2(__float_as_int(v.z), __float_as_int(v.w));
            }
        }
    };
    typedef typename std::conditional<CF, float, uint32_t>::type Acc;
    Acc yr[R], yi[R];
#pragma unroll
    for (int r = 0; r < R; ++r) yr[r] = yi[r] = Acc{};
    const int me = NCH + t;  // the lane's own block
    typedef typename std::conditional<CF, float, int32_t>::type Tap;
    ConstPtr<Tap> tp = const_view<Tap>(a.coef);
    auto chunk = [&](int c, const X2 (&cur)[RM], const X2 (&nxt)[RM], X2 (&nn)[RM]) {
        asm volatile("" : "+s"(tp));
        if (c + 1 < NCH) load(nn, me - c - 2);
#pragma unroll
        for (int i = 0; i < RM; ++i) {
            const int k = c * RM + i;
            if (k >= N) break;
            const Tap cf = tp[k];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int l = r * M - i;
                const X2 x = l >= 0 ? cur[l] : nxt[l + RM];
                if constexpr (CF) {
                    yr[r] = mac<P == 1>(cf, x.x, yr[r]);
                    yi[r] = mac<P == 1>(cf, x.y, yi[r]);
                } else if constexpr (P == 0) {  // |c| < 2^23: the low 32 bits of the exact product
                    yr[r] += (uint32_t)__mul24(cf, x.x);
                    yi[r] += (uint32_t)__mul24(cf, x.y);
                } else if constexpr (P == 1) {
                    yr[r] += (uint32_t)cf * (uint32_t)x.x;
                    yi[r] += (uint32_t)cf * (uint32_t)x.y;
                } else {  // std::operator*(short, complex<short>): int16 wrap
                    yr[r] += (uint32_t)sext16((uint32_t)__mul24(cf, x.x));
                    yi[r] += (uint32_t)sext16((uint32_t)__mul24(cf, x.y));
                }
            }
        }
    };
    load(W0, me);
    load(W1, me - 1);
    int c = 0;
    for (; c + 3 <= NCH; c += 3) {
        chunk(c, W0, W1, W2);
        chunk(c + 1, W1, W2, W0);
        chunk(c + 2, W2, W0, W1);
    }
    if (c < NCH) chunk(c, W0, W1, W2);
    if (c + 1 < NCH) chunk(c + 1, W1, W2, W0);
    const long o0 = tile * TO + (long)t * R;
    if constexpr (CF) {
        float2 *out = (float2 *)a.out + ch * a.out_stride;
        if (R % 2 == 0 && o0 + R <= a.n_out) {
#pragma unroll
            for (int r = 0; r + 1 < R; r += 2)
                store16<true>((float4 *)(out + o0 + r), make_float4(q16f(yr[r], a.shift), q16f(yi[r], a.shift),
                                                                    q16f(yr[r + 1], a.shift), q16f(yi[r + 1], a.shift)));
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (o0 + r < a.n_out) out[o0 + r] = make_float2(q16f(yr[r], a.shift), q16f(yi[r], a.shift));
        }
    } else {
        uint32_t *out = (uint32_t *)a.out + ch * a.out_stride;
        uint32_t w[R];
#pragma unroll
        for (int r = 0; r < R; ++r) w[r] = pack16(limit16((int32_t)yr[r], a.shift), limit16((int32_t)yi[r], a.shift));
        if (R % 2 == 0 && o0 + R <= a.n_out) {
#pragma unroll
            for (int r = 0; r + 1 < R; r += 2) *(uint2 *)(out + o0 + r) = make_uint2(w[r], w[r + 1]);
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (o0 + r < a.n_out) out[o0 + r] = w[r];
        }
    }
}

// Mixer table forms (TABM):
//  0: the (lr, li) word of phase k at k (N words);
//  1 (TAB2): that table stored twice (2N words), so the address of sample j of
//    staged granule i is one add of a wave-uniform tile/granule phase (SGPR)
//    and a per-lane constant (4t + j)*freq mod N -- no per-sample modulo.  The
//    lanes' words sit 4*freq apart: bank conflicts unless freq is odd*16;
//  2 (sequence table): the word of input SAMPLE s at s mod Pe (Pe = lcm(N /
//    gcd(freq, N), 4); sample s's phase (phi0 + s*freq) mod N depends on s mod
//    Pe only), stored twice (2 Pe words).  A lane's 4 samples are 4
//    consecutive words: one conflict-free ds_read_b128 per granule, any freq.
//  3 (two-word sequence table, Pe <= kSeq2Max): as 2, but both dot2 operands
//    of each sample are stored, A = (lr, -li) in one table and B = (li, lr)
//    in a second one kSeq2Off words further: re = dot2(x, A), im = dot2(x, B)
//    with no negate or half swap per sample (two conflict-free ds_read_b128
//    per granule).  |lr|, |li| <= 16383 (the LUT's amplitude), so -li fits.
//  4 (two-word sequence table stored once, Pe <= kSeq2Off): as 3 with each
//    table held once (2 Pe words: the LDS of form 2's doubled one-word table),
//    the granule's index m + lo (< 2 Pe) wrapped by one subtract and one min.
//  5 (two-word sequence in REGISTERS, Pe | SPT, 512 lanes): when the period
//    divides the tile's input span (config 4: N = 4096, any frequency, Pe a
//    power of two <= 4096), staged granule g = t + i BLOCK of every tile after
//    the first holds samples (4 t + (i odd ? 2048 : 0) + j - HS) mod Pe, so a
//    lane needs only 2 x 4 (A, B) word pairs: made once from the global LUT
//    into 16 VGPRs, no LDS table, no table fill, no table read per granule
//    (round 5's first form stored the table rotated by -HS in LDS and read
//    8 ds_read_b128 per lane-tile; form 4 spends 4 VALU per granule on the
//    index).  Tile 0 and the history read the global LUT per sample.
// Products via VOP3 dot2 and the pair clamp above.
constexpr int kSeq2Off = 4096, kSeq2Max = kSeq2Off / 2;
template <int NT, int BLOCK, bool MIX, int MINW, int TABM = 0, int MD = 4>
__global__ __launch_bounds__(BLOCK, MINW) void decim_dot2_ci16(DecimLaunch a) {
    constexpr bool TAB2 = TABM == 1, SEQT = TABM >= 2, SEQ2 = TABM >= 3, SEQ1 = TABM == 4, SEQR = TABM == 5;
    static_assert(!SEQR || BLOCK == 512, "the rotated table's two lane bases assume 4 BLOCK = 2048 samples per round");
    constexpr bool RT = NT == 0;                  // the tap count at run time (a.ntaps <= kDot2MaxTaps)
    static_assert(MD == 1 || MD == 2 || MD == 4 || MD == 8 || MD == 16, "M dividing the 16-sample lane chunk");
    static_assert(MD == 4 || RT, "tap counts are compiled in at M = 4 only");
    constexpr int R = dot2_r(MD);                 // outputs per lane (a lane chunk: 16 samples)
    constexpr int TO = BLOCK * R;                 // outputs per tile
    constexpr int SPT = MD * TO;                  // input samples per tile
    // compile-time geometry: the tap count's, or (RT) the largest tap count's,
    // which sizes the prefetch registers and the LDS image (its row length NC
    // then fixed, so every window read is a per-lane base plus immediates)
    constexpr int JC = RT ? dot2_rt_pairs(kDot2MaxTaps) : NT / 2 + 1;
    constexpr int HSC = RT ? dot2_rt_halo(kDot2MaxTaps) : 16 * ceildiv(2 * (JC - 1), 16);
    constexpr int PER = ceildiv((SPT + HSC) / 4, BLOCK);
    constexpr int PG = (SPT + HSC) / 8;           // plane granules
    constexpr int NC0 = ceildiv(PG, 2);
    constexpr int NC = NC0 + ((4 - NC0 % 8) + 8) % 8;  // slots per plane row, = 4 (mod 8)
    constexpr int LSLOTS = 4 * NC;
    constexpr int TABMAX = (MIX && !SEQR) ? (TABM ? 8192 : 4096) : 1;  // SEQR: the lane's words in registers
    static_assert(HSC % 16 == 0 && 2 * (JC - 1) <= HSC, "halo geometry");
    static_assert(BLOCK % 16 == 0, "column-major plane layout");
    // tap pairs (RT: padded with zero pairs to whole 4-pair steps), halo
    // samples (lane-chunk aligned; RT: one more plane granule pair, so the
    // window read one step ahead stays inside the image), staged granules
    const int J = RT ? dot2_rt_pairs(a.ntaps) : JC;
    const int HS = RT ? dot2_rt_halo(a.ntaps) : HSC;
    const int HG = HS / 8;                        // halo plane granules (even)
    const int TG = (SPT + HS) / 4;                // staged 16-B sample granules
    __shared__ uint4 lds[LSLOTS];
    __shared__ __attribute__((aligned(16))) uint32_t ctab[TABMAX];
#ifdef SRCDSP_PHASE_CLOCK
    unsigned long long ph_acc[8] = {0, 0, 0, 0, 0, 0, 1, 0};
#endif
    SRCDSP_PH(ph_start);

    const int ch = blockIdx.y;
    const uint32_t *in = (const uint32_t *)a.in + ch * a.in_stride;
    const uint32_t *hist = (const uint32_t *)a.hist_in[ch];
    uint32_t *out = (uint32_t *)a.out + ch * a.out_stride;
    const long n_in = a.n_in;
    const int H = RT ? a.ntaps - 1 : NT - 1;
    const int t = threadIdx.x;
    const unsigned N = a.mix_N, fr = a.mix_freq;
    const long nb = gridDim.x;
    const long b = xcd_tile(blockIdx.x, nb);
    const long per = a.ntiles / nb, rem = a.ntiles % nb;
    const long t_begin = b * per + (b < rem ? b : rem);
    const long t_end = t_begin + per + (b < rem ? 1 : 0);

    const unsigned Pe = SEQT ? a.mix_pe : 1u;
    // SEQR: every tile's staged granule t + i BLOCK reads the same 4 samples'
    // table words -- index (4 t + (i odd ? 2048 : 0) + j - HS) mod Pe -- so the
    // lane keeps its two granules' words (A = (lr, -li), B = (li, lr)) in 16
    // registers, made once from the global LUT (one 64-bit modulo per parity,
    // then a phase step per sample), and no table lives in LDS
    uint32_t rA[2][4] = {}, rB[2][4] = {};
    if constexpr (MIX && SEQR) {
        const int16_t *tab = a.mix_table;
        const unsigned hs = (unsigned)((long)HS % (long)Pe);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const unsigned m = (4u * t + (h ? 2048u % Pe : 0u) + Pe - hs) % Pe;  // sample offset of word j = 0
            unsigned k = (unsigned)(((unsigned long)a.mix_phase0 + (unsigned long)m * fr) % N);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                unsigned ic = k + N / 4;
                ic = ic >= N ? ic - N : ic;
                rA[h][j] = ((uint32_t)(uint16_t)tab[ic]) | ((uint32_t)(uint16_t)(-tab[k]) << 16);
                rB[h][j] = ((uint32_t)(uint16_t)tab[k]) | ((uint32_t)(uint16_t)tab[ic] << 16);
                k += fr;
                k = k >= N ? k - N : k;
            }
        }
    }
    if constexpr (MIX && !SEQR) {
        const int16_t *tab = a.mix_table;
        const int nw = SEQ1 ? (int)Pe : SEQT ? 2 * (int)Pe : (TAB2 ? 2 : 1) * (int)N;
        // SEQT: entry i holds the phase of sample i, (phi0 + i fr) mod N --
        // periodic in Pe, so i needs no reduction; one 64-bit
        // modulo per lane, then a step of BLOCK entries is one add and one
        // conditional subtract (a modulo per entry was ~100 VALU: ~8 per wave
        // tile of config 4 over a workgroup's tiles)
        unsigned kseq = 0, kstep = 0;
        if constexpr (SEQT) {
            kseq = (unsigned)(((unsigned long)a.mix_phase0 + (unsigned long)t * fr) % N);
            kstep = (unsigned)(((unsigned long)BLOCK * fr) % N);
        }
        for (int i = t; i < nw; i += BLOCK) {
            unsigned k;
            if constexpr (SEQT) {
                k = kseq;
                kseq += kstep;
                kseq = kseq >= N ? kseq - N : kseq;
            } else {
                k = (unsigned)i < N ? (unsigned)i : (unsigned)i - N;
            }
            unsigned ic = k + N / 4;
            ic = ic >= N ? ic - N : ic;
            if constexpr (SEQ2) {  // A = (lr, -li), B = (li, lr)
                ctab[i] = ((uint32_t)(uint16_t)tab[ic]) | ((uint32_t)(uint16_t)(-tab[k]) << 16);
                ctab[kSeq2Off + i] = ((uint32_t)(uint16_t)tab[k]) | ((uint32_t)(uint16_t)tab[ic] << 16);
            } else {
                ctab[i] = ((uint32_t)(uint16_t)tab[ic]) | ((uint32_t)(uint16_t)tab[k] << 16);
            }
        }
        __syncthreads();
    }
    auto adv = [&](unsigned p, unsigned d) { p += d; const unsigned q = p - N; return q < p ? q : p; };
    auto phase_add = [&](unsigned base, unsigned k) { return (base + (k % N) * fr) % N; };
    auto mix1 = [&](uint32_t w, unsigned ph) {
        int32_t re, im;
        if constexpr (SEQR) {  // no LDS table: ph is the phase itself, the words from the global LUT
            unsigned ic = ph + N / 4;
            ic = ic >= N ? ic - N : ic;
            const int16_t lr = a.mix_table[ic], li = a.mix_table[ph];
            re = clamp_s14(sdot2(w, ((uint32_t)(uint16_t)lr) | ((uint32_t)(uint16_t)(-li) << 16), 0));
            im = clamp_s14(sdot2(w, ((uint32_t)(uint16_t)li) | ((uint32_t)(uint16_t)lr << 16), 0));
        } else if constexpr (SEQ2) {
            re = clamp_s14(sdot2(w, ctab[ph], 0));
            im = clamp_s14(sdot2(w, ctab[kSeq2Off + ph], 0));
        } else {
            mix_dot2(w, ctab[ph], re, im);
        }
        return pack16(re, im);
    };
    // input sample s >= 0 of this call, mixed (any table form)
    auto mix_at = [&](uint32_t w, long s) {
        if constexpr (SEQR) return mix1(w, phase_add(a.mix_phase0, (unsigned)(s % (long)N)));
        else if constexpr (SEQT) return mix1(w, (unsigned)(s % (long)Pe));
        else return mix1(w, phase_add(a.mix_phase0, (unsigned)(s % (long)N)));
    };
    if (t_begin == 0 && t_end > 0) {  // new history = last H samples of (history ++ mixed input)
        uint32_t *ho = (uint32_t *)a.hist_out[ch];
        for (int k = t; k < H; k += BLOCK) {
            long idx = n_in - H + k;
            uint32_t w = idx >= 0 ? in[idx] : hist[H + idx];
            if constexpr (MIX)
                if (idx >= 0) w = mix_at(w, idx);
            ho[k] = w;
        }
    }
    const unsigned d_lane = MIX ? phase_add(0, 4 * t) : 0;
    const unsigned d_i = MIX ? phase_add(0, 4 * BLOCK) : 0;
    auto tile_phase = [&](long tile) {  // phase of the tile's first staged sample tile*SPT - HS
        return (a.mix_phase_tile0 + ((unsigned)(tile % N)) * a.mix_dtile) % N;
    };

    // staged granule of round i (one 16-B granule per lane per round), -1 past the tile
    auto sg = [&](int i) { const int g = t + i * BLOCK; return g < TG ? g : -1; };
    uint4 v[PER];
    auto stage_load = [&](long tile) {  // tile >= 1
        const long b0 = (long)SPT * tile - HS;
        const long remb = (n_in - b0) * 4;
        const unsigned nrec = (unsigned)(remb > 0xfffffff0L ? 0xfffffff0L : (remb < 0 ? 0 : remb));
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(in + b0), 0, nrec, 0x00020000);
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int g = sg(i);
            if (g >= 0) {
                auto w = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * g, 0, 0);
                v[i] = make_uint4(w[0], w[1], w[2], w[3]);
            }
        }
    };
    // staged granule g -> plane granule g>>1, half g&1
    auto lds_half = [&](int g, int plane) {
        const int G = g >> 1;
        return (uint2 *)&lds[dot2_slot<NC>(G, plane)] + (g & 1);
    };
    auto put = [&](int g, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
        *lds_half(g, 0) = make_uint2(lo16_pair(w0, w1), lo16_pair(w2, w3));
        *lds_half(g, 1) = make_uint2(hi16_pair(w0, w1), hi16_pair(w2, w3));
    };
    // mixes the granule in place (MIX) and writes both planes
    // TAB2: per-lane byte offsets of the 4 samples of a staged granule
    unsigned lj[4] = {0, 0, 0, 0};
    if constexpr (MIX && TAB2)
#pragma unroll
        for (int j = 0; j < 4; ++j) lj[j] = 4u * phase_add(0, 4 * t + j);
    auto put_mixed2 = [&](int g, uint4 w, unsigned sb) {  // sb: granule phase * 4 (uniform)
        const uint32_t *tb = ctab;
        auto ld = [&](int j) { return *(const uint32_t *)((const char *)tb + (sb + lj[j])); };
        const uint32_t c0 = ld(0), c1 = ld(1), c2 = ld(2), c3 = ld(3);
        auto neg_hi = [](uint32_t c) {
            return __builtin_bit_cast(uint32_t, __builtin_bit_cast(short2_t_, c) * (short2_t_){1, -1});
        };
        auto swp = [](uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); };
        const int32_t r0 = sdot2_0(w.x, neg_hi(c0)), i0 = sdot2_0(swp(w.x), c0);
        const int32_t r1 = sdot2_0(w.y, neg_hi(c1)), i1 = sdot2_0(swp(w.y), c1);
        const int32_t r2 = sdot2_0(w.z, neg_hi(c2)), i2 = sdot2_0(swp(w.z), c2);
        const int32_t r3 = sdot2_0(w.w, neg_hi(c3)), i3 = sdot2_0(swp(w.w), c3);
        *lds_half(g, 0) = make_uint2(clamp_pair_s14(r0, r1), clamp_pair_s14(r2, r3));
        *lds_half(g, 1) = make_uint2(clamp_pair_s14(i0, i1), clamp_pair_s14(i2, i3));
    };
    // SEQT: the granule's 4 words at ctab[m + lane offset], m = (first staged
    // sample of the granule row) mod Pe (uniform); lane offset 4t mod Pe
    const unsigned lo_t = SEQT ? (4u * t) % Pe : 0u;
    auto put_mixed_seq2 = [&](int g, uint4 w, unsigned m, unsigned lo) {
        unsigned ix = m + lo;  // < 2 Pe; a multiple of 4 words
        if constexpr (SEQ1) {
            const unsigned jx = ix - Pe;
            ix = jx < ix ? jx : ix;  // ix mod Pe (v_sub + v_min)
        }
        const uint4 A = *(const uint4 *)__builtin_assume_aligned(&ctab[ix], 16);
        const uint4 B = *(const uint4 *)__builtin_assume_aligned(&ctab[kSeq2Off + ix], 16);
        const int32_t r0 = sdot2_0(w.x, A.x), i0 = sdot2_0(w.x, B.x);
        const int32_t r1 = sdot2_0(w.y, A.y), i1 = sdot2_0(w.y, B.y);
        const int32_t r2 = sdot2_0(w.z, A.z), i2 = sdot2_0(w.z, B.z);
        const int32_t r3 = sdot2_0(w.w, A.w), i3 = sdot2_0(w.w, B.w);
        *lds_half(g, 0) = make_uint2(clamp_pair_s14(r0, r1), clamp_pair_s14(r2, r3));
        *lds_half(g, 1) = make_uint2(clamp_pair_s14(i0, i1), clamp_pair_s14(i2, i3));
    };
    auto put_mixed_seq1 = [&](int g, uint4 w, unsigned m, unsigned lo) {
        // m + lo is a multiple of 4 words: one 16-B read (the compiler, not
        // knowing that, would split it into 4-way-conflicting ds_read2_b32)
        const uint4 c = *(const uint4 *)__builtin_assume_aligned(&ctab[m + lo], 16);
        auto neg_hi = [](uint32_t x) {
            return __builtin_bit_cast(uint32_t, __builtin_bit_cast(short2_t_, x) * (short2_t_){1, -1});
        };
        auto swp = [](uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); };
        const int32_t r0 = sdot2_0(w.x, neg_hi(c.x)), i0 = sdot2_0(swp(w.x), c.x);
        const int32_t r1 = sdot2_0(w.y, neg_hi(c.y)), i1 = sdot2_0(swp(w.y), c.y);
        const int32_t r2 = sdot2_0(w.z, neg_hi(c.z)), i2 = sdot2_0(swp(w.z), c.z);
        const int32_t r3 = sdot2_0(w.w, neg_hi(c.w)), i3 = sdot2_0(swp(w.w), c.w);
        *lds_half(g, 0) = make_uint2(clamp_pair_s14(r0, r1), clamp_pair_s14(r2, r3));
        *lds_half(g, 1) = make_uint2(clamp_pair_s14(i0, i1), clamp_pair_s14(i2, i3));
    };
    // SEQR: the round's parity picks the lane's register words
    auto put_mixed_seqr = [&](int g, uint4 w, int h) {
        const uint32_t(&A)[4] = rA[h];
        const uint32_t(&B)[4] = rB[h];
        const int32_t r0 = sdot2_0(w.x, A[0]), i0 = sdot2_0(w.x, B[0]);
        const int32_t r1 = sdot2_0(w.y, A[1]), i1 = sdot2_0(w.y, B[1]);
        const int32_t r2 = sdot2_0(w.z, A[2]), i2 = sdot2_0(w.z, B[2]);
        const int32_t r3 = sdot2_0(w.w, A[3]), i3 = sdot2_0(w.w, B[3]);
        *lds_half(g, 0) = make_uint2(clamp_pair_s14(r0, r1), clamp_pair_s14(r2, r3));
        *lds_half(g, 1) = make_uint2(clamp_pair_s14(i0, i1), clamp_pair_s14(i2, i3));
    };
    auto put_mixed_seq = [&](int g, uint4 w, unsigned m, unsigned lo) {
        if constexpr (SEQ2) put_mixed_seq2(g, w, m, lo);
        else put_mixed_seq1(g, w, m, lo);
    };
    auto advp = [&](unsigned p, unsigned d) { p += d; const unsigned q = p - Pe; return q < p ? q : p; };
    // SEQT: (4*tile*TO - HS) mod Pe of the workgroup's current tile
    unsigned m_tile = 0;
    if constexpr (MIX && SEQT && !SEQR)
        if (t_begin < t_end) m_tile = (unsigned)((t_begin * (long)SPT - HS + 4 * (long)Pe * (1 + HS / 4)) % (long)Pe);
    auto put_mixed = [&](int g, uint4 w, unsigned ph) {
        if constexpr (MIX) {
            int32_t r0, i0, r1, i1, r2, i2, r3, i3;
            mix_dot2(w.x, ctab[ph], r0, i0); ph = adv(ph, fr);
            mix_dot2(w.y, ctab[ph], r1, i1); ph = adv(ph, fr);
            mix_dot2(w.z, ctab[ph], r2, i2); ph = adv(ph, fr);
            mix_dot2(w.w, ctab[ph], r3, i3);
            *lds_half(g, 0) = make_uint2(lo16_pair(r0, r1), lo16_pair(r2, r3));
            *lds_half(g, 1) = make_uint2(lo16_pair(i0, i1), lo16_pair(i2, i3));
        } else {
            put(g, w.x, w.y, w.z, w.w);
        }
    };
    if (t_begin < t_end) {
        if (t_begin == 0) {  // tile 0: halo from the (already mixed) history; mixed here, written below
            const long b0 = -HS;
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int g = sg(i);
                const long s0 = b0 + 4 * (long)g;
                if (g >= 0) {
                    uint32_t w[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        w[j] = fetch(in, hist, s0 + j, n_in, H);
                        if constexpr (MIX)
                            if (s0 + j >= 0 && s0 + j < n_in) w[j] = mix_at(w[j], s0 + j);
                    }
                    v[i] = make_uint4(w[0], w[1], w[2], w[3]);
                }
            }
        } else {
            stage_load(t_begin);
        }
    }
    SRCDSP_PH(ph_loop);
    SRCDSP_PH_ADD(0, ph_loop - ph_start);
    for (long tile = t_begin; tile < t_end; ++tile) {
        SRCDSP_PH(ph0);
        SRCDSP_LDS_BARRIER();
        SRCDSP_PH(ph1);
        if (MIX && SEQR && tile != 0) {
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int g = sg(i);
                if (g >= 0) put_mixed_seqr(g, v[i], i & 1);
            }
        } else if (MIX && SEQT && tile != 0) {
            unsigned m = m_tile;  // wave-uniform
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int g = sg(i);
                if (g >= 0) put_mixed_seq(g, v[i], m, lo_t);
                m = advp(m, a.mix_pe_drow);
            }
        } else if (MIX && TAB2 && tile != 0) {
            unsigned sp = tile_phase(tile);  // wave-uniform
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int g = t + i * BLOCK;
                if (g < TG) put_mixed2(g, v[i], 4u * sp);
                sp = adv(sp, d_i);
            }
        } else if (MIX && tile != 0) {
            unsigned ph = adv(tile_phase(tile), d_lane);
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int g = t + i * BLOCK;
                if (g < TG) put_mixed(g, v[i], ph);
                ph = adv(ph, d_i);
            }
        } else {
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int g = sg(i);
                if (g >= 0) put(g, v[i].x, v[i].y, v[i].z, v[i].w);
            }
        }
        SRCDSP_PH(ph2);
        SRCDSP_LDS_BARRIER();
        if constexpr (MIX && SEQT && !SEQR) m_tile = advp(m_tile, a.mix_pe_dtile);
        if (tile + 1 < t_end) stage_load(tile + 1);
        SRCDSP_PH(ph3);

        ConstPtr<uint32_t> tp = const_view<uint32_t>(a.coef);
        asm volatile("" : "+s"(tp));
        typedef uint32_t u4v_t __attribute__((ext_vector_type(4)));
        const unsigned sh = a.shift;
        // limitScale16 of an accumulator pair (dnsampling_filters.h:167-168);
        // Q14 taps: shift 14 (the common case), a saturating pack
        auto quant = [&](auto &yr_, auto &yi_, uint32_t *w_, int n_, int stride_) {
            if ((sh & 31u) != 0) {
#pragma unroll
                for (int k = 0; k < n_; ++k) w_[k * stride_] = limit16_pair_sh(yr_[k], yi_[k], sh);
            } else {
#pragma unroll
                for (int k = 0; k < n_; ++k) w_[k * stride_] = pack16(limit16(yr_[k], sh), limit16(yi_[k], sh));
            }
        };
        uint32_t w[R];
        if constexpr (!RT) {
            int32_t yr[R], yi[R];  // started by the first tap pair's inline-0 dot2 (no v_mov)
            // window: Dr[d + OFF], d in [-(4*NG), 8), NG = granules below the lane base
            constexpr int NG = ceildiv(JC - 1, 4);
            constexpr int OFF = 4 * NG;
            uint32_t Dr[OFF + 8], Di[OFF + 8];
            auto load_g = [&](int c) {  // plane granule lb + c -> dwords d = 4c .. 4c+3
                // granule lb + c = 2t + HG + c: row c & 1, column t + (HG + c) >> 1
                const int o = (c & 1) * NC + ((HG + c) >> 1);
                u4v_t gr = *(const u4v_t *)&lds[t + o];
                u4v_t gi = *(const u4v_t *)&lds[t + o + 2 * NC];
                // keep every read a whole ds_read_b128: at the window edges the
                // compiler would load only the words used, as ds_read2_b32 /
                // ds_read_b96, whose 4-B lane groups the layout does not spread
                asm volatile("" : "+v"(gr), "+v"(gi));
                Dr[OFF + 4 * c + 0] = gr[0]; Dr[OFF + 4 * c + 1] = gr[1]; Dr[OFF + 4 * c + 2] = gr[2]; Dr[OFF + 4 * c + 3] = gr[3];
                Di[OFF + 4 * c + 0] = gi[0]; Di[OFF + 4 * c + 1] = gi[1]; Di[OFF + 4 * c + 2] = gi[2]; Di[OFF + 4 * c + 3] = gi[3];
            };
            load_g(0);
            load_g(1);
#pragma unroll
            for (int j = 0; j < JC; ++j) {
                if ((j & 3) == 1) load_g(-1 - (j >> 2));
                if ((j & 15) == 0) asm volatile("" : "+s"(tp));
                const uint32_t P = tp[j];
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if (j == 0) {
                        yr[r] = sdot2_0(Dr[OFF + 2 * r], P);
                        yi[r] = sdot2_0(Di[OFF + 2 * r], P);
                    } else {
                        yr[r] = sdot2(Dr[OFF + 2 * r - j], P, yr[r]);
                        yi[r] = sdot2(Di[OFF + 2 * r - j], P, yi[r]);
                    }
                }
            }
            quant(yr, yi, w, R, 1);
        } else {
            // Run-time tap count: steps of 4 pairs.  Output r of a lane sits at
            // sample r M of the lane chunk; pair j multiplies (x[rM - 2j],
            // x[rM - 2j + 1]), i.e. plane dword rM/2 - j for even rM and, for
            // odd rM (M = 1), the odd-aligned pair built from dwords a and a+1,
            // a = (rM - 1)/2 - j, as (hi a, lo a+1) by one v_alignbit (reused
            // over the step's outputs).  Step q (pairs 4q..4q+3) reads window
            // granules -q-1 .. -q + EH/4 (EH = ceil((R-1) M/2)) and loads -q-2
            // for the next step: S >= EH/4 + 3 register slots (granule c in
            // slot c mod S, S even so granule parity is static) rotate with
            // static names over chunks of S steps (4S tap pairs, requested one
            // chunk ahead).  A chunk starting at step q0 reads granule e - q0
            // at column t + (HG - q0)/2 + floor(e/2) of row e & 1: one base per
            // chunk plus immediates.  At M = 1 (16 outputs per lane) the even
            // and the odd outputs run as two passes over the taps, 8
            // accumulator pairs each, in 256-lane workgroups at 3 waves per
            // SIMD (one pass of 16 spilled even at that 168-VGPR budget).
            constexpr int EH = ((R - 1) * MD + 1) / 2;
            constexpr int S = EH / 4 + 3 + (EH / 4 + 3) % 2;
            constexpr int U = S;
            constexpr int TPC = 4 * U;  // tap pairs per chunk
            constexpr int RSTEP = MD == 1 ? 2 : 1, RP = R / RSTEP;  // output stride and count of a pass
            static_assert(TPC <= dot2_pair_slack, "the pair array's zero slack covers a chunk read ahead");
            auto slot = [](int e) { return ((e % S) + S) % S; };
            auto chunk_base = [&](int q0) { return t + ((HG - q0) >> 1); };
            const int NS = J / 4;  // steps
            auto pass = [&](auto r0_tag) {
                constexpr int R0 = decltype(r0_tag)::value;  // first output of the pass
                int32_t yr[RP], yi[RP];
#pragma unroll
                for (int k = 0; k < RP; ++k) yr[k] = yi[k] = 0;
                uint32_t W[S][2][4];  // [slot][plane][dword]
                auto load_e = [&](int cb, int e) {
                    const int o = cb + (e & 1) * NC + (e >> 1);
                    u4v_t gr = *(const u4v_t *)&lds[o];
                    u4v_t gi = *(const u4v_t *)&lds[o + 2 * NC];
                    asm volatile("" : "+v"(gr), "+v"(gi));  // whole ds_read_b128 (as above)
                    uint32_t(&ww)[2][4] = W[slot(e)];
                    ww[0][0] = gr[0]; ww[0][1] = gr[1]; ww[0][2] = gr[2]; ww[0][3] = gr[3];
                    ww[1][0] = gi[0]; ww[1][1] = gi[1]; ww[1][2] = gi[2]; ww[1][3] = gi[3];
                };
                // the lgkmcnt wait for a window read then never waits on a fresh s_load
                uint32_t Tc[TPC], Tn[TPC];
                auto load_taps = [&](uint32_t(&T)[TPC], int q0) {
                    ConstPtr<uint32_t> tc = tp + 4 * q0;
                    asm volatile("" : "+s"(tc));
#pragma unroll
                    for (int i = 0; i < TPC; ++i) T[i] = tc[i];
                };
                load_taps(Tc, 0);
                auto chunk = [&](int q0, auto steps_tag) {
                    constexpr int SN = decltype(steps_tag)::value;  // steps in this chunk (U, or a tail 1..U-1)
                    const int cb = chunk_base(q0);
#pragma unroll
                    for (int s = 0; s < SN; ++s) {
                        load_e(cb, -s - 2);
                        if (SN == U && s == 0) load_taps(Tn, q0 + U);
#pragma unroll
                        for (int p = 0; p < 4; ++p) {
                            const uint32_t P = Tc[4 * s + p];
#pragma unroll
                            for (int k = 0; k < RP; ++k) {
                                const int r = R0 + k * RSTEP;
                                auto dw = [&](int pl, int d) {
                                    const int e = floordiv(d, 4);
                                    return W[slot(e)][pl][d - 4 * e];
                                };
                                if ((r * MD) % 2 == 0) {
                                    const int d = r * MD / 2 - 4 * s - p;
                                    yr[k] = sdot2(dw(0, d), P, yr[k]);
                                    yi[k] = sdot2(dw(1, d), P, yi[k]);
                                } else {  // odd-aligned pair (x[2a+1], x[2a+2])
                                    const int d = (r * MD - 1) / 2 - 4 * s - p;
                                    yr[k] = sdot2(__builtin_amdgcn_alignbit(dw(0, d + 1), dw(0, d), 16), P, yr[k]);
                                    yi[k] = sdot2(__builtin_amdgcn_alignbit(dw(1, d + 1), dw(1, d), 16), P, yi[k]);
                                }
                            }
                        }
                    }
                    if constexpr (SN == U) {
#pragma unroll
                        for (int i = 0; i < TPC; ++i) Tc[i] = Tn[i];
                    }
                };
                {
                    const int cb = chunk_base(0);
#pragma unroll
                    for (int e = EH / 4; e >= -1; --e) load_e(cb, e);
                }
                int q0 = 0;
                for (; q0 + U <= NS; q0 += U) chunk(q0, std::integral_constant<int, U>{});
                // the tail: 1 .. U-1 steps (wave-uniform), one unrolled body per length
                auto tail = [&](auto self, auto k_tag) {
                    constexpr int K = decltype(k_tag)::value;
                    if constexpr (K < U) {
                        if (NS - q0 == K) chunk(q0, k_tag);
                        else self(self, std::integral_constant<int, K + 1>{});
                    }
                };
                tail(tail, std::integral_constant<int, 1>{});
                quant(yr, yi, w + R0, RP, RSTEP);
            };
            pass(std::integral_constant<int, 0>{});
            if constexpr (RSTEP == 2) pass(std::integral_constant<int, 1>{});
        }
        SRCDSP_PH(ph4);
        const long n0 = tile * TO + (long)t * R;
        if (n0 + R <= a.n_out) {
            if constexpr (R >= 4) {
#pragma unroll
                for (int r = 0; r < R; r += 4) *(uint4 *)(out + n0 + r) = make_uint4(w[r], w[r + 1], w[r + 2], w[r + 3]);
            } else if constexpr (R == 2) {
                *(uint2 *)(out + n0) = make_uint2(w[0], w[1]);
            } else {
                out[n0] = w[0];
            }
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (n0 + r < a.n_out) out[n0 + r] = w[r];
        }
        SRCDSP_PH(ph5);
        SRCDSP_PH_ADD(1, ph1 - ph0);
        SRCDSP_PH_ADD(2, ph2 - ph1);
        SRCDSP_PH_ADD(3, ph3 - ph2);
        SRCDSP_PH_ADD(4, ph4 - ph3);
        SRCDSP_PH_ADD(5, ph5 - ph4);
        SRCDSP_PH_ADD(7, 1);
    }
#ifdef SRCDSP_PHASE_CLOCK
    if ((t & 63) == 0)
        for (int k = 0; k < 8; ++k) atomicAdd(&phase_clock[k], ph_acc[k]);
#endif
}

// ------------------------------------------------------ single-rate float FIR
// FilterFir (filters.h:133-169) for float input -> complex<float> output
// with a zero imaginary part (KV_F32_REAL), any tap count up to kFirMaxTaps
// (runtime).  complex<float> FilterFir / M = 1 decimators run on the headline
// kernel (decim_stream_cf32<0, R, ..., 1>, any N <= kCfMaxTaps), which takes
// every complex<float> shape this kernel could.
// Each lane owns R = 8 consecutive outputs; taps are walked in chunks of 4
// with a 12-sample register window held as three 4-sample blocks A|B|C (tap
// chunk q of output r reads sample r - 4q - p, p < 4).  After a chunk C drops,
// B -> C, A -> B and A is refilled from LDS, so three chunks are unrolled with
// rotating block roles and the window slides without register moves.  Each
// output is ONE sequential fma (or mul+add) chain in ascending tap order, as
// the reference's loop over n (filters.h:150-161).
// LDS: the tile span (tile outputs + P0 halo samples, P0 = 8*ceil((N-1)/8))
// as 16-B granules with one pad granule after every lane chunk (8 samples),
// so lanes' ds_read_b128 land on distinct bank slots (odd granule stride).
constexpr int kFirMaxTaps = 1024;
constexpr int kFirR = 8, kFirBlock = 256;

template <int KV>
struct FirTraits;
template <>
struct FirTraits<KV_F32_REAL> {
    typedef float S;
    static constexpr int SPG = 4;  // samples per 16-B granule
};

__device__ __forceinline__ float fir_mac(bool fma, float c, float x, float y) {
    return fma ? __builtin_fmaf(c, x, y) : y + c * x;
}

// The FIR arithmetic of one lane: R outputs from the staged LDS image `fl`
// (lane base granule gb), N taps (runtime) through the constant view tp.
template <int KV, bool FMA>
__device__ __forceinline__ void fir_lane(const float4 *fl, int gb, int N, ConstPtr<float> tp, unsigned sh,
                                         float2 (&o)[kFirR]) {
    typedef typename FirTraits<KV>::S S;
    constexpr int SPG = FirTraits<KV>::SPG;
    constexpr int R = kFirR, GPL = R / SPG;
    const int NQ = (N + 3) / 4;
    auto slot = [&](int g) { return g + g / GPL; };
    float yr[R];
    f2_t y2[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        yr[r] = 0.f;
        y2[r] = (f2_t){0.f, 0.f};
    }
    S A[4], B[4], C[4];
    // window reads through a volatile LDS view: every one a whole
    // ds_read_b128 (conflict-free at the odd granule stride).  Plain reads
    // were narrowed to the words used -- ds_read_b64 / b96 / read2_b32, whose
    // lane groups the padded layout does not spread (54.7 M conflict cycles
    // per launch at 31 taps, float in).
    typedef float f4v_t __attribute__((ext_vector_type(4)));
    auto rd = [&](int g) {
        const f4v_t w = *(const volatile __attribute__((address_space(3))) f4v_t *)(&fl[slot(g)]);
        return make_float4(w[0], w[1], w[2], w[3]);
    };
    auto fill = [&](S (&dst)[4], int m) {
        if constexpr (SPG == 4) {
            const float4 v = rd(gb + m / 4);
            dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
        } else {
            const float4 v0 = rd(gb + m / 2), v1 = rd(gb + m / 2 + 1);
            dst[0] = make_float2(v0.x, v0.y); dst[1] = make_float2(v0.z, v0.w);
            dst[2] = make_float2(v1.x, v1.y); dst[3] = make_float2(v1.z, v1.w);
        }
    };
    // chunk q: window blocks (lo = samples -4q-4.., mid = -4q.., hi = -4q+4..)
    auto chunk = [&](int q, const S (&lo)[4], const S (&mid)[4], const S (&hi)[4], bool guard) {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int k = 4 * q + p;
            if (guard && k >= N) break;
            const float c = tp[k];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int rel = r - p + 4;  // 0..11 over lo|mid|hi
                const S x = rel < 4 ? lo[rel] : (rel < 8 ? mid[rel - 4] : hi[rel - 8]);
                if constexpr (SPG == 4) {
                    yr[r] = fir_mac(FMA, c, x, yr[r]);
                } else {  // (re, im) as one packed pair: v_pk_fma_f32 / v_pk_mul + v_pk_add
                    const f2_t xv = {x.x, x.y}, cv = {c, c};
                    if constexpr (FMA) y2[r] = __builtin_elementwise_fma(cv, xv, y2[r]);
                    else y2[r] = y2[r] + cv * xv;
                }
            }
        }
    };
    fill(C, 4);
    fill(B, 0);
    int q = 0;
    for (; q + 3 <= NQ; q += 3) {
        asm volatile("" : "+s"(tp));
        fill(A, -4 * q - 4);
        chunk(q, A, B, C, false);          // A|B|C
        fill(C, -4 * q - 8);
        chunk(q + 1, C, A, B, false);      // C|A|B
        fill(B, -4 * q - 12);
        chunk(q + 2, B, C, A, q + 3 == NQ);  // B|C|A (guard the last chunk)
    }
    if (q < NQ) {
        fill(A, -4 * q - 4);
        chunk(q, A, B, C, true);
        if (q + 1 < NQ) {
            fill(C, -4 * q - 8);
            chunk(q + 1, C, A, B, true);
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
        o[r] = SPG == 4 ? make_float2(q16f(yr[r], sh), 0.f) : make_float2(q16f(y2[r].x, sh), q16f(y2[r].y, sh));
}

__host__ __device__ constexpr int fir_halo(int ntaps) { return 8 * (((ntaps + 3) / 4 + 1) / 2); }

// one tile per workgroup, any tap count up to kFirMaxTaps (dynamic LDS)
template <int KV, bool FMA>
__global__ __launch_bounds__(kFirBlock) void fir_tile_f32(DecimLaunch a) {
    typedef typename FirTraits<KV>::S S;
    constexpr int SPG = FirTraits<KV>::SPG;
    constexpr int R = kFirR, BLOCK = kFirBlock, TO = R * BLOCK;
    constexpr int GPL = R / SPG;  // granules per lane chunk
    extern __shared__ float4 fl[];
    const int N = a.ntaps, H = N - 1;
    const int P0 = fir_halo(N);  // >= 4*NQ: the last chunk's window block
    const int ch = blockIdx.y;
    const S *in = (const S *)a.in + ch * a.in_stride;
    const S *hist = (const S *)a.hist_in[ch];
    float2 *out = (float2 *)a.out + ch * a.out_stride;
    const long n_in = a.n_in;
    const int t = threadIdx.x;
    if (blockIdx.x == 0) write_history(in, n_in, hist, (S *)a.hist_out[ch], H);
    const long o0 = (long)blockIdx.x * TO;  // first output (= input sample) of the tile
    const int span = TO + P0;                // staged samples, origin o0 - P0
    auto slot = [&](int g) { return g + g / GPL; };
    // stage through the cache: the tile's own TO samples with every load of a
    // lane in flight before the LDS writes (every tile but the launch's last
    // lies inside the input), then the halo (from history on tile 0) and any
    // partial tile granule-wise
    const int GH = P0 / SPG;
    constexpr int GPB = TO / SPG / BLOCK;  // body granules per lane
    const bool body_in = o0 + TO <= n_in;
    if (body_in) {
        float4 v[GPB];
#pragma unroll
        for (int i = 0; i < GPB; ++i) v[i] = *(const float4 *)(in + o0 + (long)(t + i * BLOCK) * SPG);
#pragma unroll
        for (int i = 0; i < GPB; ++i) fl[slot(GH + t + i * BLOCK)] = v[i];
    }
    for (int g = t; g < (body_in ? GH : span / SPG); g += BLOCK) {
        const long s0 = o0 - P0 + (long)g * SPG;
        float4 v;
        if (s0 >= 0 && s0 + SPG <= n_in) {
            v = *(const float4 *)(in + s0);
        } else {
            S w[SPG];
#pragma unroll
            for (int j = 0; j < SPG; ++j) w[j] = fetch(in, hist, s0 + j, n_in, H);
            v = *(const float4 *)w;
        }
        fl[slot(g)] = v;
    }
    __syncthreads();
    float2 o[R];
    fir_lane<KV, FMA>(fl, (P0 + R * t) / SPG, N, const_view<float>(a.coef), a.shift, o);
    const long n0 = o0 + (long)t * R;
    if (n0 + R <= a.n_out) {
#pragma unroll
        for (int r = 0; r < R; r += 2) *(float4 *)(out + n0 + r) = make_float4(o[r].x, o[r].y, o[r + 1].x, o[r + 1].y);
    } else {
        for (int r = 0; r < R; ++r)
            if (n0 + r < a.n_out) out[n0 + r] = o[r];
    }
}

// Persistent variant for <= kFirStreamTaps taps (the headline decimator's
// memory schedule): grid-stride tile order, the next tile's buffer loads
// (non-temporal, range-checked zero fill past the end) issued into VGPRs
// right after this tile lands in LDS, outputs transposed across the wave's
// lanes into whole-line non-temporal stores (OST below).
constexpr int kFirStreamTaps = 128;

// OST: 1 = outputs staged through LDS (two more barriers per tile); 2 = the
// wave's outputs transposed across lanes (store_wave_lines) into whole-line
// stores, no LDS round trip.
// NTC > 0: the tap count as a compile-time constant (the tap loop unrolls
// completely); 0: a.ntaps at run time.
template <int KV, bool FMA, int OST = 2, int NTC = 0>
__global__ __launch_bounds__(kFirBlock, 4) void fir_stream_f32(DecimLaunch a) {
    typedef typename FirTraits<KV>::S S;
    constexpr int SPG = FirTraits<KV>::SPG;
    constexpr int R = kFirR, BLOCK = kFirBlock, TO = R * BLOCK;
    constexpr int GPL = R / SPG;
    constexpr int P0MAX = fir_halo(kFirStreamTaps);
    constexpr int TGMAX = (TO + P0MAX) / SPG;  // staged granules, worst case
    constexpr int PER = ceildiv(TGMAX, BLOCK);
    constexpr int LSTAGE = TGMAX + TGMAX / GPL + 1;
    constexpr int LOUT = TO * 8 / 16;          // output tile as float4
    __shared__ float4 fl[LSTAGE > LOUT ? LSTAGE : LOUT];
    const int N = NTC > 0 ? NTC : a.ntaps, H = N - 1;
    const int P0 = fir_halo(N);
    const int TG = (TO + P0) / SPG;
    const int ch = blockIdx.y;
    const S *in = (const S *)a.in + ch * a.in_stride;
    const S *hist = (const S *)a.hist_in[ch];
    float2 *out = (float2 *)a.out + ch * a.out_stride;
    const long n_in = a.n_in;
    const int t = threadIdx.x;
    const long nb = gridDim.x;
    const long b = xcd_tile(blockIdx.x, nb);
    if (b == 0) write_history(in, n_in, hist, (S *)a.hist_out[ch], H);
    auto slot = [&](int g) { return g + g / GPL; };
    float4 v[PER];
    auto stage_load = [&](long tile) {  // tile >= 1 (its halo is input, not history)
        const long s0 = tile * TO - P0;
        const long remb = (n_in - s0) * (long)sizeof(S);
        const unsigned nrec = (unsigned)(remb > 0xfffffff0L ? 0xfffffff0L : (remb < 0 ? 0 : remb));
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(in + s0), 0, nrec, 0x00020000);
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int g = t + i * BLOCK;
            if (g < TG) {
                // lane offset in the VGPR, per-load step in soffset; aux 2 = nt
                auto w = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * t, 16 * i * BLOCK, 2);
                v[i] = make_float4(__uint_as_float(w[0]), __uint_as_float(w[1]), __uint_as_float(w[2]),
                                   __uint_as_float(w[3]));
            }
        }
    };
    if (b < a.ntiles) {
        if (b == 0) {
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int g = t + i * BLOCK;
                if (g < TG) {
                    const long s0 = -P0 + (long)g * SPG;
                    S w[SPG];
#pragma unroll
                    for (int j = 0; j < SPG; ++j) w[j] = fetch(in, hist, s0 + j, n_in, H);
                    v[i] = *(const float4 *)w;
                }
            }
        } else {
            stage_load(b);
        }
    }
    ConstPtr<float> tp = const_view<float>(a.coef);
    // the staged tile lands in LDS once every wave is done with the previous
    // tile's image and output staging
    auto stage_to_lds = [&]() {
        SRCDSP_LDS_BARRIER();
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int g = t + i * BLOCK;
            if (g < TG) fl[slot(g)] = v[i];
        }
        SRCDSP_LDS_BARRIER();
    };
    // as decim_stream2_cf32: the next tile's loads are issued before this
    // tile's taps and land after its stores, in one iteration, so the wait
    // for them leaves the stores in flight
    auto do_tile = [&](long tile, auto whole_tag) {
        constexpr bool WHOLE = decltype(whole_tag)::value;
        float2 o[R];
        fir_lane<KV, FMA>(fl, (P0 + R * t) / SPG, N, tp, a.shift, o);
        const long o0 = tile * TO;
        if constexpr (OST == 2) {
            if constexpr (WHOLE) {
                store_wave_lines<R, true>(out + o0 + (t & ~63) * R, o, t & 63);
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r)
                    if (o0 + t * R + r < a.n_out) out[o0 + t * R + r] = o[r];
            }
            return;
        }
        SRCDSP_LDS_BARRIER();  // every wave is done reading the staged input
        float2 *ob = (float2 *)fl;
#pragma unroll
        for (int r = 0; r < R; ++r) ob[t * R + r] = o[r];
        SRCDSP_LDS_BARRIER();
        if constexpr (WHOLE) {
#pragma unroll
            for (int i = 0; i < LOUT / BLOCK; ++i) {
                const int k = t + i * BLOCK;
                store16<true>((float4 *)(out + o0) + k, fl[k]);
            }
        } else {
            for (int k = t; k < TO; k += BLOCK)
                if (o0 + k < a.n_out) out[o0 + k] = ob[k];
        }
    };
    // prefetching loop, the workgroup's last tile peeled (as decim_stream2_cf32)
    if (b < a.ntiles) {
        stage_to_lds();
        long tile = b;
        for (; tile + nb < a.ntiles; tile += nb) {
            stage_load(tile + nb);
            do_tile(tile, std::true_type{});
            stage_to_lds();
        }
        if ((tile + 1) * TO <= a.n_out)
            do_tile(tile, std::true_type{});
        else
            do_tile(tile, std::false_type{});
    }
}

}  // namespace srcdsp
