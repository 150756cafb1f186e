// decim_mfma.h -- complex<float> decimate-by-4 FIR on the f32-input matrix
// cores (FilterDnsamplingFir<cf32,cf32,cf32,float,4>, FMA float contract).
//
// Why matrix cores for a FIR: v_mfma_f32_16x16x4_f32 computes every output
// element as a k-ordered chain of fmas, one rounding each (D = fma(a3, b3,
// fma(a2, b2, fma(a1, b1, fma(a0, b0, C)))); MI355X_MICROARCH.md "FP32-input
// MFMA", verified here bit for bit by scripts/tune/mfma_probe.py), at the
// v_pk_fma_f32 rate, with one A and one B register per 1024 FMAs.  The VALU
// headline kernel (decim_stream2_cf32) draws enough power under that VALU load
// that the chip lowers its clock (1.2-2.0 GHz measured, profiles/r02_*ramp*)
// and its tap loop then no longer hides under the HBM stream; the matrix
// cores hold 2.4 GHz and leave the VALU idle.
//
// Formulation (dnsampling_filters.h:129-172: y[n] = sum_k c[k] x[4n-k] in
// ascending k, one fma chain per component):
//  * instruction = one 16x16 block, 4 K steps: rows i = 16 consecutive
//    outputs n_g + i of a group g, columns j = (group g = j >> 1, component
//    j & 1) -- 8 groups x 16 outputs = 128 outputs (a "sequence");
//  * K step s feeds every row of a column the SAME sample x[top_g - s]
//    (top_g = 4 (n_g + 15) + 1) and row i the tap c[4i - 61 + s]: the tap
//    its own chain needs at that sample, or 0.0 where that sample is outside
//    row i's window.  fma(0, x, acc) == acc for finite x (an fma chain from +0
//    only reaches -0 through an underflowing product, and the quantiser maps
//    -0 and +0 alike), so every output is exactly its own ascending-k chain.
//    KS = NT + 61 rounded up to 4: 188 K steps = 47 instructions for 127 taps
//    (68 % of the block's FMAs carry a tap);
//  * A (lane l: tap of row l & 15 at sub-step l >> 4) is constant for the
//    whole launch: 47 registers, loaded once;
//  * B (lane l: sample of column l & 15 at sub-step kk = l >> 4) walks its
//    column's samples 4 apart, i.e. one polyphase sub-sequence: the tile's
//    input span is staged into 8 LDS planes (re/im x sample phase mod 4) and a
//    lane reads 4 instructions' samples with one ds_read_b128.
// Non-finite inputs: a zero-tap step multiplies a sample outside the row's
// window (0 * inf = NaN).  A lane holding a non-finite accumulator recomputes
// its 4 outputs with the plain chain from LDS (never taken on finite data).
//
// LDS planes: span sample p (p = x index - S0, S0 = 4 n0 - 128) lives in plane
// (component, phi = p & 3) at float idx((p >> 2) + (phi >= 2)), idx(q) = q +
// 4 (q >> 4) (a 16-B pad every 64 B).  Plane bases are 32 floats apart mod 64
// between re and im.  With that, the 16 lanes of each ds_read_b128 lane group
// hit 16 distinct 16-B bank slots for every read (checked exhaustively).
#pragma once
#include "../../srcdsp_amd/csrc/decim_kernels.h"

namespace srcdsp {

typedef float f4m_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int mfma_idx(int q) { return q + 4 * (q >> 4); }

template <int NT>
struct MfmaGeo {
    static constexpr int KS = (NT + 61 + 3) & ~3;  // K steps
    static constexpr int MI = KS / 4;              // instructions per sequence
    static constexpr int RD = (MI + 3) / 4;        // ds_read_b128 per sequence
    static constexpr int HALO = 128;               // staged samples below 4 n0
    static constexpr int BLOCK = 256;              // 4 waves
    static constexpr int SEQ = 128;                // outputs per sequence
    static constexpr int TO = (BLOCK / 64) * 2 * SEQ;  // 2 sequences per wave
    static constexpr int SPAN = 4 * TO + HALO;     // staged samples per tile
    static constexpr int TG = SPAN / 2;            // 16-B granules (2 samples)
    static constexpr int PER = (TG + BLOCK - 1) / BLOCK;
    static constexpr int PS = ((SPAN / 4 + 2 + 4 * (SPAN / 64 + 1)) + 63) / 64 * 64;  // plane stride (floats)
    static constexpr int LDS_FLOATS = 8 * PS + 32;
    // top sample offset 4*15+1 = 61: Q of the first read (in 4-sample units)
    static constexpr int Q47 = (4 * 15 + 1 + HALO) / 4;
    static_assert(HALO % 16 == 0 && HALO >= KS - 61, "halo covers the lowest K step");
    static_assert(4 * (RD - 1) + 3 <= Q47, "reads stay inside the span");
    __host__ __device__ static constexpr int plane(int cmp, int phi) { return (4 * cmp + phi) * PS + 32 * cmp; }
};

// PROBE (tuning only): 0 = product; 1 = memory path only (no MFMA);
// 2 = compute path only (every tile reads one of 16 L2-resident spans).
template <int NT, int MINW, bool Q0, int PROBE = 0>
__global__ __launch_bounds__(256, MINW) void decim_mfma_cf32(DecimLaunch a) {
    using G = MfmaGeo<NT>;
    constexpr int MI = G::MI, RD = G::RD, TO = G::TO, TG = G::TG, PER = G::PER;
    __shared__ float lds[G::LDS_FLOATS];

    const int ch = blockIdx.y;
    const float2 *in = (const float2 *)a.in + ch * a.in_stride;
    const float2 *hist = (const float2 *)a.hist_in[ch];
    float2 *out = (float2 *)a.out + ch * a.out_stride;
    const long n_in = a.n_in;
    const int H = NT - 1;
    const int t = threadIdx.x;
    const int ln = t & 63, wv = t >> 6;
    const long nb = gridDim.x;
    const long b = xcd_tile(blockIdx.x, nb);
    const long t_begin = b, t_end = a.ntiles, t_step = nb;
    if (t_begin == 0 && t_end > 0) write_history(in, n_in, hist, (float2 *)a.hist_out[ch], H);

    // A operand of instruction m: tap of row (ln & 15) at K step 4m + (ln >> 4)
    const float *cg = (const float *)a.coef;
    float A[MI];
    {
        const int k0 = 4 * (ln & 15) + (ln >> 4) - 61;
#pragma unroll
        for (int m = 0; m < MI; ++m) {
            const int k = k0 + 4 * m;
            A[m] = (k >= 0 && k < NT) ? cg[k] : 0.0f;
        }
    }

    float4 v[PER];
    auto stage_load = [&](long tile) {  // tile >= 1: span start 4*tile*TO - HALO >= 0
        if constexpr (PROBE == 2) tile = 1 + (tile & 15);
        const long b0 = 4 * tile * TO - G::HALO;
        const long remb = (n_in - b0) * 8;
        const unsigned nrec = (unsigned)(remb > 0xfffffff0L ? 0xfffffff0L : (remb < 0 ? 0 : remb));
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(in + b0), 0, nrec, 0x00020000);
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int g = t + i * G::BLOCK;
            if (g < TG) {
                auto w = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * t, 16 * i * G::BLOCK, 2);
                v[i] = make_float4(__uint_as_float(w[0]), __uint_as_float(w[1]), __uint_as_float(w[2]),
                                   __uint_as_float(w[3]));
            }
        }
    };
    if (t_begin < t_end) {
        if (t_begin == 0) {  // tile 0: samples below 0 from the history
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int g = t + i * G::BLOCK;
                const long s = -G::HALO + 2 * (long)g;
                if (g < TG) {
                    float2 lo = fetch(in, hist, s, n_in, H), hi = fetch(in, hist, s + 1, n_in, H);
                    v[i] = make_float4(lo.x, lo.y, hi.x, hi.y);
                }
            }
        } else {
            stage_load(t_begin);
        }
    }
    // granule g = samples 2g (phase 2(g&1)) and 2g+1 (phase 2(g&1)+1), Q = g>>1.
    // Every granule of a lane has the same g & 1, and Q steps by 128 per i.
    const int godd = t & 1;
    const int wq = mfma_idx((t >> 1) + godd);  // phases 2, 3 sit one Q up
    const int w_lo = G::plane(0, 2 * godd) + wq, w_hi = G::plane(0, 2 * godd + 1) + wq;
    constexpr int CIM = G::plane(1, 0) - G::plane(0, 0);
    auto stage_to_lds = [&]() {
        SRCDSP_LDS_BARRIER();
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int g = t + i * G::BLOCK;
            if (g < TG) {
                constexpr int DI = 128 + 4 * 8;  // idx(q + 128) - idx(q)
                lds[w_lo + DI * i] = v[i].x;
                lds[w_lo + CIM + DI * i] = v[i].y;
                lds[w_hi + DI * i] = v[i].z;
                lds[w_hi + CIM + DI * i] = v[i].w;
            }
        }
        SRCDSP_LDS_BARRIER();
    };

    // lane -> B column j = ln & 15 (group gq, component cmp), sub-step kk = ln >> 4;
    // D rows 4*(ln>>4) .. +3 of column j
    const int j = ln & 15, kk = ln >> 4, gq = j >> 1, cmp = j & 1;
    const int og = wv * 2 * G::SEQ + 16 * gq;  // group's first output in the tile (h = 0)
    const int phi = (1 - kk) & 3;
    // read w covers instructions 4w .. 4w+3 at Q = og + Q47 - 4w - 3 .. og + Q47 - 4w
    const int r_base = G::plane(cmp, phi) + mfma_idx(og + G::Q47 - 4 * (RD - 1) - 3);
    // idx(Q_last + d) - idx(Q_last) for d = 4 (RD-1-w); Q_last = 16u + CL
    constexpr int CL = (G::Q47 - 3 - 4 * (RD - 1)) & 15;
    static_assert(G::Q47 - 3 - 4 * (RD - 1) >= 0, "first read inside the span");
    auto roff = [](int w) { return 4 * (RD - 1 - w) + 4 * ((CL + 4 * (RD - 1 - w)) >> 4); };
    constexpr int H1 = G::SEQ + 4 * (G::SEQ / 16);  // sequence h = 1: +128 Q

    auto do_tile = [&](long tile) {
        f4m_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
        if constexpr (PROBE == 1) {
            const float4 x0 = *(const float4 *)&lds[r_base + roff(0)];
            const float4 x1 = *(const float4 *)&lds[r_base + H1 + roff(0)];
            acc0 = (f4m_t){x0.x, x0.y, x0.z, x0.w};
            acc1 = (f4m_t){x1.x, x1.y, x1.z, x1.w};
        } else {
#pragma unroll
            for (int w = 0; w < RD; ++w) {
                const float4 x0 = *(const float4 *)&lds[r_base + roff(w)];
                const float4 x1 = *(const float4 *)&lds[r_base + H1 + roff(w)];
                const float b0[4] = {x0.w, x0.z, x0.y, x0.x}, b1[4] = {x1.w, x1.z, x1.y, x1.x};
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int m = 4 * w + u;
                    if (m < MI) {
                        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(A[m], b0[u], acc0, 0, 0, 0);
                        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(A[m], b1[u], acc1, 0, 0, 0);
                    }
                }
            }
        }
        const unsigned sh = a.shift;
        auto q = [&](float y) { return Q0 ? q16f_shift0(y) : q16f(y, sh); };
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            f4m_t d = h ? acc1 : acc0;
            const int orow = og + h * G::SEQ + 4 * kk;  // tile output of D row 0 of this lane
            const bool bad = !(__builtin_fabsf(d[0]) <= 3.4028235e38f) || !(__builtin_fabsf(d[1]) <= 3.4028235e38f) ||
                             !(__builtin_fabsf(d[2]) <= 3.4028235e38f) || !(__builtin_fabsf(d[3]) <= 3.4028235e38f);
            if (PROBE == 0 && __builtin_expect(bad, 0)) {
                // plain ascending-k chain for this lane's 4 outputs
#pragma unroll 1
                for (int r = 0; r < 4; ++r) {
                    const int p0 = 4 * (orow + r) + G::HALO;  // span position of x[4n]
                    float y = 0.f;
#pragma unroll 1
                    for (int k = 0; k < NT; ++k) {
                        const int p = p0 - k, ph = p & 3;
                        y = __builtin_fmaf(cg[k], lds[G::plane(cmp, ph) + mfma_idx((p >> 2) + (ph >> 1))], y);
                    }
                    d[r] = y;
                }
            }
            float e[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) e[r] = q(d[r]);
            // pair the re (even j) and im (odd j) lanes: the even lane stores
            // rows 0, 1 and the odd lane rows 2, 3, each as (re, im)
            const float s0 = cmp ? e[0] : e[2], s1 = cmp ? e[1] : e[3];
            const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, s0), 0xB1, 0xF, 0xF, true));
            const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, s1), 0xB1, 0xF, 0xF, true));
            const float4 o4 = cmp ? make_float4(r0, e[2], r1, e[3]) : make_float4(e[0], r0, e[1], r1);
            const long n = tile * TO + orow + (cmp ? 2 : 0);
            if (n + 2 <= a.n_out) {
                store16<true>((float4 *)(out + n), o4);
            } else if (n < a.n_out) {
                out[n] = make_float2(o4.x, o4.y);
            }
        }
    };
    if (t_begin < t_end) {
        stage_to_lds();
        long tile = t_begin;
        for (; tile + t_step < t_end; tile += t_step) {
            stage_load(tile + t_step);
            do_tile(tile);
            stage_to_lds();
        }
        do_tile(tile);
    }
}

}  // namespace srcdsp
