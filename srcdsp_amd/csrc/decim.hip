// decim.hip -- FilterDnsamplingFir (dnsampling_filters.h:49-172,
// dsptl_dnsampling_filters.h:47-220) and FilterFir (filters.h:42-169) on gfx950.
//
// Semantics restated per output n of a step over L input samples:
//   y[n] = sum_{k=0}^{N-1} c[k] * x[nM - k]          (taps in ascending k)
//   out[n] = limitScale16(y[n], coeffScaling - leftShift)
// where x[<0] is the N-1 sample history carried from the previous call.
//
// Kernels
//  * decim_tile_cf32<NT,R,BLOCK,FMA>  -- the headline path: complex<float>,
//    M = 4, NT taps.  One workgroup = one tile of BLOCK*R consecutive outputs;
//    the tile's input span (4*BLOCK*R samples + the 4*ceil(NT/4) halo) is
//    staged HBM -> VGPR -> LDS with 16-B coalesced loads into a padded layout
//    (one 16-B pad per lane chunk makes the lanes' ds_read_b128 conflict-free);
//    each lane then owns R consecutive outputs and walks the taps as 4
//    polyphase register windows that slide by one sample per 4 taps, so every
//    LDS read feeds 8R FMAs.  Coefficients are wave-uniform scalar loads
//    (SGPR operands of v_fma_f32).  Each output is ONE sequential fma chain in
//    ascending k (FMA=true), or separately rounded mul+add (FMA=false).
//  * decim_tile_ci16<NT,R,BLOCK,MIX>  -- complex<int16_t> x int32 taps (|c|<2^23,
//    v_mad_i32_i24), optionally with the NCO mixer of mixers.h fused into
//    the staging pass (config 4).
//  * decim_generic<KV,FMA>            -- any variant / M / N; one output per
//    thread, reads through the cache.  Used for shapes without a tile kernel.
// The new history (last N-1 samples of history ++ input) is written by the
// workgroup that owns tile 0 into the other ping-pong buffer, so a step is one
// launch.
#include <algorithm>

#include "ops.h"

namespace srcdsp {

// Taps of the tile kernels travel in the kernel-argument segment: wave-uniform
// constant memory, fetched with s_load into SGPRs and consumed as the scalar
// operand of each FMA (a pointer to global taps could alias the outputs, which
// forces vector loads into VGPRs).
constexpr int kMaxTileTaps = 128;
struct TapsF { float c[kMaxTileTaps]; };
struct TapsI { int32_t c[kMaxTileTaps]; };

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

// ============================================================ cf32 tiles
// Tile geometry for complex<float>, M = 4: a granule is 16 B = 2 samples,
// a 4-sample polyphase group is 2 granules.  LDS granule of tile granule g:
//   L(g) = g + (g - 2NQ + KPAD*PR) / PR, PR = 2R granules per lane chunk,
// i.e. one pad granule in front of every lane chunk, so lane t's chunk starts
// at B_t = 2NQ + KPAD + (2R+1) t and 16 lanes of a ds_read_b128 group hit 16
// distinct 16-B bank slots.
template <int NT, int R, int BLOCK, bool FMA>
__global__ __launch_bounds__(BLOCK) void decim_tile_cf32(DecimLaunch a, TapsF taps) {
    constexpr int NQ = (NT + 3) / 4;
    constexpr int TO = BLOCK * R;
    constexpr int TG = 2 * TO + 2 * NQ;
    constexpr int PR = 2 * R;
    constexpr int KPAD = ceildiv(2 * NQ, PR);
    constexpr int LG = TG + (TG + KPAD * PR) / PR + 1;
    constexpr int PER = ceildiv(TG, BLOCK);
    __shared__ float4 lds[LG];

    const int ch = blockIdx.y;
    const float2 *in = (const float2 *)a.in + ch * a.in_stride;
    const float2 *hist = (const float2 *)a.hist_in[ch];
    const long n_in = a.n_in;
    const int H = NT - 1;
    const long tile = xcd_tile(blockIdx.x, gridDim.x);
    const long o0 = tile * TO;
    const long b0 = 4 * o0 - 4 * NQ;
    const int t = threadIdx.x;

    if (tile == 0) write_history(in, n_in, hist, (float2 *)a.hist_out[ch], H);

    // ---- stage the tile: HBM -> VGPR -> LDS (all loads issued before any write)
    float4 v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int g = t + i * BLOCK;
        const long s = b0 + 2 * (long)g;
        if (g < TG) {
            if (s >= 0 && s + 1 < n_in) {
                v[i] = *(const float4 *)(in + s);
            } else {
                float2 lo = fetch(in, hist, s, n_in, H), hi = fetch(in, hist, s + 1, n_in, H);
                v[i] = make_float4(lo.x, lo.y, hi.x, hi.y);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int g = t + i * BLOCK;
        if (g < TG) lds[g + (g - 2 * NQ + KPAD * PR) / PR] = v[i];
    }
    __syncthreads();

    // ---- compute: lane t owns outputs n0 .. n0+R-1
    const int Bt = 2 * NQ + KPAD + (PR + 1) * t;
    float2 X[4 * (NQ + R)];  // X[s + 4NQ] = x[4 n0 + s]
    float yr[R], yi[R];
#pragma unroll
    for (int r = 0; r < R; ++r) yr[r] = yi[r] = 0.f;

    auto load_group = [&](int e) {  // samples 4e .. 4e+3 relative to 4 n0
        const float4 g0 = lds[Bt + 2 * e + floordiv(2 * e, PR)];
        const float4 g1 = lds[Bt + 2 * e + 1 + floordiv(2 * e + 1, PR)];
        X[4 * e + 4 * NQ + 0] = make_float2(g0.x, g0.y);
        X[4 * e + 4 * NQ + 1] = make_float2(g0.z, g0.w);
        X[4 * e + 4 * NQ + 2] = make_float2(g1.x, g1.y);
        X[4 * e + 4 * NQ + 3] = make_float2(g1.z, g1.w);
    };
#pragma unroll
    for (int e = -1; e < R; ++e) load_group(e);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        if (q + 1 < NQ) load_group(-q - 2);
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int k = 4 * q + p;
            if (k < NT) {
                const float c = taps.c[k];
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const float2 x = X[4 * (r - q) - p + 4 * NQ];
                    yr[r] = mac<FMA>(c, x.x, yr[r]);
                    yi[r] = mac<FMA>(c, x.y, yi[r]);
                }
            }
        }
    }

    // ---- quantise (limitScale16) and store
    float2 *out = (float2 *)a.out + ch * a.out_stride;
    const long n0 = o0 + (long)t * R;
    const unsigned sh = a.shift;
    if (n0 + R <= a.n_out && (R % 2) == 0) {
#pragma unroll
        for (int r = 0; r < R; r += 2)
            *(float4 *)(out + n0 + r) = make_float4(q16f(yr[r], sh), q16f(yi[r], sh), q16f(yr[r + 1], sh),
                                                    q16f(yi[r + 1], sh));
    } else {
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (n0 + r < a.n_out) out[n0 + r] = make_float2(q16f(yr[r], sh), q16f(yi[r], sh));
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

template <int NT, int R, int BLOCK, bool MIX>
__global__ __launch_bounds__(BLOCK) void decim_tile_ci16(DecimLaunch a, TapsI taps) {
    constexpr int NQ = (NT + 3) / 4;
    constexpr int TO = BLOCK * R;
    constexpr int TG = TO + NQ;                 // granules of 4 samples
    constexpr int PAD = Ci16Geo<R>::PAD;
    constexpr int PR = R;
    constexpr int KPAD = PAD ? ceildiv(NQ, PR) : 0;
    constexpr int LG = TG + (PAD ? (TG + KPAD * PR) / PR + 1 : 0);
    constexpr int PER = ceildiv(TG, BLOCK);
    constexpr int TABMAX = MIX ? 4096 : 1;
    __shared__ uint4 lds[LG];
    __shared__ int16_t tab[TABMAX];

    const int ch = blockIdx.y;
    const uint32_t *in = (const uint32_t *)a.in + ch * a.in_stride;
    const uint32_t *hist = (const uint32_t *)a.hist_in[ch];
    const long n_in = a.n_in;
    const int H = NT - 1;
    const long tile = xcd_tile(blockIdx.x, gridDim.x);
    const long o0 = tile * TO;
    const long b0 = 4 * o0 - 4 * NQ;
    const int t = threadIdx.x;
    const unsigned N = a.mix_N;

    if constexpr (MIX) {
        for (int i = t; i < (int)N; i += BLOCK) tab[i] = a.mix_table[i];
        __syncthreads();
    }
    // phase of sample idx: (phi0 + idx*freq) mod N (any sign of idx; negative
    // indices are history and never mixed, but keep the recurrence consistent)
    auto phase_of = [&](long idx) -> unsigned {
        long m = idx % (long)N;
        m = m < 0 ? m + N : m;
        return (unsigned)(((unsigned long)a.mix_phase0 + (unsigned long)m * a.mix_freq) % N);
    };
    auto adv = [&](unsigned ph, unsigned d) -> unsigned {  // (ph + d) mod N, ph,d < N
        ph += d;
        return ph >= N ? ph - N : ph;
    };
    const unsigned fstep = MIX ? (unsigned)(((unsigned long)(4 * BLOCK) % N) * a.mix_freq % N) : 0;
    unsigned ph_t = MIX ? phase_of(b0 + 4 * (long)t) : 0;  // phase of this thread's first staged sample

    if (tile == 0) {  // new history = last H samples of (history ++ mixed input)
        uint32_t *ho = (uint32_t *)a.hist_out[ch];
        for (int k = t; k < H; k += BLOCK) {
            long idx = n_in - H + k;
            uint32_t w = idx >= 0 ? in[idx] : hist[H + idx];
            if constexpr (MIX)
                if (idx >= 0) w = mix_sample(w, tab, N, phase_of(idx));
            ho[k] = w;
        }
    }

    uint4 v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int g = t + i * BLOCK;
        const long s = b0 + 4 * (long)g;
        if (g < TG) {
            if (s >= 0 && s + 3 < n_in) {
                v[i] = *(const uint4 *)(in + s);
                if constexpr (MIX) {
                    unsigned ph = ph_t;
                    v[i].x = mix_sample(v[i].x, tab, N, ph); ph = adv(ph, a.mix_freq);
                    v[i].y = mix_sample(v[i].y, tab, N, ph); ph = adv(ph, a.mix_freq);
                    v[i].z = mix_sample(v[i].z, tab, N, ph); ph = adv(ph, a.mix_freq);
                    v[i].w = mix_sample(v[i].w, tab, N, ph);
                }
            } else {
                uint32_t w[4];
                unsigned ph = ph_t;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    long idx = s + j;
                    w[j] = fetch(in, hist, idx, n_in, H);
                    if constexpr (MIX)
                        if (idx >= 0 && idx < n_in) w[j] = mix_sample(w[j], tab, N, ph);
                    if constexpr (MIX) ph = adv(ph, a.mix_freq);
                }
                v[i] = make_uint4(w[0], w[1], w[2], w[3]);
            }
        }
        if constexpr (MIX) ph_t = adv(ph_t, fstep);
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int g = t + i * BLOCK;
        if (g < TG) {
            int lg = PAD ? g + (g - NQ + KPAD * PR) / PR : g;
            lds[lg] = v[i];
        }
    }
    __syncthreads();

    const int Bt = PAD ? NQ + KPAD + (PR + 1) * t : NQ + PR * t;
    int32_t Xr[4 * (NQ + R)], Xi[4 * (NQ + R)];
    int32_t yr[R], yi[R];
#pragma unroll
    for (int r = 0; r < R; ++r) yr[r] = yi[r] = 0;
    auto load_group = [&](int e) {
        const uint4 g = lds[Bt + e + (PAD ? floordiv(e, PR) : 0)];
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
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int k = 4 * q + p;
            if (k < NT) {
                const int32_t c = taps.c[k];
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int o = 4 * (r - q) - p + 4 * NQ;
                    yr[r] += __mul24(c, Xr[o]);  // |c| < 2^23, |x| < 2^15: v_mad_i32_i24
                    yi[r] += __mul24(c, Xi[o]);
                }
            }
        }
    }
    uint32_t *out = (uint32_t *)a.out + ch * a.out_stride;
    const long n0 = o0 + (long)t * R;
    const unsigned sh = a.shift;
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (n0 + r < a.n_out) out[n0 + r] = pack16(limit16(yr[r], sh), limit16(yi[r], sh));
}

// ============================================================== dispatch
namespace {
constexpr int kCfR = 8, kCfBlock = 256;
constexpr int kCiR = 7, kCiBlock = 256;

template <int NT>
int launch_cf32(const DecimLaunch &L, const TapsF &T, int channels, bool fma, hipStream_t s) {
    constexpr int TO = kCfBlock * kCfR;
    long tiles = (L.n_out + TO - 1) / TO;
    dim3 grid((unsigned)tiles, channels);
    if (fma)
        hipLaunchKernelGGL((decim_tile_cf32<NT, kCfR, kCfBlock, true>), grid, dim3(kCfBlock), 0, s, L, T);
    else
        hipLaunchKernelGGL((decim_tile_cf32<NT, kCfR, kCfBlock, false>), grid, dim3(kCfBlock), 0, s, L, T);
    return SRCDSP_OK;
}

template <int NT>
int launch_ci16(const DecimLaunch &L, const TapsI &T, int channels, bool mixed, hipStream_t s) {
    constexpr int TO = kCiBlock * kCiR;
    long tiles = (L.n_out + TO - 1) / TO;
    dim3 grid((unsigned)tiles, channels);
    if (mixed)
        hipLaunchKernelGGL((decim_tile_ci16<NT, kCiR, kCiBlock, true>), grid, dim3(kCiBlock), 0, s, L, T);
    else
        hipLaunchKernelGGL((decim_tile_ci16<NT, kCiR, kCiBlock, false>), grid, dim3(kCiBlock), 0, s, L, T);
    return SRCDSP_OK;
}

template <int KV>
int launch_generic(const DecimLaunch &L, int channels, unsigned M, bool fma, hipStream_t s) {
    long blocks = std::max<long>(1, std::min<long>((L.n_out + 255) / 256, 4096));
    dim3 grid((unsigned)blocks, channels);
    if (fma)
        hipLaunchKernelGGL((decim_generic<KV, true>), grid, dim3(256), 0, s, L, M);
    else
        hipLaunchKernelGGL((decim_generic<KV, false>), grid, dim3(256), 0, s, L, M);
    return SRCDSP_OK;
}

bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }
}  // namespace

// Choose the kernel for one FirCore configuration and launch it.
int decim_launch(FirCore &f, const DecimLaunch &L, int channels, hipStream_t s, bool mixed) {
    const bool fma = !(f.flags & SRCDSP_FLAG_FP_STRICT);
    bool al = aligned16(L.in) && ((L.in_stride * kv_in_bytes(f.kv)) % 16 == 0);
    int rc = SRCDSP_OK;
    if (f.M == 4 && f.kv == KV_CF32 && al && (f.ntaps == 127 || f.ntaps == 128)) {
        TapsF T{};
        memcpy(T.c, f.h_coef.data(), 4 * (size_t)f.ntaps);
        rc = f.ntaps == 127 ? launch_cf32<127>(L, T, channels, fma, s) : launch_cf32<128>(L, T, channels, fma, s);
    } else if (f.M == 4 && f.kv == KV_CI16_I32 && f.coef_fits_i24 && al && (f.ntaps == 127 || f.ntaps == 128)) {
        TapsI T{};
        memcpy(T.c, f.h_coef.data(), 4 * (size_t)f.ntaps);
        rc = f.ntaps == 127 ? launch_ci16<127>(L, T, channels, mixed, s) : launch_ci16<128>(L, T, channels, mixed, s);
    } else {
        if (mixed) {
            set_error("mixer->decimator fusion needs variant 1, M=4, 127/128 taps |c|<2^23, 16-B aligned input");
            return SRCDSP_ERR_UNSUPPORTED;
        }
        switch (f.kv) {
        case KV_CF32: rc = launch_generic<KV_CF32>(L, channels, f.M, fma, s); break;
        case KV_CI16_I32: rc = launch_generic<KV_CI16_I32>(L, channels, f.M, fma, s); break;
        case KV_CI16_I16: rc = launch_generic<KV_CI16_I16>(L, channels, f.M, fma, s); break;
        case KV_CI32_I32: rc = launch_generic<KV_CI32_I32>(L, channels, f.M, fma, s); break;
        case KV_F32_REAL: rc = launch_generic<KV_F32_REAL>(L, channels, f.M, fma, s); break;
        default: set_error("bad kernel variant"); return SRCDSP_ERR_ARG;
        }
    }
    if (rc != SRCDSP_OK) return rc;
    SRCDSP_HIP_TRY(hipGetLastError());
    return SRCDSP_OK;
}

// ================================================================ FirCore
static bool coef_i24(const int32_t *c, int n) {
    for (int i = 0; i < n; ++i)
        if (c[i] >= (1 << 23) || c[i] < -(1 << 23)) return false;
    return true;
}

int FirCore::set_coeffs(const void *coeffs, int n, bool keep_history) {
    SRCDSP_ARG_CHECK(coeffs != nullptr && n >= 1, "coefficients: need at least one tap");
    int rc = order.sync();
    if (rc) return rc;
    h_coef.assign((const char *)coeffs, (size_t)n * kv_coef_bytes(kv));
    // host copy of taps widened to 4 bytes (int16 -> int32)
    std::string tmp(4 * (size_t)n, '\0');
    if (kv == KV_CI16_I16) {
        int32_t *w = (int32_t *)&tmp[0];
        for (int i = 0; i < n; ++i) w[i] = ((const int16_t *)coeffs)[i];
        coeff_scaling = coeff_scaling_i16((const int16_t *)coeffs, n);
    } else {
        memcpy(&tmp[0], coeffs, 4 * (size_t)n);
        if (kv == KV_CF32 || kv == KV_F32_REAL)
            coeff_scaling = coeff_scaling_f32((const float *)coeffs, n, (flags & SRCDSP_FLAG_ABS_FABS) != 0);
        else
            coeff_scaling = coeff_scaling_i32((const int32_t *)coeffs, n);
    }
    coef_fits_i24 = (kv == KV_CI16_I32) && coef_i24((const int32_t *)tmp.data(), n);
    if (d_coef) (void)hipFree(d_coef);
    d_coef = nullptr;
    SRCDSP_HIP_TRY(hipMalloc(&d_coef, 4 * (size_t)n));
    SRCDSP_HIP_TRY(hipMemcpy(d_coef, tmp.data(), 4 * (size_t)n, hipMemcpyHostToDevice));

    // history: resize keeping the first min(old,new) entries (vector::resize)
    const size_t es = kv_in_bytes(kv);
    const size_t new_bytes = std::max<size_t>(1, (size_t)(n - 1)) * es;
    const size_t keep = keep_history ? (size_t)std::max(0, std::min(ntaps - 1, n - 1)) * es : 0;
    void *nh[2] = {nullptr, nullptr};
    for (int b = 0; b < 2; ++b) {
        SRCDSP_HIP_TRY(hipMalloc(&nh[b], new_bytes));
        SRCDSP_HIP_TRY(hipMemset(nh[b], 0, new_bytes));
    }
    if (keep && d_hist[cur]) SRCDSP_HIP_TRY(hipMemcpy(nh[0], d_hist[cur], keep, hipMemcpyDeviceToDevice));
    for (int b = 0; b < 2; ++b)
        if (d_hist[b]) (void)hipFree(d_hist[b]);
    d_hist[0] = nh[0];
    d_hist[1] = nh[1];
    cur = 0;
    hist_cap = new_bytes;
    ntaps = n;
    return SRCDSP_OK;
}

int FirCore::init(int kv_, unsigned M_, const void *coeffs, int n, unsigned flags_) {
    kv = kv_;
    M = M_;
    flags = flags_;
    ntaps = 0;
    int rc = order.init();
    if (rc) return rc;
    rc = stage.init();
    if (rc) return rc;
    rc = set_coeffs(coeffs, n, false);
    left_shift = 0;
    return rc;
}

int FirCore::clear_history() {
    int rc = order.sync();
    if (rc) return rc;
    for (int b = 0; b < 2; ++b) SRCDSP_HIP_TRY(hipMemset(d_hist[b], 0, hist_cap));
    SRCDSP_HIP_TRY(hipDeviceSynchronize());
    return SRCDSP_OK;
}

void FirCore::destroy() {
    (void)order.sync();
    if (d_coef) (void)hipFree(d_coef);
    for (int b = 0; b < 2; ++b)
        if (d_hist[b]) (void)hipFree(d_hist[b]);
    d_coef = nullptr;
    d_hist[0] = d_hist[1] = nullptr;
    order.destroy();
    stage.destroy();
}

// one single-channel step on device buffers
static int core_step(FirCore &f, const void *d_in, size_t n_in, void *d_out, size_t n_out, hipStream_t s,
                     const MixerState *mix) {
    SRCDSP_ARG_CHECK(n_out * f.M == n_in, "step: output size * M must equal input size");
    if (n_in == 0) return SRCDSP_OK;
    SRCDSP_ARG_CHECK(d_in && d_out, "step: null buffer");
    int rc = f.order.before(s);
    if (rc) return rc;
    DecimLaunch L{};
    L.in = d_in;
    L.out = d_out;
    L.coef = f.d_coef;
    L.n_in = (long)n_in;
    L.n_out = (long)n_out;
    L.ntaps = f.ntaps;
    L.shift = f.shift();
    L.hist_in[0] = f.d_hist[f.cur];
    L.hist_out[0] = f.d_hist[f.cur ^ 1];
    if (mix) {
        L.mix_table = mix->d_table;
        L.mix_N = mix->N;
        L.mix_phase0 = (unsigned)mix->phi;
        L.mix_freq = (unsigned)mix->freq;
    }
    rc = decim_launch(f, L, 1, s, mix != nullptr);
    if (rc) return rc;
    f.cur ^= 1;
    return f.order.after(s);
}

static int core_step_host(FirCore &f, const void *in, size_t n_in, void *out, size_t n_out) {
    SRCDSP_ARG_CHECK(n_out * f.M == n_in, "step: output size * M must equal input size");
    if (n_in == 0) return SRCDSP_OK;
    const size_t ib = n_in * kv_in_bytes(f.kv), ob = n_out * kv_out_bytes(f.kv);
    const size_t ib_al = (ib + 255) & ~(size_t)255;
    int rc = f.stage.reserve(std::max(ib, ob), ib_al + ob);
    if (rc) return rc;
    hipStream_t s = f.stage.stream;
    char *d_in = (char *)f.stage.d_buf, *d_out = d_in + ib_al;
    memcpy(f.stage.h_buf, in, ib);
    SRCDSP_HIP_TRY(hipMemcpyAsync(d_in, f.stage.h_buf, ib, hipMemcpyHostToDevice, s));
    rc = core_step(f, d_in, n_in, d_out, n_out, s, nullptr);
    if (rc) return rc;
    SRCDSP_HIP_TRY(hipMemcpyAsync(f.stage.h_buf, d_out, ob, hipMemcpyDeviceToHost, s));
    SRCDSP_HIP_TRY(hipStreamSynchronize(s));
    memcpy(out, f.stage.h_buf, ob);
    return SRCDSP_OK;
}

}  // namespace srcdsp

using namespace srcdsp;

extern "C" {

// ------------------------------------------------------ FilterDnsamplingFir
SRCDSP_API int srcdsp_decim_create(srcdsp_decim_t *out, int variant, unsigned M, const void *coeffs,
                                   int ntaps, unsigned flags) {
    SRCDSP_ARG_CHECK(out != nullptr, "decim_create: null out");
    *out = nullptr;
    if (variant < 0 || variant > 3) {
        set_error("decim_create: variant must be 0..3");
        return SRCDSP_ERR_UNSUPPORTED;
    }
    SRCDSP_ARG_CHECK(M >= 1, "decim_create: M must be >= 1");
    auto *h = new srcdsp_decim();
    int rc = h->core.init(variant, M, coeffs, ntaps, flags);
    if (rc) {
        h->core.destroy();
        delete h;
        return rc;
    }
    *out = h;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_decim_destroy(srcdsp_decim_t h) {
    if (!h) return SRCDSP_OK;
    h->core.destroy();
    delete h;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_decim_set_coeffs(srcdsp_decim_t h, const void *coeffs, int ntaps, int require_multiple) {
    SRCDSP_ARG_CHECK(h != nullptr, "decim_set_coeffs: null handle");
    if (require_multiple && (ntaps % (int)h->core.M) != 0) {
        set_error("setCoeffs: number of taps must be a multiple of M (dsptl_dnsampling_filters.h:122)");
        return SRCDSP_ERR_SIZE;
    }
    int rc = h->core.set_coeffs(coeffs, ntaps, true);
    h->core.left_shift = 0;  // dsptl_dnsampling_filters.h:133
    return rc;
}

SRCDSP_API int srcdsp_decim_set_left_shift(srcdsp_decim_t h, int ls) {
    SRCDSP_ARG_CHECK(h != nullptr, "decim_set_left_shift: null handle");
    h->core.left_shift = ls;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_decim_reset(srcdsp_decim_t h) {
    SRCDSP_ARG_CHECK(h != nullptr, "decim_reset: null handle");
    return h->core.clear_history();
}

SRCDSP_API int srcdsp_decim_step(srcdsp_decim_t h, const void *d_in, size_t n_in, void *d_out, size_t n_out,
                                 void *stream) {
    SRCDSP_ARG_CHECK(h != nullptr, "decim_step: null handle");
    if (n_out * h->core.M != n_in) {
        set_error("decim_step: out.size()*M != in.size() (dnsampling_filters.h:133)");
        return SRCDSP_ERR_SIZE;
    }
    return core_step(h->core, d_in, n_in, d_out, n_out, (hipStream_t)stream, nullptr);
}

SRCDSP_API int srcdsp_decim_step_host(srcdsp_decim_t h, const void *in, size_t n_in, void *out, size_t n_out) {
    SRCDSP_ARG_CHECK(h != nullptr, "decim_step_host: null handle");
    if (n_out * h->core.M != n_in) {
        set_error("decim_step_host: out.size()*M != in.size() (dnsampling_filters.h:133)");
        return SRCDSP_ERR_SIZE;
    }
    return core_step_host(h->core, in, n_in, out, n_out);
}

SRCDSP_API int srcdsp_decim_step_batched(const srcdsp_decim_t *hs, int channels, const void *d_in,
                                         size_t in_stride, void *d_out, size_t out_stride, size_t n_in,
                                         void *stream) {
    SRCDSP_ARG_CHECK(hs != nullptr && channels >= 1, "decim_step_batched: no handles");
    FirCore &f0 = hs[0]->core;
    SRCDSP_ARG_CHECK(n_in % f0.M == 0, "decim_step_batched: n_in must be a multiple of M");
    for (int c = 1; c < channels; ++c) {
        const FirCore &fc = hs[c]->core;
        SRCDSP_ARG_CHECK(fc.kv == f0.kv && fc.M == f0.M && fc.ntaps == f0.ntaps && fc.flags == f0.flags &&
                             fc.shift() == f0.shift() && fc.h_coef == f0.h_coef,
                         "decim_step_batched: handles must share variant, M, taps, flags and shift");
    }
    if (n_in == 0) return SRCDSP_OK;
    hipStream_t s = (hipStream_t)stream;
    const size_t ib = kv_in_bytes(f0.kv), ob = kv_out_bytes(f0.kv);
    for (int c0 = 0; c0 < channels; c0 += kMaxBatch) {
        int nc = std::min(kMaxBatch, channels - c0);
        DecimLaunch L{};
        L.in = (const char *)d_in + (size_t)c0 * in_stride * ib;
        L.out = (char *)d_out + (size_t)c0 * out_stride * ob;
        L.coef = f0.d_coef;  // all channels share the taps (checked above)
        L.n_in = (long)n_in;
        L.n_out = (long)(n_in / f0.M);
        L.in_stride = (long)in_stride;
        L.out_stride = (long)out_stride;
        L.ntaps = f0.ntaps;
        L.shift = f0.shift();
        for (int c = 0; c < nc; ++c) {
            FirCore &fc = hs[c0 + c]->core;
            int rc = fc.order.before(s);
            if (rc) return rc;
            L.hist_in[c] = fc.d_hist[fc.cur];
            L.hist_out[c] = fc.d_hist[fc.cur ^ 1];
        }
        int rc = decim_launch(f0, L, nc, s, false);
        if (rc) return rc;
        for (int c = 0; c < nc; ++c) {
            FirCore &fc = hs[c0 + c]->core;
            fc.cur ^= 1;
            rc = fc.order.after(s);
            if (rc) return rc;
        }
    }
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_decim_get_state(srcdsp_decim_t h, unsigned *cs, int *ls, void *hist_host) {
    SRCDSP_ARG_CHECK(h != nullptr, "decim_get_state: null handle");
    FirCore &f = h->core;
    if (cs) *cs = f.coeff_scaling;
    if (ls) *ls = f.left_shift;
    if (hist_host && f.ntaps > 1) {
        int rc = f.order.sync();
        if (rc) return rc;
        SRCDSP_HIP_TRY(hipMemcpy(hist_host, f.d_hist[f.cur], (size_t)(f.ntaps - 1) * kv_in_bytes(f.kv),
                                 hipMemcpyDeviceToHost));
    }
    return SRCDSP_OK;
}

// ---------------------------------------------------------------- FilterFir
static const int kFirKV[3] = {KV_CF32, KV_F32_REAL, KV_CI16_I32};

SRCDSP_API int srcdsp_fir_create(srcdsp_fir_t *out, int variant, const void *coeffs, int ntaps, unsigned flags) {
    SRCDSP_ARG_CHECK(out != nullptr, "fir_create: null out");
    *out = nullptr;
    if (variant < 0 || variant > 2) {
        set_error("fir_create: variant must be 0..2");
        return SRCDSP_ERR_UNSUPPORTED;
    }
    auto *h = new srcdsp_fir();
    int rc = h->core.init(kFirKV[variant], 1, coeffs, ntaps, flags);
    if (rc) {
        h->core.destroy();
        delete h;
        return rc;
    }
    *out = h;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_fir_destroy(srcdsp_fir_t h) {
    if (!h) return SRCDSP_OK;
    h->core.destroy();
    delete h;
    return SRCDSP_OK;
}

// setCoeffs (filters.h:86-97) ends in reset(): the buffer is cleared.
SRCDSP_API int srcdsp_fir_set_coeffs(srcdsp_fir_t h, const void *coeffs, int ntaps) {
    SRCDSP_ARG_CHECK(h != nullptr, "fir_set_coeffs: null handle");
    return h->core.set_coeffs(coeffs, ntaps, false);
}

SRCDSP_API int srcdsp_fir_reset(srcdsp_fir_t h) {
    SRCDSP_ARG_CHECK(h != nullptr, "fir_reset: null handle");
    return h->core.clear_history();
}

SRCDSP_API int srcdsp_fir_step(srcdsp_fir_t h, const void *d_in, size_t n_in, void *d_out, size_t n_out,
                               void *stream) {
    SRCDSP_ARG_CHECK(h != nullptr, "fir_step: null handle");
    if (n_in != n_out) {
        set_error("fir_step: signal.size() != filteredSignal.size() (filters.h:136)");
        return SRCDSP_ERR_SIZE;
    }
    return core_step(h->core, d_in, n_in, d_out, n_out, (hipStream_t)stream, nullptr);
}

SRCDSP_API int srcdsp_fir_step_host(srcdsp_fir_t h, const void *in, size_t n_in, void *out, size_t n_out) {
    SRCDSP_ARG_CHECK(h != nullptr, "fir_step_host: null handle");
    if (n_in != n_out) {
        set_error("fir_step_host: signal.size() != filteredSignal.size() (filters.h:136)");
        return SRCDSP_ERR_SIZE;
    }
    return core_step_host(h->core, in, n_in, out, n_out);
}

// -------------------------------------------------- Mixer -> decimator chain
SRCDSP_API int srcdsp_mixdecim_step(srcdsp_mixer_t mixer, srcdsp_decim_t decim, const void *d_in, size_t n_in,
                                    void *d_out, size_t n_out, void *stream) {
    SRCDSP_ARG_CHECK(mixer != nullptr && decim != nullptr, "mixdecim_step: null handle");
    FirCore &f = decim->core;
    MixerState &m = mixer->m;
    if (f.kv != KV_CI16_I32) {
        set_error("mixdecim_step: the decimator must be variant 1 (ci16 x int32 taps)");
        return SRCDSP_ERR_UNSUPPORTED;
    }
    if (m.N > 4096) {
        set_error("mixdecim_step: fused mixer table limited to N <= 4096");
        return SRCDSP_ERR_UNSUPPORTED;
    }
    if (n_out * f.M != n_in) {
        set_error("mixdecim_step: out.size()*M != in.size() (dnsampling_filters.h:133)");
        return SRCDSP_ERR_SIZE;
    }
    hipStream_t s = (hipStream_t)stream;
    int rc = m.order.before(s);
    if (rc) return rc;
    rc = core_step(f, d_in, n_in, d_out, n_out, s, &m);
    if (rc) return rc;
    // mixer phase after the call: phi += n_in * freq (mod N), mixers.h:177
    m.phi = (int16_t)(((unsigned long)(unsigned)m.phi + (unsigned long)(n_in % m.N) * (unsigned)m.freq) % m.N);
    return m.order.after(s);
}

}  // extern "C"
