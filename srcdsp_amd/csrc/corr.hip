// corr.hip -- dsptl::FixedPatternCorrelator<int16_t, int32_t, N, S>
// (correlators.h:54-316) on gfx950.
//
// The reference walks the input one sample at a time and stops at the first
// detection.  Everything it computes per sample depends only on the window of
// N*S samples ending there, so the step is split into
//   1. corr_eval   : every sample's scaled correlation |C_i>>2|^2 and scaled
//                    window energy, in parallel (int32 wrap-around arithmetic
//                    as the reference's complex<int32_t>/uint32 registers);
//   2. corr_detect : the 3-point peak + threshold test of correlators.h:262-268
//                    on each index, reduced to the FIRST index with atomicMin;
//   3. host        : state update -- the registers, the N*S-1 sample history
//                    (the detected sample is dropped: the reference `break`s
//                    without advancing `top`, correlators.h:291), bitSamples.
// The double-precision threshold sqrt(c) > sqrt(e)*2.7 is evaluated exactly:
// sqrt(e) > 300 <=> e > 90000 for integer e, and the correctly rounded sqrt of
// a uint32 is obtained from the hardware estimate by an exact 128-bit
// neighbour check, so no tolerance is involved.
#include <algorithm>
#include <vector>

#include "ops.h"
#include "decim_kernels.h"
#include "corr_hit.h"

namespace srcdsp {

typedef short short2_t __attribute__((ext_vector_type(2)));

struct srcdsp_corr_state {
    unsigned N = 0, S = 1, NS = 0;
    unsigned NP = 0;             // N rounded up to 16 (the dot2 tap array is front-padded with zero taps)
    int32_t *d_coef = nullptr;   // conj(pattern), N complex<int32_t> (2N int32)
    std::vector<int32_t> h_coef;
    uint32_t *d_ptaps = nullptr; // packed int16 pairs for v_dot2: (p.re,p.im),(-p.im,p.re) per tap, NP taps
    bool taps16 = false;         // every pattern component fits int16 (always true when the
                                 // reference's energy assert holds)
    uint32_t *d_hist[2] = {nullptr, nullptr};  // last NS-1 effective samples (packed ci16)
    int cur = 0;
    uint32_t *d_corr = nullptr, *d_en = nullptr;  // per-sample scratch
    size_t scratch_cap = 0;
    unsigned *d_best = nullptr;
    // CorrState (correlators.h:59-81)
    uint32_t energy[3] = {0, 0, 0}, corr[3] = {0, 0, 0};
    uint32_t coeffs_energy = 0;
    int coeff_scaling = 0;
    double threshold_factor = 0;
    std::vector<int16_t> bits;  // bitSamples, N complex<int16_t>
    Ordering order;
    HostStage stage;
};

// the detection test (correlators.h:262-268): corr_hit / corr_hit_exact in corr_hit.h

// ------------------------------------------------------------------ kernels
__device__ __forceinline__ uint32_t corr_fetch(const uint32_t *in, const uint32_t *hist, long j, long NSm1) {
    return j >= 0 ? in[j] : (j + NSm1 >= 0 ? hist[j + NSm1] : 0u);
}

constexpr int kCorrBlock = 256;
constexpr size_t kCorrEvalMaxSmem = 64 * 1024;  // corr_eval's staged window + taps; longer: corr_eval_g
constexpr unsigned kCorrMaxGridY = 65535;       // corr_eval_dot2 runs one stride phase per grid row

// one output per lane; the block's window span and the taps are staged in LDS
__global__ __launch_bounds__(kCorrBlock) void corr_eval(const uint32_t *__restrict__ in, long n, long i_begin,
                                                        long i_end, const uint32_t *__restrict__ hist,
                                                        const int32_t *__restrict__ coef, unsigned N, unsigned S,
                                                        unsigned cs, uint32_t *__restrict__ corr_out,
                                                        uint32_t *__restrict__ en_out, const unsigned *stop) {
    if ((long)*stop < i_begin) return;  // an earlier segment already detected
    extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
    const long NSm1 = (long)N * S - 1;
    const long span = kCorrBlock + NSm1;  // samples i0-NSm1 .. i0+255
    uint32_t *xs = sm;
    int2 *cs2 = (int2 *)(sm + ((span + 3) & ~3l));
    const long i0 = i_begin + (long)blockIdx.x * kCorrBlock;
    for (long k = threadIdx.x; k < span; k += kCorrBlock) {
        long j = i0 - NSm1 + k;
        xs[k] = j < n ? corr_fetch(in, hist, j, NSm1) : 0u;
    }
    for (unsigned m = threadIdx.x; m < N; m += kCorrBlock) cs2[m] = make_int2(coef[2 * m], coef[2 * m + 1]);
    __syncthreads();
    const long i = i0 + threadIdx.x;
    if (i >= i_end) return;
    uint32_t tr = 0, ti = 0, e = 0;
    // window sample of tap m: x[i - (N-1-m) S]  ->  xs[threadIdx.x + (S-1) + m S]
    const uint32_t *xw = xs + threadIdx.x + (S - 1);
    for (unsigned m = 0; m < N; ++m) {
        const uint32_t w = xw[m * S];
        const int32_t hr = sext16(w), hi = sext16_hi(w);
        const int2 c = cs2[m];
        tr += (uint32_t)hr * (uint32_t)c.x - (uint32_t)hi * (uint32_t)c.y;
        ti += (uint32_t)hr * (uint32_t)c.y + (uint32_t)hi * (uint32_t)c.x;
        e += (uint32_t)hr * (uint32_t)hr + (uint32_t)hi * (uint32_t)hi;
    }
    const int32_t sr = (int32_t)tr >> (cs & 31u), si = (int32_t)ti >> (cs & 31u);  // scale32 :244
    const int32_t ar = sr >> 2, ai = si >> 2;                                       // :250
    corr_out[i] = (uint32_t)ar * (uint32_t)ar + (uint32_t)ai * (uint32_t)ai;
    en_out[i] = e >> ((unsigned)((int)cs / 2) & 31u);                                // :245
}

// -------------------------------------------------- register-tiled eval
// For stride 1 the correlation is a complex FIR over the last N samples:
//   C_i = sum_m x[i-(N-1)+m] * conj(p[m]).
// With packed complex<int16_t> words both real products of a tap are one
// v_dot2_i32_i16 (int16 x int16 -> int32, wrap-around accumulate, as the
// reference's complex<int32_t> arithmetic):
//   Re = dot2(x, (p.re, p.im)),  Im = dot2(x, (-p.im, p.re)).
// Each lane owns CR consecutive outputs and slides a register window over the
// taps (16 taps per chunk: CR+15 window words, 4 new ds_read_b128 per chunk for
// 2*16*CR dot2).  Window energy: direct sum for the lane's first output
// (one dot2(x,x) per tap), then E_{i+1} = E_i + |x_{i+1}|^2 - |x_{i+1-N}|^2.
// Taps (2N packed words) are scalar loads through a constant view.  The LDS
// image gets one 16-B pad per lane chunk (CR words), so the 16 lanes of a
// ds_read_b128 group touch 16 distinct bank slots.
// Any stride S and tap count N: outputs i = k S + ph of one phase ph (grid.y)
// correlate the phase stream x_ph[k] = x[k S + ph] with the pattern, a stride-1
// correlation of that stream, so each workgroup stages one phase's samples
// (a strided gather, through L2) and runs the stride-1 tiles on them.  The
// taps are front-padded with zero taps to NP = 16 ceil(N/16) (exact: a zero
// tap adds 0); the window energy covers the N real taps only (the padded
// positions' |x|^2 are taken off the direct sum, and the sliding update drops
// the oldest real sample).
constexpr int kCR = 16;       // outputs per lane
constexpr int kCBlock = 256;  // lanes per workgroup
// corr_scan_s1 at 5 waves per SIMD (<= 96 VGPRs, no spills): -1.4 % against 4
// (profiles/tuning/r04_corr_ab.txt)
#ifndef SRCDSP_CORR_MINW
#define SRCDSP_CORR_MINW 5
#endif
// Dynamic LDS of the dot2 tiles: the staged window, corr_lds_words(NP) words
// (chunks of 16 samples + 4 pad words); corr_scan_s1 appends its chunk sums,
// kCBlock + NP/16 words.  At the largest NP, 8192: 61.6 KB + 3.0 KB (gfx950
// gives a workgroup up to 160 KB).
constexpr unsigned kCorrDot2MaxTaps = 8192;
__host__ __device__ constexpr int corr_lds_words(int NP) { return ((kCBlock * kCR + NP + 1) / kCR + 2) * (kCR + 4); }
__host__ __device__ constexpr int corr_scan_lds_words(int NP) { return corr_lds_words(NP) + kCBlock + NP / 16; }

// corr_eval's arithmetic for windows too long to stage (N*S + 255 samples
// past kCorrEvalMaxSmem of LDS, e.g. S in the thousands): one output per lane,
// window samples and taps read through the cache (adjacent lanes read
// adjacent samples, so every tap is one coalesced load per wave)
__global__ __launch_bounds__(kCorrBlock) void corr_eval_g(const uint32_t *__restrict__ in, long n, long i_begin,
                                                          long i_end, const uint32_t *__restrict__ hist,
                                                          const int32_t *__restrict__ coef, unsigned N, unsigned S,
                                                          unsigned cs, uint32_t *__restrict__ corr_out,
                                                          uint32_t *__restrict__ en_out, const unsigned *stop) {
    if ((long)*stop < i_begin) return;
    const long i = i_begin + (long)blockIdx.x * kCorrBlock + threadIdx.x;
    if (i >= i_end) return;
    const long NSm1 = (long)N * S - 1;
    uint32_t tr = 0, ti = 0, e = 0;
    // tap m multiplies x[i - (N-1-m) S]
    long j = i - (long)(N - 1) * S;
    for (unsigned m = 0; m < N; ++m, j += S) {
        const uint32_t w = j < n ? corr_fetch(in, hist, j, NSm1) : 0u;
        const int32_t hr = sext16(w), hi = sext16_hi(w);
        const int32_t cr = coef[2 * m], ci = coef[2 * m + 1];
        tr += (uint32_t)hr * (uint32_t)cr - (uint32_t)hi * (uint32_t)ci;
        ti += (uint32_t)hr * (uint32_t)ci + (uint32_t)hi * (uint32_t)cr;
        e += (uint32_t)hr * (uint32_t)hr + (uint32_t)hi * (uint32_t)hi;
    }
    const int32_t sr = (int32_t)tr >> (cs & 31u), si = (int32_t)ti >> (cs & 31u);  // scale32 :244
    const int32_t ar = sr >> 2, ai = si >> 2;                                       // :250
    corr_out[i] = (uint32_t)ar * (uint32_t)ar + (uint32_t)ai * (uint32_t)ai;
    en_out[i] = e >> ((unsigned)((int)cs / 2) & 31u);                                // :245
}

__global__ __launch_bounds__(kCBlock) void corr_eval_dot2(const uint32_t *__restrict__ in, long n, long i_begin,
                                                           long i_end, const uint32_t *__restrict__ hist,
                                                           const uint32_t *__restrict__ ptaps, int N, int NP, int S,
                                                           unsigned cs, uint32_t *__restrict__ corr_out,
                                                           uint32_t *__restrict__ en_out, const unsigned *stop) {
    if ((long)*stop < i_begin) return;  // an earlier segment already detected
    extern __shared__ __attribute__((aligned(16))) uint32_t xs[];
    constexpr int TO = kCBlock * kCR;
    const int ph = blockIdx.y;
    const long NSm1 = (long)N * S - 1;
    // this phase's outputs of the segment: k in [kb, ke), i = k S + ph
    const long kb = (i_begin - ph + S - 1) / S, ke = (i_end - ph + S - 1) / S;
    const long k0 = kb + (long)blockIdx.x * TO;  // first output of the tile (phase stream)
    if (k0 >= ke) return;
    const long base = k0 - (NP - 1);             // first phase-stream sample the tile needs
    const int span = TO + NP - 1;
    const int pad = NP - N;
    // LDS word of tile sample l (l = sample - base): lp = l + 1 (aligns the lane
    // windows' new words to 16 B), one 4-word pad per kCR = 16 words, i.e.
    // 20-word chunks of which the last 4 are padding
    static_assert(kCR == 16, "LDS chunk geometry assumes 16 outputs per lane");
    auto lw = [&](int l) { int lp = l + 1; return lp + 4 * (lp / kCR); };
    for (int l = threadIdx.x; l < span; l += kCBlock) {
        const long j = (base + l) * S + ph;
        uint32_t w = 0;
        if (j < n) w = j >= 0 ? in[j] : (j + NSm1 >= 0 ? hist[j + NSm1] : 0u);
        xs[lw(l)] = w;
    }
    __syncthreads();
    const int t = threadIdx.x;
    // lane window W[j] = sample base + t*kCR + j  ->  LDS lw(t*kCR + j)
    int32_t ar[kCR], ai[kCR];
#pragma unroll
    for (int r = 0; r < kCR; ++r) ar[r] = ai[r] = 0;
    int32_t e0 = 0;
    const int lb = t * kCR;  // lane base in sample units
    // Window words j = 0..30 of a 16-tap chunk: j < 15 were loaded by the
    // previous chunk (its words 16..30), j >= 15 are the chunk's 16 new words.
    // Two register sets alternate roles (unrolled by 2), so sliding the window
    // costs no moves.
    uint32_t A[kCR + 15], B[kCR + 15];
#pragma unroll
    for (int j = 0; j < kCR - 1; ++j) B[16 + j] = xs[lw(lb + j)];
    ConstPtr<uint32_t> tp = const_view<uint32_t>(ptaps);
    auto chunk = [&](int m0, uint32_t(&cur)[kCR + 15], const uint32_t(&prev)[kCR + 15]) {
        asm volatile("" : "+s"(tp));
        uint32_t pw[32];  // this chunk's 16 taps (2 x s_load_dwordx16)
#pragma unroll
        for (int k = 0; k < 32; ++k) pw[k] = tp[2 * m0 + k];
        // new words: the whole 16-word LDS chunk t+1+m0/16 = uint4 slots 5(t+1+m0/16)..+3
        const uint4 *src = (const uint4 *)xs + 5 * (t + 1 + (m0 >> 4));
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const uint4 q = src[g];
            cur[kCR - 1 + 4 * g + 0] = q.x;
            cur[kCR - 1 + 4 * g + 1] = q.y;
            cur[kCR - 1 + 4 * g + 2] = q.z;
            cur[kCR - 1 + 4 * g + 3] = q.w;
        }
        auto word = [&](int j) { return j < kCR - 1 ? prev[16 + j] : cur[j]; };
#pragma unroll
        for (int mm = 0; mm < 16; ++mm) {
            const uint32_t p0 = pw[2 * mm], p1 = pw[2 * mm + 1];
            const short2_t x0 = __builtin_bit_cast(short2_t, word(mm));
            e0 = __builtin_amdgcn_sdot2(x0, x0, e0, false);
#pragma unroll
            for (int r = 0; r < kCR; ++r) {
                const short2_t x = __builtin_bit_cast(short2_t, word(mm + r));
                ar[r] = __builtin_amdgcn_sdot2(x, __builtin_bit_cast(short2_t, p0), ar[r], false);
                ai[r] = __builtin_amdgcn_sdot2(x, __builtin_bit_cast(short2_t, p1), ai[r], false);
            }
        }
    };
    int m0 = 0;
    for (; m0 + 32 <= NP; m0 += 32) {  // NP % 16 == 0
        chunk(m0, A, B);
        chunk(m0 + 16, B, A);
    }
    if (m0 < NP) chunk(m0, A, B);
    // outputs, energies (sliding) and stores; the direct sum ran over the NP
    // window words, the first pad of them before the real window
    uint32_t e = (uint32_t)e0;
    for (int q = 0; q < pad; ++q) {
        const short2_t a = __builtin_bit_cast(short2_t, xs[lw(lb + q)]);
        e -= (uint32_t)__builtin_amdgcn_sdot2(a, a, 0, false);
    }
    for (int r = 0; r < kCR; ++r) {
        const long k = k0 + lb + r;
        if (r > 0) {  // E_{k} = E_{k-1} + |x_k|^2 - |x_{k-N}|^2 (phase stream)
            const uint32_t xn = xs[lw(lb + r + NP - 1)], xo = xs[lw(lb + r - 1 + pad)];
            const short2_t a = __builtin_bit_cast(short2_t, xn), b = __builtin_bit_cast(short2_t, xo);
            e += (uint32_t)__builtin_amdgcn_sdot2(a, a, 0, false) - (uint32_t)__builtin_amdgcn_sdot2(b, b, 0, false);
        }
        if (k < ke) {
            const long i = k * S + ph;
            const int32_t sr = ar[r] >> (cs & 31u), si = ai[r] >> (cs & 31u);
            const int32_t qr = sr >> 2, qi = si >> 2;
            corr_out[i] = (uint32_t)qr * (uint32_t)qr + (uint32_t)qi * (uint32_t)qi;
            en_out[i] = e >> ((unsigned)((int)cs / 2) & 31u);
        }
    }
}

// ------------------------------------ S == 1: one launch, detection fused
// corr_eval_dot2's arithmetic at S = 1 (taps front-padded to NP) over the whole call in ONE launch, with the
// peak/threshold test of correlators.h:262-268 evaluated by each block on its
// own 4096 outputs and reduced to the first hit with atomicMin(best).
//  * the test at a block's first two outputs needs corr/energy of the two
//    samples before it: wave 0 computes those two outputs itself (16 taps per
//    lane from L2, wave reduction), or takes the previous call's registers at
//    index 0;
//  * a block whose first output lies past a recorded hit returns at once, and
//    a running block re-reads `best` every 256 taps and stops computing once
//    a hit before it is known -- the scan ends near the first detection, as
//    the reference's `break` does, with no host round trip.
__device__ __forceinline__ uint32_t corr_value(int32_t ar, int32_t ai, unsigned cs) {
    const int32_t sr = ar >> (cs & 31u), si = ai >> (cs & 31u);  // scale32 :244
    const int32_t qr = sr >> 2, qi = si >> 2;                    // :250
    return (uint32_t)qr * (uint32_t)qr + (uint32_t)qi * (uint32_t)qi;
}

__device__ __forceinline__ unsigned load_best(const unsigned *best) {
    return __hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kCBlock, SRCDSP_CORR_MINW) void corr_scan_s1(const uint32_t *__restrict__ in, long n,
                                                         const uint32_t *__restrict__ hist,
                                                         const uint32_t *__restrict__ ptaps, int N, int NP, unsigned cs,
                                                         uint32_t c_prev0, uint32_t c_prev1, uint32_t e_prev0,
                                                         unsigned *best) {
    extern __shared__ __attribute__((aligned(16))) uint32_t xs[];
    __shared__ uint32_t prev_c[kCBlock + 1][2], prev_e[kCBlock + 1];
    __shared__ unsigned dead_any, best0;
    constexpr int TO = kCBlock * kCR;
    const long i0 = (long)blockIdx.x * TO;  // first output of the tile
    if (threadIdx.x == 0) best0 = load_best(best);
    __syncthreads();
    if ((long)best0 < i0) return;  // a hit before this tile is already known (block-uniform)
    // taps front-padded with NP - N zero taps (NP = 16 ceil(N/16), as corr_eval_dot2)
    const int pad = NP - N;
    // tile sample l (input word i0 - (NP - 1) + l, l = 0 .. TO + NP - 2) -> LDS word
    // lp + 4 (lp / 16), lp = l + 1: chunks of 16 samples + 4 pad words
    // Staging by 16-B granules: LDS chunk c (20 words, the last 4 padding)
    // holds tile samples 16c - 1 .. 16c + 14, i.e. input words j0 + 16c + 4q +
    // (0..3), j0 = i0 - NP: 16-aligned, so an aligned input is read with one
    // dwordx4 per granule; granules that reach before sample 0 or past n, and
    // misaligned inputs, go word by word (history before 0, zeros past n).
    const int NC = (TO + NP) / kCR;  // chunks: tile samples -1 .. TO + NP - 2
    const long j0 = i0 - NP;
    const bool al16 = ((uintptr_t)in & 15u) == 0;
    uint4 *xs4 = (uint4 *)xs;
    for (int gq = threadIdx.x; gq < 4 * NC; gq += kCBlock) {
        const int c = gq >> 2, q = gq & 3;
        const long j = j0 + 16L * c + 4 * q;
        uint4 v;
        if (al16 && j >= 0 && j + 4 <= n) {
            v = *(const uint4 *)(in + j);
        } else {
            uint32_t w[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const long jk = j + k;
                w[k] = jk < n ? (jk >= 0 ? in[jk] : (jk + (N - 1) >= 0 ? hist[jk + (N - 1)] : 0u)) : 0u;
            }
            v = make_uint4(w[0], w[1], w[2], w[3]);
        }
        xs4[5 * c + q] = v;
    }
    if (threadIdx.x == 0) dead_any = 0;
    __syncthreads();
    const int t = threadIdx.x;
    int32_t ar[kCR], ai[kCR];
#pragma unroll
    for (int r = 0; r < kCR; ++r) ar[r] = ai[r] = 0;
    int32_t e0 = 0;
    const int lb = t * kCR;
    // The window energy of each lane's first output from 16-sample chunk sums
    // instead of one dot2(x, x) per tap beside the 32 correlation dot2.  Lane
    // t's window is tile samples lb .. lb + NP - 1 (lb = 16 t); LDS chunks
    // t .. t + NP/16 - 1 hold samples lb - 1 .. lb + NP - 2, so the sum of their
    // chunk sums, less |x[lb - 1]|^2, plus |x[lb + NP - 1]|^2 (word 0 of chunk
    // t + NP/16).  A chunk sum reads its chunk as 4 ds_read_b128 (conflict-free
    // at the 80-B chunk stride).  Wrap-around uint32 sums: equal to the direct sum.
    {
        uint32_t *csum = xs + corr_lds_words(NP);  // kCBlock + NP/16 words (dynamic, sized by the host)
        const int NCk = NP / 16;
        auto sq = [](uint32_t w) {
            const short2_t a = __builtin_bit_cast(short2_t, w);
            return (uint32_t)__builtin_amdgcn_sdot2(a, a, 0, false);
        };
        for (int g = t; g < kCBlock + NCk - 1; g += kCBlock) {
            uint32_t sg = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                typedef uint32_t u4v_t __attribute__((ext_vector_type(4)));
                u4v_t v = *(const u4v_t *)&xs4[5 * g + q];
                asm volatile("" : "+v"(v));  // one ds_read_b128 (not 4-B pieces, 4-way conflicting at the 80-B stride)
                sg += sq(v.x) + sq(v.y) + sq(v.z) + sq(v.w);
            }
            csum[g] = sg;
        }
        __syncthreads();
        uint32_t eu = sq(xs[20 * (t + NCk)]) - sq(xs[20 * t]);
        for (int g = 0; g < NCk; ++g) eu += csum[t + g];
        e0 = (int32_t)eu;
    }
    // Each 16-tap chunk reads its whole 31-word window from LDS (LDS chunks
    // c0 = t + m0/16 and c0 + 1: 8 ds_read_b128, words j = -1 .. 30 of the
    // lane window) instead of carrying the previous chunk's 15 words in
    // registers: the carried words came back from the compiler's early reads
    // through 15 v_mov per 32 taps, the extra reads cost LDS slots only.
    ConstPtr<uint32_t> tp = const_view<uint32_t>(ptaps);
    auto chunk = [&](int m0) {
        asm volatile("" : "+s"(tp));
        uint32_t pw[32];
#pragma unroll
        for (int k = 0; k < 32; ++k) pw[k] = tp[2 * m0 + k];
        const uint4 *src = (const uint4 *)xs + 5 * (t + (m0 >> 4));
        uint32_t W[32];  // W[j + 1] = window word j
        typedef uint32_t u4v_t __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            // chunk c0 granules 0..3, chunk c0 + 1 granules 0..3; each a whole
            // ds_read_b128 (W[0] is unused: left alone the compiler reads chunk
            // c0 as 4-B pieces, which the 80-B lane stride does not spread)
            u4v_t q = *(const u4v_t *)(src + (g < 4 ? g : g + 1));
            asm volatile("" : "+v"(q));
            W[4 * g + 0] = q.x;
            W[4 * g + 1] = q.y;
            W[4 * g + 2] = q.z;
            W[4 * g + 3] = q.w;
        }
#pragma unroll
        for (int mm = 0; mm < 16; ++mm) {
            const uint32_t p0 = pw[2 * mm], p1 = pw[2 * mm + 1];
#pragma unroll
            for (int r = 0; r < kCR; ++r) {
                const short2_t x = __builtin_bit_cast(short2_t, W[mm + r + 1]);
                ar[r] = __builtin_amdgcn_sdot2(x, __builtin_bit_cast(short2_t, p0), ar[r], false);
                ai[r] = __builtin_amdgcn_sdot2(x, __builtin_bit_cast(short2_t, p1), ai[r], false);
            }
        }
    };
    bool dead = false;
    for (int m0 = 0, it = 0; m0 < NP; m0 += 16, ++it) {  // NP % 16 == 0
        chunk(m0);
        if ((it & 15) == 15) {  // every 256 taps: has a hit before this tile been found?
            const unsigned bb = __builtin_amdgcn_readfirstlane(load_best(best));
            if ((long)bb < i0) {
                dead = true;
                break;
            }
        }
    }
    // the two outputs before the tile (for the test at its first two indices)
    if (t < 64) {
        uint32_t ex_c[2] = {c_prev0, c_prev1}, ex_e = e_prev0;
        if (i0 > 0 && !dead) {
            int32_t r1 = 0, q1 = 0, r2 = 0, q2 = 0, en1 = 0;
            for (int m = t; m < N; m += 64) {  // output i0-1-u: sample i0-1-u-(N-1)+m
                const uint32_t xa = corr_fetch(in, hist, i0 - N + m, N - 1);      // u = 0
                const uint32_t xb = corr_fetch(in, hist, i0 - N - 1 + m, N - 1);  // u = 1
                const short2_t sa = __builtin_bit_cast(short2_t, xa), sb = __builtin_bit_cast(short2_t, xb);
                const short2_t p0 = __builtin_bit_cast(short2_t, (uint32_t)tp[2 * (m + pad)]);
                const short2_t p1 = __builtin_bit_cast(short2_t, (uint32_t)tp[2 * (m + pad) + 1]);
                r1 = __builtin_amdgcn_sdot2(sa, p0, r1, false);
                q1 = __builtin_amdgcn_sdot2(sa, p1, q1, false);
                r2 = __builtin_amdgcn_sdot2(sb, p0, r2, false);
                q2 = __builtin_amdgcn_sdot2(sb, p1, q2, false);
                en1 = __builtin_amdgcn_sdot2(sa, sa, en1, false);
            }
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) {
                r1 += __shfl_xor(r1, off);
                q1 += __shfl_xor(q1, off);
                r2 += __shfl_xor(r2, off);
                q2 += __shfl_xor(q2, off);
                en1 += __shfl_xor(en1, off);
            }
            ex_c[0] = corr_value(r1, q1, cs);
            ex_c[1] = corr_value(r2, q2, cs);
            ex_e = (uint32_t)en1 >> ((unsigned)((int)cs / 2) & 31u);
        }
        if (t == 0) {
            prev_c[0][0] = ex_c[0];
            prev_c[0][1] = ex_c[1];
            prev_e[0] = ex_e;
        }
    }
    // this lane's correlation values and (sliding) energies, tested as they are
    // formed: outputs 2..15 need only the lane's own values, so only outputs 0
    // and 1 (which need the previous lane's last values) wait for the barrier,
    // and three values per lane live across it instead of 32 (at 5 waves per
    // SIMD the 32 spilled to scratch: 2.25 x the algorithmic HBM bytes)
    // LDS words of the sliding energy, from per-lane bases (no per-output
    // index arithmetic): the sample entering output r's window is tile sample
    // lb + r + NP - 1, word 20 (t + NP/16) + r; the one leaving is tile sample
    // lb + r - 1 + pad, word 20 t + q + 4 (q >> 4) with q = r + pad (uniform)
    const uint32_t *xn_base = xs + 20 * (t + NP / 16), *xo_base = xs + 20 * t;
    auto xo_word = [&](int q) { return xo_base[q + 4 * (q >> 4)]; };
    uint32_t e = (uint32_t)e0;  // the direct sum ran over NP window words, the first pad before the real window
    for (int q = 0; q < pad; ++q) {  // tile samples lb .. lb + pad - 1 (q + 1 <= 15: one LDS chunk)
        const short2_t a = __builtin_bit_cast(short2_t, xo_base[q + 1]);
        e -= (uint32_t)__builtin_amdgcn_sdot2(a, a, 0, false);
    }
    // outputs of this lane inside the call: r < nrem (int compares, no 64-bit index per output)
    const int nrem = (int)std::min<long>(kCR, n - (i0 + lb));
    uint32_t c_0 = 0, c_1 = 0, e_0 = 0;  // outputs 0 and 1, for the tests after the barrier
    uint32_t cm2 = 0, cm1 = 0, em1 = 0;  // the two outputs before r, the energy before r
    int hit = -1;                        // first hit among outputs 2..15 (lane-relative)
#pragma unroll
    for (int r = 0; r < kCR; ++r) {
        if (r > 0) {  // E_i = E_{i-1} + |x_i|^2 - |x_{i-N}|^2
            const uint32_t xn = xn_base[r], xo = xo_word(r + pad);
            const short2_t a = __builtin_bit_cast(short2_t, xn), b = __builtin_bit_cast(short2_t, xo);
            e += (uint32_t)__builtin_amdgcn_sdot2(a, a, 0, false) - (uint32_t)__builtin_amdgcn_sdot2(b, b, 0, false);
        }
        const uint32_t c = corr_value(ar[r], ai[r], cs), ev = e >> ((unsigned)((int)cs / 2) & 31u);
        if (r == 0) {
            c_0 = c;
            e_0 = ev;
        } else if (r == 1) {
            c_1 = c;
        } else if (!dead && hit < 0 && r < nrem && corr_hit(cm2, cm1, c, em1)) {
            hit = r;
        }
        cm2 = cm1;
        cm1 = c;
        em1 = ev;
    }
    prev_c[t + 1][0] = cm1;  // output 15
    prev_c[t + 1][1] = cm2;  // output 14
    prev_e[t + 1] = em1;
    if (dead) dead_any = 1;
    __syncthreads();
    if (dead_any) return;  // outputs past a known hit: nothing to record
    const uint32_t pc1 = prev_c[t][0], pc2 = prev_c[t][1], pe1 = prev_e[t];
    if (1 < nrem && corr_hit(pc1, c_0, c_1, e_0)) hit = 1;
    if (0 < nrem && corr_hit(pc2, pc1, c_0, pe1)) hit = 0;
    if (hit >= 0) atomicMin(best, (unsigned)(i0 + lb + hit));
}

__global__ void corr_detect(const uint32_t *__restrict__ corr, const uint32_t *__restrict__ en, long i_begin,
                            long i_end, uint32_t c_prev0, uint32_t c_prev1, uint32_t e_prev0, unsigned *best) {
    // skip when an EARLIER segment detected (a hit of this segment is >= i_begin,
    // so blocks of this launch never stop each other)
    if ((long)*(volatile unsigned *)best < i_begin) return;
    for (long i = i_begin + (long)blockIdx.x * blockDim.x + threadIdx.x; i < i_end;
         i += (long)gridDim.x * blockDim.x) {
        const uint32_t c0 = corr[i];
        const uint32_t c1 = i >= 1 ? corr[i - 1] : c_prev0;
        const uint32_t c2 = i >= 2 ? corr[i - 2] : (i == 1 ? c_prev0 : c_prev1);
        const uint32_t e1 = i >= 1 ? en[i - 1] : e_prev0;
        if (corr_hit(c2, c1, c0, e1)) atomicMin(best, (unsigned)i);
    }
}

// new_hist[k] = effective stream sample (last - NSm1 + 1 + k), from input or old history
__global__ void corr_history(const uint32_t *in, const uint32_t *hist_in, uint32_t *hist_out, long last,
                             long NSm1) {
    for (long k = (long)blockIdx.x * blockDim.x + threadIdx.x; k < NSm1; k += (long)gridDim.x * blockDim.x)
        hist_out[k] = corr_fetch(in, hist_in, last - NSm1 + 1 + k, NSm1);
}

// The registers after a fused scan (corr_scan_s1 stores no per-sample values):
// corr and energy at last-2 .. last, last = the detected sample (*best) or
// n - 1, each a direct sum over the N taps with corr_eval's arithmetic
// (int32 wrap-around sums, so equal to the scan's sliding energy).  One block;
// out[k] = corr(last - k), out[3 + k] = energy(last - k) for last - k >= 0.
__global__ __launch_bounds__(256) void corr_point(const uint32_t *__restrict__ in, long n,
                                                  const uint32_t *__restrict__ hist,
                                                  const int32_t *__restrict__ coef, unsigned N, unsigned S, unsigned cs,
                                                  const unsigned *__restrict__ best, uint32_t *__restrict__ out) {
    __shared__ uint32_t red[3][3][256];
    const unsigned b = *best;
    const long last = b != 0xffffffffu ? (long)b : n - 1;
    const long NSm1 = (long)N * S - 1;
    for (int k = 0; k < 3; ++k) {
        uint32_t tr = 0, ti = 0, e = 0;
        const long i = last - k;
        if (i >= 0)
            for (unsigned m = threadIdx.x; m < N; m += blockDim.x) {
                const uint32_t w = corr_fetch(in, hist, i - (long)(N - 1 - m) * S, NSm1);
                const int32_t hr = sext16(w), hi = sext16_hi(w);
                const int32_t cr = coef[2 * m], ci = coef[2 * m + 1];
                tr += (uint32_t)hr * (uint32_t)cr - (uint32_t)hi * (uint32_t)ci;
                ti += (uint32_t)hr * (uint32_t)ci + (uint32_t)hi * (uint32_t)cr;
                e += (uint32_t)hr * (uint32_t)hr + (uint32_t)hi * (uint32_t)hi;
            }
        red[k][0][threadIdx.x] = tr;
        red[k][1][threadIdx.x] = ti;
        red[k][2][threadIdx.x] = e;
    }
    __syncthreads();
    for (int w = 128; w >= 1; w >>= 1) {
        if ((int)threadIdx.x < w)
            for (int k = 0; k < 3; ++k)
                for (int q = 0; q < 3; ++q) red[k][q][threadIdx.x] += red[k][q][threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x < 3) {
        const int k = threadIdx.x;
        const int32_t sr = (int32_t)red[k][0][0] >> (cs & 31u), si = (int32_t)red[k][1][0] >> (cs & 31u);
        const int32_t ar = sr >> 2, ai = si >> 2;
        out[k] = (uint32_t)ar * (uint32_t)ar + (uint32_t)ai * (uint32_t)ai;
        out[3 + k] = red[k][2][0] >> ((unsigned)((int)cs / 2) & 31u);
    }
}

// ---------------------------------------------------------------- host side
static int corr_alloc_scratch(srcdsp_corr_state &c, size_t n) {
    if (n <= c.scratch_cap) return SRCDSP_OK;
    if (c.d_corr) (void)hipFree(c.d_corr);
    if (c.d_en) (void)hipFree(c.d_en);
    c.d_corr = c.d_en = nullptr;
    SRCDSP_HIP_TRY(hipMalloc(&c.d_corr, 4 * n));
    SRCDSP_HIP_TRY(hipMalloc(&c.d_en, 4 * n));
    c.scratch_cap = n;
    return SRCDSP_OK;
}

// detect = false: stream the samples with no detection test (corr_prime):
// only the last three positions are evaluated (they feed the registers).
// trace (CREATE_DEBUG_FILES, correlators.h:253-257): host arrays of n_
// entries receive corrValue[0] / energyValue[0] after each processed sample
// (*trace_n of them: corrIndex + 2 on a detection, else n_); the segmented
// kernels run, since only they keep per-sample values.
struct CorrTrace {
    uint32_t *corr = nullptr, *energy = nullptr;
    size_t *count = nullptr;
};

static int corr_run(srcdsp_corr_state &c, const uint32_t *d_in, size_t n_, int *found, int *corr_index,
                    hipStream_t s, bool detect = true, const CorrTrace *trace = nullptr) {
    *found = 0;
    if (trace) *trace->count = 0;
    if (n_ == 0) return SRCDSP_OK;
    const long n = (long)n_;
    if (n > 0x7fffffffL) {
        set_error("corr_step: input longer than INT_MAX samples (correlators.h:212 uses int)");
        return SRCDSP_ERR_SIZE;
    }
    int rc = c.order.before(s);
    if (rc) return rc;
    const long NSm1 = (long)c.NS - 1;
    const uint32_t *hist = c.d_hist[c.cur];
    const unsigned cs = (unsigned)c.coeff_scaling;
    // dot2 tiles for int16-range patterns (48 <= N <= kCorrDot2MaxTaps at
    // S > 1: below 48 taps there the strided staging costs more than the taps,
    // 0.277 vs 0.468 ms at N = 31, S = 3 on 2^24 samples); at S = 1 (config 5
    // and every N <= kCorrDot2MaxTaps) one launch scans with detection fused
    const bool dot2 = c.taps16 && c.NP <= kCorrDot2MaxTaps && c.S <= kCorrMaxGridY &&
                      (c.N >= 48 || c.S == 1);
    const bool fast = dot2 && c.S == 1;
    // the fused scan keeps no per-sample values (corr_point computes the three
    // the registers need); the segmented kernels write corr/energy per sample
    // for corr_detect
    const bool fused = fast && detect && !trace;
    if (!fused) {
        rc = corr_alloc_scratch(c, n_);
        if (rc) return rc;
    }
    // The reference stops at the first detection (break, correlators.h:291).
    // All segments are queued at once; each launch returns at its start when
    // an earlier segment's detect kernel has recorded a hit, so the scan stops
    // one segment after the detection with no host round trip in between.
    const long seg = std::max<long>(1L << 22, (n + 15) / 16);
    const unsigned none = 0xffffffffu;
    unsigned best = none;
    SRCDSP_HIP_TRY(hipMemsetAsync(c.d_best, 0xff, 4, s));
    if (fused) {  // one launch, detection fused, in-flight early exit
        constexpr long TO = (long)kCBlock * kCR;
        const long blocks = (n + TO - 1) / TO;
        const size_t smem = 4 * (size_t)corr_scan_lds_words((int)c.NP);
        hipLaunchKernelGGL(corr_scan_s1, dim3((unsigned)blocks), dim3(kCBlock), smem, s, d_in, n, hist, c.d_ptaps,
                           (int)c.N, (int)c.NP, cs, c.corr[0], c.corr[1], c.energy[0], c.d_best);
        SRCDSP_HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(corr_point, dim3(1), dim3(256), 0, s, d_in, n, hist, c.d_coef, c.N, c.S, cs,
                           (const unsigned *)c.d_best, c.d_best + 2);
        SRCDSP_HIP_TRY(hipGetLastError());
    }
    // the segmented path: priming (the last 3 positions only) and the generic
    // kernels (S > 1 or N % 16 != 0)
    for (long sb = detect ? (fused ? n : 0) : std::max(0L, n - 3); sb < n; sb += seg) {
        const long se = std::min(n, sb + seg);
        if (dot2) {  // grid.y = phase of the stride
            constexpr long TO = (long)kCBlock * kCR;
            const long per_phase = (se - sb + c.S - 1) / c.S;
            const long blocks = (per_phase + TO - 1) / TO;
            const size_t smem = 4 * (size_t)corr_lds_words((int)c.NP);
            hipLaunchKernelGGL(corr_eval_dot2, dim3((unsigned)blocks, c.S), dim3(kCBlock), smem, s, d_in, n, sb, se,
                               hist, c.d_ptaps, (int)c.N, (int)c.NP, (int)c.S, cs, c.d_corr, c.d_en,
                               (const unsigned *)c.d_best);
        } else {
            const size_t smem = 4 * (size_t)((kCorrBlock + NSm1 + 3) & ~3l) + 8 * (size_t)c.N;
            const long blocks = (se - sb + kCorrBlock - 1) / kCorrBlock;
            if (smem <= kCorrEvalMaxSmem)
                hipLaunchKernelGGL(corr_eval, dim3((unsigned)blocks), dim3(kCorrBlock), smem, s, d_in, n, sb, se, hist,
                                   c.d_coef, c.N, c.S, cs, c.d_corr, c.d_en, (const unsigned *)c.d_best);
            else
                hipLaunchKernelGGL(corr_eval_g, dim3((unsigned)blocks), dim3(kCorrBlock), 0, s, d_in, n, sb, se, hist,
                                   c.d_coef, c.N, c.S, cs, c.d_corr, c.d_en, (const unsigned *)c.d_best);
        }
        SRCDSP_HIP_TRY(hipGetLastError());
        if (!detect) continue;
        const int db = (int)std::max<long>(1, std::min<long>((se - sb + 255) / 256, 4096));
        hipLaunchKernelGGL(corr_detect, dim3(db), dim3(256), 0, s, c.d_corr, c.d_en, sb, se, c.corr[0], c.corr[1],
                           c.energy[0], c.d_best);
        SRCDSP_HIP_TRY(hipGetLastError());
    }
    unsigned words[8];  // best, pad, corr_point's corr[3] and energy[3]
    SRCDSP_HIP_TRY(hipMemcpyAsync(words, c.d_best, fused ? sizeof words : 4, hipMemcpyDeviceToHost, s));
    SRCDSP_HIP_TRY(hipStreamSynchronize(s));
    best = words[0];

    const bool hit = best != none;
    const long last = hit ? (long)best : n - 1;  // last processed sample
    if (trace) {  // every processed sample's registers (the segmented kernels computed them all up to `last`)
        SRCDSP_HIP_TRY(hipMemcpyAsync(trace->corr, c.d_corr, 4 * (size_t)(last + 1), hipMemcpyDeviceToHost, s));
        SRCDSP_HIP_TRY(hipMemcpyAsync(trace->energy, c.d_en, 4 * (size_t)(last + 1), hipMemcpyDeviceToHost, s));
        SRCDSP_HIP_TRY(hipStreamSynchronize(s));
        *trace->count = (size_t)(last + 1);
    }
    // registers after processing `last` (correlators.h:228-230, 248-250)
    uint32_t cw[3] = {0, 0, 0}, ew[3] = {0, 0, 0};
    const long lo = std::max(0L, last - 2);
    const long cnt = last - lo + 1;
    if (fused) {
        for (long idx = lo; idx <= last; ++idx) {
            cw[idx - lo] = words[2 + (last - idx)];
            ew[idx - lo] = words[5 + (last - idx)];
        }
    } else {
        SRCDSP_HIP_TRY(hipMemcpyAsync(cw, c.d_corr + lo, 4 * cnt, hipMemcpyDeviceToHost, s));
        SRCDSP_HIP_TRY(hipMemcpyAsync(ew, c.d_en + lo, 4 * cnt, hipMemcpyDeviceToHost, s));
        SRCDSP_HIP_TRY(hipStreamSynchronize(s));
    }
    uint32_t nc[3], ne[3];
    for (int k = 0; k < 3; ++k) {  // nc[k] = corr of sample last-k
        long idx = last - k;
        if (idx >= 0) {
            nc[k] = cw[idx - lo];
            ne[k] = ew[idx - lo];
        } else {  // reach back into the previous registers
            nc[k] = c.corr[-idx - 1];
            ne[k] = c.energy[-idx - 1];
        }
    }
    if (hit) {
        // bitSamples (correlators.h:278-288): ring read backwards from the peak
        // sample best-1 with stride S; with S == 1 the oldest slot already
        // holds the detected sample (the ring wrapped onto it).
        std::vector<uint32_t> win((size_t)c.NS + 1);
        // effective stream positions best-NS .. best
        const long first = (long)best - (long)c.NS;
        std::vector<uint32_t> h_hist(NSm1 > 0 ? NSm1 : 1);
        if (NSm1 > 0) SRCDSP_HIP_TRY(hipMemcpyAsync(h_hist.data(), hist, 4 * NSm1, hipMemcpyDeviceToHost, s));
        const long in_lo = std::max(0L, first);
        const long in_cnt = (long)best - in_lo + 1;
        std::vector<uint32_t> h_in(in_cnt);
        SRCDSP_HIP_TRY(hipMemcpyAsync(h_in.data(), d_in + in_lo, 4 * in_cnt, hipMemcpyDeviceToHost, s));
        SRCDSP_HIP_TRY(hipStreamSynchronize(s));
        for (long j = first; j <= (long)best; ++j) {
            uint32_t v;
            if (j >= 0) v = h_in[j - in_lo];
            else v = (j + NSm1 >= 0) ? h_hist[j + NSm1] : 0u;
            win[j - first] = v;
        }
        for (unsigned m = 0; m < c.N; ++m) {
            const long d = (long)(c.N - 1 - m) * c.S;
            uint32_t v = (d == NSm1) ? win[c.NS] : win[((long)best - 1 - d) - first];
            c.bits[2 * m] = (int16_t)(v & 0xffff);
            c.bits[2 * m + 1] = (int16_t)(v >> 16);
        }
    }
    // history: last NS-1 samples of the effective stream (the detected sample is
    // overwritten by the next call's first sample)
    const long last_eff = hit ? (long)best - 1 : n - 1;
    if (NSm1 > 0) {
        const int hb = (int)std::max<long>(1, std::min<long>((NSm1 + 255) / 256, 1024));
        hipLaunchKernelGGL(corr_history, dim3(hb), dim3(256), 0, s, d_in, hist, c.d_hist[c.cur ^ 1], last_eff, NSm1);
        SRCDSP_HIP_TRY(hipGetLastError());
        c.cur ^= 1;
    }
    for (int k = 0; k < 3; ++k) {
        c.corr[k] = nc[k];
        c.energy[k] = ne[k];
    }
    if (hit) {
        *found = 1;
        *corr_index = (int)best - 1;
    }
    return c.order.after(s);
}

}  // namespace srcdsp

using namespace srcdsp;
struct srcdsp_corr { srcdsp_corr_state c; };

// The build's test switches, reported by a kernel of this library (so a
// process holding two copies of the library -- the product and a test build,
// tests/test_gpu_corr_hit.py -- can tell which copy's kernels a call ran).
__global__ void corr_build_flags_kernel(unsigned *out) {
    if (threadIdx.x == 0) {
#ifdef SRCDSP_CORR_ALWAYS_EXACT
        *out = SRCDSP_BUILD_CORR_ALWAYS_EXACT;
#else
        *out = 0u;
#endif
    }
}

extern "C" {

SRCDSP_API int srcdsp_build_flags(unsigned *flags) {
    SRCDSP_ARG_CHECK(flags != nullptr, "build_flags: null flags");
    unsigned *d = nullptr;
    if (hipMalloc(&d, sizeof(unsigned)) != hipSuccess) {
        set_error("build_flags: device allocation failed");
        return SRCDSP_ERR_HIP;
    }
    hipLaunchKernelGGL(corr_build_flags_kernel, dim3(1), dim3(64), 0, nullptr, d);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpy(flags, d, sizeof(unsigned), hipMemcpyDeviceToHost);
    hipFree(d);
    if (e != hipSuccess) {
        set_error(hipGetErrorString(e));
        return SRCDSP_ERR_HIP;
    }
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_corr_create(srcdsp_corr_t *out, unsigned N, unsigned S) {
    SRCDSP_ARG_CHECK(out != nullptr, "corr_create: null out");
    *out = nullptr;
    SRCDSP_ARG_CHECK(N >= 1 && S >= 1 && (unsigned long)N * S <= (1ul << 24), "corr_create: bad N/S");
    auto *h = new srcdsp_corr();
    srcdsp_corr_state &c = h->c;
    c.N = N;
    c.S = S;
    c.NS = N * S;
    c.NP = (N + 15) / 16 * 16;
    c.h_coef.assign(2 * N, 0);
    c.bits.assign(2 * N, 0);
    int rc = c.order.init();
    if (!rc) rc = c.stage.init();
    if (rc) {
        delete h;
        return rc;
    }
    const size_t hb = 4 * (size_t)std::max(1u, c.NS - 1);
    if (hipMalloc(&c.d_coef, 8 * (size_t)N) != hipSuccess || hipMemset(c.d_coef, 0, 8 * (size_t)N) != hipSuccess ||
        hipMalloc(&c.d_ptaps, 8 * (size_t)c.NP) != hipSuccess || hipMemset(c.d_ptaps, 0, 8 * (size_t)c.NP) != hipSuccess ||
        hipMalloc(&c.d_hist[0], hb) != hipSuccess || hipMalloc(&c.d_hist[1], hb) != hipSuccess ||
        hipMemset(c.d_hist[0], 0, hb) != hipSuccess || hipMalloc(&c.d_best, 32) != hipSuccess) {
        set_error("corr_create: device allocation failed");
        srcdsp_corr_destroy(h);
        return SRCDSP_ERR_HIP;
    }
    *out = h;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_corr_destroy(srcdsp_corr_t h) {
    if (!h) return SRCDSP_OK;
    srcdsp_corr_state &c = h->c;
    (void)c.order.sync();
    for (void *p : {(void *)c.d_coef, (void *)c.d_ptaps, (void *)c.d_hist[0], (void *)c.d_hist[1], (void *)c.d_corr, (void *)c.d_en,
                    (void *)c.d_best})
        if (p) (void)hipFree(p);
    c.order.destroy();
    c.stage.destroy();
    delete h;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_corr_clone(srcdsp_corr_t h, srcdsp_corr_t *out) {
    SRCDSP_ARG_CHECK(h != nullptr && out != nullptr, "corr_clone: null argument");
    *out = nullptr;
    srcdsp_corr_state &s = h->c;
    int rc = s.order.sync();
    if (rc) return rc;
    srcdsp_corr_t n = nullptr;
    rc = srcdsp_corr_create(&n, s.N, s.S);
    if (rc) return rc;
    srcdsp_corr_state &c = n->c;
    c.h_coef = s.h_coef;
    c.taps16 = s.taps16;
    for (int k = 0; k < 3; ++k) {
        c.energy[k] = s.energy[k];
        c.corr[k] = s.corr[k];
    }
    c.coeffs_energy = s.coeffs_energy;
    c.coeff_scaling = s.coeff_scaling;
    c.threshold_factor = s.threshold_factor;
    c.bits = s.bits;
    const size_t hb = 4 * (size_t)std::max(1u, s.NS - 1);
    if (hipMemcpy(c.d_coef, s.d_coef, 8 * (size_t)s.N, hipMemcpyDeviceToDevice) != hipSuccess ||
        hipMemcpy(c.d_ptaps, s.d_ptaps, 8 * (size_t)s.NP, hipMemcpyDeviceToDevice) != hipSuccess ||
        hipMemcpy(c.d_hist[0], s.d_hist[s.cur], hb, hipMemcpyDeviceToDevice) != hipSuccess) {
        srcdsp_corr_destroy(n);
        set_error("corr_clone: device copy failed");
        return SRCDSP_ERR_HIP;
    }
    c.cur = 0;
    *out = n;
    return SRCDSP_OK;
}

// setPattern (correlators.h:167-194)
SRCDSP_API int srcdsp_corr_set_pattern(srcdsp_corr_t h, const int32_t *p, double th) {
    SRCDSP_ARG_CHECK(h != nullptr && p != nullptr, "corr_set_pattern: null argument");
    srcdsp_corr_state &c = h->c;
    double tmp = 0;
    for (unsigned i = 0; i < c.N; ++i) {
        const int32_t re = p[2 * i], im = (int32_t)(0u - (uint32_t)p[2 * i + 1]);  // conjugate
        c.h_coef[2 * i] = re;
        c.h_coef[2 * i + 1] = im;
        tmp += (double)(int32_t)((uint32_t)re * (uint32_t)re + (uint32_t)im * (uint32_t)im);
    }
    if (!(tmp <= 1073217600)) {
        set_error("setPattern: pattern energy above 1073217600 (correlators.h:185 assert)");
        return SRCDSP_ERR_ARG;
    }
    int rc = c.order.sync();
    if (rc) return rc;
    c.coeffs_energy = (uint32_t)(uint64_t)(int64_t)tmp;
    c.threshold_factor = th * std::sqrt((double)c.coeffs_energy);
    c.coeff_scaling = cvt_d2i_x86(std::floor(std::log2(std::sqrt((double)c.coeffs_energy))));
    SRCDSP_HIP_TRY(hipMemcpy(c.d_coef, c.h_coef.data(), 8 * (size_t)c.N, hipMemcpyHostToDevice));
    c.taps16 = true;
    std::vector<uint32_t> pk(2 * (size_t)c.NP, 0u);  // front-padded with NP - N zero taps
    for (unsigned i = 0; i < c.N; ++i) {
        const int32_t pr = p[2 * i], pi = p[2 * i + 1];
        if (pr < -32767 || pr > 32767 || pi < -32767 || pi > 32767) c.taps16 = false;
        const size_t m = (size_t)(c.NP - c.N) + i;
        pk[2 * m] = ((uint32_t)pr & 0xffffu) | ((uint32_t)pi << 16);       // Re = x.re*p.re + x.im*p.im
        pk[2 * m + 1] = ((uint32_t)(-pi) & 0xffffu) | ((uint32_t)pr << 16);  // Im = -x.re*p.im + x.im*p.re
    }
    SRCDSP_HIP_TRY(hipMemcpy(c.d_ptaps, pk.data(), 8 * (size_t)c.NP, hipMemcpyHostToDevice));
    return SRCDSP_OK;
}

// reset (correlators.h:146-159): registers, history and bitSamples cleared
SRCDSP_API int srcdsp_corr_reset(srcdsp_corr_t h) {
    SRCDSP_ARG_CHECK(h != nullptr, "corr_reset: null handle");
    srcdsp_corr_state &c = h->c;
    int rc = c.order.sync();
    if (rc) return rc;
    for (int k = 0; k < 3; ++k) c.energy[k] = c.corr[k] = 0;
    std::fill(c.bits.begin(), c.bits.end(), 0);
    const size_t hb = 4 * (size_t)std::max(1u, c.NS - 1);
    // on the handle's own stream: no wait on other streams' work
    SRCDSP_HIP_TRY(hipMemsetAsync(c.d_hist[c.cur], 0, hb, c.stage.stream));
    SRCDSP_HIP_TRY(hipStreamSynchronize(c.stage.stream));
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_corr_prime(srcdsp_corr_t h, const void *d_in, size_t n, void *stream) {
    SRCDSP_ARG_CHECK(h != nullptr && (d_in != nullptr || n == 0), "corr_prime: null argument");
    int found = 0, idx = 0;
    return corr_run(h->c, (const uint32_t *)d_in, n, &found, &idx, (hipStream_t)stream, false);
}

SRCDSP_API int srcdsp_corr_step(srcdsp_corr_t h, const void *d_in, size_t n, int *found, int *corr_index,
                                void *stream) {
    SRCDSP_ARG_CHECK(h != nullptr && found != nullptr && corr_index != nullptr, "corr_step: null argument");
    SRCDSP_ARG_CHECK(d_in != nullptr || n == 0, "corr_step: null input");
    return corr_run(h->c, (const uint32_t *)d_in, n, found, corr_index, (hipStream_t)stream);
}

SRCDSP_API int srcdsp_corr_step_host(srcdsp_corr_t h, const void *in, size_t n, int *found, int *corr_index) {
    SRCDSP_ARG_CHECK(h != nullptr && found != nullptr && corr_index != nullptr, "corr_step_host: null argument");
    *found = 0;
    if (n == 0) return SRCDSP_OK;
    srcdsp_corr_state &c = h->c;
    int rc = c.stage.reserve(4 * n, 4 * n);
    if (rc) return rc;
    host_copy(c.stage.h_buf, in, 4 * n);
    SRCDSP_HIP_TRY(hipMemcpyAsync(c.stage.d_buf, c.stage.h_buf, 4 * n, hipMemcpyHostToDevice, c.stage.stream));
    return corr_run(c, (const uint32_t *)c.stage.d_buf, n, found, corr_index, c.stage.stream);
}

SRCDSP_API int srcdsp_corr_step_trace(srcdsp_corr_t h, const void *d_in, size_t n, int *found, int *corr_index,
                                      uint32_t *corr_out, uint32_t *energy_out, size_t *count, void *stream) {
    SRCDSP_ARG_CHECK(h != nullptr && found != nullptr && corr_index != nullptr && count != nullptr,
                     "corr_step_trace: null argument");
    SRCDSP_ARG_CHECK(d_in != nullptr || n == 0, "corr_step_trace: null input");
    SRCDSP_ARG_CHECK(n == 0 || (corr_out != nullptr && energy_out != nullptr), "corr_step_trace: null trace array");
    const CorrTrace t{corr_out, energy_out, count};
    return corr_run(h->c, (const uint32_t *)d_in, n, found, corr_index, (hipStream_t)stream, true, &t);
}

SRCDSP_API int srcdsp_corr_step_host_trace(srcdsp_corr_t h, const void *in, size_t n, int *found, int *corr_index,
                                           uint32_t *corr_out, uint32_t *energy_out, size_t *count) {
    SRCDSP_ARG_CHECK(h != nullptr && found != nullptr && corr_index != nullptr && count != nullptr,
                     "corr_step_host_trace: null argument");
    SRCDSP_ARG_CHECK(n == 0 || (in != nullptr && corr_out != nullptr && energy_out != nullptr),
                     "corr_step_host_trace: null argument");
    *found = 0;
    *count = 0;
    if (n == 0) return SRCDSP_OK;
    srcdsp_corr_state &c = h->c;
    int rc = c.stage.reserve(4 * n, 4 * n);
    if (rc) return rc;
    host_copy(c.stage.h_buf, in, 4 * n);
    SRCDSP_HIP_TRY(hipMemcpyAsync(c.stage.d_buf, c.stage.h_buf, 4 * n, hipMemcpyHostToDevice, c.stage.stream));
    const CorrTrace t{corr_out, energy_out, count};
    return corr_run(c, (const uint32_t *)c.stage.d_buf, n, found, corr_index, c.stage.stream, true, &t);
}

SRCDSP_API int srcdsp_corr_get_bit_samples(srcdsp_corr_t h, int16_t *bits) {
    SRCDSP_ARG_CHECK(h != nullptr && bits != nullptr, "corr_get_bit_samples: null argument");
    memcpy(bits, h->c.bits.data(), 4 * (size_t)h->c.N);
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_corr_get_status(srcdsp_corr_t h, uint32_t *e3, uint32_t *c3, uint32_t *ce, int *cs,
                                      double *tf) {
    SRCDSP_ARG_CHECK(h != nullptr, "corr_get_status: null handle");
    const srcdsp_corr_state &c = h->c;
    for (int k = 0; k < 3; ++k) {
        if (e3) e3[k] = c.energy[k];
        if (c3) c3[k] = c.corr[k];
    }
    if (ce) *ce = c.coeffs_energy;
    if (cs) *cs = c.coeff_scaling;
    if (tf) *tf = c.threshold_factor;
    return SRCDSP_OK;
}

}  // extern "C"
