// upsamp.hip -- dsptl::FilterUpsamplingFir<In,Out,Internal,Coef,L>
// (upsampling_filters.h:36-326) on gfx950.
//
// Polyphase interpolation restated per output: input sample j produces L
// outputs  y[L j + o] = sum_{i=0}^{H-1} c[o + iL] * x[j - i],  H = ntaps / L,
// x[<0] from the H-1 sample history, then limitScale<Out>(y, shift) with the
// ASYMMETRIC int16 clamp (dsp_complex.h:83-108).  The vector overload of
// step() shifts by 15 - round(log2 L) (:120,189), the iterator overload by 0
// (:244).  flush appends length/L zero inputs (:196), `length` excluding the
// trailing zero taps (:121-123).  Integer arithmetic wraps modulo 2^32, so the
// tap order is free: the polyphase taps of each phase are kept contiguous in
// LDS (c_o[i] = c[o + iL]) and one lane computes the L phases of one input
// sample from a register copy of its H-sample window.
#include <algorithm>
#include <string>
#include <vector>

#include "ops.h"

namespace srcdsp {

enum { UV_CI16_I32 = 0, UV_CI16_I16 = 1, UV_I16_I32 = 2 };
typedef short short2_t_u __attribute__((ext_vector_type(2)));

struct srcdsp_up_state {
    int variant = 0;
    unsigned L = 1;
    int ntaps = 0, H = 0;
    unsigned length = 0;
    int left_shift_factor = 0;
    std::string h_raw;          // the taps as given (CoefType bytes), for copies
    int32_t *d_coef = nullptr;  // polyphase order: d_coef[o*H + i] = c[o + i*L]
    bool coef_i24 = false;      // every tap in (-2^23, 2^23): v_mad_i32_i24
    bool coef_i16 = false;      // every tap in int16 range: v_dot2 tap pairs (variant 0)
    uint32_t *d_pair = nullptr; // per phase o: pairs[o*(H/2+1) + p] = (lo c_o[2p], hi c_o[2p-1])
    void *d_hist[2] = {nullptr, nullptr};
    size_t hist_cap = 0;
    int cur = 0;
    Ordering order;
    HostStage stage;
};

template <int UV>
__device__ __forceinline__ void up_mac(uint32_t &yr, uint32_t &yi, int32_t c, uint32_t w) {
    if constexpr (UV == UV_I16_I32) {
        yr += (uint32_t)c * (uint32_t)sext16(w);
    } else if constexpr (UV == UV_CI16_I16) {  // std::operator*(short, complex<short>): int16 wrap
        yr += (uint32_t)sext16((uint32_t)c * (uint32_t)sext16(w));
        yi += (uint32_t)sext16((uint32_t)c * (uint32_t)sext16_hi(w));
    } else {  // ::operator*(complex<int32_t>(c,0), complex<int16_t>) (dsp_complex.cpp:23-29)
        yr += (uint32_t)c * (uint32_t)sext16(w);
        yi += (uint32_t)c * (uint32_t)sext16_hi(w);
    }
}

// sample j of the virtual stream (history ++ input ++ flush zeros), as a packed word
template <int UV>
__device__ __forceinline__ uint32_t up_fetch(const void *in, const void *hist, long j, long n_in, int Hm1) {
    if (j < 0) {
        long h = j + Hm1;
        if (h < 0) return 0;
        return UV == UV_I16_I32 ? (uint32_t)(uint16_t)((const int16_t *)hist)[h] : ((const uint32_t *)hist)[h];
    }
    if (j >= n_in) return 0;
    return UV == UV_I16_I32 ? (uint32_t)(uint16_t)((const int16_t *)in)[j] : ((const uint32_t *)in)[j];
}

template <int UV, bool LDS = true>
__global__ __launch_bounds__(256) void up_kernel(const void *in, long n_in, long n_total, const void *hist_in,
                                                 void *hist_out, const int32_t *coef, int H, unsigned L,
                                                 unsigned shift, void *out) {
    // L*H polyphase taps: staged in LDS, or (!LDS: past kUpKernelMaxSmem) read
    // through the cache, wave-uniform
    extern __shared__ int32_t sc_lds[];
    if constexpr (LDS) {
        for (int i = threadIdx.x; i < (int)(L * H); i += blockDim.x) sc_lds[i] = coef[i];
        __syncthreads();
    }
    const int32_t *sc = LDS ? sc_lds : coef;
    const int Hm1 = H - 1;
    if (blockIdx.x == 0) {  // new history: last H-1 samples of the virtual stream
        for (int k = threadIdx.x; k < Hm1; k += blockDim.x) {
            long j = n_total - Hm1 + k;
            uint32_t w = up_fetch<UV>(in, hist_in, j, n_in, Hm1);
            if (UV == UV_I16_I32) ((int16_t *)hist_out)[k] = (int16_t)w;
            else ((uint32_t *)hist_out)[k] = w;
        }
    }
    for (long j = (long)blockIdx.x * blockDim.x + threadIdx.x; j < n_total; j += (long)gridDim.x * blockDim.x) {
        for (unsigned o = 0; o < L; ++o) {
            uint32_t yr = 0, yi = 0;
            const int32_t *c = sc + o * H;
            for (int i = 0; i < H; ++i) up_mac<UV>(yr, yi, c[i], up_fetch<UV>(in, hist_in, j - i, n_in, Hm1));
            const long oi = (long)L * j + o;
            if (UV == UV_I16_I32) ((int16_t *)out)[oi] = (int16_t)limit_t16((int32_t)yr, shift);
            else ((uint32_t *)out)[oi] = limit_t16_pair((int32_t)yr, (int32_t)yi, shift);
        }
    }
}

// Tiled polyphase interpolator for complex<int16_t> input (UV_CI16_I32 /
// UV_CI16_I16), ratio LR in {2, 4, 8} (template), H = ntaps / L taps per phase
// (runtime).  Each lane owns R = 4 consecutive input samples (4L outputs) and
// keeps a 8-sample register window as two 4-sample blocks lo|hi that rotate
// roles every 4 taps (tap i of input r reads sample r - i); the L phases share
// each window sample.  Taps are wave-uniform SGPR operands (polyphase order:
// coef[o*H + i]).  The tile's input span (1024 samples + H-1 halo rounded to
// 4) is staged through LDS as packed words; lanes read whole 16-B granules at
// granule stride 1 (conflict-free).  Products: v_mad_i32_i24 when the host
// has checked |c| < 2^23 (I24), exact 32-bit multiply otherwise; the int16
// variant wraps each product to int16 (std::operator*, UV_CI16_I16).
constexpr int kUpR = 4, kUpBlock = 256, kUpMaxTaps = 4096;
constexpr size_t kUpKernelMaxSmem = 64 * 1024;  // up_kernel's taps in LDS; longer filters read them through the cache

template <int UV, int LR, bool I24>
__global__ __launch_bounds__(kUpBlock) void up_tile(const uint32_t *in, long n_in, long n_total,
                                                    const uint32_t *hist_in, uint32_t *hist_out,
                                                    const int32_t *coef, int H, unsigned shift, uint32_t *out) {
    constexpr int R = kUpR, TI = R * kUpBlock;
    extern __shared__ uint4 ug[];
    const int Hm1 = H - 1;
    const int NQ = (H + 3) / 4;
    const int P0 = 4 * NQ;  // halo samples staged in front of the tile (>= H-1, block aligned)
    const int t = threadIdx.x;
    if (blockIdx.x == 0) {
        for (int k = t; k < Hm1; k += kUpBlock) {
            const long j = n_total - Hm1 + k;
            hist_out[k] = up_fetch<UV>(in, hist_in, j, n_in, Hm1);
        }
    }
    const long j0 = (long)blockIdx.x * TI;
    const int ng = (TI + P0) / 4;
    for (int g = t; g < ng; g += kUpBlock) {
        const long s0 = j0 - P0 + 4L * g;
        uint4 v;
        if (s0 >= 0 && s0 + 4 <= n_in) {
            v = *(const uint4 *)(in + s0);
        } else {
            v = make_uint4(up_fetch<UV>(in, hist_in, s0, n_in, Hm1), up_fetch<UV>(in, hist_in, s0 + 1, n_in, Hm1),
                           up_fetch<UV>(in, hist_in, s0 + 2, n_in, Hm1), up_fetch<UV>(in, hist_in, s0 + 3, n_in, Hm1));
        }
        ug[g] = v;
    }
    __syncthreads();
    const int gb = NQ + t;  // lane's first granule (sample P0 + 4t)
    int32_t xr_lo[4], xi_lo[4], xr_hi[4], xi_hi[4];
    auto fill = [&](int32_t (&dr)[4], int32_t (&di)[4], int c) {
        const uint4 v = ug[gb + c];
        dr[0] = sext16(v.x); di[0] = sext16_hi(v.x);
        dr[1] = sext16(v.y); di[1] = sext16_hi(v.y);
        dr[2] = sext16(v.z); di[2] = sext16_hi(v.z);
        dr[3] = sext16(v.w); di[3] = sext16_hi(v.w);
    };
    uint32_t yr[LR][R], yi[LR][R];
#pragma unroll
    for (int o = 0; o < LR; ++o)
#pragma unroll
        for (int r = 0; r < R; ++r) yr[o][r] = yi[o][r] = 0;
    ConstPtr<int32_t> tp = const_view<int32_t>(coef);
    auto mac = [&](int32_t c, int32_t x) -> uint32_t {
        uint32_t p = I24 ? (uint32_t)__mul24(c, x) : (uint32_t)c * (uint32_t)x;
        if constexpr (UV == UV_CI16_I16) p = (uint32_t)sext16(p);
        return p;
    };
    // chunk q (taps 4q..4q+3): input r reads sample r - i, i.e. block lo
    // (samples -4q-4..-4q-1) or hi (-4q..-4q+3)
    auto chunk = [&](int q, const int32_t (&lr)[4], const int32_t (&li)[4], const int32_t (&hr)[4],
                     const int32_t (&hi)[4], bool guard) {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int i = 4 * q + p;
            if (guard && i >= H) break;
            int32_t c[LR];
#pragma unroll
            for (int o = 0; o < LR; ++o) c[o] = tp[o * H + i];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int rel = r - p + 4;  // 1..7 over lo|hi
                const int32_t xr = rel < 4 ? lr[rel] : hr[rel - 4];
                const int32_t xi = rel < 4 ? li[rel] : hi[rel - 4];
#pragma unroll
                for (int o = 0; o < LR; ++o) {
                    yr[o][r] += mac(c[o], xr);
                    yi[o][r] += mac(c[o], xi);
                }
            }
        }
    };
    int32_t ar[4], ai[4], br[4], bi[4];
    fill(br, bi, 0);  // hi block of chunk 0
    int q = 0;
    for (; q + 2 <= NQ; q += 2) {
        asm volatile("" : "+s"(tp));
        fill(ar, ai, -q - 1);
        chunk(q, ar, ai, br, bi, false);
        fill(br, bi, -q - 2);
        chunk(q + 1, br, bi, ar, ai, q + 2 == NQ);
    }
    if (q < NQ) {
        fill(ar, ai, -q - 1);
        chunk(q, ar, ai, br, bi, true);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const long j = j0 + 4L * t + r;
        if (j >= n_total) break;
        uint32_t w[LR];
#pragma unroll
        for (int o = 0; o < LR; ++o) w[o] = limit_t16_pair((int32_t)yr[o][r], (int32_t)yi[o][r], shift);
        uint32_t *dst = out + (long)LR * j;
#pragma unroll
        for (int o = 0; o < LR; o += 2) *(uint2 *)(dst + o) = make_uint2(w[o], w[o + 1]);
    }
}

// Tiled polyphase interpolator on v_dot2_i32_i16 (variant 0 with int16-range
// taps, LR in {2, 4}).  Each lane owns RD = 8 consecutive input samples.  Taps
// of phase o are paired Q_p = (lo c_o[2p+1], hi c_o[2p]) (c_o[H] = 0), p <
// ceil(H/2); the pair of input j multiplies the packed samples (x[j-2p-1],
// x[j-2p]), which for even j = 2m is dword m-p-1 of an odd-aligned plane
// O[e] = (x[2e+1], x[2e+2]) and for odd j = 2m+1 dword m-p of an even-aligned
// plane E[e] = (x[2e], x[2e+1]).  A lane's 8 inputs read O[4t'+r/2-1-p] (even
// r) / E[4t'+(r-1)/2-p] (odd r): one 4-dword register window per plane and
// component sliding one dword per pair, one ds_read_b128 per plane every 4
// pairs.  ceil(H/2) dot2 per phase and component (the (c[2p], c[2p-1])
// pairing needed H/2 + 1).  int16 x int16 -> int32 products, wrap-around
// accumulate: exactly the reference's complex<int32_t> arithmetic.
constexpr int kUpRD = 8, kUpBlockD = 256;

// WS: window register sets (3: the next granule is read a chunk ahead, 150
// VGPRs at LR = 4; 2: it is read at the end of the chunk into the set that
// chunk is done with, <= 128 VGPRs -> 4 waves per SIMD); MINW as launch bound
// PPC: pairs per phase as a compile-time constant (0: runtime, from H): the
// chunk loop unrolls completely, the window sets rotate without register
// copies and each accumulator starts with a dot2 into an inline 0.
template <int LR, bool NTS = false, int WS = 3, int MINW = 1, int PPC = 0>
__global__ __launch_bounds__(kUpBlockD, MINW) void up_tile_dot2(const uint32_t *in, long n_in, long n_total,
                                                         const uint32_t *hist_in, uint32_t *hist_out,
                                                         const uint32_t *pairs, int H, unsigned shift, uint32_t *out) {
    constexpr int R = kUpRD, TI = R * kUpBlockD;
    extern __shared__ uint4 ug[];  // 4 planes (E_re, E_im, O_re, O_im) of PGR granules each
    const int Hm1 = H - 1;
    const int PP = PPC ? PPC : (H + 1) / 2;  // pairs per phase
    const int HG = (PP + 3) / 4;         // halo granules per plane (window reach: dword D0 - PP)
    const int PGR = TI / 8 + HG;         // granules per plane (4 dwords = 8 samples)
    const int t = threadIdx.x;
    if (blockIdx.x == 0) {
        for (int k = t; k < Hm1; k += kUpBlockD) {
            const long j = n_total - Hm1 + k;
            hist_out[k] = up_fetch<UV_CI16_I32>(in, hist_in, j, n_in, Hm1);
        }
    }
    const long j0 = (long)blockIdx.x * TI;
    // staging: sample granule g (4 samples from j0 - 8*HG + 4g) -> plane dwords 2g, 2g+1
    uint32_t *pl = (uint32_t *)ug;
    const int PDW = 4 * PGR;  // dwords per plane
    const int ng = 2 * PGR;
    auto lo = [](uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x05040100u); };
    auto hi = [](uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x07060302u); };
    auto put = [&](int g, const uint32_t (&w)[5]) {
        *(uint2 *)&pl[0 * PDW + 2 * g] = make_uint2(lo(w[0], w[1]), lo(w[2], w[3]));
        *(uint2 *)&pl[1 * PDW + 2 * g] = make_uint2(hi(w[0], w[1]), hi(w[2], w[3]));
        *(uint2 *)&pl[2 * PDW + 2 * g] = make_uint2(lo(w[1], w[2]), lo(w[3], w[4]));
        *(uint2 *)&pl[3 * PDW + 2 * g] = make_uint2(hi(w[1], w[2]), hi(w[3], w[4]));
    };
    // a tile whose whole span (halo included) lies inside the input: the
    // lane's first three granules are loaded together, then written (one
    // exposed load latency per tile instead of one per granule)
    constexpr int NI = 3;
    const bool interior = j0 - 8L * HG >= 0 && j0 + TI + 1 <= n_in;
    int g1 = t;  // first granule of the generic loop
    if (interior) {
        uint32_t w[NI][5];
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int g = t + i * kUpBlockD;
            if (i < 2 || g < ng) {  // ng >= 2 * kUpBlockD
                const long s0 = j0 - 8L * HG + 4L * g;
                const uint4 v = *(const uint4 *)(in + s0);
                w[i][0] = v.x; w[i][1] = v.y; w[i][2] = v.z; w[i][3] = v.w;
                w[i][4] = in[s0 + 4];
            }
        }
#pragma unroll
        for (int i = 0; i < NI; ++i)
            if (i < 2 || t + i * kUpBlockD < ng) put(t + i * kUpBlockD, w[i]);
        g1 = t + NI * kUpBlockD;
    }
    for (int g = g1; g < ng; g += kUpBlockD) {
        const long s0 = j0 - 8L * HG + 4L * g;
        uint32_t w[5];
        if (s0 >= 0 && s0 + 5 <= n_in) {
            const uint4 v = *(const uint4 *)(in + s0);
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
            w[4] = in[s0 + 4];
        } else {
#pragma unroll
            for (int k = 0; k < 5; ++k) w[k] = up_fetch<UV_CI16_I32>(in, hist_in, s0 + k, n_in, Hm1);
        }
        put(g, w);
    }
    __syncthreads();
    // lane base: input j0 + 8t = plane dword D0 = 4t + 4*HG (granule gb).  Input
    // r, pair p reads dword D0 + k - p, k = r/2 - 1 in plane O for even r,
    // k = (r-1)/2 in plane E for odd r:
    // for the chunk of pairs 4q..4q+3 those are dwords of granules gb - q
    // (`cur`) and gb - q - 1 (`nxt`), two register sets that swap roles.
    const int gb = t + HG;
    int32_t yr[LR][R], yi[LR][R];
    if constexpr (PPC == 0) {
#pragma unroll
        for (int o = 0; o < LR; ++o)
#pragma unroll
            for (int r = 0; r < R; ++r) yr[o][r] = yi[o][r] = 0;
    }
    ConstPtr<uint32_t> tp = const_view<uint32_t>(pairs);
    // Three window register sets rotate over the chunks and the taps of a
    // chunk (4 pairs x LR phases, contiguous: dword (4q + pp) LR + o) arrive in
    // one s_load; both for chunk q+1 are requested after chunk q's first pair,
    // so the lgkmcnt wait at chunk q+1 lands three pairs of dot2 after them
    // (waiting on a tap s_load drains every LDS read in flight too).
    uint32_t W0[4][4], W1[4][4], W2[4][4];  // [plane][dword]
    constexpr int TPC = 4 * LR;            // tap dwords per chunk
    uint32_t Tc[TPC], Tn[TPC];
    auto load = [&](uint32_t (&w)[4][4], int gi) {
#pragma unroll
        for (int pl4 = 0; pl4 < 4; ++pl4) {
            typedef uint32_t u4v_t __attribute__((ext_vector_type(4)));
            // volatile keeps every window read a whole ds_read_b128
            // (conflict-free at the lanes' 16-B stride): at the window's far end
            // the compiler would read only the dwords used, as ds_read_b32 /
            // ds_read2_b32, whose 32-lane groups at a 16-B stride hit 8 banks
            typedef const volatile __attribute__((address_space(3))) u4v_t *lds_u4v;
            const u4v_t v = *(lds_u4v)(&ug[pl4 * PGR + gi]);
            w[pl4][0] = v[0]; w[pl4][1] = v[1]; w[pl4][2] = v[2]; w[pl4][3] = v[3];
        }
    };
    auto load_taps = [&](uint32_t (&T)[TPC], int q) {
        asm volatile("" : "+s"(tp));
#pragma unroll
        for (int i = 0; i < TPC; ++i) T[i] = tp[q * TPC + i];
    };
    const int NQ = (PP + 3) / 4;
    auto chunk = [&](int q, const uint32_t (&cur)[4][4], const uint32_t (&nxt)[4][4], uint32_t (&nn)[4][4]) {
#pragma unroll
        for (int pp = 0; pp < 4; ++pp) {
            const int p = 4 * q + pp;
            if (p >= PP) break;  // the last chunk only
            if (WS == 3 && pp == 1 && q + 1 < NQ) {
                load(nn, gb - q - 2);
                load_taps(Tn, q + 1);
            }
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int k = (r & 1) ? (r >> 1) : (r >> 1) - 1, rel = k - pp;  // -4..3
                const int pr = (r & 1) ? 0 : 2, pi = pr + 1;  // planes E_re/E_im or O_re/O_im
                const uint32_t xr = rel >= 0 ? cur[pr][rel] : nxt[pr][rel + 4];
                const uint32_t xi = rel >= 0 ? cur[pi][rel] : nxt[pi][rel + 4];
#pragma unroll
                for (int o = 0; o < LR; ++o) {
                    const uint32_t P = Tc[pp * LR + o];
                    if (PPC && q == 0 && pp == 0) {  // first pair: into an inline 0
                        asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(yr[o][r]) : "v"(xr), "s"(P));
                        asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(yi[o][r]) : "v"(xi), "s"(P));
                    } else {
                        yr[o][r] = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t_u, xr),
                                                          __builtin_bit_cast(short2_t_u, P), yr[o][r], false);
                        yi[o][r] = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t_u, xi),
                                                          __builtin_bit_cast(short2_t_u, P), yi[o][r], false);
                    }
                }
            }
        }
        if constexpr (WS == 3) {
#pragma unroll
            for (int i = 0; i < TPC; ++i) Tc[i] = Tn[i];
        }
    };
    load(W0, gb);
    load(W1, gb - 1);
    load_taps(Tc, 0);
    int q = 0;
    if constexpr (WS == 3) {
#pragma unroll
        for (; q + 3 <= NQ; q += 3) {
            chunk(q, W0, W1, W2);
            chunk(q + 1, W1, W2, W0);
            chunk(q + 2, W2, W0, W1);
        }
        if (q < NQ) chunk(q, W0, W1, W2);
        if (q + 1 < NQ) chunk(q + 1, W1, W2, W0);
    } else {
        // chunk q reads granules gb-q (cur) and gb-q-1 (nxt); the next chunk's
        // new granule gb-q-2 goes into cur once this chunk is done with it
        (void)W2;
        auto chunk2 = [&](int qq, uint32_t (&cur)[4][4], const uint32_t (&nxt)[4][4]) {
            uint32_t none[4][4];
            chunk(qq, cur, nxt, none);  // no early read (nn unused when WS == 2)
            if (qq + 1 < NQ) {
                load(cur, gb - qq - 2);
                load_taps(Tc, qq + 1);
            }
        };
#pragma unroll
        for (; q + 2 <= NQ; q += 2) {
            chunk2(q, W0, W1);
            chunk2(q + 1, W1, W0);
        }
        if (q < NQ) chunk2(q, W0, W1);
    }
    // outputs -> LDS (lane chunk of 8*LR words at a 9-granule stride for LR = 4,
    // conflict-free) -> whole-line 16-B stores of the tile's contiguous output
    constexpr int GPLo = R * LR / 4;    // output granules per lane
    constexpr int STR = GPLo + 1;       // padded lane stride (odd)
    // (each lane storing its own 128-B output line directly, 8 x 16 B at a
    // 128-B lane stride, measured 30 % slower with plain stores and 5.5x
    // slower with nt stores than this LDS transpose into whole-line stores:
    // profiles/tuning/r03_up_stage_ab.txt)
    __syncthreads();                    // every wave is done reading the planes
    uint4 *ob = ug;
#pragma unroll
    for (int k = 0; k < GPLo; ++k) {
        uint32_t w4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int idx = 4 * k + u, r = idx / LR, o = idx % LR;
            w4[u] = limit_t16_pair(yr[o][r], yi[o][r], shift);
        }
        ob[t * STR + k] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
    }
    __syncthreads();
    const long wbase = (long)LR * j0;             // first output word of the tile
    const long wend = (long)LR * n_total;         // output words of the call
    // one whole ds_read_b128 per granule (volatile: the compiler split these
    // reads into ds_read_b32 / ds_read2_b32 for the partial-tile branch, whose
    // 32-lane groups at a 16-B stride hit 8 banks: 25 M conflict cycles per
    // launch at L = 4, 2^26 inputs)
    typedef uint32_t o4v_t __attribute__((ext_vector_type(4)));
    typedef const volatile __attribute__((address_space(3))) o4v_t *lds_o4v;
    auto oread = [&](int G) { return *(lds_o4v)(&ob[(G / GPLo) * STR + (G % GPLo)]); };
    if (wbase + 4L * GPLo * kUpBlockD <= wend) {
        // whole tile: every granule read, then every store issued, at one
        // base address (no per-store range checks)
        o4v_t v[GPLo];
#pragma unroll
        for (int i = 0; i < GPLo; ++i) v[i] = oread(i * kUpBlockD + t);
        uint32_t *o = out + wbase + 4L * t;
#pragma unroll
        for (int i = 0; i < GPLo; ++i) {
            if constexpr (NTS) {  // streaming store: the output is written once, 4L x the input bytes
                __builtin_nontemporal_store(v[i], (o4v_t *)(o + 4 * i * kUpBlockD));
            } else {
                *(o4v_t *)(o + 4 * i * kUpBlockD) = v[i];
            }
        }
        return;
    }
    for (int i = 0; i < GPLo; ++i) {  // the call's last, partial tile
        const int G = i * kUpBlockD + t;          // output granule within the tile
        const o4v_t vv4 = oread(G);
        const long w0 = wbase + 4L * G;
        for (int u = 0; u < 4; ++u)
            if (w0 + u < wend) out[w0 + u] = vv4[u];
    }
}

static int in_bytes(int v) { return v == UV_I16_I32 ? 2 : 4; }

static int up_set(srcdsp_up_state &u, const void *coeffs, int n) {
    SRCDSP_ARG_CHECK(coeffs != nullptr && n >= 1, "setCoefficients: empty coefficient vector (upsampling_filters.h:110)");
    if (n % (int)u.L) {
        set_error("setCoefficients: number of taps must be a multiple of L (upsampling_filters.h:113)");
        return SRCDSP_ERR_SIZE;
    }
    int rc = u.order.sync();
    if (rc) return rc;
    std::vector<int32_t> c(n);
    for (int i = 0; i < n; ++i)
        c[i] = u.variant == UV_CI16_I16 ? ((const int16_t *)coeffs)[i] : ((const int32_t *)coeffs)[i];
    unsigned len = (unsigned)n;
    while (len > 0 && c[len - 1] == 0) --len;  // :121-123
    if (len == 0) {
        set_error("setCoefficients: all taps are zero (the reference reads coeff[-1])");
        return SRCDSP_ERR_ARG;
    }
    const int H = n / (int)u.L;
    u.coef_i24 = true;
    u.coef_i16 = u.variant == UV_CI16_I32;
    for (int i = 0; i < n; ++i) {
        u.coef_i24 = u.coef_i24 && c[i] < (1 << 23) && c[i] >= -(1 << 23);
        u.coef_i16 = u.coef_i16 && c[i] <= 32767 && c[i] >= -32768;
    }
    std::vector<int32_t> poly((size_t)n);
    for (unsigned o = 0; o < u.L; ++o)
        for (int i = 0; i < H; ++i) poly[o * H + i] = c[o + i * u.L];
    if (u.d_coef) (void)hipFree(u.d_coef);
    u.d_coef = nullptr;
    SRCDSP_HIP_TRY(hipMalloc(&u.d_coef, 4 * (size_t)n));
    SRCDSP_HIP_TRY(hipMemcpy(u.d_coef, poly.data(), 4 * (size_t)n, hipMemcpyHostToDevice));
    if (u.d_pair) (void)hipFree(u.d_pair);
    u.d_pair = nullptr;
    if (u.coef_i16) {  // tap pairs of each phase: (lo c_o[2p], hi c_o[2p-1]), c_o[-1] = c_o[H] = 0
        // chunk-major for up_tile_dot2: the 4 pairs x L phases of chunk q are
        // the contiguous dwords [4qL, 4(q+1)L), pair p of phase o at p L + o,
        // zero-padded to whole chunks; pair p = (lo c_o[2p+1], hi c_o[2p])
        const int Hh = n / (int)u.L, PP = (Hh + 1) / 2, NQ = (PP + 3) / 4;
        std::vector<uint32_t> pr((size_t)u.L * 4 * NQ, 0u);
        auto tap = [&](unsigned o, int i) {
            return (i >= 0 && i < Hh) ? (uint32_t)(uint16_t)(int16_t)c[o + (size_t)i * u.L] : 0u;
        };
        for (unsigned o = 0; o < u.L; ++o)
            for (int q = 0; q < PP; ++q) pr[(size_t)q * u.L + o] = tap(o, 2 * q + 1) | (tap(o, 2 * q) << 16);
        SRCDSP_HIP_TRY(hipMalloc(&u.d_pair, 4 * pr.size()));
        SRCDSP_HIP_TRY(hipMemcpy(u.d_pair, pr.data(), 4 * pr.size(), hipMemcpyHostToDevice));
    }
    // buffer.resize(N/L) (:117) keeps the first entries of the ring; a new
    // coefficient set starts from a cleared history here (documented deviation
    // only when H changes and the ring was not reset).
    const size_t hb = (size_t)std::max(1, H - 1) * in_bytes(u.variant);
    for (int b = 0; b < 2; ++b) {
        if (u.d_hist[b]) (void)hipFree(u.d_hist[b]);
        u.d_hist[b] = nullptr;
        SRCDSP_HIP_TRY(hipMalloc(&u.d_hist[b], hb));
        SRCDSP_HIP_TRY(hipMemset(u.d_hist[b], 0, hb));
    }
    u.hist_cap = hb;
    u.cur = 0;
    u.ntaps = n;
    u.H = H;
    u.length = len;
    u.left_shift_factor = (int)std::round(std::log2((double)u.L));  // :119
    u.h_raw.assign((const char *)coeffs, (size_t)n * (u.variant == UV_CI16_I16 ? 2 : 4));
    return SRCDSP_OK;
}

static int up_launch(srcdsp_up_state &u, const void *d_in, size_t n_in, void *d_out, size_t n_out, bool flush,
                     bool iter, hipStream_t s) {
    const long extra = flush ? (long)(u.length / u.L) : 0;
    const size_t need = (size_t)u.L * (n_in + extra);
    if (flush ? n_out < need : n_out != need) {
        set_error("up_step: output must hold L*in.size() samples (+ L*(length/L) when flushing) "
                  "(upsampling_filters.h:152)");
        return SRCDSP_ERR_SIZE;
    }
    const long n_total = (long)n_in + extra;
    if (n_total == 0) return SRCDSP_OK;
    SRCDSP_ARG_CHECK(d_out && (d_in || n_in == 0), "up_step: null buffer");
    int rc = u.order.before(s);
    if (rc) return rc;
    const unsigned shift = iter ? 0u : (unsigned)(15 - u.left_shift_factor);
    const void *hin0 = u.d_hist[u.cur];
    void *hout0 = u.d_hist[u.cur ^ 1];
    const bool tiled = u.variant != UV_I16_I32 && (u.L == 2 || u.L == 4 || u.L == 8) && u.ntaps <= kUpMaxTaps &&
                       ((uintptr_t)d_in & 15u) == 0 && ((uintptr_t)d_out & 7u) == 0;
    const bool dot2_l = u.L >= 2 && u.L <= 8;  // up_tile_dot2: LR in 2..8
    if (u.variant == UV_CI16_I32 && u.coef_i16 && dot2_l && u.ntaps <= kUpMaxTaps && ((uintptr_t)d_in & 15u) == 0 &&
        ((uintptr_t)d_out & 15u) == 0) {
        constexpr int TI = kUpRD * kUpBlockD;
        const int PP = (u.H + 1) / 2, HG = (PP + 3) / 4, PGR = TI / 8 + HG;
        const size_t out_lds = 16 * (size_t)kUpBlockD * (kUpRD * u.L / 4 + 1);  // staged output tile
        const size_t smem = std::max(4 * 16 * (size_t)PGR, out_lds);
        const dim3 grid((unsigned)((n_total + TI - 1) / TI));
        // non-temporal output stores: 0.414 -> 0.385 ms at L = 4, 128 taps, 2^26 inputs
#define SRCDSP_UP_DOT2(LR)                                                                                        \
    hipLaunchKernelGGL((up_tile_dot2<LR, true, WSV, MW, PPV>), grid, dim3(kUpBlockD), smem, s, (const uint32_t *)d_in, (long)n_in, \
                       n_total, (const uint32_t *)hin0, (uint32_t *)hout0, u.d_pair, u.H, shift, (uint32_t *)d_out)
        // 16, 32 or 64 taps per phase (L = 4 x 64 / 128 / 256 taps, L = 2 x 32 /
        // 64 / 128): compile-time shapes
#define SRCDSP_UP_PP(LR, P)                              \
    if (u.L == LR && PP == P) {                          \
        constexpr int WSV = 3, MW = 1, PPV = P;          \
        SRCDSP_UP_DOT2(LR);                              \
    } else
        SRCDSP_UP_PP(2, 8)
        SRCDSP_UP_PP(2, 16)
        SRCDSP_UP_PP(2, 32)
        SRCDSP_UP_PP(4, 8)
        SRCDSP_UP_PP(4, 16)
        SRCDSP_UP_PP(4, 32)
        SRCDSP_UP_PP(8, 8)
        SRCDSP_UP_PP(8, 16)
#undef SRCDSP_UP_PP
        if (u.L == 2) {
            constexpr int WSV = 3, MW = 1, PPV = 0;
            SRCDSP_UP_DOT2(2);
        } else {
            constexpr int WSV = 3, MW = 1, PPV = 0;
            switch (u.L) {
            case 3: SRCDSP_UP_DOT2(3); break;
            case 4: SRCDSP_UP_DOT2(4); break;
            case 5: SRCDSP_UP_DOT2(5); break;
            case 6: SRCDSP_UP_DOT2(6); break;
            case 7: SRCDSP_UP_DOT2(7); break;
            default: SRCDSP_UP_DOT2(8); break;
            }
        }
#undef SRCDSP_UP_DOT2
        SRCDSP_HIP_TRY(hipGetLastError());
        u.cur ^= 1;
        return u.order.after(s);
    }
    if (tiled) {
        constexpr int TI = kUpR * kUpBlock;
        const int NQ = (u.H + 3) / 4;
        const size_t smem = 16 * (size_t)((TI + 4 * NQ) / 4);
        const dim3 grid((unsigned)((n_total + TI - 1) / TI));
        const uint32_t *i32 = (const uint32_t *)d_in;
        const uint32_t *h32 = (const uint32_t *)hin0;
        uint32_t *ho32 = (uint32_t *)hout0, *o32 = (uint32_t *)d_out;
#define SRCDSP_UP_TILE(UVV, LL, I24)                                                                             \
    hipLaunchKernelGGL((up_tile<UVV, LL, I24>), grid, dim3(kUpBlock), smem, s, i32, (long)n_in, n_total, h32, ho32, \
                       u.d_coef, u.H, shift, o32)
#define SRCDSP_UP_L(UVV, I24)                 \
    switch (u.L) {                             \
    case 2: SRCDSP_UP_TILE(UVV, 2, I24); break; \
    case 4: SRCDSP_UP_TILE(UVV, 4, I24); break; \
    default: SRCDSP_UP_TILE(UVV, 8, I24); break; \
    }
        if (u.variant == UV_CI16_I16) {
            SRCDSP_UP_L(UV_CI16_I16, true)  // int16 taps always fit i24
        } else if (u.coef_i24) {
            SRCDSP_UP_L(UV_CI16_I32, true)
        } else {
            SRCDSP_UP_L(UV_CI16_I32, false)
        }
#undef SRCDSP_UP_L
#undef SRCDSP_UP_TILE
        SRCDSP_HIP_TRY(hipGetLastError());
        u.cur ^= 1;
        return u.order.after(s);
    }
    const int blocks = (int)std::max<long>(1, std::min<long>((n_total + 255) / 256, 4096));
    const size_t smem = 4 * (size_t)u.ntaps;
    const void *hin = u.d_hist[u.cur];
    void *hout = u.d_hist[u.cur ^ 1];
#define SRCDSP_UP_GENERIC(UVV)                                                                                      \
    if (smem <= kUpKernelMaxSmem)                                                                                   \
        hipLaunchKernelGGL((up_kernel<UVV, true>), dim3(blocks), dim3(256), smem, s, d_in, (long)n_in, n_total, hin, \
                           hout, u.d_coef, u.H, u.L, shift, d_out);                                                \
    else                                                                                                            \
        hipLaunchKernelGGL((up_kernel<UVV, false>), dim3(blocks), dim3(256), 0, s, d_in, (long)n_in, n_total, hin,  \
                           hout, u.d_coef, u.H, u.L, shift, d_out);
    switch (u.variant) {
    case UV_CI16_I32: SRCDSP_UP_GENERIC(UV_CI16_I32) break;
    case UV_CI16_I16: SRCDSP_UP_GENERIC(UV_CI16_I16) break;
    default: SRCDSP_UP_GENERIC(UV_I16_I32) break;
    }
#undef SRCDSP_UP_GENERIC
    SRCDSP_HIP_TRY(hipGetLastError());
    u.cur ^= 1;
    return u.order.after(s);
}

}  // namespace srcdsp

using namespace srcdsp;
struct srcdsp_up { srcdsp_up_state u; };

extern "C" {

SRCDSP_API int srcdsp_up_create(srcdsp_up_t *out, int variant, unsigned L, const void *coeffs, int ntaps) {
    SRCDSP_ARG_CHECK(out != nullptr, "up_create: null out");
    *out = nullptr;
    if (variant < 0 || variant > 2) {
        set_error("up_create: variant must be 0..2");
        return SRCDSP_ERR_UNSUPPORTED;
    }
    SRCDSP_ARG_CHECK(L >= 1, "up_create: L must be >= 1");
    auto *h = new srcdsp_up();
    h->u.variant = variant;
    h->u.L = L;
    int rc = h->u.order.init();
    if (!rc) rc = h->u.stage.init();
    if (!rc) rc = up_set(h->u, coeffs, ntaps);
    if (rc) {
        srcdsp_up_destroy(h);
        return rc;
    }
    *out = h;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_up_destroy(srcdsp_up_t h) {
    if (!h) return SRCDSP_OK;
    (void)h->u.order.sync();
    if (h->u.d_coef) (void)hipFree(h->u.d_coef);
    if (h->u.d_pair) (void)hipFree(h->u.d_pair);
    for (int b = 0; b < 2; ++b)
        if (h->u.d_hist[b]) (void)hipFree(h->u.d_hist[b]);
    h->u.order.destroy();
    h->u.stage.destroy();
    delete h;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_up_clone(srcdsp_up_t h, srcdsp_up_t *out) {
    SRCDSP_ARG_CHECK(h != nullptr && out != nullptr, "up_clone: null argument");
    *out = nullptr;
    srcdsp_up_state &u = h->u;
    int rc = u.order.sync();
    if (rc) return rc;
    srcdsp_up_t c = nullptr;
    rc = srcdsp_up_create(&c, u.variant, u.L, u.h_raw.data(), u.ntaps);
    if (rc) return rc;
    if (hipMemcpy(c->u.d_hist[0], u.d_hist[u.cur], u.hist_cap, hipMemcpyDeviceToDevice) != hipSuccess) {
        srcdsp_up_destroy(c);
        set_error("up_clone: history copy failed");
        return SRCDSP_ERR_HIP;
    }
    c->u.cur = 0;
    *out = c;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_up_set_coeffs(srcdsp_up_t h, const void *coeffs, int ntaps) {
    SRCDSP_ARG_CHECK(h != nullptr, "up_set_coeffs: null handle");
    return up_set(h->u, coeffs, ntaps);
}

SRCDSP_API int srcdsp_up_reset(srcdsp_up_t h) {
    SRCDSP_ARG_CHECK(h != nullptr, "up_reset: null handle");
    int rc = h->u.order.sync();
    if (rc) return rc;
    // on the handle's own stream: no wait on other streams' work
    for (int b = 0; b < 2; ++b) SRCDSP_HIP_TRY(hipMemsetAsync(h->u.d_hist[b], 0, h->u.hist_cap, h->u.stage.stream));
    SRCDSP_HIP_TRY(hipStreamSynchronize(h->u.stage.stream));
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_up_get_length(srcdsp_up_t h, int *length, int *imp_length, int *ratio) {
    SRCDSP_ARG_CHECK(h != nullptr, "up_get_length: null handle");
    if (length) *length = (int)h->u.length;
    if (imp_length) *imp_length = h->u.ntaps;
    if (ratio) *ratio = (int)h->u.L;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_up_step(srcdsp_up_t h, const void *d_in, size_t n_in, void *d_out, size_t n_out, int flush,
                              int iterator, void *stream) {
    SRCDSP_ARG_CHECK(h != nullptr, "up_step: null handle");
    return up_launch(h->u, d_in, n_in, d_out, n_out, flush != 0, iterator != 0, (hipStream_t)stream);
}

SRCDSP_API int srcdsp_up_step_host(srcdsp_up_t h, const void *in, size_t n_in, void *out, size_t n_out, int flush,
                                   int iterator) {
    SRCDSP_ARG_CHECK(h != nullptr, "up_step_host: null handle");
    srcdsp_up_state &u = h->u;
    const size_t eb = in_bytes(u.variant);
    const size_t ib = n_in * eb, ob = n_out * eb, ib_al = (ib + 255) & ~(size_t)255;
    if (n_out == 0 && n_in == 0) return SRCDSP_OK;
    int rc = u.stage.reserve(std::max(ib, ob), ib_al + ob);
    if (rc) return rc;
    hipStream_t s = u.stage.stream;
    char *d_in = (char *)u.stage.d_buf, *d_out = d_in + ib_al;
    if (ib) {
        host_copy(u.stage.h_buf, in, ib);
        SRCDSP_HIP_TRY(hipMemcpyAsync(d_in, u.stage.h_buf, ib, hipMemcpyHostToDevice, s));
    }
    rc = up_launch(u, d_in, n_in, d_out, n_out, flush != 0, iterator != 0, s);
    if (rc) return rc;
    // only the L*(n_in [+ length/L]) written samples go back; a larger caller
    // vector keeps its tail untouched, as with the reference
    const size_t wb = std::min(ob, (size_t)u.L * (n_in + (flush ? u.length / u.L : 0)) * eb);
    SRCDSP_HIP_TRY(hipMemcpyAsync(u.stage.h_buf, d_out, wb, hipMemcpyDeviceToHost, s));
    SRCDSP_HIP_TRY(hipStreamSynchronize(s));
    host_copy(out, u.stage.h_buf, wb);
    return SRCDSP_OK;
}

}  // extern "C"
