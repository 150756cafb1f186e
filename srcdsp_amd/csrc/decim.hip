// decim.hip -- FilterDnsamplingFir (dnsampling_filters.h:49-172,
// dsptl_dnsampling_filters.h:47-220) and FilterFir (filters.h:42-169) on gfx950.
//
// Semantics restated per output n of a step over L input samples:
//   y[n] = sum_{k=0}^{N-1} c[k] * x[nM - k]          (taps in ascending k)
//   out[n] = limitScale16(y[n], coeffScaling - leftShift)
// where x[<0] is the N-1 sample history carried from the previous call.
//
// Kernels (decim_kernels.h)
//  * decim_stream_cf32<NT,R,BLOCK,FMA,MINW,Q0,M> -- the headline path:
//    complex<float>, M = 4, 127 taps (and M = 1/2/3/8/16, any N <= 1024 with
//    NT = 0: the tap count at run time).  A persistent grid of 512-lane
//    workgroups taking tiles of BLOCK*R outputs in grid-stride order.  A
//    tile's input span (4*BLOCK*R samples + the 4*ceil(NT/4) halo) is staged
//    HBM -> VGPR -> LDS (non-temporal buffer_load_dwordx4, padded
//    conflict-free layout) and the NEXT tile's loads are issued before this
//    tile's FMA work.  Each lane owns R consecutive outputs and walks the taps
//    as 4 polyphase register windows that slide one sample per 4 taps; taps
//    are wave-uniform SGPR operands; each output is ONE sequential fma chain
//    in ascending k (FMA) or separately rounded mul+add (!FMA).  Outputs are
//    paired across the two half-waves (v_permlane32_swap) so each store
//    instruction writes 1 KiB of whole lines, non-temporal.
//  * decim_dot2_ci16<NT,BLOCK,MIX,MINW,TAB2> -- complex<int16_t> x int16-range
//    taps on v_dot2 tap pairs over planar int16 LDS images, optionally with
//    the NCO mixer of mixers.h fused into the staging pass (config 4).
//  * decim_stream_ci16<NT,R,BLOCK,MIX,MINW> -- the same for |c| < 2^23 taps
//    (v_mad_i32_i24).
//  * fir_stream_f32 / fir_tile_f32 -- M = 1 (FilterFir) for float input.
//  * decim_generic<KV,FMA> -- any variant / M / N; one output per thread,
//    reads through the cache.  Used for shapes without a tile kernel.
// The new history (last N-1 samples of history ++ input) is written by the
// workgroup that owns tile 0 into the other ping-pong buffer, so a step is one
// launch.
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "ops.h"

#include "decim_kernels.h"

namespace srcdsp {

// ============================================================== dispatch
namespace {
constexpr int kCiR_ = 4, kCiBlock_ = 256;
}
// phase advance of the fused mixer over `samples` input samples (one tile)
unsigned phase_step(unsigned long N, unsigned long fr, unsigned long samples) {
    return (unsigned)((samples % N) * fr % N);
}
namespace {
// cf32 tiles: 4 outputs per lane, 512 lanes -> 8192 input samples per tile,
// 75 KB LDS and 128 VGPRs = 2 resident workgroups (16 waves) per CU; the
// persistent grid is 2x the resident capacity (measured best on MI355X:
// scripts/tune, profiles/).
constexpr int kCfGridCap = 2048;  // persistent grid of the streaming kernels
constexpr int kCiR = 4, kCiBlock = 256;

template <int NT>
int launch_ci16(DecimLaunch L, int channels, bool mixed, hipStream_t s) {
    constexpr int TO = kCiBlock * kCiR;
    L.ntiles = (L.n_out + TO - 1) / TO;
    dim3 grid((unsigned)std::min<long>(L.ntiles, kCfGridCap), channels);
    if (mixed)
        hipLaunchKernelGGL((decim_stream_ci16<NT, kCiR, kCiBlock, true, 4>), grid, dim3(kCiBlock), 0, s, L);
    else
        hipLaunchKernelGGL((decim_stream_ci16<NT, kCiR, kCiBlock, false, 4>), grid, dim3(kCiBlock), 0, s, L);
    return SRCDSP_OK;
}

// dot2 ci16 kernel shape: tile lanes and mixer table form.  The product ships
// one shape (512 lanes, sequence mixer table: measured best, profiles/); a
// tuning build (-DSRCDSP_TUNING, scripts/tune) can pick another with
// SRCDSP_CI16_VARIANT = 0: 256 lanes, 1: 512 lanes, 2: 256 lanes + doubled
// table, 3: 512 lanes + doubled table, 4 (product): 512 lanes + sequence table.
#ifdef SRCDSP_TUNING
static int ci16_variant() {
    static const int v = [] {
        const char *e = std::getenv("SRCDSP_CI16_VARIANT");
        return e ? std::atoi(e) : 4;
    }();
    return v;
}
#endif

#ifdef SRCDSP_PHASE_CLOCK
// tuning build: read (and clear) decim_dot2_ci16's phase clock sums
extern "C" SRCDSP_API int srcdsp_tune_phase_clock(unsigned long long *out8) {
    SRCDSP_HIP_TRY(hipDeviceSynchronize());
    SRCDSP_HIP_TRY(hipMemcpyFromSymbol(out8, HIP_SYMBOL(phase_clock), 8 * sizeof(unsigned long long)));
    unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    SRCDSP_HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(phase_clock), z, sizeof z));
    return SRCDSP_OK;
}
#endif

// period of the fused mixer's table index over input samples, extended to a
// multiple of 4 (one 16-B table read per staged granule): lcm(N / gcd(freq, N), 4)
static unsigned mixer_seq_period(unsigned N, unsigned fr) {
    unsigned a = N, b = fr;
    while (b) { const unsigned r = a % b; a = b; b = r; }
    const unsigned P = N / a;
    return P % 4 == 0 ? P : (P % 2 == 0 ? 2 * P : 4 * P);
}
constexpr unsigned kSeqMax = 4096;  // 2 x 4096 words of LDS, as the doubled phase table

template <int NT, int BLOCK, int TABM, int MD = 4>
int launch_ci16_dot2_shape(DecimLaunch L, int channels, bool mixed, hipStream_t s) {
    constexpr int TO = BLOCK * dot2_r(MD), SPT = MD * TO;  // outputs / input samples per tile
    L.ntiles = (L.n_out + TO - 1) / TO;
    if (mixed) L.mix_dtile = phase_step(L.mix_N, L.mix_freq, SPT);
    if (mixed && NT == 0) {
        // phase of tile 0's first staged sample, -dot2_rt_halo(N) (the
        // caller's value is for the 127/128-tap halo of 128 samples)
        const unsigned long N = L.mix_N, h = (unsigned long)dot2_rt_halo(L.ntaps) % N;
        L.mix_phase_tile0 = (unsigned)((L.mix_phase0 + ((N - h) % N) * L.mix_freq) % N);
    }
    if (mixed && TABM >= 2) {
        L.mix_pe = mixer_seq_period(L.mix_N, L.mix_freq);
        L.mix_pe_dtile = (unsigned)((unsigned long)SPT % L.mix_pe);
        L.mix_pe_drow = (unsigned)((4ul * BLOCK) % L.mix_pe);
    }
    dim3 grid((unsigned)std::min<long>(L.ntiles, kCfGridCap * 256 / BLOCK), channels);
    // M = 1 (16 outputs per lane) needs more than 128 VGPRs: 3 waves per SIMD
    constexpr int MINW = MD == 1 ? 3 : 4;
    if (mixed)
        hipLaunchKernelGGL((decim_dot2_ci16<NT, BLOCK, true, MINW, TABM, MD>), grid, dim3(BLOCK), 0, s, L);
    else
        hipLaunchKernelGGL((decim_dot2_ci16<NT, BLOCK, false, MINW, 0, MD>), grid, dim3(BLOCK), 0, s, L);
    return SRCDSP_OK;
}

template <int NT, int MD = 4>
int launch_ci16_dot2(DecimLaunch L, int channels, bool mixed, hipStream_t s) {
#ifdef SRCDSP_TUNING
    switch (ci16_variant()) {
    case 0: return launch_ci16_dot2_shape<NT, 256, 0>(L, channels, mixed, s);
    case 1: return launch_ci16_dot2_shape<NT, 512, 0>(L, channels, mixed, s);
    case 2: return launch_ci16_dot2_shape<NT, 256, 1>(L, channels, mixed, s);
    case 3: return launch_ci16_dot2_shape<NT, 512, 1>(L, channels, mixed, s);
    default: break;
    }
#endif
    // the product shape: 512 lanes; the two-word sequence mixer table
    // (conflict-free reads for any frequency, no per-sample negate or swap)
    // when its period fits the LDS budget, else the doubled phase table
    // (only these instantiations are compiled outside the tuning build)
    constexpr int BLOCK = MD == 1 ? 256 : 512;  // M = 1: 3 workgroups of 4 waves per CU
    if (!mixed) return launch_ci16_dot2_shape<NT, BLOCK, 2, MD>(L, channels, mixed, s);
    const unsigned pe = mixer_seq_period(L.mix_N, L.mix_freq);
    if (pe > kSeqMax) return launch_ci16_dot2_shape<NT, BLOCK, 1, MD>(L, channels, mixed, s);
    // two-word sequence tables: stored twice up to Pe = 2048, once (index
    // wrapped) up to 4096 -- config 4's mixer (N = 4096, f = 0.1: freq word
    // 205, Pe = 4096) takes the latter
    // the period dividing the tile's input span (16 BLOCK samples): the lane's
    // table words in registers (config 4: Pe = 4096 | 8192); not for runtime
    // taps at M = 2, whose 16 more VGPRs would spill past the 128 of MINW = 4
    if constexpr (BLOCK == 512 && !(NT == 0 && MD == 2))
        if ((16u * BLOCK) % pe == 0) return launch_ci16_dot2_shape<NT, BLOCK, 5, MD>(L, channels, mixed, s);
    if (pe <= (unsigned)kSeq2Max) return launch_ci16_dot2_shape<NT, BLOCK, 3, MD>(L, channels, mixed, s);
    return launch_ci16_dot2_shape<NT, BLOCK, 4, MD>(L, channels, mixed, s);
}

template <int KV>
int launch_fir_tile(const DecimLaunch &L0, int channels, bool fma, hipStream_t s) {
    constexpr int TO = kFirR * kFirBlock;
    constexpr int SPG = FirTraits<KV>::SPG;
    DecimLaunch L = L0;
    L.ntiles = (L.n_out + TO - 1) / TO;
    if (L.ntaps <= kFirStreamTaps) {  // persistent, prefetching
        // grid 512..2048 measure alike (0.650-0.660 ms, 2^28 samples, 31 taps); 256 is 1.7x slower
        dim3 grid((unsigned)std::min<long>(L.ntiles, kCfGridCap), channels);
#define SRCDSP_FIR_STREAM(NTC)                                                               \
    if (fma)                                                                                 \
        hipLaunchKernelGGL((fir_stream_f32<KV, true, 2, NTC>), grid, dim3(kFirBlock), 0, s, L); \
    else                                                                                     \
        hipLaunchKernelGGL((fir_stream_f32<KV, false, 2, NTC>), grid, dim3(kFirBlock), 0, s, L)
        // 31 taps (the reference's FilterFir example length) with the tap
        // count compiled in; at 63 the unrolled loop spills, so longer
        // filters keep the runtime loop
        if (L.ntaps == 31) {
            SRCDSP_FIR_STREAM(31);
        } else {
            SRCDSP_FIR_STREAM(0);
        }
#undef SRCDSP_FIR_STREAM
        return SRCDSP_OK;
    }
    const int span = TO + fir_halo(L.ntaps);
    const size_t smem = 16 * (size_t)(span / SPG + span / SPG / (kFirR / SPG) + 1);
    dim3 grid((unsigned)L.ntiles, channels);
    if (fma)
        hipLaunchKernelGGL((fir_tile_f32<KV, true>), grid, dim3(kFirBlock), smem, s, L);
    else
        hipLaunchKernelGGL((fir_tile_f32<KV, false>), grid, dim3(kFirBlock), smem, s, L);
    return SRCDSP_OK;
}

template <int KV, int M, int P>
int launch_decim_tile(const DecimLaunch &L0, int channels, hipStream_t s) {
    constexpr int RM = dt_rm(M), TO = kDtBlock * (RM / M);
    DecimLaunch L = L0;
    L.ntiles = (L.n_out + TO - 1) / TO;
    const int nch = (L.ntaps + RM - 1) / RM;
    const size_t smem = 16 * (size_t)dt_bs(M) * (size_t)(nch + kDtBlock);
    dim3 grid((unsigned)L.ntiles, channels);
    hipLaunchKernelGGL((decim_tile<KV, M, P>), grid, dim3(kDtBlock), smem, s, L);
    return SRCDSP_OK;
}

template <int KV, int P>
int launch_decim_tile_m(const DecimLaunch &L, int channels, unsigned M, hipStream_t s) {
    switch (M) {
    case 1: return launch_decim_tile<KV, 1, P>(L, channels, s);
    case 2: return launch_decim_tile<KV, 2, P>(L, channels, s);
    case 3: return launch_decim_tile<KV, 3, P>(L, channels, s);
    case 4: return launch_decim_tile<KV, 4, P>(L, channels, s);
    case 5: return launch_decim_tile<KV, 5, P>(L, channels, s);
    case 6: return launch_decim_tile<KV, 6, P>(L, channels, s);
    case 8: return launch_decim_tile<KV, 8, P>(L, channels, s);
    default: return launch_decim_tile<KV, 16, P>(L, channels, s);
    }
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
bool aligned8(const void *p) { return ((uintptr_t)p & 7u) == 0; }
}  // namespace

// Choose the kernel for one FirCore configuration and launch it.
int decim_launch(FirCore &f, const DecimLaunch &L, int channels, hipStream_t s, bool mixed) {
    const bool fma = !(f.flags & SRCDSP_FLAG_FP_STRICT);
    bool al = aligned16(L.in) && ((L.in_stride * kv_in_bytes(f.kv)) % 16 == 0);
    int rc = SRCDSP_OK;
    const bool out_al = aligned16(L.out) && ((L.out_stride * kv_out_bytes(f.kv)) % 16 == 0);
    if (f.kv == KV_CF32 && al && out_al && !mixed && f.ntaps <= kCfMaxTaps &&
        (f.M == 1 || f.M == 2 || f.M == 3 || f.M == 4 || (f.M == 6 && f.ntaps >= 48) || f.M == 8 || f.M == 12 ||
         f.M == 16)) {
        // (M = 6 below 48 taps: decim_tile streams faster, 0.107 vs 0.119 ms at
        // 31 taps on 2^26 samples; profiles/r03_cf32_envelope_m6_m12.txt)
        // complex<float>: the headline kernel.  The tap count is compiled in at the
        // BASELINE lengths (127/128: configs 2 and 3) and the common neighbouring
        // power-of-two lengths; any other N <= 1024 takes the same kernel with
        // the tap count at run time
        // A batch of long channels runs as one launch per channel on the
        // stream, so the channels' persistent sweeps do not overlap: one launch
        // with grid.y = channel measured 3.7 % slower per channel at 8 x 2^28
        // samples, as the next channel's workgroups start beside the last ones
        // of the previous (profiles/tuning/r03_batched_ab.txt).  Short channels
        // (under 2^22 samples, where one channel does not fill the persistent
        // grid for long) keep the single grid.y launch.
        const int per = (channels > 1 && L.n_in >= (1L << 22)) ? 1 : channels;
        for (int c = 0; c < channels && rc == SRCDSP_OK; c += per) {
            DecimLaunch Lc = L;
            Lc.in = (const float2 *)L.in + c * L.in_stride;
            Lc.out = (float2 *)L.out + c * L.out_stride;
            for (int k = 0; k < per; ++k) {
                Lc.hist_in[k] = L.hist_in[c + k];
                Lc.hist_out[k] = L.hist_out[c + k];
            }
            rc = launch_cf32_compiled(Lc, per, f.M, f.ntaps, fma, s);
            if (rc == SRCDSP_ERR_UNSUPPORTED) rc = launch_cf32_rt(Lc, per, f.M, fma, s);
        }
    } else if (f.M == 1 && f.kv == KV_F32_REAL && al && out_al && f.ntaps <= kFirMaxTaps && !mixed) {
        rc = launch_fir_tile<KV_F32_REAL>(L, channels, fma, s);
    } else if ((f.M == 1 || f.M == 2 || f.M == 4 || f.M == 8 || f.M == 16) && f.kv == KV_CI16_I32 &&
               f.coef_fits_i16 && al && out_al && f.ntaps <= kDot2MaxTaps) {
        // complex<int16_t> x int16-range taps on v_dot2 tap pairs, the mixer
        // fused when chained: at M = 4 the tap count compiled in at 127/128
        // (config 4) and, unmixed, 63/64/255/256; any other N <= kDot2MaxTaps
        // and M = 1 (FilterFir) / 2 / 8 / 16 at run time
        DecimLaunch L2 = L;
        L2.coef = f.d_cpair;
        if (f.M != 4) {
            switch (f.M) {
            case 1: rc = launch_ci16_dot2<0, 1>(L2, channels, mixed, s); break;
            case 2: rc = launch_ci16_dot2<0, 2>(L2, channels, mixed, s); break;
            case 8: rc = launch_ci16_dot2<0, 8>(L2, channels, mixed, s); break;
            default: rc = launch_ci16_dot2<0, 16>(L2, channels, mixed, s); break;
            }
        } else if (f.ntaps == 127 || f.ntaps == 128) {
            rc = f.ntaps == 127 ? launch_ci16_dot2<127>(L2, channels, mixed, s) : launch_ci16_dot2<128>(L2, channels, mixed, s);
        } else if (!mixed && (f.ntaps == 63 || f.ntaps == 64 || f.ntaps == 255 || f.ntaps == 256)) {
            switch (f.ntaps) {
            case 63: rc = launch_ci16_dot2_shape<63, 512, 0>(L2, channels, false, s); break;
            case 64: rc = launch_ci16_dot2_shape<64, 512, 0>(L2, channels, false, s); break;
            case 255: rc = launch_ci16_dot2_shape<255, 512, 0>(L2, channels, false, s); break;
            default: rc = launch_ci16_dot2_shape<256, 512, 0>(L2, channels, false, s); break;
            }
        } else {
            rc = launch_ci16_dot2<0>(L2, channels, mixed, s);
        }
    } else if (f.M == 4 && f.kv == KV_CI16_I32 && f.coef_fits_i24 && al && out_al && (f.ntaps == 127 || f.ntaps == 128)) {
        rc = f.ntaps == 127 ? launch_ci16<127>(L, channels, mixed, s) : launch_ci16<128>(L, channels, mixed, s);
    } else if ((f.kv == KV_CF32 || f.kv == KV_CI16_I32 || f.kv == KV_CI16_I16) &&
               (f.M <= 6 || f.M == 8 || f.M == 16) &&
               (f.kv == KV_CF32 ? al : aligned8(L.in) && (L.in_stride * 4) % 8 == 0) &&
               (f.kv == KV_CF32 ? out_al : aligned8(L.out) && (L.out_stride * 4) % 8 == 0) &&
               f.ntaps <= kDtMaxTaps && !mixed && L.n_out > 0) {
        // any tap count <= 1024 at M = 1..6, 8, 16 (M = 1: FilterFir on complex<int16_t>)
        if (f.kv == KV_CF32)
            rc = fma ? launch_decim_tile_m<KV_CF32, 1>(L, channels, f.M, s) : launch_decim_tile_m<KV_CF32, 0>(L, channels, f.M, s);
        else if (f.kv == KV_CI16_I16)
            rc = launch_decim_tile_m<KV_CI16_I16, 2>(L, channels, f.M, s);
        else if (f.coef_fits_i24)
            rc = launch_decim_tile_m<KV_CI16_I32, 0>(L, channels, f.M, s);
        else
            rc = launch_decim_tile_m<KV_CI16_I32, 1>(L, channels, f.M, s);
    } else {
        if (mixed) {
            set_error("mixer->decimator fusion needs variant 1, M = 1/2/4/8/16 with int16-range taps (N <= 1024) or M = 4 with "
                      "127/128 taps |c|<2^23, "
                      "16-B aligned input and output");
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
static bool coef_i16(const int32_t *c, int n) {
    for (int i = 0; i < n; ++i)
        if (c[i] > 32767 || c[i] < -32768) return false;
    return true;
}

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
    coef_fits_i16 = (kv == KV_CI16_I32) && coef_i16((const int32_t *)tmp.data(), n);
    if (d_coef) (void)hipFree(d_coef);
    d_coef = nullptr;
    if (d_cpair) (void)hipFree(d_cpair);
    d_cpair = nullptr;
    if (coef_fits_i16) {  // tap pairs for v_dot2: P_j = (lo c[2j], hi c[2j-1]), c[-1] = c[n] = 0
        const int32_t *c = (const int32_t *)tmp.data();
        auto tap = [&](int k) { return (k >= 0 && k < n) ? (uint32_t)(uint16_t)(int16_t)c[k] : 0u; };
        // zero pairs after the N/2+1 real ones: the run-time-tap kernel's
        // padded steps and its chunks' 16-pair s_loads read them
        const int J = n / 2 + 1, JA = std::max(J, dot2_pair_alloc(n));
        std::vector<uint32_t> pr((size_t)JA, 0u);
        for (int j = 0; j < J; ++j) pr[j] = tap(2 * j) | (tap(2 * j - 1) << 16);
        SRCDSP_HIP_TRY(hipMalloc(&d_cpair, 4 * (size_t)JA));
        SRCDSP_HIP_TRY(hipMemcpy(d_cpair, pr.data(), 4 * (size_t)JA, hipMemcpyHostToDevice));
    }
    // 32 zero taps of slack: the tap chunks of decim_tile end on 12/16/20-tap
    // boundaries (taps past N are never applied, but their s_load stays in bounds)
    tmp.resize(4 * ((size_t)n + 32), '\0');
    SRCDSP_HIP_TRY(hipMalloc(&d_coef, tmp.size()));
    SRCDSP_HIP_TRY(hipMemcpy(d_coef, tmp.data(), tmp.size(), hipMemcpyHostToDevice));

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

// a copy of the object as the reference's implicit copy constructor makes it:
// coefficients, coeffScaling, leftShift and the current history (src settled)
int FirCore::clone_from(FirCore &src) {
    int rc = src.order.sync();
    if (rc) return rc;
    rc = init(src.kv, src.M, src.h_coef.data(), src.ntaps, src.flags);
    if (rc) return rc;
    left_shift = src.left_shift;
    coeff_scaling = src.coeff_scaling;
    if (src.ntaps > 1)
        SRCDSP_HIP_TRY(hipMemcpy(d_hist[0], src.d_hist[src.cur], (size_t)(src.ntaps - 1) * kv_in_bytes(kv),
                                 hipMemcpyDeviceToDevice));
    cur = 0;
    return SRCDSP_OK;
}

int FirCore::clear_history() {
    int rc = order.sync();
    if (rc) return rc;
    // on the handle's own stream: no wait on other streams' work
    for (int b = 0; b < 2; ++b) SRCDSP_HIP_TRY(hipMemsetAsync(d_hist[b], 0, hist_cap, stage.stream));
    SRCDSP_HIP_TRY(hipStreamSynchronize(stage.stream));
    return SRCDSP_OK;
}

void FirCore::destroy() {
    (void)order.sync();
    if (d_coef) (void)hipFree(d_coef);
    if (d_cpair) (void)hipFree(d_cpair);
    d_cpair = nullptr;
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
        const unsigned long N = mix->N, fr = (unsigned)mix->freq, phi0 = (unsigned)mix->phi;
        // phase of sample i: (phi0 + i*fr) mod N, for any sign of i
        auto phase = [&](long i) {
            long m = i % (long)N;
            if (m < 0) m += (long)N;
            return (unsigned)((phi0 + (unsigned long)m * fr) % N);
        };
        constexpr long kNQ = 32;  // taps 127/128: ceil(N/4) polyphase steps
        L.mix_table = mix->d_table;
        L.mix_N = mix->N;
        L.mix_phase0 = (unsigned)phi0;
        L.mix_freq = (unsigned)fr;
        L.mix_phase_tile0 = phase(-4 * kNQ);
        L.mix_dtile = phase_step(N, fr, 4ul * kCiBlock_ * kCiR_);  // reset per kernel tile
        L.mix_phase_hist = phase((long)n_in - (f.ntaps - 1));
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
    host_copy(f.stage.h_buf, in, ib);
    SRCDSP_HIP_TRY(hipMemcpyAsync(d_in, f.stage.h_buf, ib, hipMemcpyHostToDevice, s));
    rc = core_step(f, d_in, n_in, d_out, n_out, s, nullptr);
    if (rc) return rc;
    SRCDSP_HIP_TRY(hipMemcpyAsync(f.stage.h_buf, d_out, ob, hipMemcpyDeviceToHost, s));
    SRCDSP_HIP_TRY(hipStreamSynchronize(s));
    host_copy(out, f.stage.h_buf, ob);
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

SRCDSP_API int srcdsp_decim_clone(srcdsp_decim_t h, srcdsp_decim_t *out) {
    SRCDSP_ARG_CHECK(h != nullptr && out != nullptr, "decim_clone: null argument");
    *out = nullptr;
    auto *c = new srcdsp_decim();
    int rc = c->core.clone_from(h->core);
    if (rc) {
        c->core.destroy();
        delete c;
        return rc;
    }
    *out = c;
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

SRCDSP_API int srcdsp_fir_clone(srcdsp_fir_t h, srcdsp_fir_t *out) {
    SRCDSP_ARG_CHECK(h != nullptr && out != nullptr, "fir_clone: null argument");
    *out = nullptr;
    auto *c = new srcdsp_fir();
    int rc = c->core.clone_from(h->core);
    if (rc) {
        c->core.destroy();
        delete c;
        return rc;
    }
    *out = c;
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
// The two reference calls as two launches, through the mixer handle's
// grow-only scratch buffer: the configurations the fused kernel does not
// cover.  The mixer's ordering event is recorded after the DECIMATOR launch
// (the scratch's reader), so the next mixer write into the scratch -- from
// whichever decimator and stream the mixer feeds next -- waits for the last
// read of it, not only for the last mixer kernel.
static int mixdecim_unfused(srcdsp_mixer_t mixer, FirCore &f, const void *d_in, size_t n_in, void *d_out,
                            size_t n_out, hipStream_t s) {
    MixerState &m = mixer->m;
    if (m.scratch_cap < n_in * 4) {  // grow: only after every earlier use is done
        int rc = f.order.sync();
        if (!rc) rc = m.order.sync();
        if (rc) return rc;
        SRCDSP_HIP_TRY(hipStreamSynchronize(s));
        if (m.d_scratch) (void)hipFree(m.d_scratch);
        m.d_scratch = nullptr;
        m.scratch_cap = 0;
        SRCDSP_HIP_TRY(hipMalloc(&m.d_scratch, n_in * 4));
        m.scratch_cap = n_in * 4;
    }
    int rc = f.order.before(s);
    if (rc) return rc;
    rc = srcdsp_mixer_step(mixer, d_in, n_in, m.d_scratch, s);  // mixers.h:169-188
    if (rc == SRCDSP_OK) rc = core_step(f, m.d_scratch, n_in, d_out, n_out, s, nullptr);
    if (rc == SRCDSP_OK) rc = m.order.after(s);  // scratch released after its reader
    return rc;
}

SRCDSP_API int srcdsp_mixdecim_step(srcdsp_mixer_t mixer, srcdsp_decim_t decim, const void *d_in, size_t n_in,
                                    void *d_out, size_t n_out, void *stream) {
    SRCDSP_ARG_CHECK(mixer != nullptr && decim != nullptr, "mixdecim_step: null handle");
    FirCore &f = decim->core;
    MixerState &m = mixer->m;
    if (f.kv != KV_CI16_I32 && f.kv != KV_CI16_I16) {
        set_error("mixdecim_step: the decimator must take complex<int16_t> input (the mixer's output)");
        return SRCDSP_ERR_UNSUPPORTED;
    }
    if (n_out * f.M != n_in) {
        set_error("mixdecim_step: out.size()*M != in.size() (dnsampling_filters.h:133)");
        return SRCDSP_ERR_SIZE;
    }
    if (n_in == 0) return SRCDSP_OK;
    SRCDSP_ARG_CHECK(d_in && d_out, "mixdecim_step: null buffer");
    hipStream_t s = (hipStream_t)stream;
    // fused: variant 1, M = 4, int16-range taps (any N <= 1024) or 127/128 taps
    // with |c| < 2^23, a table of <= 4096 entries, 16-B aligned buffers
    // (decim_launch refuses the rest unchanged)
    if (f.kv != KV_CI16_I32 || m.N > 4096) return mixdecim_unfused(mixer, f, d_in, n_in, d_out, n_out, s);
    int rc = m.order.before(s);
    if (rc) return rc;
    rc = core_step(f, d_in, n_in, d_out, n_out, s, &m);
    if (rc == SRCDSP_ERR_UNSUPPORTED) {
        set_error("");  // not an error: the unfused pair of launches serves this configuration
        return mixdecim_unfused(mixer, f, d_in, n_in, d_out, n_out, s);
    }
    if (rc) return rc;
    // mixer phase after the call: phi += n_in * freq (mod N), mixers.h:177
    m.phi = (int16_t)(((unsigned long)(unsigned)m.phi + (unsigned long)(n_in % m.N) * (unsigned)m.freq) % m.N);
    return m.order.after(s);
}

}  // extern "C"
