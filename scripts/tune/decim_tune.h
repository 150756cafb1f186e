// decim_tune.h -- TUNING ONLY (scripts/tune), never built into the product.
// The headline complex<float> decimator with every knob the tuning rounds
// varied (probe paths, cache-policy overrides, store shapes, issue order),
// plus the measured-and-rejected wave-private variant.  The product kernel is
// srcdsp_amd/csrc/decim_kernels.h decim_stream_cf32 (no knobs).
#pragma once
#include "../../srcdsp_amd/csrc/decim_kernels.h"

namespace srcdsp {
// OST: 0 = each lane stores its own R outputs (two 16-B stores at a 32-B lane
// stride: every store instruction half-covers its lines); 1 = outputs staged
// through LDS (two barriers per tile); 2 (R == 4 only) = a v_permlane32_swap
// per dword pairs lane i's first output pair with lane i+32's and lane i+32's
// second pair with lane i's, so each of the two store instructions writes
// 1 KiB of whole lines, with no LDS round trip and no barrier.
template <int NT, int R, int BLOCK, bool FMA, int MINW, bool Q0, int PROBE = 0, bool NTL = false, int OST = 0,
          bool NTS = false, bool GS = false, int LAUX = -1, int SAUX = -1, bool ILV = false, int M = 4>
__global__ __launch_bounds__(BLOCK, MINW) void decim_stream2_cf32_tune(DecimLaunch a) {
    static_assert(OST != 2 || R == 1 || R == 2 || R == 4 || R == 8, "whole-line stores assume 1, 2, 4 or 8 outputs per lane");
    static_assert((M * R) % 4 == 0 && M * R <= 32 && (M == 4 || ILV),
                  "a lane chunk is 4, 8, 12 or 16 input samples; M != 4 takes the ILV tap loop");
    constexpr int NQ = (NT + 3) / 4;
    constexpr int TO = BLOCK * R;
    constexpr int TG = M * TO / 2 + 2 * NQ;  // staged granules: M TO input samples + the halo
    constexpr int PR = M * R / 2;  // granules per lane chunk (M R samples)
    constexpr int KPAD = ceildiv(2 * NQ, PR);
    constexpr int LG = TG + (TG + KPAD * PR) / PR + 1;
    constexpr int PER = ceildiv(TG, BLOCK);
    __shared__ float4 lds[LG];

    const int ch = blockIdx.y;
    const float2 *in = (const float2 *)a.in + ch * a.in_stride;
    const float2 *hist = (const float2 *)a.hist_in[ch];
    float2 *out = (float2 *)a.out + ch * a.out_stride;
    const long n_in = a.n_in;
    const int H = NT - 1;
    const int t = threadIdx.x;
    const long nb = gridDim.x;
    const long b = xcd_tile(blockIdx.x, nb);
    const long per = a.ntiles / nb, rem = a.ntiles % nb;
    // GS: tiles b, b+nb, b+2nb, ... (the whole grid sweeps one contiguous
    // window of the input at a time); else a contiguous run of tiles per block
    const long t_begin = GS ? b : b * per + (b < rem ? b : rem);
    const long t_end = GS ? a.ntiles : t_begin + per + (b < rem ? 1 : 0);
    constexpr long kStep1 = 1;
    const long t_step = GS ? nb : kStep1;
    if (t_begin == 0 && t_end > 0) write_history(in, n_in, hist, (float2 *)a.hist_out[ch], H);

    float4 v[PER];
    // tiles >= 1: one descriptor per tile, 32-bit lane offsets, range-checked
    auto stage_load = [&](float4 (&v)[PER], long tile) {
        if constexpr (PROBE >= 2) tile = 1 + (tile & 15);
        const long b0 = M * tile * TO - 4 * NQ;  // >= 0 for tile >= 1
        const long remb = (n_in - b0) * 8;
        const unsigned nrec = (unsigned)(remb > 0xfffffff0L ? 0xfffffff0L : (remb < 0 ? 0 : remb));
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(in + b0), 0, nrec, 0x00020000);
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int g = t + i * BLOCK;
            if (g < TG) {
                // aux: bit0 sc0, bit1 nt, bit4 sc1 (LAUX >= 0: tuning override)
                // lane offset in the VGPR, the per-load step in soffset (an
                // SGPR constant): one offset VGPR for all PER loads
                auto w = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * t, 16 * i * BLOCK,
                                                              LAUX >= 0 ? LAUX : (NTL ? 2 : 0));
                v[i] = make_float4(__uint_as_float(w[0]), __uint_as_float(w[1]), __uint_as_float(w[2]),
                                   __uint_as_float(w[3]));
            }
        }
    };
    if (t_begin < t_end) {
        if (t_begin == 0) {  // tile 0: the halo comes from the history
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
            stage_load(v, t_begin);
        }
    }
    const int Bt = 2 * NQ + KPAD + (PR + 1) * t;
    // the staged tile lands in LDS once every wave is done with the previous
    // tile's image (and its output staging, which reuses it)
    auto stage_to_lds = [&]() {
        SRCDSP_LDS_BARRIER();
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int g = t + i * BLOCK;
            if (g < TG) lds[g + (g - 2 * NQ + KPAD * PR) / PR] = v[i];
        }
        SRCDSP_LDS_BARRIER();
    };
    // one tile: taps over the LDS image, outputs stored.  The loop below
    // issues the next tile's loads before this and lands them in LDS after
    // it, all in one iteration: the compiler then waits for the loads with
    // vmcnt(this tile's stores) and the stores stay in flight.
    // WHOLE: the tile's TO outputs all exist (every tile but a partial last one)
    auto do_tile = [&](long tile, auto whole_tag) {
        constexpr bool WHOLE = decltype(whole_tag)::value;
        ConstPtr<float> tp = const_view<float>(a.coef);
        asm volatile("" : "+s"(tp));
        constexpr int GPC = M * R / 4;  // 4-sample groups per lane chunk
        float2 X[4 * (NQ + GPC)];
        float yr[R], yi[R];
#pragma unroll
        for (int r = 0; r < R; ++r) yr[r] = yi[r] = 0.f;
        auto load_group = [&](int e) {
            const float4 g0 = lds[Bt + 2 * e + floordiv(2 * e, PR)];
            const float4 g1 = lds[Bt + 2 * e + 1 + floordiv(2 * e + 1, PR)];
            X[4 * e + 4 * NQ + 0] = make_float2(g0.x, g0.y);
            X[4 * e + 4 * NQ + 1] = make_float2(g0.z, g0.w);
            X[4 * e + 4 * NQ + 2] = make_float2(g1.x, g1.y);
            X[4 * e + 4 * NQ + 3] = make_float2(g1.z, g1.w);
        };
#pragma unroll
        for (int e = -1; e < GPC; ++e) load_group(e);
        if constexpr (PROBE == 1 || PROBE == 3) {
#pragma unroll
            for (int r = 0; r < R; ++r) { yr[r] = X[M * r + 4 * NQ].x; yi[r] = X[M * r + 4 * NQ].y; }
        } else if constexpr (ILV && PROBE != 3) {
            // tap-major issue order through inline asm: R independent chains
            // round-robin, taps as SGPR pairs (c[2m], c[2m+1]); FMA: one
            // pk_fma per tap and output; strict: R products, then R sums
            ConstPtr<unsigned long long> tp2 = const_view<unsigned long long>(a.coef);
            asm volatile("" : "+s"(tp2));
            f2_t acc[R];
            if constexpr (!FMA) {
#pragma unroll
                for (int r = 0; r < R; ++r) acc[r] = f2_t{0.f, 0.f};
            }
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                if (q + 1 < NQ) load_group(-q - 2);
                if ((q & 3) == 0) asm volatile("" : "+s"(tp2));
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    const int k = 4 * q + p;
                    if (k < NT) {
                        const unsigned long long cp = tp2[k >> 1];
                        if constexpr (FMA) {
#pragma unroll
                            for (int r = 0; r < R; ++r) {
                                const float2 x = X[M * r - 4 * q - p + 4 * NQ];
                                const f2_t xv = {x.x, x.y};
                                if (k == 0) pk_fma_tap<false, true>(acc[r], cp, xv);
                                else if (k & 1) pk_fma_tap<true, false>(acc[r], cp, xv);
                                else pk_fma_tap<false, false>(acc[r], cp, xv);
                            }
                        } else {
                            f2_t pr[R];
#pragma unroll
                            for (int r = 0; r < R; ++r) {
                                const float2 x = X[M * r - 4 * q - p + 4 * NQ];
                                const f2_t xv = {x.x, x.y};
                                if (k & 1) pk_mul_tap<true>(pr[r], cp, xv);
                                else pk_mul_tap<false>(pr[r], cp, xv);
                            }
#pragma unroll
                            for (int r = 0; r < R; ++r) pk_add_acc(acc[r], pr[r]);
                        }
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < R; ++r) { yr[r] = acc[r].x; yi[r] = acc[r].y; }
        } else
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            if (q + 1 < NQ) load_group(-q - 2);
            if ((q & 3) == 0) asm volatile("" : "+s"(tp));
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const int k = 4 * q + p;
                if (k < NT) {
                    // PROBE 3 (timing only): compute path with one tap value, no tap loads
                    const float c = PROBE == 3 ? __builtin_bit_cast(float, a.shift | 0x3c000000u) : tp[k];
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const float2 x = X[4 * (r - q) - p + 4 * NQ];
                        yr[r] = mac<FMA>(c, x.x, yr[r]);
                        yi[r] = mac<FMA>(c, x.y, yi[r]);
                    }
                }
            }
        }
        const long n0 = tile * TO + (long)t * R;
        const unsigned sh = a.shift;
        auto q = [&](float y) { return Q0 ? q16f_shift0(y) : q16f(y, sh); };
        if (PROBE == 5 && a.ntaps != 12345) {  // tuning: no stores
        } else if constexpr (OST == 2 && WHOLE && R == 2) {  // 16 B per lane: whole lines as they stand
            store16<NTS>((float4 *)(out + n0), make_float4(q(yr[0]), q(yi[0]), q(yr[1]), q(yi[1])));
        } else if constexpr (OST == 2 && WHOLE && R == 1) {  // 8 B per lane, lane-contiguous
            out[n0] = make_float2(q(yr[0]), q(yi[0]));
        } else if constexpr (OST == 2 && WHOLE) {
            float2 o[R];
#pragma unroll
            for (int r = 0; r < R; ++r) o[r] = make_float2(q(yr[r]), q(yi[r]));
            store_wave_lines<R, NTS>(out + tile * TO + (t & ~63) * R, o, t & 63);
        } else if constexpr (OST == 2) {
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (n0 + r < a.n_out) out[n0 + r] = make_float2(q(yr[r]), q(yi[r]));
        } else if constexpr (OST == 1) {
            // outputs -> LDS (reusing the tile image once every wave is done
            // reading it) -> 16-B lane-contiguous stores of the whole tile
            const long o0 = tile * TO;
            SRCDSP_LDS_BARRIER();
            float2 *ob = (float2 *)lds;
#pragma unroll
            for (int r = 0; r < R; ++r) ob[t * R + r] = make_float2(q(yr[r]), q(yi[r]));
            SRCDSP_LDS_BARRIER();
            const float4 *ob4 = (const float4 *)lds;
            if constexpr (WHOLE) {
#pragma unroll
                for (int i = 0; i < TO / 2 / BLOCK; ++i) {
                    const int k = t + i * BLOCK;
                    if constexpr (SAUX >= 0) {  // tuning override of the store policy
                        __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
                            (void *)(out + o0), 0, 0x7ffffff0, 0x00020000);
                        const float4 v4 = ob4[k];
                        typedef unsigned u4_t __attribute__((ext_vector_type(4)));
                        const u4_t u = {__float_as_uint(v4.x), __float_as_uint(v4.y), __float_as_uint(v4.z),
                                        __float_as_uint(v4.w)};
                        __builtin_amdgcn_raw_buffer_store_b128(u, ro, 16 * k, 0, SAUX);
                    } else {
                        store16<NTS>((float4 *)(out + o0 + 2 * k), ob4[k]);
                    }
                }
            } else {
                for (int k = t; k < TO; k += BLOCK)
                    if (o0 + k < a.n_out) out[o0 + k] = ob[k];
            }
        } else if (WHOLE && (R % 2) == 0) {
#pragma unroll
            for (int r = 0; r < R; r += 2)
                store16<NTS>((float4 *)(out + n0 + r), make_float4(q(yr[r]), q(yi[r]), q(yr[r + 1]), q(yi[r + 1])));
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (n0 + r < a.n_out) out[n0 + r] = make_float2(q(yr[r]), q(yi[r]));
        }
        };
    // Every iteration of the loop prefetches (the workgroup's last tile is
    // peeled off after it), and only the launch's last tile can be partial, so
    // the loop body is one straight path with a fixed number of stores: the
    // compiler waits for the prefetch with a counted vmcnt and the stores stay
    // in flight across iterations.
    if (t_begin < t_end) {
        stage_to_lds();
        long tile = t_begin;
        for (; tile + t_step < t_end; tile += t_step) {
            if constexpr (PROBE < 4) stage_load(v, tile + t_step);
            do_tile(tile, std::true_type{});
            if constexpr (PROBE < 4) stage_to_lds();
        }
        if ((tile + 1) * TO <= a.n_out)
            do_tile(tile, std::true_type{});
        else
            do_tile(tile, std::false_type{});
    }

}

// ------------------------------------------------- wave-private cf32 (headline)
// Persistent complex<float> decimator, M = 4, with NO workgroup barrier: every
// wave owns wave tiles of 64 lanes x 4 outputs (1024 input samples + the
// 4*NQ-sample halo) end to end -- loads, LDS image, taps, stores.
//
// The wave's LDS image is stored column-major: image granule g (16 B, two
// samples) = column g/8, row g%8 sits at slot row*NCOL + column.  Column c is
// lane (c - HC)'s 8-granule chunk (HC halo columns first).  So
//  * lane t's read of its frame group e (granules 2e, 2e+1 of its chunk) is
//    slot ((2e)&7)*NCOL + HC + t + floor(2e/8): a per-lane base (16 t) plus a
//    compile-time immediate, and the 16 lanes of a ds_read_b128 group read 16
//    consecutive slots -- conflict-free without any pad granules;
//  * load instruction i, lane l fetches the contiguous image granule 64 i + l
//    and writes it to slot (l&7)*NCOL + 8i + l/8; with NCOL = 1 (mod 8) the 8
//    lanes of a ds_write_b128 group land in 8 distinct 16-B bank slots.
// One image is 8*NCOL*16 B (9,344 B at NQ = 32), so 16 waves fit a CU's LDS
// with one image each.  A wave lands its prefetched next tile as soon as its
// own reads of the current image are done (LDS operations of one wave execute
// in order), so no wave ever waits for another: the four waves of a SIMD
// drift apart and keep the VALU fed.  The halo (the previous wave tile's
// tail) is re-read by every wave tile, an L2 hit.
// Taps: wave-uniform SGPR pairs, issued tap-major (pk_fma_tap) for the FMA
// contract; the strict contract keeps separately rounded mul/add.
// PROBE (tuning only): 1 = memory path only (no tap loop); 2 = compute path
// only (every wave tile loads one of 16 L2-resident spans)
// 3 = memory path without the halo load; LAUX: load cache policy (2 = nt)
// SYNC (tuning): one workgroup barrier per wave tile, before its loads issue
template <int NT, int BLOCK, bool FMA, int MINW, bool Q0, int PROBE = 0, int LAUX = 2, bool SYNC = false>
__global__ __launch_bounds__(BLOCK, MINW) void decim_wave_cf32(DecimLaunch a) {
    constexpr int R = 4;                      // outputs per lane
    constexpr int NQ = (NT + 3) / 4;          // 4-tap polyphase groups
    constexpr int HC = ceildiv(2 * NQ, 8);    // halo columns (8 granules each)
    constexpr int COLS = 64 + HC;             // loaded columns
    constexpr int NCOL = COLS + ((1 - COLS % 8) + 8) % 8;  // = 1 (mod 8)
    constexpr int WG = 8 * COLS;              // image granules (loaded)
    static_assert(WG % 64 == 0, "whole load instructions per image");
    constexpr int PER = WG / 64;              // loads per lane
    constexpr int WPB = BLOCK / 64;
    constexpr int TO = 64 * R;                // outputs per wave tile
    constexpr int HALO = 8 * HC * 2;          // halo samples (>= 4 NQ)
    __shared__ float4 lds[WPB][8 * NCOL];

    const int ch = blockIdx.y;
    const float2 *in = (const float2 *)a.in + ch * a.in_stride;
    const float2 *hist = (const float2 *)a.hist_in[ch];
    float2 *out = (float2 *)a.out + ch * a.out_stride;
    const long n_in = a.n_in;
    const int H = NT - 1;
    const int ln = threadIdx.x & 63;
    // wave index made wave-uniform for the compiler: tiles, descriptors and
    // the image base live in SGPRs
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long nb = gridDim.x;
    const long b = xcd_tile(blockIdx.x, nb);
    if (b == 0) write_history(in, n_in, hist, (float2 *)a.hist_out[ch], H);
    float4 *img = lds[wv];
    const long step = nb * WPB;
    long tile = b * WPB + wv;

    float4 v[PER];
    // image granule 64 i + ln of wave tile `tile` (>= 1): one descriptor per
    // tile, range-checked (zero past the input end), non-temporal
    auto stage_load = [&](long tl) {
        if constexpr (PROBE == 2) tl = 1 + (tl & 15);
        const long s0 = (long)TO * 4 * tl - HALO;
        const long remb = (n_in - s0) * 8;
        const unsigned nrec = (unsigned)(remb > 0xfffffff0L ? 0xfffffff0L : (remb < 0 ? 0 : remb));
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(in + s0), 0, nrec, 0x00020000);
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            if (PROBE == 3 && i == 0) { v[i] = make_float4(0.f, 0.f, 0.f, 0.f); continue; }
            auto w = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * ln, 1024 * i, LAUX);
            v[i] = make_float4(__uint_as_float(w[0]), __uint_as_float(w[1]), __uint_as_float(w[2]),
                               __uint_as_float(w[3]));
        }
    };
    auto stage_first = [&]() {  // wave tile 0: the halo comes from the history
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const long s = -HALO + 2 * (long)(64 * i + ln);
            const float2 lo = fetch(in, hist, s, n_in, H), hi = fetch(in, hist, s + 1, n_in, H);
            v[i] = make_float4(lo.x, lo.y, hi.x, hi.y);
        }
    };
    const int wslot = (ln & 7) * NCOL + (ln >> 3);
    auto land = [&]() {
#pragma unroll
        for (int i = 0; i < PER; ++i) img[wslot + 8 * i] = v[i];
    };
    // own frame of lane ln: granule 2e (+1) -> slot ((2e)&7)*NCOL + HC + ln + floor(2e/8)
    const float4 *rd = img + HC + ln;
    auto do_tile = [&](long tl, auto whole_tag) {
        constexpr bool WHOLE = decltype(whole_tag)::value;
        float2 X[4 * (NQ + R)];
        auto load_group = [&](int e) {
            const int o = ((2 * e) & 7) * NCOL + floordiv(2 * e, 8);
            const float4 g0 = rd[o], g1 = rd[o + NCOL];
            X[4 * e + 4 * NQ + 0] = make_float2(g0.x, g0.y);
            X[4 * e + 4 * NQ + 1] = make_float2(g0.z, g0.w);
            X[4 * e + 4 * NQ + 2] = make_float2(g1.x, g1.y);
            X[4 * e + 4 * NQ + 3] = make_float2(g1.z, g1.w);
        };
#pragma unroll
        for (int e = -1; e < R; ++e) load_group(e);
        float yr[R], yi[R];
        if constexpr (PROBE == 1 || PROBE == 3) {
#pragma unroll
            for (int r = 0; r < R; ++r) { yr[r] = X[4 * r + 4 * NQ].x; yi[r] = X[4 * r + 4 * NQ - 4].y; }
        } else if constexpr (FMA) {
            ConstPtr<unsigned long long> tp2 = const_view<unsigned long long>(a.coef);
            asm volatile("" : "+s"(tp2));
            f2_t acc[R];
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                if (q + 1 < NQ) load_group(-q - 2);
                if ((q & 3) == 0) asm volatile("" : "+s"(tp2));
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    const int k = 4 * q + p;
                    if (k < NT) {
                        const unsigned long long cp = tp2[k >> 1];
#pragma unroll
                        for (int r = 0; r < R; ++r) {
                            const float2 x = X[4 * (r - q) - p + 4 * NQ];
                            const f2_t xv = {x.x, x.y};
                            if (k == 0) pk_fma_tap<false, true>(acc[r], cp, xv);
                            else if (k & 1) pk_fma_tap<true, false>(acc[r], cp, xv);
                            else pk_fma_tap<false, false>(acc[r], cp, xv);
                        }
                    }
                }
            }
#pragma unroll
            for (int r = 0; r < R; ++r) { yr[r] = acc[r].x; yi[r] = acc[r].y; }
        } else {
            ConstPtr<float> tp = const_view<float>(a.coef);
            asm volatile("" : "+s"(tp));
#pragma unroll
            for (int r = 0; r < R; ++r) yr[r] = yi[r] = 0.f;
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                if (q + 1 < NQ) load_group(-q - 2);
                if ((q & 3) == 0) asm volatile("" : "+s"(tp));
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    const int k = 4 * q + p;
                    if (k < NT) {
                        const float c = tp[k];
#pragma unroll
                        for (int r = 0; r < R; ++r) {
                            const float2 x = X[4 * (r - q) - p + 4 * NQ];
                            yr[r] = mac<false>(c, x.x, yr[r]);
                            yi[r] = mac<false>(c, x.y, yi[r]);
                        }
                    }
                }
            }
        }
        const unsigned sh = a.shift;
        auto qz = [&](float y) { return Q0 ? q16f_shift0(y) : q16f(y, sh); };
        const long o0 = tl * TO;
        if constexpr (WHOLE) {
            float2 o[R];
#pragma unroll
            for (int r = 0; r < R; ++r) o[r] = make_float2(qz(yr[r]), qz(yi[r]));
            store_wave_lines<R, true>(out + o0, o, ln);
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const long n = o0 + (long)ln * R + r;
                if (n < a.n_out) out[n] = make_float2(qz(yr[r]), qz(yi[r]));
            }
        }
    };
    if (tile >= a.ntiles) return;
    if (tile == 0) stage_first(); else stage_load(tile);
    // land this tile, issue the next one's loads, then the taps and stores:
    // the wait for the prefetch (next iteration's land) leaves the stores in
    // flight; the wave's last tile is peeled so the loop body is straight
    for (; tile + step < a.ntiles; tile += step) {
        land();
        if constexpr (SYNC) __builtin_amdgcn_s_barrier();
        stage_load(tile + step);
        do_tile(tile, std::true_type{});
    }
    land();
    if ((tile + 1) * TO <= a.n_out)
        do_tile(tile, std::true_type{});
    else
        do_tile(tile, std::false_type{});
}

}  // namespace srcdsp

namespace srcdsp {
// ---------------------------------------------------------------- round 3
// The round-3 product kernel (decim_stream_cf32, compile-time taps, M = 4)
// with the staging experiments of VERDICT r2 item 1:
//  STAG  > 0: workgroups on an odd workgroup slot of their CU (HW_ID.TG_ID)
//        start STAG x 2048 clocks late, so the two workgroups of a CU do not
//        reach their barriers / LDS staging together (a stagger)
//  EPI   1: the finished tile's quantise + permlane + stores issue after the
//        next tile's ds_writes, between the two barriers (VALU work beside
//        the LDS write transfer instead of before the first barrier)
//  PRIO  1: waves 4..7 of each workgroup at s_setprio 1 (static priority
//        for the younger half, MI355X_MICROARCH.md "two waves per SIMD" 4)
template <int NT, int R, int BLOCK, int MINW, int STAG, int EPI, int PRIO>
__global__ __launch_bounds__(BLOCK, MINW) void decim_stream_x(DecimLaunch a) {
    constexpr int M = 4;
    constexpr int NQ = (NT + 3) / 4;
    constexpr int TO = BLOCK * R;
    constexpr int PR = M * R / 2;
    constexpr int PER = ceildiv(M * TO / 2 + 2 * NQ, BLOCK);
    constexpr int TG = M * TO / 2 + 2 * NQ;
    constexpr int KPAD = ceildiv(2 * NQ, PR);
    __shared__ float4 lds[TG + (TG + KPAD * PR) / PR + 1];
    const float2 *in = (const float2 *)a.in;
    const float2 *hist = (const float2 *)a.hist_in[0];
    float2 *out = (float2 *)a.out;
    const long n_in = a.n_in;
    const int H = NT - 1;
    const int t = threadIdx.x;
    const long nb = gridDim.x;
    const long b = xcd_tile(blockIdx.x, nb);
    if constexpr (PRIO) {
        if (t >= 256) __builtin_amdgcn_s_setprio(1);
    }
    if constexpr (STAG > 0) {
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_REG_HW_ID
        if ((hw >> 16) & 1)
            for (int i = 0; i < STAG; ++i) __builtin_amdgcn_s_sleep(32);
    }
    if (b == 0 && a.ntiles > 0) write_history(in, n_in, hist, (float2 *)a.hist_out[0], H);
    float4 v[PER];
    auto stage_load = [&](long tile) {
        const long b0 = M * tile * TO - 4 * NQ;
        const long remb = (n_in - b0) * 8;
        const unsigned nrec = (unsigned)(remb > 0xfffffff0L ? 0xfffffff0L : (remb < 0 ? 0 : remb));
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(in + b0), 0, nrec, 0x00020000);
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int g = t + i * BLOCK;
            if ((i + 1) * BLOCK <= M * TO / 2 || g < TG) {
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
                const long s = -4 * NQ + 2 * (long)g;
                if (g < TG) {
                    float2 lo = fetch(in, hist, s, n_in, H), hi = fetch(in, hist, s + 1, n_in, H);
                    v[i] = make_float4(lo.x, lo.y, hi.x, hi.y);
                }
            }
        } else {
            stage_load(b);
        }
    }
    const int Bt = 2 * NQ + KPAD + (PR + 1) * t;
    const int lq = (t - 2 * NQ + KPAD * PR) / PR;
    auto write_image = [&]() {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int g = t + i * BLOCK;
            if ((i + 1) * BLOCK <= M * TO / 2 || g < TG) lds[g + lq + i * (BLOCK / PR)] = v[i];
        }
    };
    auto taps = [&](f2_t (&acc)[R]) {
        ConstPtr<unsigned long long> tp2 = const_view<unsigned long long>(a.coef);
        asm volatile("" : "+s"(tp2));
        constexpr int GPC = M * R / 4;
        float2 X[4 * (NQ + GPC)];
        auto load_group = [&](int e) {
            const float4 g0 = lds[Bt + 2 * e + floordiv(2 * e, PR)];
            const float4 g1 = lds[Bt + 2 * e + 1 + floordiv(2 * e + 1, PR)];
            X[4 * e + 4 * NQ + 0] = make_float2(g0.x, g0.y);
            X[4 * e + 4 * NQ + 1] = make_float2(g0.z, g0.w);
            X[4 * e + 4 * NQ + 2] = make_float2(g1.x, g1.y);
            X[4 * e + 4 * NQ + 3] = make_float2(g1.z, g1.w);
        };
#pragma unroll
        for (int e = -1; e < GPC; ++e) load_group(e);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            if (q + 1 < NQ) load_group(-q - 2);
            if ((q & 3) == 0) asm volatile("" : "+s"(tp2));
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const int k = 4 * q + p;
                if (k < NT) {
                    const unsigned long long cp = tp2[k >> 1];
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const float2 x = X[M * r - 4 * q - p + 4 * NQ];
                        const f2_t xv = {x.x, x.y};
                        if (k == 0) pk_fma_tap<false, true>(acc[r], cp, xv);
                        else if (k & 1) pk_fma_tap<true, false>(acc[r], cp, xv);
                        else pk_fma_tap<false, false>(acc[r], cp, xv);
                    }
                }
            }
        }
    };
    auto epilogue = [&](long tile, const f2_t (&acc)[R], bool whole) {
        const long n0 = tile * TO + (long)t * R;
        if (whole) {
            float2 o[R];
#pragma unroll
            for (int r = 0; r < R; ++r) o[r] = make_float2(q16f_shift0(acc[r].x), q16f_shift0(acc[r].y));
            store_wave_lines<R, true>(out + tile * TO + (t & ~63) * R, o, t & 63);
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (n0 + r < a.n_out) out[n0 + r] = make_float2(q16f_shift0(acc[r].x), q16f_shift0(acc[r].y));
        }
    };
    if (b < a.ntiles) {
        SRCDSP_LDS_BARRIER();
        write_image();
        SRCDSP_LDS_BARRIER();
        long tile = b;
        for (; tile + nb < a.ntiles; tile += nb) {
            stage_load(tile + nb);
            f2_t acc[R];
            taps(acc);
            if constexpr (EPI) {
                SRCDSP_LDS_BARRIER();
                write_image();
                epilogue(tile, acc, true);
                SRCDSP_LDS_BARRIER();
            } else {
                epilogue(tile, acc, true);
                SRCDSP_LDS_BARRIER();
                write_image();
                SRCDSP_LDS_BARRIER();
            }
        }
        f2_t acc[R];
        taps(acc);
        epilogue(tile, acc, (tile + 1) * TO <= a.n_out);
    }
}

// census of workgroup placement: one record per workgroup (HW_ID, XCC_ID)
__global__ void wg_census(unsigned *out) {
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
        out[2 * blockIdx.x + 1] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
        __builtin_amdgcn_s_sleep(127);  // stay resident while the rest of the grid lands
        __builtin_amdgcn_s_sleep(127);
    }
}

}  // namespace srcdsp
