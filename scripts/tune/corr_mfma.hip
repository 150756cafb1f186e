// Config 5's correlator on the integer matrix cores: a TUNING PROBE, not the
// product (BASELINE north_star says the product path uses no
// MFMA, so this kernel never ships in libsrcdsp_hip.so).
//
// What it computes, for every sample i of one fresh FixedPatternCorrelator<
// int16_t, int32_t, 1024, 1> stream (history zeros before sample 0): the two
// registers the reference forms before its peak test (correlators.h:233-250)
//   C_i    = sum_k x[i - 1023 + k] * c[k]           complex, int32 wrap
//            (c = conj(pattern), dsp_complex.cpp:31-37 products)
//   corr_i = ((C_i.re >> cs) >> 2)^2 + ((C_i.im >> cs) >> 2)^2   uint32
//   e_i    = (sum_k |x[i - 1023 + k]|^2) >> (cs / 2)             uint32 wrap
// and stores both (8 B per sample) for a bit-exact comparison with the oracle.
//
// Formulation (exact modulo 2^32, as the reference's wrap-around sums):
// * Limbs.  x = 256 xh + xl + 128 with xh = x >> 8 (the int16's high byte) and
//   xl = (x & 255) - 128 (its low byte XOR 0x80), both in [-128, 127]; a zero
//   sample (the history before the stream) is (0, -128).  A coefficient value
//   v = 256 vh + vl, vl in [-128, 127], vh = (v - vl) / 256 (the host checks
//   vh in [-128, 127]).  So x * v = 65536 xh vh + 256 (xh vl + xl vh) + xl vl
//   + 128 v, and the window's sum of the last term is the constant
//   bias = 128 sum_k v[k] (every window holds all 1024 taps).
// * Toeplitz tiles.  A wave's tile is 1024 consecutive outputs
//   i = i_w + 32 row + col (row, col in 0..31).  For chunk t (0..65) of 16
//   samples, A_t[row][(s, comp)] = limb of x_comp[i_w + 32 row - 1024 + 16 t + s]
//   (a pure reshape of the staged stream: row r of chunk t is the 16 samples at
//   32 r + 16 t) and B_t[(s, comp)][col] = limb of the coefficient of output
//   col for that sample, k = 16 t + s - col - 1 (zero outside [0, 1023]).
//   66 chunks cover every (output, tap) pair exactly once: 1056 / 1024 = 3 %
//   zero products.  Per chunk: 2 A fragments (xl, xh) and 4 B fragments
//   (re/im output x low/high coefficient limb), 8 v_mfma_i32_32x32x32_i8 into
//   6 accumulators S0 = xl.vl, S1 = xl.vh + xh.vl, S2 = xh.vh per component;
//   C = S0 + (S1 << 8) + (S2 << 16) + bias.
// * K order.  The 32 k of a lane group hold 16 samples x (re, im); lane
//   (row or col = l & 31, group h = l >> 5) holds samples 8h..8h+7, 16 bytes,
//   in the same byte order for A and B (scripts/tune/mfma_i8_probe.py checks
//   that the instruction sums A byte j of lane (r, h) with B byte j of lane
//   (c, h) for every j and h).
// * LDS.  A: two byte planes (xl, xh), (re, im) per sample, 64 B per 32
//   samples with the four 16-B slots of a group XOR-swizzled by bits 2-3 of
//   the group index (the 16 lanes of a ds_read_b128 quarter, 16 consecutive
//   groups, hit 16 different bank quads; round 6's first version padded each
//   group to 80 B instead).  B: per kind, 4 copies of the limb array shifted by
//   0..3 entries so every lane's 8 entries start 8-B aligned (2 ds_read_b64);
//   built on the host, copied once per workgroup.  Energy: the inclusive
//   prefix P of |x|^2 over the staged span (uint32 wrap), e_i = P[i] - P[i-1024].
// * Grid.  Persistent, one 512-lane workgroup per CU (8 waves, 2 per SIMD),
//   8192 outputs per workgroup tile.  (Two 256-lane workgroups per CU, 4096
//   outputs each, measured level with one -- 0.8355 against 0.8384 ms -- and
//   no longer fit with the bank-conflict-free B copies.)
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v2i __attribute__((ext_vector_type(2)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

namespace {
constexpr int NP = 1024;                 // pattern length (config 5)
#ifndef WG_DESYNC
#define WG_DESYNC 0                      // s_sleep(127) rounds (~8k cycles each) for the second workgroup per CU
#endif
#ifndef PROBE_SKIP_SCAN
#define PROBE_SKIP_SCAN 0                // timing tests (wrong results): no energy prefix scan
#endif
#ifndef PROBE_SKIP_STAGE
#define PROBE_SKIP_STAGE 0               // ... or no staging after the first tile
#endif
#ifndef PROBE_SKIP_A
#define PROBE_SKIP_A 0
#endif
#ifndef PROBE_SKIP_B
#define PROBE_SKIP_B 0
#endif
#ifndef CORR_SCHED_BARRIER
#define CORR_SCHED_BARRIER 1             // sched_barrier around the MFMAs (the prefetch stays a prefetch); 0: without
#endif
#ifndef CORR_PREFETCH
#define CORR_PREFETCH 1                  // 0: no register prefetch of the next tile / next chunk (fewer VGPRs)
#endif
#ifndef CORR_WAVES
#define CORR_WAVES 8                     // waves per workgroup (8: one workgroup per CU)
#endif
#ifndef CORR_A_DPP
#define CORR_A_DPP 0                     // 1: A of chunk t+2 = A of chunk t one row on (DPP wave_shl:1), LDS only for row 31
#endif
constexpr int WAVES = CORR_WAVES;
constexpr int LANES = 64 * WAVES;
constexpr int TILE = 1024 * WAVES;       // outputs per workgroup tile
constexpr int SPAN = TILE + NP;          // staged samples per tile
constexpr int GROUPS = SPAN / 32;        // 32-sample groups
constexpr int PLANE = GROUPS * 64;       // bytes per limb plane (64 B per 32-sample group, swizzled)
constexpr int CHUNKS = (NP + 32) / 16;   // 66
constexpr int BENT = 1096;               // entries per B copy (2 B each)
constexpr int BSTRIDE = 2 * BENT;        // bytes per B copy
// copy sigma's base inside a kind: {0, 56, 120, 184} mod 256, so the 32 lanes of
// a ds_read_b64 (8 lanes per copy, 64 contiguous bytes each) cover the 64 banks
// exactly once (no bank conflicts; a uniform copy stride leaves 2-way ones)
constexpr int BKIND = 7096 + BSTRIDE;    // 4 shifted copies per kind
// B kinds: 2 pattern limbs -> re lo, re hi, im lo, im hi; 1 limb -> re, im
template <int PL> constexpr int BBYTES = 2 * PL * BKIND;
constexpr int LDS_A = 2 * PLANE;
constexpr int LDS_P = SPAN * 4;
template <int PL> constexpr int LDS_TOTAL = BBYTES<PL> + LDS_A + LDS_P + WAVES * 4;
constexpr int WG_PER_CU = WAVES >= 8 ? 1 : 8 / WAVES;  // 4, 8: 2 waves per SIMD; 12: 3
static_assert(2360 >= BSTRIDE && 4728 - 2360 >= BSTRIDE && 7096 - 4728 >= BSTRIDE, "B copies overlap");
static_assert(SPAN % 32 == 0 && TILE % 1024 == 0, "tile shape");
static_assert(WG_PER_CU * LDS_TOTAL<2> <= 160 * 1024, "LDS");
}  // namespace

// byte address of staged sample js in a limb plane: group js >> 5 (64 B), its
// 16-B slot (js >> 3) & 3 XOR-swizzled by bits 2-3 of the group, 2 B per sample
__device__ __forceinline__ int sample_addr(int js)
{
    const int g = js >> 5;
    return 64 * g + 16 * (((js >> 3) & 3) ^ ((g >> 2) & 3)) + 2 * (js & 7);
}

// a B fragment: 16 bytes at an 8-B aligned LDS address, as two b64 halves (a
// v4i load would be emitted as one ds_read_b128, which the LDS accepts at 8-B
// alignment in unaligned mode but serves ~2.4x slower: measured, round 6)
__device__ __forceinline__ v4i ld_b64x2(const unsigned char* p)
{
    const v2i a = *(const v2i*)p, b = *(const v2i*)(p + 8);
    return v4i{a[0], a[1], b[0], b[1]};
}

__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel)
{
    return __builtin_amdgcn_perm(hi, lo, sel);
}

// PL = 2: any pattern with |component| < 32640 (two limbs, S0..S2 per
// component, 8 MFMAs per chunk).  PL = 1: pattern = scale * q with every q
// component in [-128, 127] (the host factors out the gcd of the components,
// e.g. 500 for config 5's +-500 QPSK pattern): one limb, S0 = xl.q,
// S1 = xh.q, 4 MFMAs per chunk, C = scale (S0 + (S1 << 8) + bias) mod 2^32
// (exact: C = sum x (scale q) = scale sum x q in Z/2^32).
template <int PL>
__global__ void __launch_bounds__(LANES, WG_PER_CU)
corr_mfma_i8(const uint32_t* __restrict__ x, long n, const v4u* __restrict__ btab, int cs, uint32_t bias_re,
             uint32_t bias_im, uint32_t scale, uint32_t* __restrict__ corr_out, uint32_t* __restrict__ e_out,
             long n_tiles, int store_all)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    unsigned char* ldsB = lds;
    unsigned char* ldsA = lds + BBYTES<PL>;                 // xl plane, then xh plane
    uint32_t* ldsP = (uint32_t*)(lds + BBYTES<PL> + LDS_A);  // prefix of |x|^2
    uint32_t* ldsW = ldsP + SPAN;                        // per-wave totals of the scan

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int w = tid >> 6;
    const int h = lane >> 5;
    const int rc = lane & 31;  // A row / B col / D col

    // B tables, once per workgroup
    for (int i = tid; i < BBYTES<PL> / 16; i += LANES)
        ((v4u*)ldsB)[i] = btab[i];

    // per-lane LDS bases
    // A: group g = 32 w + row + (t >> 1), 16-B slot 2 (t & 1) + h of it, stored
    // at slot ^ ((g >> 2) & 3) (sample_addr): 16 consecutive rows are 16
    // consecutive groups, so a ds_read_b128 quarter hits 16 bank quads
    const int a_g0 = 32 * w + rc;
    // B: copy sigma = (col + 1) & 3, entry e = 16 t + 8 h - col + 31 + sigma (multiple of 4)
    const int sig = (rc + 1) & 3;
    const int copy_off[4] = {0, 2360, 4728, 7096};
    const int b_base = copy_off[sig] + 2 * (8 * h - rc + 31 + sig);

    // next tile's input, fetched into registers before the current tile's
    // MFMA work: granule g = tid + 512 k of the span; the buffer descriptor's
    // range check returns zeros past the end and, through the wrapped 32-bit
    // offset, before sample 0 (tile 0's history), i.e. the limbs of 0
    constexpr int NG = (SPAN / 4 + LANES - 1) / LANES;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, (int)(4 * n), 0x00020000);
    v4u pre[NG];
    auto fetch = [&](long tile) {
        const long j0 = tile * TILE - NP;
#pragma unroll
        for (int k = 0; k < NG; ++k) {
            const int g = tid + LANES * k;
            const uint32_t voff = (uint32_t)(4 * (j0 + 4 * g));
            pre[k] = v4u{0u, 0u, 0u, 0u};
            if (g < SPAN / 4)
                pre[k] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, 0));
        }
    };
    if (CORR_PREFETCH && blockIdx.x < n_tiles) fetch(blockIdx.x);
#if WG_DESYNC
    // two workgroups per CU start in phase and, doing identical work, stay in
    // phase: their staging / scan / epilogue phases coincide and the MFMAs
    // idle.  The second half of the grid (the second workgroup a CU receives)
    // starts about half a tile later, so one's non-MFMA phases run under the
    // other's MFMAs (tuning experiment).
    if (WG_PER_CU > 1 && blockIdx.x >= gridDim.x / 2)
        for (int i = 0; i < WG_DESYNC; ++i) __builtin_amdgcn_s_sleep(127);
#endif

    for (long tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const long i0 = tile * TILE;
        if (!CORR_PREFETCH) fetch(tile);
        __syncthreads();          // previous tile's readers are done with A and P
        // ---- staging: the prefetched granules -> limb planes and |x|^2
#pragma unroll
        for (int k = 0; k < (PROBE_SKIP_STAGE && tile != blockIdx.x ? 0 : NG); ++k) {
            const int g = tid + LANES * k;
            if (g >= SPAN / 4) break;
            const v4u v = pre[k];
            const int js = 4 * g;
            const int off = sample_addr(js);
            uint32_t lo0 = perm(v[1], v[0], 0x06040200u) ^ 0x80808080u;
            uint32_t lo1 = perm(v[3], v[2], 0x06040200u) ^ 0x80808080u;
            uint32_t hi0 = perm(v[1], v[0], 0x07050301u);
            uint32_t hi1 = perm(v[3], v[2], 0x07050301u);
            *(v2i*)(ldsA + off) = v2i{(int)lo0, (int)lo1};
            *(v2i*)(ldsA + PLANE + off) = v2i{(int)hi0, (int)hi1};
            v4u p;
#pragma unroll
            for (int q = 0; q < 4; ++q) {  // |x|^2 = re^2 + im^2, int32 wrap (correlators.h:237)
                const int re = (int16_t)(v[q] & 0xFFFFu), im = (int16_t)(v[q] >> 16);
                p[q] = (uint32_t)re * (uint32_t)re + (uint32_t)im * (uint32_t)im;
            }
            *(v4u*)(ldsP + js) = p;
        }
        __syncthreads();
        if (CORR_PREFETCH && tile + gridDim.x < n_tiles) fetch(tile + gridDim.x);
        // ---- energy: inclusive prefix of |x|^2 over the span (18 samples per lane)
        if (!PROBE_SKIP_SCAN) {
            constexpr int PER = (SPAN + LANES - 1) / LANES;  // 18 (a ragged last lane when LANES does not divide SPAN)
            uint32_t loc[PER];
            uint32_t s = 0;
#pragma unroll
            for (int q = 0; q < PER; ++q) {
                if (SPAN % LANES == 0 || PER * tid + q < SPAN) s += ldsP[PER * tid + q];
                loc[q] = s;
            }
            // wave-inclusive scan of the lane totals
            uint32_t incl = s;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                uint32_t o = __shfl_up(incl, d, 64);
                if (lane >= d) incl += o;
            }
            if (lane == 63) ldsW[w] = incl;
            __syncthreads();
            uint32_t base = incl - s;
            for (int q = 0; q < w; ++q) base += ldsW[q];
#pragma unroll
            for (int q = 0; q < PER; ++q)
                if (SPAN % LANES == 0 || PER * tid + q < SPAN) ldsP[PER * tid + q] = loc[q] + base;
        }
        __syncthreads();

        // ---- correlation: 66 chunks x 8 (PL = 2) or 4 (PL = 1) MFMAs; the
        // next chunk's fragments are read before the current chunk's MFMAs
        v16i s0r = {}, s1r = {}, s2r = {}, s0i = {}, s1i = {}, s2i = {};
        const unsigned char* pa = ldsA;
        const unsigned char* pb = ldsB + b_base;
        struct Frags { v4i xl, xh, rl, rh, il, ih; };
        auto load = [&](int t) {
            Frags f;
            const int g = a_g0 + (t >> 1);
            const int ao = 64 * g + 16 * ((2 * (t & 1) + h) ^ ((g >> 2) & 3));
            f.xl = *(const v4i*)(pa + ao);
            f.xh = *(const v4i*)(pa + PLANE + ao);
            const int bo = 32 * t;
            f.rl = ld_b64x2(pb + bo);
            if constexpr (PL == 2) {
                f.rh = ld_b64x2(pb + BKIND + bo);
                f.il = ld_b64x2(pb + 2 * BKIND + bo);
                f.ih = ld_b64x2(pb + 3 * BKIND + bo);
            } else {
                f.il = ld_b64x2(pb + BKIND + bo);
            }
            return f;
        };
        Frags cur = load(0);
#if CORR_A_DPP
        // A_{t+2}[row] = A_t[row + 1] (32 (row + 1) + 16 t = 32 row + 16 (t + 2)): the
        // next-but-one chunk's A fragments are this chunk's one lane on (DPP
        // wave_shl:1, lane l <- lane l + 1); only row 31 of each lane group (lanes
        // 31 and 63) reads its 16 bytes from LDS.  Halves the LDS bytes per chunk
        // with one limb (B stays 2 fragments from LDS).
        v4i a1l, a1h;
        {
            const Frags f1 = load(1);
            a1l = f1.xl;
            a1h = f1.xh;
        }
        auto shl1 = [](v4i v) {
            v4i r;
#pragma unroll
            for (int q = 0; q < 4; ++q) r[q] = __builtin_amdgcn_update_dpp(0, v[q], 0x130, 0xf, 0xf, false);
            return r;
        };
#pragma unroll 2
        for (int t = 0; t < CHUNKS; ++t) {
            const int tb = t + 1 < CHUNKS ? t + 1 : t;
            const unsigned char* pbt = pb + 32 * tb;
            v4i nrl = ld_b64x2(pbt), nrh = {}, nil, nih = {};
            if constexpr (PL == 2) {
                nrh = ld_b64x2(pbt + BKIND);
                nil = ld_b64x2(pbt + 2 * BKIND);
                nih = ld_b64x2(pbt + 3 * BKIND);
            } else {
                nil = ld_b64x2(pbt + BKIND);
            }
            v4i a2l = shl1(cur.xl), a2h = shl1(cur.xh);
            if (rc == 31) {
                const int t2 = t + 2 < CHUNKS ? t + 2 : t;
                const int g = a_g0 + (t2 >> 1);
                const int ao = 64 * g + 16 * ((2 * (t2 & 1) + h) ^ ((g >> 2) & 3));
                a2l = *(const v4i*)(pa + ao);
                a2h = *(const v4i*)(pa + PLANE + ao);
            }
#if CORR_SCHED_BARRIER
            __builtin_amdgcn_sched_barrier(0);
#endif
            s0r = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xl, cur.rl, s0r, 0, 0, 0);
            s0i = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xl, cur.il, s0i, 0, 0, 0);
            if constexpr (PL == 2) {
                s1r = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xl, cur.rh, s1r, 0, 0, 0);
                s1i = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xl, cur.ih, s1i, 0, 0, 0);
                s2r = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xh, cur.rh, s2r, 0, 0, 0);
                s2i = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xh, cur.ih, s2i, 0, 0, 0);
            }
            s1r = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xh, cur.rl, s1r, 0, 0, 0);
            s1i = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xh, cur.il, s1i, 0, 0, 0);
#if CORR_SCHED_BARRIER
            __builtin_amdgcn_sched_barrier(0);
#endif
            cur.xl = a1l;
            cur.xh = a1h;
            cur.rl = nrl;
            cur.rh = nrh;
            cur.il = nil;
            cur.ih = nih;
            a1l = a2l;
            a1h = a2h;
        }
#else
#pragma unroll 2
        for (int t = 0; t < CHUNKS; ++t) {
#if PROBE_SKIP_A || PROBE_SKIP_B
            // LDS-bound test (wrong results): odd chunks reuse the previous
            // chunk's A (or B) fragments instead of reading them
            Frags nxt = load(t + 1 < CHUNKS ? t + 1 : t);
            if ((t + 1) & 1) {
                if (PROBE_SKIP_A) { nxt.xl = cur.xl; nxt.xh = cur.xh; }
                if (PROBE_SKIP_B) { nxt.rl = cur.rl; nxt.rh = cur.rh; nxt.il = cur.il; nxt.ih = cur.ih; }
            }
#elif CORR_PREFETCH
            const Frags nxt = load(t + 1 < CHUNKS ? t + 1 : t);
#if CORR_SCHED_BARRIER
            // keep the next chunk's LDS reads above this chunk's MFMAs (the
            // scheduler otherwise sinks them next to their use, exposing the
            // LDS latency before an MFMA: measured, round 6)
            __builtin_amdgcn_sched_barrier(0);
#endif
#else
            cur = load(t);
#endif
            s0r = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xl, cur.rl, s0r, 0, 0, 0);
            s0i = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xl, cur.il, s0i, 0, 0, 0);
            if constexpr (PL == 2) {
                s1r = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xl, cur.rh, s1r, 0, 0, 0);
                s1i = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xl, cur.ih, s1i, 0, 0, 0);
                s2r = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xh, cur.rh, s2r, 0, 0, 0);
                s2i = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xh, cur.ih, s2i, 0, 0, 0);
            }
            s1r = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xh, cur.rl, s1r, 0, 0, 0);
            s1i = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xh, cur.il, s1i, 0, 0, 0);
#if CORR_PREFETCH || PROBE_SKIP_A || PROBE_SKIP_B
#if CORR_SCHED_BARRIER
            __builtin_amdgcn_sched_barrier(0);
#endif
            cur = nxt;
#endif
        }
#endif  // CORR_A_DPP

        // ---- epilogue: D layout col = l & 15.. 31, row = (r & 3) + 8 (r >> 2) + 4 h
        const unsigned es = (unsigned)(cs / 2) & 31u;
        const long iw = i0 + 1024 * w;
        const bool full = iw + 1024 <= n;
        uint32_t* co = corr_out + iw;
        uint32_t* eo = e_out + iw;
        // the window energies first: 32 LDS words read back to back (one wait),
        // not one wait per output between the conditional stores below
        uint32_t ew[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
            const int li = 1024 * w + 32 * row + rc + NP;  // local index of output iw + 32 row + rc
            ew[r] = ldsP[li] - ldsP[li - NP];
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
            const int o = 32 * row + rc;  // output iw + o
            uint32_t cr, ci;
            if constexpr (PL == 2) {
                cr = (uint32_t)s0r[r] + ((uint32_t)s1r[r] << 8) + ((uint32_t)s2r[r] << 16) + bias_re;
                ci = (uint32_t)s0i[r] + ((uint32_t)s1i[r] << 8) + ((uint32_t)s2i[r] << 16) + bias_im;
            } else {
                cr = scale * ((uint32_t)s0r[r] + ((uint32_t)s1r[r] << 8) + bias_re);
                ci = scale * ((uint32_t)s0i[r] + ((uint32_t)s1i[r] << 8) + bias_im);
            }
            // scale32 (dsp_complex.cpp:43-46), then :250; |t| < 2^22 for cs >= 7 (host check), so the
            // 24-bit multiplier gives the wrapped int32 squares
            // (the shift pair as one arithmetic shift by cs + 2; the sign extension from 24 bits is
            // exact here and lets the compiler use v_mul_i32_i24)
            const int sh = (cs & 31) + 2;
            const int32_t tr = (((int32_t)cr >> sh) << 8) >> 8;
            const int32_t ti = (((int32_t)ci >> sh) << 8) >> 8;
            const uint32_t corr = (uint32_t)(tr * tr) + (uint32_t)(ti * ti);
            // window (li - 1024, li] of local sample li = 1024 w + o + NP
            const uint32_t e = ew[r] >> es;
            if (store_all) {
                if (full || iw + o < n) {
                    co[o] = corr;
                    eo[o] = e;
                }
            } else if ((corr & e) == 0xFFFFFFFFu) {  // never (keeps the work live for timing)
                co[o] = corr;
                eo[o] = e;
            }
        }
    }
}

#ifndef CORR_ROWB
#define CORR_ROWB 1
#endif
#if CORR_ROWB == 2
// CORR_ROWB = 2 (one limb only): each wave owns TWO 32 x 32 output blocks
// (2048 consecutive outputs), so every B fragment read from LDS feeds two
// MFMAs (4 A + 2 B fragment reads per 8 MFMAs instead of 4 + 4): a third fewer
// LDS instructions per MFMA.  Tile 16384 outputs; its A planes and energy
// prefix take 139 KB of LDS (the two-limb B tables do not fit beside them); no
// register prefetch of the next tile (that would need 36 more VGPRs beside the
// 8 accumulators).
namespace {
constexpr int RB_TILE = 2048 * WAVES;
constexpr int RB_SPAN = RB_TILE + NP;
constexpr int RB_GROUPS = RB_SPAN / 32;
constexpr int RB_PLANE = RB_GROUPS * 64;
constexpr int RB_LDS = BBYTES<1> + 2 * RB_PLANE + RB_SPAN * 4 + WAVES * 4;
static_assert(RB_LDS <= 160 * 1024, "LDS");
}  // namespace

__global__ void __launch_bounds__(LANES, 1)
corr_mfma_i8_rb2(const uint32_t* __restrict__ x, long n, const v4u* __restrict__ btab, int cs, uint32_t bias_re,
                 uint32_t bias_im, uint32_t scale, uint32_t* __restrict__ corr_out, uint32_t* __restrict__ e_out,
                 long n_tiles, int store_all)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    unsigned char* ldsB = lds;
    unsigned char* ldsA = lds + BBYTES<1>;
    uint32_t* ldsP = (uint32_t*)(lds + BBYTES<1> + 2 * RB_PLANE);
    uint32_t* ldsW = ldsP + RB_SPAN;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, rc = lane & 31;
    for (int i = tid; i < BBYTES<1> / 16; i += LANES)
        ((v4u*)ldsB)[i] = btab[i];
    const int sig = (rc + 1) & 3;
    const int copy_off[4] = {0, 2360, 4728, 7096};
    const int b_base = copy_off[sig] + 2 * (8 * h - rc + 31 + sig);
    constexpr int NG2 = (RB_SPAN / 4 + LANES - 1) / LANES;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, (int)(4 * n), 0x00020000);
    for (long tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const long i0 = tile * RB_TILE;
        const long j0 = i0 - NP;
        v4u pre[NG2];
#pragma unroll
        for (int k = 0; k < NG2; ++k) {
            const int g = tid + LANES * k;
            pre[k] = v4u{0u, 0u, 0u, 0u};
            if (g < RB_SPAN / 4)
                pre[k] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(4 * (j0 + 4 * g)), 0, 0));
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < NG2; ++k) {
            const int g = tid + LANES * k;
            if (g >= RB_SPAN / 4) continue;  // (continue, not break: the loop must unroll, pre[] in registers)
            const v4u v = pre[k];
            const int js = 4 * g;
            const int off = sample_addr(js);
            *(v2i*)(ldsA + off) = v2i{(int)(perm(v[1], v[0], 0x06040200u) ^ 0x80808080u),
                                      (int)(perm(v[3], v[2], 0x06040200u) ^ 0x80808080u)};
            *(v2i*)(ldsA + RB_PLANE + off) = v2i{(int)perm(v[1], v[0], 0x07050301u), (int)perm(v[3], v[2], 0x07050301u)};
            v4u p;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int re = (int16_t)(v[q] & 0xFFFFu), im = (int16_t)(v[q] >> 16);
                p[q] = (uint32_t)re * (uint32_t)re + (uint32_t)im * (uint32_t)im;
            }
            *(v4u*)(ldsP + js) = p;
        }
        __syncthreads();
        {
            // (the lane's running sums are re-read in the second pass: 34 registers of
            // partial sums would not fit beside the 8 accumulators)
            constexpr int PER = (RB_SPAN + LANES - 1) / LANES;
            uint32_t s = 0;
            for (int q = 0; q < PER; ++q)
                if (RB_SPAN % LANES == 0 || PER * tid + q < RB_SPAN) s += ldsP[PER * tid + q];
            uint32_t incl = s;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t o = __shfl_up(incl, d, 64);
                if (lane >= d) incl += o;
            }
            if (lane == 63) ldsW[w] = incl;
            __syncthreads();
            uint32_t base = incl - s;
            for (int q = 0; q < w; ++q) base += ldsW[q];
            for (int q = 0; q < PER; ++q)
                if (RB_SPAN % LANES == 0 || PER * tid + q < RB_SPAN) {
                    base += ldsP[PER * tid + q];
                    ldsP[PER * tid + q] = base;
                }
        }
        __syncthreads();
        v16i s0r[2] = {}, s1r[2] = {}, s0i[2] = {}, s1i[2] = {};
        const unsigned char* pb = ldsB + b_base;
        struct F { v4i xl[2], xh[2], rl, il; };
        auto load = [&](int t) {
            F f;
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const int g = 32 * (2 * w + b) + rc + (t >> 1);
                const int ao = 64 * g + 16 * ((2 * (t & 1) + h) ^ ((g >> 2) & 3));
                f.xl[b] = *(const v4i*)(ldsA + ao);
                f.xh[b] = *(const v4i*)(ldsA + RB_PLANE + ao);
            }
            f.rl = ld_b64x2(pb + 32 * t);
            f.il = ld_b64x2(pb + BKIND + 32 * t);
            return f;
        };
        F cur = load(0);
#pragma unroll 2
        for (int t = 0; t < CHUNKS; ++t) {
            const F nxt = load(t + 1 < CHUNKS ? t + 1 : t);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                s0r[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xl[b], cur.rl, s0r[b], 0, 0, 0);
                s0i[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xl[b], cur.il, s0i[b], 0, 0, 0);
                s1r[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xh[b], cur.rl, s1r[b], 0, 0, 0);
                s1i[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xh[b], cur.il, s1i[b], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            cur = nxt;
        }
        const unsigned es = (unsigned)(cs / 2) & 31u;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const long iw = i0 + 2048 * w + 1024 * b;
            const bool full = iw + 1024 <= n;
            uint32_t ew[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
                const int li = 2048 * w + 1024 * b + 32 * row + rc + NP;
                ew[r] = ldsP[li] - ldsP[li - NP];
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
                const int o = 32 * row + rc;
                const uint32_t cr = scale * ((uint32_t)s0r[b][r] + ((uint32_t)s1r[b][r] << 8) + bias_re);
                const uint32_t ci = scale * ((uint32_t)s0i[b][r] + ((uint32_t)s1i[b][r] << 8) + bias_im);
                const int sh = (cs & 31) + 2;
                const int32_t tr = (((int32_t)cr >> sh) << 8) >> 8;
                const int32_t ti = (((int32_t)ci >> sh) << 8) >> 8;
                const uint32_t corr = (uint32_t)(tr * tr) + (uint32_t)(ti * ti);
                const uint32_t e = ew[r] >> es;
                if (store_all) {
                    if (full || iw + o < n) {
                        corr_out[iw + o] = corr;
                        e_out[iw + o] = e;
                    }
                } else if ((corr & e) == 0xFFFFFFFFu) {
                    corr_out[iw + o] = corr;
                    e_out[iw + o] = e;
                }
            }
        }
    }
}
#endif  // CORR_ROWB == 2

extern "C" int tune_corr_mfma_geometry(int* out)
{
    out[0] = TILE; out[1] = CHUNKS; out[2] = BENT; out[3] = BSTRIDE; out[4] = BKIND; out[5] = BBYTES<2>;
    out[6] = PLANE; out[7] = LDS_TOTAL<2>;
    return 0;
}

template <int PL>
static int launch(const void* x, long n, const void* btab, int cs, uint32_t bias_re, uint32_t bias_im,
                  uint32_t scale, void* corr_out, void* e_out, int grid, int store_all, hipStream_t s)
{
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)corr_mfma_i8<PL>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, LDS_TOTAL<PL>);
        if (e != hipSuccess) return (int)e;
        attr = true;
    }
    const long n_tiles = (n + TILE - 1) / TILE;
    if (n % 4 != 0 || 4 * n >= (1l << 31)) return 1;  // granule loads and the wrapped-offset zero fill
    if (cs < 7 || cs > 29) return 2;                      // the epilogue's shift by cs + 2 and 24-bit squares
    if (grid <= 0) grid = 256 * WG_PER_CU;
    if (grid > n_tiles) grid = (int)n_tiles;
    hipLaunchKernelGGL(corr_mfma_i8<PL>, dim3(grid), dim3(LANES), LDS_TOTAL<PL>, s, (const uint32_t*)x, n,
                       (const v4u*)btab, cs, bias_re, bias_im, scale, (uint32_t*)corr_out, (uint32_t*)e_out,
                       n_tiles, store_all);
    return (int)hipGetLastError();
}

// pattern_limbs 2: btab = 4 kinds, scale unused; 1: btab = 2 kinds of the
// pattern divided by `scale`, biases of that quotient pattern
extern "C" int tune_corr_mfma(const void* x, long n, const void* btab, int cs, uint32_t bias_re, uint32_t bias_im,
                              void* corr_out, void* e_out, int grid, int store_all, int pattern_limbs, uint32_t scale,
                              hipStream_t s)
{
#if CORR_ROWB == 2
    if (pattern_limbs != 1) return 3;  // the two-limb B tables do not fit beside the 16 k-output tile
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)corr_mfma_i8_rb2, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           RB_LDS);
        if (e != hipSuccess) return (int)e;
        attr = true;
    }
    if (n % 4 != 0 || 4 * n >= (1l << 31)) return 1;
    if (cs < 7 || cs > 29) return 2;
    const long n_tiles = (n + RB_TILE - 1) / RB_TILE;
    if (grid <= 0) grid = 256;
    if (grid > n_tiles) grid = (int)n_tiles;
    hipLaunchKernelGGL(corr_mfma_i8_rb2, dim3(grid), dim3(LANES), RB_LDS, s, (const uint32_t*)x, n, (const v4u*)btab,
                       cs, bias_re, bias_im, scale, (uint32_t*)corr_out, (uint32_t*)e_out, n_tiles, store_all);
    return (int)hipGetLastError();
#endif
    if (pattern_limbs == 1)
        return launch<1>(x, n, btab, cs, bias_re, bias_im, scale, corr_out, e_out, grid, store_all, s);
    return launch<2>(x, n, btab, cs, bias_re, bias_im, 1u, corr_out, e_out, grid, store_all, s);
}
