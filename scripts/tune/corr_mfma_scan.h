// corr_mfma_scan.h -- TUNING VARIANT, never the product.  Included into a
// patched copy of srcdsp_amd/csrc/corr.hip by scripts/tune/variant_lib.py
// ("corrmfma" -> scripts/tune/ab/libsrcdsp_hip_corrmfma.so); BASELINE
// north_star says the product path uses no MFMA, so libsrcdsp_hip.so never
// contains this code.
//
// What it is: scripts/tune/corr_mfma.hip's i8 matrix-core correlator (the
// limb / Toeplitz-tile formulation is described there) behind the product's
// own C ABI, in place of corr_scan_s1 on the path the bench's config 5 takes
// (srcdsp_corr_step, detect on, no debug trace, N = 1024, S = 1), with the
// parts the probe left out:
// * the stream's history: samples before the call come from the N*S-1 history
//   words (corr_fetch's rule), so a continued stream is exact too;
// * detection fused into the tile: each tile's corr / energy words go to LDS
//   (over the A planes and the energy prefix, which the tile no longer needs)
//   and every output but the tile's first two takes the 3-point test there;
//   corr_mfma_seams tests the first two of each tile from the words the tile
//   before it left in a small seam array;
// * early exit: a workgroup stops at the first tile that starts after a
//   recorded hit (the first detection is the atomicMin over all hits, so no
//   hit past it matters); the registers after the call come from corr_point,
//   as on the product's fused path.
// Per-sample HBM traffic is the 4 B input read (no per-sample scratch).
// * one limb: each wave owns two 32 x 32 output blocks (RB = 2, 16 k-output
//   tiles), so each B fragment read feeds two MFMAs (the probe's CORR_ROWB = 2:
//   -8 %); two limbs keep one block per wave (their B tables leave no LDS for
//   the larger tile).

namespace cmf {
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v2i __attribute__((ext_vector_type(2)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

constexpr int NP = 1024;
constexpr int WAVES = 8;
constexpr int LANES = 64 * WAVES;
constexpr int CHUNKS = (NP + 32) / 16;
constexpr int BENT = 1096;
constexpr int BSTRIDE = 2 * BENT;
constexpr int BKIND = 7096 + BSTRIDE;
constexpr int COPY_OFF[4] = {0, 2360, 4728, 7096};
template <int PL> constexpr int BBYTES = 2 * PL * BKIND;
// RB = output row blocks (32 x 32) per wave: 1, or 2 (one limb only: each B
// fragment read feeds two MFMAs; the 16 k-output tile's planes and prefix take
// 139 KB of LDS, no room for the two-limb B tables)
template <int RB> constexpr int TILE = 1024 * WAVES * RB;
template <int RB> constexpr int SPAN = TILE<RB> + NP;
template <int RB> constexpr int PLANE = SPAN<RB> / 32 * 64;
template <int PL, int RB> constexpr int LDS_TOTAL = BBYTES<PL> + 2 * PLANE<RB> + 4 * SPAN<RB> + 16 * 4;
constexpr int SEAM_WORDS = 8;
static_assert(4 * TILE<2> <= 2 * PLANE<2> && 4 * TILE<1> <= 2 * PLANE<1>, "corr words reuse the A planes");
static_assert(LDS_TOTAL<2, 1> <= 160 * 1024 && LDS_TOTAL<1, 2> <= 160 * 1024, "LDS");

__device__ __forceinline__ int sample_addr(int js)
{
    const int g = js >> 5;
    return 64 * g + 16 * (((js >> 3) & 3) ^ ((g >> 2) & 3)) + 2 * (js & 7);
}

__device__ __forceinline__ v4i ld_b64x2(const unsigned char* p)
{
    const v2i a = *(const v2i*)p, b = *(const v2i*)(p + 8);
    return v4i{a[0], a[1], b[0], b[1]};
}
}  // namespace cmf

template <int PL, int RB>
__global__ void __launch_bounds__(cmf::LANES, 1)
corr_scan_mfma(const uint32_t* __restrict__ x, long n, const uint32_t* __restrict__ hist,
               const cmf::v4u* __restrict__ btab, int cs, uint32_t bias_re, uint32_t bias_im, uint32_t scale,
               uint32_t* __restrict__ seams, unsigned* best)
{
    using namespace cmf;
    static_assert(RB == 1 || PL == 1, "two row blocks per wave: one limb only");
    constexpr int T = TILE<RB>, SP = SPAN<RB>, PLN = PLANE<RB>;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    unsigned char* ldsB = lds;
    unsigned char* ldsA = lds + BBYTES<PL>;
    uint32_t* ldsP = (uint32_t*)(lds + BBYTES<PL> + 2 * PLN);
    uint32_t* ldsW = ldsP + SP;        // per-wave scan totals, then the stop word
    uint32_t* ldsC = (uint32_t*)ldsA;  // the tile's corr words (after the MFMAs)

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int w = tid >> 6;
    const int h = lane >> 5;
    const int rc = lane & 31;
    const long n_tiles = (n + T - 1) / T;

    for (int i = tid; i < BBYTES<PL> / 16; i += LANES)
        ((v4u*)ldsB)[i] = btab[i];
    const int sig = (rc + 1) & 3;
    const int b_base = COPY_OFF[sig] + 2 * (8 * h - rc + 31 + sig);

    // RB = 1: the next tile's input is fetched into registers before this
    // tile's MFMAs; RB = 2: at the tile's start (no VGPRs for a prefetch beside
    // the 8 accumulators)
    constexpr int NG = (SP / 4 + LANES - 1) / LANES;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, (int)(4 * n), 0x00020000);
    v4u pre[NG];
    auto fetch = [&](long tile) {
        const long j0 = tile * T - NP;
#pragma unroll
        for (int k = 0; k < NG; ++k) {
            const int g = tid + LANES * k;
            pre[k] = v4u{0u, 0u, 0u, 0u};
            if (g < SP / 4) {
                const long j = j0 + 4 * g;
                if (j >= 0) {  // past the end: the descriptor's range check returns zeros
                    pre[k] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(4 * j), 0, 0));
                } else {  // before the call: the history (N*S-1 = 1023 words), zeros before it
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        pre[k][q] = j + q + (NP - 1) >= 0 ? hist[j + q + (NP - 1)] : 0u;
                }
            }
        }
    };
    if (RB == 1 && blockIdx.x < n_tiles) fetch(blockIdx.x);

    for (long tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const long i0 = tile * T;
        if (tid == 0) ldsW[WAVES] = __hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();  // previous tile's readers are done; the stop word is visible
        if ((long)ldsW[WAVES] < i0) break;  // a hit before this tile: nothing here can be the first
        if constexpr (RB == 2) fetch(tile);
#pragma unroll
        for (int k = 0; k < NG; ++k) {
            const int g = tid + LANES * k;
            if (g >= SP / 4) continue;  // (not break: the loop must unroll, pre[] stays in registers)
            const v4u v = pre[k];
            const int js = 4 * g;
            const int off = sample_addr(js);
            const uint32_t lo0 = __builtin_amdgcn_perm(v[1], v[0], 0x06040200u) ^ 0x80808080u;
            const uint32_t lo1 = __builtin_amdgcn_perm(v[3], v[2], 0x06040200u) ^ 0x80808080u;
            const uint32_t hi0 = __builtin_amdgcn_perm(v[1], v[0], 0x07050301u);
            const uint32_t hi1 = __builtin_amdgcn_perm(v[3], v[2], 0x07050301u);
            *(v2i*)(ldsA + off) = v2i{(int)lo0, (int)lo1};
            *(v2i*)(ldsA + PLN + off) = v2i{(int)hi0, (int)hi1};
            v4u p;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int re = (int16_t)(v[q] & 0xFFFFu), im = (int16_t)(v[q] >> 16);
                p[q] = (uint32_t)re * (uint32_t)re + (uint32_t)im * (uint32_t)im;
            }
            *(v4u*)(ldsP + js) = p;
        }
        __syncthreads();
        if (RB == 1 && tile + gridDim.x < n_tiles) fetch(tile + gridDim.x);
        {   // energy: inclusive prefix of |x|^2 over the span
            constexpr int PER = (SP + LANES - 1) / LANES;
            uint32_t s = 0;
            uint32_t loc[RB == 1 ? PER : 1];  // RB = 2: the running sums are re-read instead
#pragma unroll
            for (int q = 0; q < PER; ++q) {
                if (SP % LANES == 0 || PER * tid + q < SP) s += ldsP[PER * tid + q];
                if constexpr (RB == 1) loc[q] = s;
            }
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
#pragma unroll
            for (int q = 0; q < PER; ++q)
                if (SP % LANES == 0 || PER * tid + q < SP) {
                    if constexpr (RB == 1) {
                        ldsP[PER * tid + q] = loc[q] + base;
                    } else {
                        base += ldsP[PER * tid + q];
                        ldsP[PER * tid + q] = base;
                    }
                }
        }
        __syncthreads();

        // ---- correlation: wave w owns row blocks RB w .. RB w + RB - 1 (1024 outputs each)
        v16i s0r[RB] = {}, s1r[RB] = {}, s2r[RB] = {}, s0i[RB] = {}, s1i[RB] = {}, s2i[RB] = {};
        const unsigned char* pb = ldsB + b_base;
        struct Frags { v4i xl[RB], xh[RB], rl, rh, il, ih; };
        auto load = [&](int t) {
            Frags f;
#pragma unroll
            for (int b = 0; b < RB; ++b) {
                const int g = 32 * (RB * w + b) + rc + (t >> 1);
                const int ao = 64 * g + 16 * ((2 * (t & 1) + h) ^ ((g >> 2) & 3));
                f.xl[b] = *(const v4i*)(ldsA + ao);
                f.xh[b] = *(const v4i*)(ldsA + PLN + ao);
            }
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
#pragma unroll 2
        for (int t = 0; t < CHUNKS; ++t) {
            const Frags nxt = load(t + 1 < CHUNKS ? t + 1 : t);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int b = 0; b < RB; ++b) {
                s0r[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xl[b], cur.rl, s0r[b], 0, 0, 0);
                s0i[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xl[b], cur.il, s0i[b], 0, 0, 0);
                if constexpr (PL == 2) {
                    s1r[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xl[b], cur.rh, s1r[b], 0, 0, 0);
                    s1i[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xl[b], cur.ih, s1i[b], 0, 0, 0);
                    s2r[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xh[b], cur.rh, s2r[b], 0, 0, 0);
                    s2i[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xh[b], cur.ih, s2i[b], 0, 0, 0);
                }
                s1r[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xh[b], cur.rl, s1r[b], 0, 0, 0);
                s1i[b] = __builtin_amdgcn_mfma_i32_32x32x32_i8(cur.xh[b], cur.il, s1i[b], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            cur = nxt;
        }

        // corr (correlators.h:233-250 via scale32, dsp_complex.cpp:43-46) and
        // energy words of the wave's outputs, D layout row = (r & 3) + 8 (r >> 2)
        // + 4 h, col = rc, in block b at tile output 1024 (RB w + b)
        const unsigned es = (unsigned)(cs / 2) & 31u;
        uint32_t cv[RB][16], ev[RB][16];
#pragma unroll
        for (int b = 0; b < RB; ++b) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
                const int li = 1024 * (RB * w + b) + 32 * row + rc + NP;
                ev[b][r] = (ldsP[li] - ldsP[li - NP]) >> es;
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                uint32_t cr, ci;
                if constexpr (PL == 2) {
                    cr = (uint32_t)s0r[b][r] + ((uint32_t)s1r[b][r] << 8) + ((uint32_t)s2r[b][r] << 16) + bias_re;
                    ci = (uint32_t)s0i[b][r] + ((uint32_t)s1i[b][r] << 8) + ((uint32_t)s2i[b][r] << 16) + bias_im;
                } else {
                    cr = scale * ((uint32_t)s0r[b][r] + ((uint32_t)s1r[b][r] << 8) + bias_re);
                    ci = scale * ((uint32_t)s0i[b][r] + ((uint32_t)s1i[b][r] << 8) + bias_im);
                }
                const int sh = (cs & 31) + 2;
                const int32_t tr = (((int32_t)cr >> sh) << 8) >> 8;
                const int32_t ti = (((int32_t)ci >> sh) << 8) >> 8;
                cv[b][r] = (uint32_t)(tr * tr) + (uint32_t)(ti * ti);
            }
        }
        __syncthreads();  // every wave is done with the A planes and the prefix
#pragma unroll
        for (int b = 0; b < RB; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
                const int o = 1024 * (RB * w + b) + 32 * row + rc;
                ldsC[o] = cv[b][r];
                ldsP[o] = ev[b][r];
            }
        __syncthreads();
        // the 3-point test (correlators.h:262-268) of tile outputs o >= 2,
        // o = 1024 RB w + 64 q + lane: consecutive lanes read consecutive words
        const long nrem = n - i0;
        int hit = -1;
#pragma unroll 4
        for (int q = 0; q < 16 * RB; ++q) {
            const int o = 1024 * RB * w + 64 * q + lane;
            if (o >= 2 && o < nrem && corr_hit(ldsC[o - 2], ldsC[o - 1], ldsC[o], ldsP[o - 1])) {
                hit = o;
                break;
            }
        }
        if (hit >= 0) atomicMin(best, (unsigned)(i0 + hit));
        if (tid < 6) {  // the seam words: corr[0], corr[1], en[0], corr[T-2], corr[T-1], en[T-1]
            const int src[6] = {0, 1, 0, T - 2, T - 1, T - 1};
            const uint32_t v = (tid == 2 || tid == 5) ? ldsP[src[tid]] : ldsC[src[tid]];
            seams[SEAM_WORDS * tile + tid] = v;
        }
    }
}

// the first two outputs of every scanned tile, from the seam words of the tile
// and of the one before it (tile 0: the registers from before the call, as
// corr_detect's c_prev0 / c_prev1 / e_prev0)
__global__ void corr_mfma_seams(const uint32_t* __restrict__ seams, long n, long tile_outputs, uint32_t c_prev0,
                                uint32_t c_prev1, uint32_t e_prev0, unsigned* best)
{
    const long n_tiles = (n + tile_outputs - 1) / tile_outputs;
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_tiles) return;
    const long i0 = t * tile_outputs;
    if ((long)__hip_atomic_load(best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < i0) return;  // not scanned
    const uint32_t* s = seams + cmf::SEAM_WORDS * t;
    uint32_t pc2 = c_prev1, pc1 = c_prev0, pe1 = e_prev0;  // corr[i0-2], corr[i0-1], en[i0-1]
    if (t > 0) {
        const uint32_t* p = seams + cmf::SEAM_WORDS * (t - 1);
        pc2 = p[3];
        pc1 = p[4];
        pe1 = p[5];
    }
    const uint32_t c0 = s[0], c1 = s[1], e0 = s[2];
    unsigned hit = 0xffffffffu;
    if (i0 + 1 < n && corr_hit(pc1, c0, c1, e0)) hit = (unsigned)(i0 + 1);
    if (corr_hit(pc2, pc1, c0, pe1)) hit = (unsigned)i0;
    if (hit != 0xffffffffu) atomicMin(best, hit);
}

// ---- host side: the B tables of the pattern (scripts/tune/corr_mfma.py btables)
static uint32_t cmf_gcd(uint32_t a, uint32_t b)
{
    while (b) {
        const uint32_t t = a % b;
        a = b;
        b = t;
    }
    return a;
}

// from the conjugated pattern h_coef (c = conj(p)): re output pair (c.re, -c.im),
// im output pair (c.im, c.re) per tap, components (x.re, x.im)
static int corr_mfma_prepare(srcdsp_corr_state& c)
{
    using namespace cmf;
    c.mfma_pl = 0;
    const char* off = getenv("SRCDSP_CORR_MFMA");
    if (off && off[0] == '0') return SRCDSP_OK;
    if (c.N != (unsigned)NP || c.S != 1 || !c.taps16) return SRCDSP_OK;
    std::vector<int32_t> pair[2];
    pair[0].resize(2 * NP);
    pair[1].resize(2 * NP);
    uint32_t g = 0;
    for (int k = 0; k < NP; ++k) {
        const int32_t cr = c.h_coef[2 * k], ci = c.h_coef[2 * k + 1];
        pair[0][2 * k] = cr;
        pair[0][2 * k + 1] = -ci;
        pair[1][2 * k] = ci;
        pair[1][2 * k + 1] = cr;
        g = cmf_gcd(g, (uint32_t)std::abs(cr));
        g = cmf_gcd(g, (uint32_t)std::abs(ci));
    }
    if (g == 0) return SRCDSP_OK;  // the zero pattern: no scaling exponent (the product path)
    int pl = 1;
    for (int o = 0; o < 2 && pl == 1; ++o)
        for (int32_t v : pair[o])
            if (v / (int32_t)g < -128 || v / (int32_t)g > 127) {
                pl = 2;
                break;
            }
    const char* force = getenv("SRCDSP_CORR_MFMA_PL");
    if (force && force[0] == '2') pl = 2;
    const uint32_t scale = pl == 1 ? g : 1u;
    std::vector<uint8_t> img((size_t)BBYTES<2>, 0);
    uint32_t bias[2] = {0u, 0u};
    for (int o = 0; o < 2; ++o) {
        std::vector<int8_t> limb[2];
        limb[0].resize(2 * NP);
        limb[1].resize(2 * NP);
        for (int m = 0; m < 2 * NP; ++m) {
            const int32_t v = pl == 1 ? pair[o][m] / (int32_t)scale : pair[o][m];
            bias[o] += 128u * (uint32_t)v;
            if (pl == 1) {
                limb[0][m] = (int8_t)v;
            } else {
                const int32_t vl = ((v + 128) & 255) - 128, vh = (v - vl) >> 8;
                if (vh < -128 || vh > 127) return SRCDSP_OK;  // outside two limbs: the product path
                limb[0][m] = (int8_t)vl;
                limb[1][m] = (int8_t)vh;
            }
        }
        for (int lb = 0; lb < pl; ++lb) {
            const int kind = pl * o + lb;  // pl 2: re lo, re hi, im lo, im hi; pl 1: re, im
            for (int sg = 0; sg < 4; ++sg) {
                uint8_t* base = img.data() + (size_t)kind * BKIND + COPY_OFF[sg];
                for (int e = 0; e < BENT; ++e) {
                    const int k = e - sg - 32;
                    if (k < 0 || k >= NP) continue;
                    base[2 * e] = (uint8_t)limb[lb][2 * k];
                    base[2 * e + 1] = (uint8_t)limb[lb][2 * k + 1];
                }
            }
        }
    }
    if (!c.d_mfma_b) SRCDSP_HIP_TRY(hipMalloc(&c.d_mfma_b, (size_t)BBYTES<2>));
    SRCDSP_HIP_TRY(hipMemcpy(c.d_mfma_b, img.data(), (size_t)BBYTES<2>, hipMemcpyHostToDevice));
    c.mfma_pl = pl;
    c.mfma_scale = scale;
    c.mfma_bias[0] = bias[0];
    c.mfma_bias[1] = bias[1];
    return SRCDSP_OK;
}

static bool corr_mfma_usable(const srcdsp_corr_state& c, const uint32_t* d_in, long n)
{
    const int cs = c.coeff_scaling;
    return c.mfma_pl != 0 && cs >= 7 && cs <= 29 && n % 4 == 0 && 4 * n < (1L << 31) &&
           ((uintptr_t)d_in & 15) == 0;
}

template <int PL, int RB>
static int corr_mfma_launch_t(srcdsp_corr_state& c, const uint32_t* d_in, long n, const uint32_t* hist,
                              hipStream_t s)
{
    using namespace cmf;
    static bool attr = false;
    if (!attr) {
        SRCDSP_HIP_TRY(hipFuncSetAttribute((const void*)corr_scan_mfma<PL, RB>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, LDS_TOTAL<PL, RB>));
        attr = true;
    }
    const long n_tiles = (n + TILE<RB> - 1) / TILE<RB>;
    if ((size_t)n_tiles > c.seams_cap) {
        if (c.d_seams) (void)hipFree(c.d_seams);
        c.d_seams = nullptr;
        c.seams_cap = 0;
        SRCDSP_HIP_TRY(hipMalloc(&c.d_seams, 4 * SEAM_WORDS * (size_t)n_tiles));
        c.seams_cap = (size_t)n_tiles;
    }
    const int grid = (int)std::min<long>(256, n_tiles);
    hipLaunchKernelGGL((corr_scan_mfma<PL, RB>), dim3(grid), dim3(LANES), (LDS_TOTAL<PL, RB>), s, d_in, n, hist,
                       (const v4u*)c.d_mfma_b, c.coeff_scaling, c.mfma_bias[0], c.mfma_bias[1], c.mfma_scale,
                       c.d_seams, c.d_best);
    SRCDSP_HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(corr_mfma_seams, dim3((unsigned)((n_tiles + 255) / 256)), dim3(256), 0, s,
                       (const uint32_t*)c.d_seams, n, (long)TILE<RB>, c.corr[0], c.corr[1], c.energy[0], c.d_best);
    SRCDSP_HIP_TRY(hipGetLastError());
    return SRCDSP_OK;
}

static long g_corr_mfma_launches = 0;  // calls that took the matrix-core scan (the A/B scripts check it)

extern "C" __attribute__((visibility("default"))) long srcdsp_tune_corr_mfma_launches() { return g_corr_mfma_launches; }

static int corr_mfma_launch(srcdsp_corr_state& c, const uint32_t* d_in, long n, const uint32_t* hist, hipStream_t s)
{
    ++g_corr_mfma_launches;
    if (c.mfma_pl == 2) return corr_mfma_launch_t<2, 1>(c, d_in, n, hist, s);
    // one limb: two row blocks per wave unless SRCDSP_CORR_MFMA_RB=1 (A/B)
    const char* rb = getenv("SRCDSP_CORR_MFMA_RB");
    if (rb && rb[0] == '1') return corr_mfma_launch_t<1, 1>(c, d_in, n, hist, s);
    return corr_mfma_launch_t<1, 2>(c, d_in, n, hist, s);
}
