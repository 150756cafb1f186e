// mixdecim_mfma_step.h -- TUNING VARIANT, never the product.  Included into a
// patched copy of srcdsp_amd/csrc/decim.hip by scripts/tune/variant_lib.py
// ("mixmfma" -> scripts/tune/ab/libsrcdsp_hip_mixmfma.so); BASELINE north_star
// says the product path uses no MFMA, so libsrcdsp_hip.so never contains it.
//
// scripts/tune/mixdecim_mfma.hip's kernel (config 4's tap loop on
// v_mfma_i32_16x16x64_i8 through int8 limbs; the layout is described there)
// behind the product's own srcdsp_mixdecim_step, with what the probe left out:
// * the decimator's history: staged samples before the call are the H = N-1
//   history words (already mixed), zeros before them; workgroup 0 writes the
//   new history (the last H samples of history ++ mixed input) first;
// * the mixer's state: phase phi0 and step freq of the call (any power-of-two
//   table length up to 4096, so every tile's lane phases are the same: N
//   divides the tile's 8192 input samples), words made from the mixer's own
//   table on the device;
// * any tap count up to 128 with |c| < 32640 (two limbs), any shift 1..31
//   (limitScale16 as the product's limit16_pair_sh), any length (the last tile
//   reads zeros past the end and stores only outputs < n_out);
// * the tap fragments built on the host per decimator, rebuilt when its taps
//   change (a side table keyed by the decimator's address and its taps);
// * the same kernel without the mixer serves the plain complex<int16_t>
//   decimator's step (row a2, core_step).

namespace mmf {
typedef int v4i __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef short v2s __attribute__((ext_vector_type(2)));

constexpr int LANES = 512;
constexpr int WAVES = LANES / 64;
constexpr int TILE = 2048;
constexpr int HALO = 128;
constexpr int SPAN = 4 * TILE + HALO;
constexpr int GRAN = SPAN / 4;
constexpr int NG = (GRAN + LANES - 1) / LANES;
constexpr int BLK64 = SPAN / 64;
constexpr int PLANE = BLK64 * 80;
constexpr int P_RE_LO = 0, P_IM_LO = 10624, P_RE_HI = 21248, P_IM_HI = 31872;
constexpr int LDS_TOTAL = P_IM_HI + PLANE;
constexpr int WT_PER_TILE = TILE / 128;
constexpr int MAX_TAPS = 128;
static_assert(2 * LDS_TOTAL <= 160 * 1024, "2 workgroups per CU");

__device__ __forceinline__ int32_t sdot2w(uint32_t a, uint32_t b)
{
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(v2s, a), __builtin_bit_cast(v2s, b), 0, false);
}

// limitScale16 pair (dsp_complex.cpp:63-73) after an arithmetic shift 1..31
__device__ __forceinline__ uint32_t pack_clamp_sh(int re, int im, unsigned sh)
{
    const v2s v = __builtin_bit_cast(v2s, __builtin_amdgcn_cvt_pk_i16(re >> sh, im >> sh));
    const v2s lo = {-32767, -32767};
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(v, lo));
}

// the mixer (mixers.h:169-188) on one packed sample at table phase ph:
// A = (cos, -sin), B = (sin, cos), cos = T[(ph + N/4) mod N], sin = T[ph]
__device__ __forceinline__ v2u mix_words(const int16_t* tab, unsigned ph, unsigned N)
{
    const unsigned ic = (ph + N / 4) & (N - 1);
    const uint32_t c = (uint16_t)tab[ic], s = (uint16_t)tab[ph];
    return v2u{c | ((uint32_t)(uint16_t)(-tab[ph]) << 16), s | (c << 16)};
}
}  // namespace mmf

// MIX = false: the plain complex<int16_t> decimator (row a2's srcdsp_decim_step):
// the staged samples are the input itself
template <bool MIX>
__global__ void __launch_bounds__(mmf::LANES, 2)
mixdecim_mfma_step_i8(const uint32_t* __restrict__ x, long n_in, const uint32_t* __restrict__ hist, int H,
                      uint32_t* __restrict__ hist_out, const mmf::v4i* __restrict__ bfrag,
                      const int16_t* __restrict__ tab, unsigned N, uint32_t phi0, uint32_t freq, uint32_t bias, unsigned sh, uint32_t* __restrict__ y, long n_tiles)
{
    using namespace mmf;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int w = tid >> 6;

    // lane tid's granules g = tid + LANES k start at staged sample 4 g of every
    // tile (global sample tile * 4 TILE - HALO + 4 g); N | 4 TILE, so their
    // phases are the same in every tile (mod 2^32 arithmetic: N is a power of 2)
    v2u tw[MIX ? NG : 1][4];
    if constexpr (MIX) {
#pragma unroll
        for (int k = 0; k < NG; ++k) {
            const int g = tid + LANES * k;
            uint32_t ph = (phi0 + (uint32_t)(4 * g - HALO) * freq) & (N - 1);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                tw[k][q] = mix_words(tab, ph, N);
                ph = (ph + freq) & (N - 1);
            }
        }
    }
    v4i B[6];
#pragma unroll
    for (int f = 0; f < 6; ++f)
        B[f] = bfrag[64 * f + lane];

    const long n_out = n_in / 4;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, (int)(4 * n_in), 0x00020000);
    v4u pre[NG];
    auto fetch = [&](long tile) {
        const long j0 = tile * (4 * TILE) - HALO;
#pragma unroll
        for (int k = 0; k < NG; ++k) {
            const int g = tid + LANES * k;
            pre[k] = v4u{0u, 0u, 0u, 0u};
            if (g < GRAN)  // before the call (tile 0): out of range (wrapped offset) -> 0; history at staging
                pre[k] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(
                                                     rs, (uint32_t)(4 * (j0 + 4 * g)), 0, 2));
        }
    };
    if (blockIdx.x < n_tiles) fetch(blockIdx.x);
    if (blockIdx.x == 0) {  // the new history: (hist ++ mixed input)[n_in + k], k < H
        for (int k = tid; k < H; k += LANES) {
            const long idx = n_in - H + k;
            uint32_t wv;
            if (idx >= 0) {
                wv = x[idx];
                if constexpr (MIX) {
                    const v2u t = mix_words(tab, (phi0 + (uint32_t)idx * freq) & (N - 1), N);
                    wv = pack_clamp_sh(sdot2w(wv, t[0]), sdot2w(wv, t[1]), 14u);
                }
            } else {
                wv = hist[H + idx];
            }
            hist_out[k] = wv;
        }
    }

    const int row = lane & 15, h = lane >> 4;
    const int a_re_im = (row & 1) ? (P_IM_LO - P_RE_LO) : 0;
    const int col = lane & 15, g4 = lane >> 4;

    for (long tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        __syncthreads();
#pragma unroll
        for (int k = 0; k < NG; ++k) {
            const int g = tid + LANES * k;
            if (g >= GRAN) break;
            const v4u v = pre[k];
            uint32_t m[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if constexpr (MIX) {
                    const v2u t = tw[k][q];
                    m[q] = pack_clamp_sh(sdot2w(v[q], t[0]), sdot2w(v[q], t[1]), 14u);
                } else {
                    m[q] = v[q];
                }
            }
            const uint32_t t0 = __builtin_amdgcn_perm(m[1], m[0], 0x05010400u);
            const uint32_t t1 = __builtin_amdgcn_perm(m[3], m[2], 0x05010400u);
            const uint32_t u0 = __builtin_amdgcn_perm(m[1], m[0], 0x07030602u);
            const uint32_t u1 = __builtin_amdgcn_perm(m[3], m[2], 0x07030602u);
            const int js = 4 * g;
            const int off = 80 * (js >> 6) + (js & 63);
            *(uint32_t*)(lds + P_RE_LO + off) = __builtin_amdgcn_perm(t1, t0, 0x05040100u) ^ 0x80808080u;
            *(uint32_t*)(lds + P_RE_HI + off) = __builtin_amdgcn_perm(t1, t0, 0x07060302u);
            *(uint32_t*)(lds + P_IM_LO + off) = __builtin_amdgcn_perm(u1, u0, 0x05040100u) ^ 0x80808080u;
            *(uint32_t*)(lds + P_IM_HI + off) = __builtin_amdgcn_perm(u1, u0, 0x07060302u);
        }
        __syncthreads();
        if (tile == 0 && H > 0) {
            // the decimator's history (mixed samples) in place of the staged
            // samples before the call (staged as 0: the buffer's range check);
            // once, outside the staging loop (a per-granule branch there cost
            // 56 VGPRs: one workgroup per CU instead of two)
            for (int js = HALO - H + tid; js < HALO; js += LANES) {
                const uint32_t mv = hist[js - HALO + H];
                const int off = 80 * (js >> 6) + (js & 63);
                lds[P_RE_LO + off] = (unsigned char)((mv & 0xFFu) ^ 0x80u);
                lds[P_RE_HI + off] = (unsigned char)(mv >> 8);
                lds[P_IM_LO + off] = (unsigned char)(((mv >> 16) & 0xFFu) ^ 0x80u);
                lds[P_IM_HI + off] = (unsigned char)(mv >> 24);
            }
            __syncthreads();
        }
        if (tile + gridDim.x < n_tiles) fetch(tile + gridDim.x);

        for (int wt = w; wt < WT_PER_TILE; wt += WAVES) {
            const int s0 = HALO + 512 * wt + 64 * (row >> 1) - 128 + 16 * h;
            v4i s0a = {0, 0, 0, 0}, s1a = {0, 0, 0, 0}, s2a = {0, 0, 0, 0};
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                const int sj = s0 + 64 * t;
                const int off = 80 * (sj >> 6) + (sj & 63) + a_re_im;
                const v4i al = *(const v4i*)(lds + P_RE_LO + off);
                const v4i ah = *(const v4i*)(lds + P_RE_HI + off);
                s0a = __builtin_amdgcn_mfma_i32_16x16x64_i8(al, B[2 * t], s0a, 0, 0, 0);
                s1a = __builtin_amdgcn_mfma_i32_16x16x64_i8(al, B[2 * t + 1], s1a, 0, 0, 0);
                s1a = __builtin_amdgcn_mfma_i32_16x16x64_i8(ah, B[2 * t], s1a, 0, 0, 0);
                s2a = __builtin_amdgcn_mfma_i32_16x16x64_i8(ah, B[2 * t + 1], s2a, 0, 0, 0);
            }
            int v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i)
                v[i] = (int32_t)((uint32_t)s0a[i] + ((uint32_t)s1a[i] << 8) + ((uint32_t)s2a[i] << 16) + bias);
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const long o = tile * TILE + 128 * wt + 16 * (2 * g4 + b) + col;
                if (o < n_out) y[o] = pack_clamp_sh(v[2 * b], v[2 * b + 1], sh);
            }
        }
    }
}

// ---- host side
struct MixMfmaTaps {
    std::string taps;       // the decimator's taps the fragments were built from
    void* d_frag = nullptr; // 6 x 64 lanes x 16 B
    uint32_t bias = 0;
    bool ok = false;
};

static MixMfmaTaps& mixmfma_taps(FirCore& f)
{
    static std::vector<std::pair<const FirCore*, MixMfmaTaps*>> cache;  // entries live for the process
    for (auto& e : cache)
        if (e.first == &f) return *e.second;
    cache.emplace_back(&f, new MixMfmaTaps());
    return *cache.back().second;
}

// B fragment f = 2 t + limb, lane (col = l & 15, h = l >> 4), byte j: the limb
// of c[4 col - (-128 + 64 t) - (16 h + j)], zero outside [0, ntaps)
static int mixmfma_prepare(FirCore& f, MixMfmaTaps& e)
{
    if (e.d_frag && e.taps == f.h_coef) return SRCDSP_OK;
    e.ok = false;
    e.taps = f.h_coef;
    const int32_t* c = (const int32_t*)f.h_coef.data();
    const int n = f.ntaps;
    std::vector<int8_t> lo(n), hi(n);
    uint32_t bias = 0;
    for (int k = 0; k < n; ++k) {
        const int32_t v = c[k], vl = ((v + 128) & 255) - 128, vh = (v - vl) >> 8;
        if (vh < -128 || vh > 127) return SRCDSP_OK;  // past two limbs: the product path
        lo[k] = (int8_t)vl;
        hi[k] = (int8_t)vh;
        bias += 128u * (uint32_t)v;
    }
    std::vector<int8_t> img(6 * 64 * 16, 0);
    for (int t = 0; t < 3; ++t)
        for (int lane = 0; lane < 64; ++lane)
            for (int j = 0; j < 16; ++j) {
                const int k = 4 * (lane & 15) + 128 - 64 * t - (16 * (lane >> 4) + j);
                if (k < 0 || k >= n) continue;
                img[((2 * t) * 64 + lane) * 16 + j] = lo[k];
                img[((2 * t + 1) * 64 + lane) * 16 + j] = hi[k];
            }
    if (!e.d_frag) SRCDSP_HIP_TRY(hipMalloc(&e.d_frag, img.size()));
    SRCDSP_HIP_TRY(hipMemcpy(e.d_frag, img.data(), img.size(), hipMemcpyHostToDevice));
    e.bias = bias;
    e.ok = true;
    return SRCDSP_OK;
}

static long g_mixmfma_launches = 0;  // calls that took the matrix-core path (the check scripts read them)
static long g_decmfma_launches = 0;

extern "C" __attribute__((visibility("default"))) long srcdsp_tune_mixdecim_mfma_launches() { return g_mixmfma_launches; }
extern "C" __attribute__((visibility("default"))) long srcdsp_tune_decim_mfma_launches() { return g_decmfma_launches; }

static bool decmfma_usable(FirCore& f, const void* d_in, size_t n_in, const void* d_out)
{
    const unsigned sh = f.shift() & 31u;
    return f.kv == KV_CI16_I32 && f.M == 4 && f.ntaps >= 1 && f.ntaps <= mmf::MAX_TAPS && sh != 0 &&
           n_in % 4 == 0 && 4 * n_in < (1ul << 31) && ((uintptr_t)d_in & 15) == 0 && ((uintptr_t)d_out & 15) == 0;
}

static bool mixmfma_usable(FirCore& f, const MixerState& m, const void* d_in, size_t n_in, const void* d_out)
{
    const char* off = getenv("SRCDSP_MIXDECIM_MFMA");
    if (off && off[0] == '0') return false;
    return decmfma_usable(f, d_in, n_in, d_out) && m.N >= 4 && m.N <= 4096 && (m.N & (m.N - 1)) == 0;
}

// the plain decimator (core_step without a mixer); SRCDSP_DECIM_MFMA=0: off
static bool plainmfma_usable(FirCore& f, const void* d_in, size_t n_in, const void* d_out)
{
    const char* off = getenv("SRCDSP_DECIM_MFMA");
    if (off && off[0] == '0') return false;
    return decmfma_usable(f, d_in, n_in, d_out);
}

// core_step's contract (ordering, history double buffer) with the matrix-core kernel;
// SRCDSP_ERR_UNSUPPORTED when the taps do not fit two limbs (the caller then takes core_step)
template <bool MIX>
static int mfma_decim_step(FirCore& f, const MixerState* m, const void* d_in, size_t n_in, void* d_out, hipStream_t s)
{
    MixMfmaTaps& e = mixmfma_taps(f);
    int rc = mixmfma_prepare(f, e);
    if (rc) return rc;
    if (!e.ok) return SRCDSP_ERR_UNSUPPORTED;
    static bool attr = false;
    if (!attr) {
        SRCDSP_HIP_TRY(hipFuncSetAttribute((const void*)mixdecim_mfma_step_i8<MIX>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, mmf::LDS_TOTAL));
        attr = true;
    }
    rc = f.order.before(s);
    if (rc) return rc;
    const long n = (long)n_in;
    const long n_tiles = (n + 4 * mmf::TILE - 1) / (4 * mmf::TILE);
    const uint32_t phi0 = MIX ? (uint32_t)(int32_t)m->phi : 0u, fr = MIX ? (uint32_t)(int32_t)m->freq : 0u;
    const int H = f.ntaps - 1;
    const int grid = (int)std::min<long>(512, n_tiles);
    ++(MIX ? g_mixmfma_launches : g_decmfma_launches);
    hipLaunchKernelGGL(mixdecim_mfma_step_i8<MIX>, dim3(grid), dim3(mmf::LANES), mmf::LDS_TOTAL, s, (const uint32_t*)d_in,
                       n, (const uint32_t*)f.d_hist[f.cur], H, (uint32_t*)f.d_hist[f.cur ^ 1],
                       (const mmf::v4i*)e.d_frag, MIX ? (const int16_t*)m->d_table : nullptr,
                       MIX ? m->N : 1u, phi0, fr, e.bias, f.shift() & 31u, (uint32_t*)d_out, n_tiles);
    SRCDSP_HIP_TRY(hipGetLastError());
    f.cur ^= 1;
    return f.order.after(s);
}

static int mixmfma_step(FirCore& f, const MixerState& m, const void* d_in, size_t n_in, void* d_out, hipStream_t s)
{
    return mfma_decim_step<true>(f, &m, d_in, n_in, d_out, s);
}
