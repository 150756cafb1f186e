// Config 4's tap loop on the integer matrix cores: a TUNING PROBE, not the
// product (BASELINE north_star: the product path uses no
// MFMA, so this kernel never ships in libsrcdsp_hip.so).
//
// The fused chain of config 4 on a fresh pair of objects, one call:
//   m[j] = limitScale16(x[j] * (T[(phi_j + N/4) % N], T[phi_j]), 14)
//          phi_j = (phi0 + j freq) mod N                     (mixers.h:169-188)
//   y[n] = limitScale16(sum_{k<127} c[k] m[4n - k], 14)      (dnsampling_filters.h:150-167)
// with m[j < 0] = 0 (the decimator's zero history), exactly the product's
// MixerDecimatorChain (mixer.step(in, tmp); decim.step(tmp, out)).
//
// The mixer stays on the VALU (v_dot2 per component, shift, saturating pack,
// -32768 -> -32767); the 127-tap sum moves to v_mfma_i32_16x16x64_i8:
// * limbs: m = 256 mh + ml + 128 (mh = the int16's high byte, ml = low byte
//   XOR 0x80), Q14 taps c = 256 ch + cl (|c| < 32640); S0 = ml.cl,
//   S1 = ml.ch + mh.cl, S2 = mh.ch; sum = S0 + (S1 << 8) + (S2 << 16) + 128 sum(c)
//   (mod 2^32, the reference's complex<int32_t> wrap; every window holds all
//   127 taps, zero history included, since m = 0 is its limbs too);
// * rows = (block, component): a wave tile is 8 blocks of 16 outputs (512
//   input samples); A row r reads component r & 1 of block r >> 1: 16 bytes of
//   one limb plane (re lo, re hi, im lo, im hi; one byte per sample); cols =
//   the 16 outputs of a block; K = 64 samples per chunk, 3 chunks at offsets
//   -128, -64, 0 from the block's first sample cover its window [-126, 60];
//   B_t[s][col] = limb of c[4 col - base_t - s] (Toeplitz, zero outside
//   [0, 126]) is the same for every tile: 6 fragments (3 chunks x 2 limbs) held
//   in 24 VGPRs for the kernel's lifetime;
// * per wave tile: 6 ds_read_b128 (3 chunks x 2 limbs) and 12 MFMAs; the D
//   layout (col = l & 15, row = 4 (l >> 4) + i) gives each lane the (re, im)
//   of 2 outputs, packed and stored as complex<int16_t>.
// * staging: persistent 512-lane workgroups, 2 per CU, tiles of 2048 outputs
//   (8192 + 128 input samples), next tile's input prefetched into VGPRs
//   (buffer loads: zeros before sample 0 and past the end); the mixer's
//   8-byte (A = (cos, -sin), B = (sin, cos)) words of a lane's samples in
//   registers (the same in every tile when N divides the tile's input span,
//   as for config 4; the first version read them from an LDS table: 4-way
//   bank conflicts, 0.266 ms); limb planes by v_perm.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
typedef short v2s __attribute__((ext_vector_type(2)));

namespace {
constexpr int LANES = 512;
constexpr int WAVES = LANES / 64;
constexpr int TILE = 2048;                 // outputs per workgroup tile
constexpr int HALO = 128;                  // staged samples before the tile (>= 126)
constexpr int SPAN = 4 * TILE + HALO;      // 8320 staged samples
constexpr int GRAN = SPAN / 4;             // 2080 granules of 4 samples
constexpr int NG = (GRAN + LANES - 1) / LANES;  // 5
constexpr int BLK64 = SPAN / 64;           // 130 blocks of 64 samples
constexpr int PLANE = BLK64 * 80;          // 10400 B: 64 B + 16 B pad per 64 samples
// plane bases: re and im planes 128 B apart modulo 256, so the 16 lanes of a
// ds_read_b128 quarter (8 blocks x 2 components) hit 16 different bank quads
constexpr int P_RE_LO = 0, P_IM_LO = 10624, P_RE_HI = 21248, P_IM_HI = 31872;
constexpr int LDS_PLANES = P_IM_HI + PLANE;
constexpr int LDS_TOTAL = LDS_PLANES;
constexpr int WT_PER_TILE = TILE / 128;    // 16 wave tiles of 128 outputs
static_assert(P_IM_LO % 256 == 128 && P_RE_HI % 256 == 0 && P_IM_HI % 256 == 128, "plane banks");
static_assert(P_IM_LO >= PLANE && P_RE_HI - P_IM_LO >= PLANE && P_IM_HI - P_RE_HI >= PLANE, "planes");
static_assert(2 * LDS_TOTAL <= 160 * 1024, "2 workgroups per CU");
}  // namespace

__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel)
{
    return __builtin_amdgcn_perm(hi, lo, sel);
}

__device__ __forceinline__ int32_t sdot2(uint32_t a, uint32_t b)
{
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(v2s, a), __builtin_bit_cast(v2s, b), 0, false);
}

// the clamp of limitScale16 (dsp_complex.cpp:63-73) on an already shifted
// pair: saturating pack to [-32768, 32767] (v_cvt_pk_i16_i32), then -32768 ->
// -32767 (v_pk_max_i16); complex<int16_t> word (re low, im high)
__device__ __forceinline__ uint32_t pack_clamp(int re, int im)
{
    const v2s v = __builtin_bit_cast(v2s, __builtin_amdgcn_cvt_pk_i16(re, im));
    const v2s lo = {-32767, -32767};
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(v, lo));
}

__global__ void __launch_bounds__(LANES, 2)
mixdecim_mfma_i8(const uint32_t* __restrict__ x, long n_in, const v4i* __restrict__ bfrag,
                 const v2u* __restrict__ table, uint32_t phi0, uint32_t freq, uint32_t bias,
                 uint32_t* __restrict__ y, long n_tiles)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int w = tid >> 6;

    // mixer words in registers: lane tid's granules g = tid + LANES k start at
    // staged sample 4 g of every tile, i.e. at global sample tile * 4 TILE - HALO
    // + 4 g, and tile * 4 TILE * freq = 0 mod N (N = 4096 divides 4 TILE), so
    // their phases are the same in every tile (the product's register-table
    // form): 2 words x 4 samples x NG granules, read once
    v2u tw[NG][4];
#pragma unroll
    for (int k = 0; k < NG; ++k) {
        const int g = tid + LANES * k;
        uint32_t ph = (phi0 + (uint32_t)(4 * g - HALO) * freq) & 4095u;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            tw[k][q] = table[ph];
            ph = (ph + freq) & 4095u;
        }
    }
    // taps: fragment f = 2 t + limb, lane-major
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
            if (g < GRAN)  // before sample 0: the wrapped 32-bit offset is out of range -> 0
                pre[k] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(
                                                     rs, (uint32_t)(4 * (j0 + 4 * g)), 0, 2));
        }
    };
    if (blockIdx.x < n_tiles) fetch(blockIdx.x);

    // A fragment: lane (row = l & 15, h = l >> 4): component row & 1, block row >> 1
    const int row = lane & 15, h = lane >> 4;
    const int a_re_im = (row & 1) ? (P_IM_LO - P_RE_LO) : 0;
    const int col = lane & 15, g4 = lane >> 4;

    for (long tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const long j0 = tile * (4 * TILE) - HALO;
        __syncthreads();
        // ---- staging: mixer, limitScale16, limb planes
#pragma unroll
        for (int k = 0; k < NG; ++k) {
            const int g = tid + LANES * k;
            if (g >= GRAN) break;
            const v4u v = pre[k];
            const long j = j0 + 4 * g;
            uint32_t m[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const v2u t = tw[k][q];
                const uint32_t xq = v[q];
                const int re = sdot2(xq, t[0]);  // x.re cos - x.im sin (mixers.h:175-176, dsp_complex.cpp:31-37)
                const int im = sdot2(xq, t[1]);  // x.re sin + x.im cos
                // limitScale16(., 14); before the stream: the decimator's zero history
                m[q] = (j + q >= 0) ? pack_clamp(re >> 14, im >> 14) : 0u;
            }
            // bytes: m = (re.b0, re.b1, im.b0, im.b1)
            const uint32_t t0 = perm(m[1], m[0], 0x05010400u);  // (m0.b0, m1.b0, m0.b1, m1.b1)
            const uint32_t t1 = perm(m[3], m[2], 0x05010400u);
            const uint32_t u0 = perm(m[1], m[0], 0x07030602u);  // (m0.b2, m1.b2, m0.b3, m1.b3)
            const uint32_t u1 = perm(m[3], m[2], 0x07030602u);
            const uint32_t re_lo = perm(t1, t0, 0x05040100u) ^ 0x80808080u;
            const uint32_t re_hi = perm(t1, t0, 0x07060302u);
            const uint32_t im_lo = perm(u1, u0, 0x05040100u) ^ 0x80808080u;
            const uint32_t im_hi = perm(u1, u0, 0x07060302u);
            const int js = 4 * g;
            const int off = 80 * (js >> 6) + (js & 63);
            *(uint32_t*)(lds + P_RE_LO + off) = re_lo;
            *(uint32_t*)(lds + P_RE_HI + off) = re_hi;
            *(uint32_t*)(lds + P_IM_LO + off) = im_lo;
            *(uint32_t*)(lds + P_IM_HI + off) = im_hi;
        }
        __syncthreads();
        if (tile + gridDim.x < n_tiles) fetch(tile + gridDim.x);

        // ---- taps: wave tiles wt = w, w + 8 (128 outputs = 512 samples each)
        for (int wt = w; wt < WT_PER_TILE; wt += WAVES) {
            // block b = row >> 1 of the wave tile starts at staged sample HALO + 512 wt + 64 b;
            // chunk t covers offsets -128 + 64 t + 16 h .. +15 from it
            const int s0 = HALO + 512 * wt + 64 * (row >> 1) - 128 + 16 * h;  // chunk 0
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
            // D: lane (col, g4) holds rows 4 g4 + i = (block 2 g4 + (i >> 1), component i & 1)
            int v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t acc = (uint32_t)s0a[i] + ((uint32_t)s1a[i] << 8) + ((uint32_t)s2a[i] << 16) + bias;
                v[i] = (int32_t)acc >> 14;  // limitScale16 shift (coeffScaling 14, leftShift 0)
            }
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const long o = tile * TILE + 128 * wt + 16 * (2 * g4 + b) + col;
                if (o < n_out) y[o] = pack_clamp(v[2 * b], v[2 * b + 1]);
            }
        }
    }
}

extern "C" int tune_mixdecim_mfma(const void* x, long n_in, const void* bfrag, const void* table, uint32_t phi0,
                                  uint32_t freq, uint32_t bias, void* y, int grid, hipStream_t s)
{
    static bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute((const void*)mixdecim_mfma_i8, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           LDS_TOTAL);
        if (e != hipSuccess) return (int)e;
        attr = true;
    }
    if (n_in % (4 * TILE) != 0 || 4 * n_in >= (1l << 31)) return 1;
    const long n_tiles = n_in / (4 * TILE);
    if (grid <= 0) grid = 512;
    if (grid > n_tiles) grid = (int)n_tiles;
    hipLaunchKernelGGL(mixdecim_mfma_i8, dim3(grid), dim3(LANES), LDS_TOTAL, s, (const uint32_t*)x, n_in,
                       (const v4i*)bfrag, (const v2u*)table, phi0, freq, bias, (uint32_t*)y, n_tiles);
    return (int)hipGetLastError();
}
