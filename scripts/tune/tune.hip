// Tuning harness (not part of the product): instantiates decimator kernel
// variants from srcdsp_amd/csrc/decim_kernels.h and an FMA-rate microbenchmark
// so they can be timed side by side, interleaved, in one process.
#include "decim_tune.h"
#include "decim_mfma.h"
#include "decim_ring.h"

using namespace srcdsp;

// ---- FMA issue-rate microbenchmark: 16 independent chains per lane
template <int MODE>
__global__ __launch_bounds__(256) void fma_rate(float *out, int iters, float c0) {
    float a[16];
    float2 p[8];
#pragma unroll
    for (int j = 0; j < 16; ++j) a[j] = threadIdx.x * 0.001f + j;
#pragma unroll
    for (int j = 0; j < 8; ++j) p[j] = make_float2(a[2 * j], a[2 * j + 1]);
    const float2 cc = make_float2(c0, c0);
    const float2 xx = make_float2(1.0001f, 0.9999f);
    for (int i = 0; i < iters; ++i) {
        if constexpr (MODE == 0) {
#pragma unroll
            for (int j = 0; j < 16; ++j) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[j]) : "s"(c0), "v"(xx.x));
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j)
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p[j]) : "v"(cc), "v"(xx));
        }
    }
    float s = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) s += a[j];
#pragma unroll
    for (int j = 0; j < 8; ++j) s += p[j].x + p[j].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// ---- pure streaming probe: read 8 B/sample (dwordx4), write 2 B/sample (1 of 4)
__global__ __launch_bounds__(256) void stream_probe(const float4 *in, float4 *out, long n16) {
    // n16 = input granules; each lane reads 4 consecutive granules (8 samples) and writes
    // one granule (2 samples) -> 4:1 like the decimator
    long stride = (long)gridDim.x * blockDim.x;
    for (long k = (long)blockIdx.x * blockDim.x + threadIdx.x; 4 * k + 3 < n16; k += stride) {
        float4 a = in[4 * k], b = in[4 * k + 1], c = in[4 * k + 2], d = in[4 * k + 3];
        out[k] = make_float4(a.x + b.y, a.z + c.w, b.x + d.y, c.z + d.w);
    }
}
// coalesced variant: every load instruction reads 1 KiB contiguous per wave,
// 4 loads in flight per lane, 1 coalesced store per 4 loads
__global__ __launch_bounds__(256) void stream_probe2(const float4 *in, float4 *out, long n16) {
    const long nth = (long)gridDim.x * blockDim.x;
    const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    for (long base = 0; base + 4 * nth <= n16; base += 4 * nth) {
        float4 a = in[base + tid], b = in[base + nth + tid], c = in[base + 2 * nth + tid], d = in[base + 3 * nth + tid];
        out[base / 4 + tid] = make_float4(a.x + b.y, a.z + c.w, b.x + d.y, c.z + d.w);
    }
}
// read-only ceiling
__global__ __launch_bounds__(256) void read_probe(const float4 *in, float *out, long n16) {
    const long nth = (long)gridDim.x * blockDim.x;
    float acc = 0;
    for (long k = (long)blockIdx.x * blockDim.x + threadIdx.x; k < n16; k += nth) {
        float4 a = in[k];
        acc += a.x + a.y + a.z + a.w;
    }
    if (acc == 12345.678f) out[0] = acc;
}
extern "C" int tune_stream_probe2(int mode, int blocks, const void *in, void *out, long n_samples, void *stream) {
    if (mode == 0)
        hipLaunchKernelGGL(stream_probe2, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const float4 *)in,
                           (float4 *)out, n_samples / 2);
    else
        hipLaunchKernelGGL(read_probe, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const float4 *)in,
                           (float *)out, n_samples / 2);
    return hipGetLastError();
}
extern "C" int tune_stream_probe(int blocks, const void *in, void *out, long n_samples, void *stream) {
    hipLaunchKernelGGL(stream_probe, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const float4 *)in,
                       (float4 *)out, n_samples / 2);
    return hipGetLastError();
}

extern "C" int tune_fma_rate(int mode, int blocks, int iters, float *out, void *stream) {
    if (mode == 0)
        hipLaunchKernelGGL(fma_rate<0>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, out, iters, 1.0f);
    else
        hipLaunchKernelGGL(fma_rate<1>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, out, iters, 1.0f);
    return hipGetLastError();
}

// ---- decimator variants (cf32, M=4, 127 taps, FMA)
template <class K>
static int launch(K kern, int blocks, int threads, const DecimLaunch &L, hipStream_t s) {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, s, L);
    return hipGetLastError();
}

extern "C" int tune_decim(int variant, int grid, const float *d_coef, const void *in, void *out, long n_in,
                          const void *hist_in, void *hist_out, void *stream) {
    DecimLaunch L{};
    L.in = in; L.out = out; L.n_in = n_in; L.n_out = n_in / 4; L.ntaps = 127; L.shift = 0;
    L.hist_in[0] = hist_in; L.hist_out[0] = hist_out;
    L.coef = d_coef;
    hipStream_t s = (hipStream_t)stream;
    auto tiles = [&](int TO) { return (L.n_out + TO - 1) / TO; };
    switch (variant) {
    // v2: buffer loads + shift-0 quantiser
    case 10: L.ntiles = tiles(256 * 4); return launch(decim_stream2_cf32_tune<127, 4, 256, true, 4, false>, grid, 256, L, s);
    case 11: L.ntiles = tiles(256 * 4); return launch(decim_stream2_cf32_tune<127, 4, 256, true, 4, true>, grid, 256, L, s);
    case 12: L.ntiles = tiles(128 * 4); return launch(decim_stream2_cf32_tune<127, 4, 128, true, 4, true>, grid, 128, L, s);
    case 13: L.ntiles = tiles(64 * 4); return launch(decim_stream2_cf32_tune<127, 4, 64, true, 4, true>, grid, 64, L, s);
    case 15: L.ntiles = tiles(128 * 6); return launch(decim_stream2_cf32_tune<127, 6, 128, true, 3, true>, grid, 128, L, s);
    case 16: L.ntiles = tiles(64 * 6); return launch(decim_stream2_cf32_tune<127, 6, 64, true, 3, true>, grid, 64, L, s);
    case 20: L.ntiles = tiles(256 * 4); return launch(decim_stream2_cf32_tune<127, 4, 256, true, 4, true, 1>, grid, 256, L, s);
    case 21: L.ntiles = tiles(256 * 4); return launch(decim_stream2_cf32_tune<127, 4, 256, true, 4, true, 2>, grid, 256, L, s);
    case 30: L.ntiles = tiles(256 * 4); return launch(decim_stream2_cf32_tune<127, 4, 256, true, 4, true, 0, true, false>, grid, 256, L, s);
    case 31: L.ntiles = tiles(256 * 4); return launch(decim_stream2_cf32_tune<127, 4, 256, true, 4, true, 0, false, true>, grid, 256, L, s);
    case 32: L.ntiles = tiles(256 * 4); return launch(decim_stream2_cf32_tune<127, 4, 256, true, 4, true, 0, true, true>, grid, 256, L, s);
    case 33: L.ntiles = tiles(256 * 4); return launch(decim_stream2_cf32_tune<127, 4, 256, true, 4, true, 1, true, true>, grid, 256, L, s);
    case 34: L.ntiles = tiles(256 * 4); return launch(decim_stream2_cf32_tune<127, 4, 256, true, 4, true, 0, false, false, true>, grid, 256, L, s);
    case 35: L.ntiles = tiles(256 * 4); return launch(decim_stream2_cf32_tune<127, 4, 256, true, 4, true, 0, true, false, true>, grid, 256, L, s);
    case 36: L.ntiles = tiles(256 * 4); return launch(decim_stream2_cf32_tune<127, 4, 256, true, 4, true, 0, false, true, true>, grid, 256, L, s);
    case 37: L.ntiles = tiles(256 * 4); return launch(decim_stream2_cf32_tune<127, 4, 256, true, 4, true, 0, true, true, true>, grid, 256, L, s);
    case 38: L.ntiles = tiles(256 * 4); return launch(decim_stream2_cf32_tune<127, 4, 256, true, 4, true, 1, true, true, true>, grid, 256, L, s);
    case 40: L.ntiles = tiles(256 * 4); return launch(decim_stream2_cf32_tune<127, 4, 256, true, 4, true, 0, false, false, false, true>, grid, 256, L, s);
    case 41: L.ntiles = tiles(256 * 4); return launch(decim_stream2_cf32_tune<127, 4, 256, true, 4, true, 0, true, false, false, true>, grid, 256, L, s);
    case 42: L.ntiles = tiles(256 * 4); return launch(decim_stream2_cf32_tune<127, 4, 256, true, 4, true, 0, true, true, true, true>, grid, 256, L, s);
    case 43: L.ntiles = tiles(256 * 4); return launch(decim_stream2_cf32_tune<127, 4, 256, true, 4, true, 1, false, false, false, true>, grid, 256, L, s);
    case 44: L.ntiles = tiles(256 * 4); return launch(decim_stream2_cf32_tune<127, 4, 256, true, 4, true, 0, false, true, true, true>, grid, 256, L, s);
    case 48: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 0, true, true, true, true>, grid, 512, L, s);
    case 49: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 3, true, 0, true, true, true, true>, grid, 512, L, s);
    case 50: L.ntiles = tiles(1024 * 4); return launch(decim_stream2_cf32_tune<127, 4, 1024, true, 4, true, 0, true, true, true, true>, grid, 1024, L, s);
    case 51: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 0, true, true, true, false>, grid, 512, L, s);
    case 52: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 0, false, true, true, true>, grid, 512, L, s);
    case 60: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 0, true, true, true, true, 2, 2>, grid, 512, L, s);
    case 61: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 0, true, true, true, true, 2, 3>, grid, 512, L, s);
    case 62: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 0, true, true, true, true, 3, 2>, grid, 512, L, s);
    case 63: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 0, true, true, true, true, 3, 3>, grid, 512, L, s);
    case 64: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 0, true, true, true, true, 18, 18>, grid, 512, L, s);
    case 65: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 0, true, true, true, true, 2, 19>, grid, 512, L, s);
    case 66: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 0, true, true, true, true, 19, 2>, grid, 512, L, s);
    case 80: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 1, true, true, true, true>, grid, 512, L, s);
    case 84: L.ntiles = tiles(256 * 4); return launch(decim_stream2_cf32_tune<127, 4, 256, true, 4, true, 1, true, true, true, true>, grid, 256, L, s);
    case 88: L.ntiles = tiles(256 * 4); return launch(decim_stream2_cf32_tune<127, 4, 256, true, 4, true, 0, true, true, true, true>, grid, 256, L, s);
    case 90: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 2, true, 1, true, true, true, true>, grid, 512, L, s);
    // compute path only (PROBE=2: every tile re-reads one of 16 L2-resident spans)
    case 110: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 2, true, true, true, true>, grid, 512, L, s);
    case 111: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 2, true, 2, true, true, true, true>, grid, 512, L, s);
    case 112: L.ntiles = tiles(1024 * 4); return launch(decim_stream2_cf32_tune<127, 4, 1024, true, 4, true, 2, true, true, true, true>, grid, 1024, L, s);
    case 113: L.ntiles = tiles(1024 * 4); return launch(decim_stream2_cf32_tune<127, 4, 1024, true, 4, true, 0, true, true, true, true>, grid, 1024, L, s);
    case 114: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 3, true, true, true, true>, grid, 512, L, s);
    case 120: L.ntiles = tiles(256 * 8); return launch(decim_stream2_cf32_tune<127, 8, 256, true, 2, true, 0, true, true, true, true>, grid, 256, L, s);
    // OST 2: permlane32-paired whole-line stores (no LDS output staging, 2 barriers per tile)
    // matrix-core decimator (decim_mfma.h): 1024-output tiles, 2 workgroups per CU
    case 300: L.ntiles = tiles(1024); return launch(decim_mfma_cf32<127, 2, true, 0>, grid, 256, L, s);
    case 301: L.ntiles = tiles(1024); return launch(decim_mfma_cf32<127, 2, true, 2>, grid, 256, L, s);
    case 302: L.ntiles = tiles(1024); return launch(decim_mfma_cf32<127, 2, true, 1>, grid, 256, L, s);
    case 303: L.ntiles = tiles(1024); return launch(decim_mfma_cf32<127, 3, true, 0>, grid, 256, L, s);
    case 304: L.ntiles = tiles(1024); return launch(decim_mfma_cf32<127, 3, true, 2>, grid, 256, L, s);
    // ILV: tap-major pk_fma issue order (inline asm)
    case 200: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 0, true, 2, true, true, -1, -1, true>, grid, 512, L, s);
    case 201: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 2, true, 2, true, true, -1, -1, true>, grid, 512, L, s);
    case 202: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 2, true, 0, true, 2, true, true, -1, -1, true>, grid, 512, L, s);
    case 203: L.ntiles = tiles(256 * 4); return launch(decim_stream2_cf32_tune<127, 4, 256, true, 4, true, 0, true, 2, true, true, -1, -1, true>, grid, 256, L, s);
    case 204: L.ntiles = tiles(256 * 8); return launch(decim_stream2_cf32_tune<127, 8, 256, true, 2, true, 0, true, 2, true, true, -1, -1, true>, grid, 256, L, s);
    case 610: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 0, true, 2, true, true, 0, -1, true>, grid, 512, L, s);  // ILV, load aux 0
    case 611: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 0, true, 2, true, true, 1, -1, true>, grid, 512, L, s);  // ILV, load aux 1
    case 612: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 0, true, 2, true, true, 3, -1, true>, grid, 512, L, s);  // ILV, load aux 3
    case 613: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 0, true, 2, true, true, 16, -1, true>, grid, 512, L, s);  // ILV, load aux 16
    case 614: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 0, true, 2, true, true, 18, -1, true>, grid, 512, L, s);  // ILV, load aux 18
    case 70: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 0, true, 2, true, true>, grid, 512, L, s);
    case 71: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 1, true, 2, true, true>, grid, 512, L, s);
    case 72: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 2, true, 0, true, 2, true, true>, grid, 512, L, s);
    case 73: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 2, true, 2, true, true>, grid, 512, L, s);
    case 74: L.ntiles = tiles(256 * 4); return launch(decim_stream2_cf32_tune<127, 4, 256, true, 4, true, 0, true, 2, true, true>, grid, 256, L, s);
    // 12 waves per CU: 2 x 384 lanes or 1 x 768 lanes (up to 168 VGPRs)
    case 92: L.ntiles = tiles(384 * 4); return launch(decim_stream2_cf32_tune<127, 4, 384, true, 3, true, 0, true, 2, true, true>, grid, 384, L, s);
    case 93: L.ntiles = tiles(768 * 4); return launch(decim_stream2_cf32_tune<127, 4, 768, true, 3, true, 0, true, 2, true, true>, grid, 768, L, s);
    case 94: L.ntiles = tiles(384 * 4); return launch(decim_stream2_cf32_tune<127, 4, 384, true, 3, true, 1, true, 2, true, true>, grid, 384, L, s);
    case 95: L.ntiles = tiles(768 * 4); return launch(decim_stream2_cf32_tune<127, 4, 768, true, 3, true, 1, true, 2, true, true>, grid, 768, L, s);
    case 96: L.ntiles = tiles(384 * 4); return launch(decim_stream2_cf32_tune<127, 4, 384, true, 4, true, 0, true, 2, true, true>, grid, 384, L, s);
    case 76: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 4, true, 2, true, true>, grid, 512, L, s);
    case 77: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 5, true, 2, true, true>, grid, 512, L, s);
    case 205: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 4, true, 2, true, true, -1, -1, true>, grid, 512, L, s);
    case 206: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 5, true, 2, true, true, -1, -1, true>, grid, 512, L, s);
    // wave-private images, no barriers (decim_wave_cf32): 256-output wave tiles
    case 400: L.ntiles = tiles(256); return launch(decim_wave_cf32<127, 512, true, 4, true>, grid, 512, L, s);
    case 401: L.ntiles = tiles(256); return launch(decim_wave_cf32<127, 256, true, 4, true>, grid, 256, L, s);
    case 402: L.ntiles = tiles(256); return launch(decim_wave_cf32<127, 512, true, 4, true, 1>, grid, 512, L, s);
    case 403: L.ntiles = tiles(256); return launch(decim_wave_cf32<127, 512, true, 4, true, 2>, grid, 512, L, s);
    case 404: L.ntiles = tiles(256); return launch(decim_wave_cf32<127, 512, true, 4, true, 1, 0>, grid, 512, L, s);
    case 405: L.ntiles = tiles(256); return launch(decim_wave_cf32<127, 512, true, 4, true, 3>, grid, 512, L, s);
    case 406: L.ntiles = tiles(256); return launch(decim_wave_cf32<127, 512, true, 4, true, 0, 0>, grid, 512, L, s);
    case 407: L.ntiles = tiles(256); return launch(decim_wave_cf32<127, 256, true, 4, true, 1>, grid, 256, L, s);
    case 408: L.ntiles = tiles(256); return launch(decim_wave_cf32<127, 512, true, 4, true, 1, 2, true>, grid, 512, L, s);
    case 409: L.ntiles = tiles(256); return launch(decim_wave_cf32<127, 512, true, 4, true, 0, 2, true>, grid, 512, L, s);
    case 75: L.ntiles = tiles(512 * 4); return launch(decim_stream2_cf32_tune<127, 4, 512, true, 4, true, 0, true, 0, true, true>, grid, 512, L, s);
    // LDS-DMA loader/consumer ring (decim_ring.h): one workgroup per CU (grid 256 whatever is asked),
    // <NCONS consumer waves, NSLOT slots, NPF slots in flight, CH wave tiles per chunk>; whole chunks only
#define RING(V, NC, NS, NP, CHK)                                                                  \
    case V:                                                                                       \
        if (L.n_out % (256L * 256 * CHK)) return -2;                                              \
        L.ntiles = L.n_out / 256;                                                                 \
        return launch(decim_ring_cf32<NC, NS, NP, CHK>, 256, 64 * (NC + 1), L, s);
    RING(500, 12, 15, 3, 8)
    RING(501, 12, 15, 2, 8)
    RING(502, 10, 15, 4, 8)
    RING(503, 12, 15, 3, 1)
    RING(504, 8, 15, 5, 8)
    RING(505, 12, 15, 3, 32)
#undef RING
    // round 3: the product kernel with the staging experiments (decim_stream_x<NT, R, BLOCK, MINW, STAG, EPI, PRIO>)
    case 600: L.ntiles = tiles(512 * 4); return launch(decim_stream_x<127, 4, 512, 4, 0, 0, 0>, grid, 512, L, s);
    case 601: L.ntiles = tiles(512 * 4); return launch(decim_stream_x<127, 4, 512, 4, 2, 0, 0>, grid, 512, L, s);
    case 602: L.ntiles = tiles(512 * 4); return launch(decim_stream_x<127, 4, 512, 4, 4, 0, 0>, grid, 512, L, s);
    case 603: L.ntiles = tiles(512 * 4); return launch(decim_stream_x<127, 4, 512, 4, 0, 1, 0>, grid, 512, L, s);
    case 604: L.ntiles = tiles(512 * 4); return launch(decim_stream_x<127, 4, 512, 4, 0, 0, 1>, grid, 512, L, s);
    case 605: L.ntiles = tiles(512 * 4); return launch(decim_stream_x<127, 4, 512, 4, 2, 1, 0>, grid, 512, L, s);
    case 606: L.ntiles = tiles(512 * 4); return launch(decim_stream_x<127, 4, 512, 4, 0, 1, 1>, grid, 512, L, s);
    case 607: L.ntiles = tiles(512 * 4); return launch(decim_stream_x<127, 4, 512, 4, 2, 1, 1>, grid, 512, L, s);
    case 608: L.ntiles = tiles(256 * 4); return launch(decim_stream_x<127, 4, 256, 4, 0, 1, 0>, grid, 256, L, s);
    case 609: L.ntiles = tiles(256 * 4); return launch(decim_stream_x<127, 4, 256, 4, 2, 1, 0>, grid, 256, L, s);
    default: return -1;
    }
}

// workgroup placement census: blocks x 512 threads, 75 KB of LDS each (the
// headline's residency: 2 per CU); out[2 b] = HW_ID, out[2 b + 1] = XCC_ID
extern "C" int tune_census(int blocks, unsigned *out, void *stream) {
    hipLaunchKernelGGL(wg_census, dim3(blocks), dim3(512), 75 * 1024, (hipStream_t)stream, out);
    return hipGetLastError();
}

// ---- FilterFir stream kernel (float in, 31 taps): output store shapes
extern "C" int tune_fir(int variant, int grid, const float *d_coef, const void *in, void *out, long n_in, int ntaps,
                        unsigned shift, const void *hist_in, void *hist_out, void *stream) {
    DecimLaunch L{};
    L.in = in; L.out = out; L.n_in = n_in; L.n_out = n_in; L.ntaps = ntaps; L.shift = shift;
    L.hist_in[0] = hist_in; L.hist_out[0] = hist_out;
    L.coef = d_coef;
    L.ntiles = (L.n_out + kFirR * kFirBlock - 1) / (kFirR * kFirBlock);
    hipStream_t s = (hipStream_t)stream;
    switch (variant) {
    case 0: return launch(fir_stream_f32<KV_F32_REAL, true, 1>, grid, kFirBlock, L, s);
    case 1: return launch(fir_stream_f32<KV_F32_REAL, true, 2>, grid, kFirBlock, L, s);
    // variants 2, 3 (complex<float> input) are gone: fir_stream_f32 is the
    // float -> complex<float> kernel only (FirTraits<KV_F32_REAL>); complex<float>
    // FIRs run on the decimator kernels at M = 1
    }
    return -1;
}

// ---- clock probe (tuning only): one lane records (s_memtime, s_memrealtime)
// every `gap` ticks of the 100 MHz real-time counter, n times, while other
// kernels run beside it on another stream; d(memtime)/d(realtime) x 100 MHz is
// the shader clock the chip holds at that moment (MI355X_MICROARCH.md, DVFS).
__global__ void clock_probe(unsigned long long *out, int n, int gap) {
    if (threadIdx.x != 0) return;
    for (int i = 0; i < n; ++i) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)gap) __builtin_amdgcn_s_sleep(4);
        const unsigned long long c = __builtin_amdgcn_s_memtime();
        const unsigned long long r = __builtin_amdgcn_s_memrealtime();
        out[2 * i] = c;
        out[2 * i + 1] = r;
    }
}
__global__ void realtime_stamp(unsigned long long *out) {
    if (threadIdx.x == 0) out[0] = __builtin_amdgcn_s_memrealtime();
}
extern "C" int tune_clock_probe(unsigned long long *out, int n, int gap, void *stream) {
    hipLaunchKernelGGL(clock_probe, dim3(1), dim3(64), 0, (hipStream_t)stream, out, n, gap);
    return hipGetLastError();
}
extern "C" int tune_realtime_stamp(unsigned long long *out, void *stream) {
    hipLaunchKernelGGL(realtime_stamp, dim3(1), dim3(64), 0, (hipStream_t)stream, out);
    return hipGetLastError();
}

// ---- layout / numerics probe of v_mfma_f32_4x4x1_16b_f32: K steps of
// per-lane A and B values (a[k*64 + lane], b[k*64 + lane]) accumulated from 0;
// D (4 floats per lane) written to d[lane*4 + r]
__global__ void mfma4x4_probe(const float *a, const float *b, float *d, int K) {
    const int l = threadIdx.x;
    f4m_t acc = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < K; ++k) acc = __builtin_amdgcn_mfma_f32_4x4x1f32(a[k * 64 + l], b[k * 64 + l], acc, 0, 0, 0);
    for (int r = 0; r < 4; ++r) d[l * 4 + r] = acc[r];
}
extern "C" int tune_mfma4x4_probe(const float *a, const float *b, float *d, int K, void *stream) {
    hipLaunchKernelGGL(mfma4x4_probe, dim3(1), dim3(64), 0, (hipStream_t)stream, a, b, d, K);
    return hipGetLastError();
}
