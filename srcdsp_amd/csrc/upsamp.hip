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
#include <vector>

#include "ops.h"

namespace srcdsp {

enum { UV_CI16_I32 = 0, UV_CI16_I16 = 1, UV_I16_I32 = 2 };

struct srcdsp_up_state {
    int variant = 0;
    unsigned L = 1;
    int ntaps = 0, H = 0;
    unsigned length = 0;
    int left_shift_factor = 0;
    int32_t *d_coef = nullptr;  // polyphase order: d_coef[o*H + i] = c[o + i*L]
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

template <int UV>
__global__ __launch_bounds__(256) void up_kernel(const void *in, long n_in, long n_total, const void *hist_in,
                                                 void *hist_out, const int32_t *coef, int H, unsigned L,
                                                 unsigned shift, void *out) {
    extern __shared__ int32_t sc[];  // L*H polyphase taps
    for (int i = threadIdx.x; i < (int)(L * H); i += blockDim.x) sc[i] = coef[i];
    __syncthreads();
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
            else ((uint32_t *)out)[oi] = pack16(limit_t16((int32_t)yr, shift), limit_t16((int32_t)yi, shift));
        }
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
    std::vector<int32_t> poly((size_t)n);
    for (unsigned o = 0; o < u.L; ++o)
        for (int i = 0; i < H; ++i) poly[o * H + i] = c[o + i * u.L];
    if (u.d_coef) (void)hipFree(u.d_coef);
    u.d_coef = nullptr;
    SRCDSP_HIP_TRY(hipMalloc(&u.d_coef, 4 * (size_t)n));
    SRCDSP_HIP_TRY(hipMemcpy(u.d_coef, poly.data(), 4 * (size_t)n, hipMemcpyHostToDevice));
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
    const int blocks = (int)std::max<long>(1, std::min<long>((n_total + 255) / 256, 4096));
    const size_t smem = 4 * (size_t)u.ntaps;
    const void *hin = u.d_hist[u.cur];
    void *hout = u.d_hist[u.cur ^ 1];
    switch (u.variant) {
    case UV_CI16_I32:
        hipLaunchKernelGGL(up_kernel<UV_CI16_I32>, dim3(blocks), dim3(256), smem, s, d_in, (long)n_in, n_total, hin,
                           hout, u.d_coef, u.H, u.L, shift, d_out);
        break;
    case UV_CI16_I16:
        hipLaunchKernelGGL(up_kernel<UV_CI16_I16>, dim3(blocks), dim3(256), smem, s, d_in, (long)n_in, n_total, hin,
                           hout, u.d_coef, u.H, u.L, shift, d_out);
        break;
    default:
        hipLaunchKernelGGL(up_kernel<UV_I16_I32>, dim3(blocks), dim3(256), smem, s, d_in, (long)n_in, n_total, hin,
                           hout, u.d_coef, u.H, u.L, shift, d_out);
        break;
    }
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
    for (int b = 0; b < 2; ++b)
        if (h->u.d_hist[b]) (void)hipFree(h->u.d_hist[b]);
    h->u.order.destroy();
    h->u.stage.destroy();
    delete h;
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
    for (int b = 0; b < 2; ++b) SRCDSP_HIP_TRY(hipMemset(h->u.d_hist[b], 0, h->u.hist_cap));
    SRCDSP_HIP_TRY(hipDeviceSynchronize());
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
        memcpy(u.stage.h_buf, in, ib);
        SRCDSP_HIP_TRY(hipMemcpyAsync(d_in, u.stage.h_buf, ib, hipMemcpyHostToDevice, s));
    }
    rc = up_launch(u, d_in, n_in, d_out, n_out, flush != 0, iterator != 0, s);
    if (rc) return rc;
    // only the L*(n_in [+ length/L]) written samples go back; a larger caller
    // vector keeps its tail untouched, as with the reference
    const size_t wb = std::min(ob, (size_t)u.L * (n_in + (flush ? u.length / u.L : 0)) * eb);
    SRCDSP_HIP_TRY(hipMemcpyAsync(u.stage.h_buf, d_out, wb, hipMemcpyDeviceToHost, s));
    SRCDSP_HIP_TRY(hipStreamSynchronize(s));
    memcpy(out, u.stage.h_buf, wb);
    return SRCDSP_OK;
}

}  // extern "C"
