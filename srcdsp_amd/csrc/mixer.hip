// mixer.hip -- dsptl::Mixer<complex<int16_t>, complex<int16_t>, int16_t, N>
// (mixers.h:27-188) on gfx950.
//
// The reference advances phi by freq (mod N) per sample (mixers.h:177), a
// loop-carried recurrence; its closed form phi_i = (phi_0 + i*freq) mod N lets
// every lane start anywhere.  Each lane streams 4 samples (16 B) per
// iteration of a grid-stride loop and advances its phase by a precomputed
// stride increment, so the only modulo per lane is the one at its start.  The
// N-entry LUT is built on the host with libm sin() exactly as mixers.h:155-158
// and staged once per workgroup into LDS.
#include <algorithm>

#include "ops.h"

namespace srcdsp {

__device__ __forceinline__ uint32_t nco_mix(uint32_t w, const int16_t *tab, unsigned N, unsigned phi) {
    unsigned ic = phi + N / 4;  // (phi + N/4) % N, phi < N
    ic = ic >= N ? ic - N : ic;
    const int32_t lr = tab[ic], li = tab[phi];
    const int32_t ar = sext16(w), ai = sext16_hi(w);
    // ::operator*(complex<int16_t>, complex<int32_t>) (dsp_complex.cpp:31-37); |T| <= 16383 so no wrap
    const int32_t r = ar * lr - ai * li;
    const int32_t i = ai * lr + li * ar;
    return pack16(limit16(r, 14), limit16(i, 14));
}

__device__ __forceinline__ unsigned phase_at(unsigned long idx, unsigned phi0, unsigned freq, unsigned N) {
    return (unsigned)(((unsigned long)phi0 + (idx % N) * (unsigned long)freq) % N);
}

template <bool LDS_TABLE>
__global__ __launch_bounds__(256) void mixer_kernel(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                    unsigned long n, const int16_t *__restrict__ gtab,
                                                    unsigned N, unsigned phi0, unsigned freq,
                                                    unsigned dphase) {
    extern __shared__ __attribute__((aligned(16))) int16_t stab[];
    const int16_t *tab = gtab;
    if constexpr (LDS_TABLE) {
        for (unsigned i = threadIdx.x; i < N; i += blockDim.x) stab[i] = gtab[i];
        __syncthreads();
        tab = stab;
    }
    const unsigned long nchunk = n / 4;
    const unsigned long stride = (unsigned long)gridDim.x * blockDim.x;
    unsigned long c = (unsigned long)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned ph = phase_at(4 * c, phi0, freq, N);
    auto adv = [&](unsigned p, unsigned d) { p += d; return p >= N ? p - N : p; };
    for (; c < nchunk; c += stride) {
        uint4 v = ((const uint4 *)in)[c];
        unsigned p = ph;
        v.x = nco_mix(v.x, tab, N, p); p = adv(p, freq);
        v.y = nco_mix(v.y, tab, N, p); p = adv(p, freq);
        v.z = nco_mix(v.z, tab, N, p); p = adv(p, freq);
        v.w = nco_mix(v.w, tab, N, p);
        ((uint4 *)out)[c] = v;
        ph = adv(ph, dphase);
    }
    // tail (n % 4 samples) by the first lanes
    const unsigned long t0 = 4 * nchunk;
    unsigned long i = t0 + (unsigned long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = nco_mix(in[i], tab, N, phase_at(i, phi0, freq, N));
}

// any alignment: one sample per lane
__global__ void mixer_kernel_unaligned(const uint32_t *in, uint32_t *out, unsigned long n, const int16_t *tab,
                                       unsigned N, unsigned phi0, unsigned freq) {
    for (unsigned long i = (unsigned long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (unsigned long)gridDim.x * blockDim.x)
        out[i] = nco_mix(in[i], tab, N, phase_at(i, phi0, freq, N));
}

// _Mixer::setFrequency (mixers.h:51-67): the products are float, the
// rounding is ::round(double); a tiny negative frequency maps N to 0.
static void set_frequency(MixerState &m, float lo) {
    m.nominal = lo;
    const float Nf = (float)m.N;
    if (lo >= 0) {
        float v = lo * Nf / 2;
        m.freq = (int16_t)std::round((double)v);
    } else {
        float v = -lo * Nf / 2;
        m.freq = (int16_t)std::round((double)m.N - std::round((double)v));
        if (m.freq == (int16_t)m.N) m.freq = 0;
    }
}

static int mixer_launch(MixerState &m, const void *d_in, size_t n, void *d_out, hipStream_t s) {
    if (n == 0) return SRCDSP_OK;
    SRCDSP_ARG_CHECK(d_in && d_out, "mixer_step: null buffer");
    int rc = m.order.before(s);
    if (rc) return rc;
    const unsigned N = m.N, phi = (unsigned)m.phi, fr = (unsigned)m.freq;
    const bool aligned = (((uintptr_t)d_in | (uintptr_t)d_out) & 15u) == 0;
    if (aligned) {
        const unsigned long chunks = n / 4;
        int blocks = (int)std::max<unsigned long>(1, std::min<unsigned long>((chunks + 255) / 256, 256 * 16));
        const unsigned long stride_samples = 4ul * (unsigned long)blocks * 256ul;
        const unsigned dphase = (unsigned)(((stride_samples % N) * fr) % N);
        const bool lds = N <= 16384;
        if (lds)
            hipLaunchKernelGGL(mixer_kernel<true>, dim3(blocks), dim3(256), N * sizeof(int16_t), s,
                               (const uint32_t *)d_in, (uint32_t *)d_out, (unsigned long)n, m.d_table, N, phi, fr,
                               dphase);
        else
            hipLaunchKernelGGL(mixer_kernel<false>, dim3(blocks), dim3(256), 0, s, (const uint32_t *)d_in,
                               (uint32_t *)d_out, (unsigned long)n, m.d_table, N, phi, fr, dphase);
    } else {
        int blocks = (int)std::max<size_t>(1, std::min<size_t>((n + 255) / 256, 4096));
        hipLaunchKernelGGL(mixer_kernel_unaligned, dim3(blocks), dim3(256), 0, s, (const uint32_t *)d_in,
                           (uint32_t *)d_out, (unsigned long)n, m.d_table, N, phi, fr);
    }
    SRCDSP_HIP_TRY(hipGetLastError());
    // phi after n samples: (phi + n*freq) mod N  (mixers.h:177 iterated)
    m.phi = (int16_t)(((unsigned long)phi + (unsigned long)(n % N) * fr) % N);
    return m.order.after(s);
}

}  // namespace srcdsp

using namespace srcdsp;

extern "C" {

SRCDSP_API int srcdsp_mixer_create(srcdsp_mixer_t *out, unsigned N) {
    SRCDSP_ARG_CHECK(out != nullptr, "mixer_create: null out");
    *out = nullptr;
    SRCDSP_ARG_CHECK(N >= 4 && N <= 32768, "mixer_create: N must be in [4, 32768] (int16_t phase)");
    auto *h = new srcdsp_mixer();
    MixerState &m = h->m;
    m.N = N;
    int rc = m.order.init();
    if (!rc) rc = m.stage.init();
    if (rc) {
        delete h;
        return rc;
    }
    // LUT: (int16_t)(16383 * sin(2*pi*k/N)) in double (mixers.h:155-158, constants.h:21)
    const double pi = 3.141592653589793238462643383279502884;
    const int16_t amp = INT16_MAX >> 1;
    m.h_table = new int16_t[N];
    for (unsigned k = 0; k < N; ++k) m.h_table[k] = (int16_t)(amp * std::sin(2 * pi * (double)k / N));
    if (hipMalloc(&m.d_table, N * sizeof(int16_t)) != hipSuccess ||
        hipMemcpy(m.d_table, m.h_table, N * sizeof(int16_t), hipMemcpyHostToDevice) != hipSuccess) {
        set_error("mixer_create: device table allocation failed");
        delete[] m.h_table;
        delete h;
        return SRCDSP_ERR_HIP;
    }
    m.phi = 0;
    m.freq = 0;
    m.nominal = 0.f;
    *out = h;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_mixer_destroy(srcdsp_mixer_t h) {
    if (!h) return SRCDSP_OK;
    (void)h->m.order.sync();
    if (h->m.d_table) (void)hipFree(h->m.d_table);
    if (h->m.d_scratch) (void)hipFree(h->m.d_scratch);
    delete[] h->m.h_table;
    h->m.order.destroy();
    h->m.stage.destroy();
    delete h;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_mixer_clone(srcdsp_mixer_t h, srcdsp_mixer_t *out) {
    SRCDSP_ARG_CHECK(h != nullptr && out != nullptr, "mixer_clone: null argument");
    *out = nullptr;
    int rc = h->m.order.sync();
    if (rc) return rc;
    srcdsp_mixer_t c = nullptr;
    rc = srcdsp_mixer_create(&c, h->m.N);  // the same table: built from N alone (mixers.h:155-158)
    if (rc) return rc;
    c->m.phi = h->m.phi;
    c->m.freq = h->m.freq;
    c->m.nominal = h->m.nominal;
    *out = c;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_mixer_set_frequency(srcdsp_mixer_t h, float f) {
    SRCDSP_ARG_CHECK(h != nullptr, "mixer_set_frequency: null handle");
    SRCDSP_ARG_CHECK(f <= 1 && f >= -1, "setFrequency: loFreq must be in [-1, 1] (mixers.h:54)");
    set_frequency(h->m, f);
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_mixer_reset(srcdsp_mixer_t h, float f) {
    SRCDSP_ARG_CHECK(h != nullptr, "mixer_reset: null handle");
    SRCDSP_ARG_CHECK(f <= 1 && f >= -1, "reset: loFreq must be in [-1, 1] (mixers.h:54)");
    h->m.phi = 0;
    set_frequency(h->m, f);
    return SRCDSP_OK;
}

// adjustFrequency (mixers.h:91-98): continuous phase, wrap nominal into [-1,1]
SRCDSP_API int srcdsp_mixer_adjust_frequency(srcdsp_mixer_t h, float adj) {
    SRCDSP_ARG_CHECK(h != nullptr, "mixer_adjust_frequency: null handle");
    float nf = h->m.nominal + adj;
    if (nf > 1) nf -= 2;
    if (nf < -1) nf += 2;
    SRCDSP_ARG_CHECK(nf <= 1 && nf >= -1, "adjustFrequency: result outside [-1, 1] (mixers.h:54)");
    set_frequency(h->m, nf);
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_mixer_set_phase(srcdsp_mixer_t h, int phi) {
    SRCDSP_ARG_CHECK(h != nullptr, "mixer_set_phase: null handle");
    SRCDSP_ARG_CHECK(phi >= 0 && (unsigned)phi < h->m.N, "mixer_set_phase: phi must be in [0, N)");
    int rc = h->m.order.sync();
    if (rc) return rc;
    h->m.phi = (int16_t)phi;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_mixer_get_state(srcdsp_mixer_t h, int *phi, int *freq, float *nominal) {
    SRCDSP_ARG_CHECK(h != nullptr, "mixer_get_state: null handle");
    if (phi) *phi = h->m.phi;
    if (freq) *freq = h->m.freq;
    if (nominal) *nominal = h->m.nominal;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_mixer_get_table(srcdsp_mixer_t h, int16_t *t) {
    SRCDSP_ARG_CHECK(h != nullptr && t != nullptr, "mixer_get_table: null argument");
    memcpy(t, h->m.h_table, h->m.N * sizeof(int16_t));
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_mixer_step(srcdsp_mixer_t h, const void *d_in, size_t n, void *d_out, void *stream) {
    SRCDSP_ARG_CHECK(h != nullptr, "mixer_step: null handle");
    return mixer_launch(h->m, d_in, n, d_out, (hipStream_t)stream);
}

SRCDSP_API int srcdsp_mixer_step_host(srcdsp_mixer_t h, const void *in, size_t n, void *out) {
    SRCDSP_ARG_CHECK(h != nullptr, "mixer_step_host: null handle");
    if (n == 0) return SRCDSP_OK;
    MixerState &m = h->m;
    const size_t b = 4 * n, bal = (b + 255) & ~(size_t)255;
    int rc = m.stage.reserve(b, 2 * bal);
    if (rc) return rc;
    hipStream_t s = m.stage.stream;
    char *d_in = (char *)m.stage.d_buf, *d_out = d_in + bal;
    host_copy(m.stage.h_buf, in, b);
    SRCDSP_HIP_TRY(hipMemcpyAsync(d_in, m.stage.h_buf, b, hipMemcpyHostToDevice, s));
    rc = mixer_launch(m, d_in, n, d_out, s);
    if (rc) return rc;
    SRCDSP_HIP_TRY(hipMemcpyAsync(m.stage.h_buf, d_out, b, hipMemcpyDeviceToHost, s));
    SRCDSP_HIP_TRY(hipStreamSynchronize(s));
    host_copy(out, m.stage.h_buf, b);
    return SRCDSP_OK;
}

}  // extern "C"
