/*
 * srcdsp_oracle.c -- scalar C restatement of SrcDsp's hot-path operators.
 *
 * TEST INFRASTRUCTURE ONLY (see srcdsp_oracle.h).  This is the checker the HIP
 * path is compared against; it is never linked into libsrcdsp_hip.so.
 * Parity: pinned bit-exactly against tests/golden/ (generated from the real
 * reference headers by tests/golden/gen_golden.py through oracle/_ref).
 *
 * Built with -O2 -ffp-contract=off: the "strict" flavour below is a separately
 * rounded multiply then add even when the ISA has FMA; the "fma" flavour calls
 * fmaf() explicitly.  Signed-overflow wrap of the reference's int32 arithmetic is
 * restated with uint32 arithmetic to stay defined in C.
 */
#include "srcdsp_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ======================= L0: dsp_complex.cpp / .h ======================= */

/* float -> int32 as x86 cvttss2si does it: truncation, INT_MIN when out of
 * range or NaN.  This is what `complex<int32_t>(complex<float>)` compiles to
 * when limitScale16 is fed a float accumulator (dnsampling_filters.h:167). */
int32_t orc_cvt_f2i(float f) {
    if (!(f >= -2147483648.0f && f < 2147483648.0f)) return INT32_MIN;
    return (int32_t)f;
}

/* double -> int32 as x86 cvttsd2si (static_cast<int>(floor(log2(...))),
 * dnsampling_filters.h:95, filters.h:96, correlators.h:192). */
int32_t orc_cvt_d2i(double d) {
    if (!(d > -2147483649.0 && d < 2147483648.0)) return INT32_MIN;
    return (int32_t)d;
}

static inline int32_t sar32(int32_t v, unsigned s) { return v >> (s & 31u); } /* x86 sar masks */
static inline uint32_t shr32(uint32_t v, unsigned s) { return v >> (s & 31u); }
static inline int32_t wadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
static inline int32_t wsub(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
static inline int32_t wmul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }

/* limitScale16 (dsp_complex.cpp:63-73), one component: arithmetic shift, then a
 * SYMMETRIC clamp to +-32767 decided by abs(); abs(INT_MIN) stays negative, so
 * INT_MIN passes unclamped and its int16 truncation is 0 (verified on the
 * reference build, tests/golden case decim_edge). */
int16_t orc_limit16(int32_t v, unsigned shift) {
    int32_t a = sar32(v, shift);
    if (a != INT32_MIN && (a > 32767 || a < -32767)) a = a > 0 ? 32767 : -32767;
    return (int16_t)(uint16_t)(uint32_t)a;
}

/* limitScale<T,U> (dsp_complex.h:45-63 scalar, :83-108 complex): shift then an
 * ASYMMETRIC clamp to [-32768, 32767] for an int16 output type. */
static inline int16_t limit_t16(int32_t v, unsigned shift) {
    int32_t a = sar32(v, shift);
    if (a > 32767) a = 32767;
    else if (a < -32768) a = -32768;
    return (int16_t)a;
}

/* abs() as bound in the canonical TU: with <cmath> only,
 * `abs(float)` resolves to ::abs(int), so the coefficient is first truncated. */
static double abs_bound_f32(float c, int abs_mode) {
    if (abs_mode == ORC_ABS_FABS) return (double)fabsf(c);
    int32_t i = orc_cvt_f2i(c);
    return (double)(i == INT32_MIN ? INT32_MIN : (i < 0 ? -i : i));
}

static unsigned scaling_from_sum(double sum) {
    /* coeffScaling = static_cast<int>(floor(log2(sumMagnitude)))
     * (dnsampling_filters.h:95); stored unsigned in the decimator. */
    return (unsigned)orc_cvt_d2i(floor(log2(sum)));
}

unsigned orc_coeff_scaling_f32(const float *c, int n, int abs_mode) {
    double s = 0;
    for (int i = 0; i < n; ++i) s += abs_bound_f32(c[i], abs_mode);
    return scaling_from_sum(s);
}
unsigned orc_coeff_scaling_i32(const int32_t *c, int n) {
    double s = 0;
    for (int i = 0; i < n; ++i) s += (double)(c[i] == INT32_MIN ? INT32_MIN : abs(c[i]));
    return scaling_from_sum(s);
}
unsigned orc_coeff_scaling_i16(const int16_t *c, int n) {
    double s = 0;
    for (int i = 0; i < n; ++i) s += (double)abs((int)c[i]);
    return scaling_from_sum(s);
}

/* one tap of a complex<float> accumulation, y += c * x
 * (std::operator*(float, complex<float>) then complex<float>::operator+=). */
static inline void cmac_f32(float *yr, float *yi, float c, float xr, float xi, int fp_mode) {
    if (fp_mode == ORC_FP_FMA) {
        *yr = fmaf(c, xr, *yr);
        *yi = fmaf(c, xi, *yi);
    } else {
        float pr = xr * c, pi = xi * c;
        *yr = *yr + pr;
        *yi = *yi + pi;
    }
}

/* ================= FilterDnsamplingFir (dnsampling_filters.h) ================= */

/* sample sizes per In type of each decimator variant (ref_api.h codes) */
static size_t decim_in_size(int v) { return v == 0 ? 8 : (v == 3 ? 8 : 4); }

struct orc_decim {
    int variant, ntaps, fp_mode, left_shift;
    unsigned M, coeff_scaling;
    float *cf;      /* variant 0 */
    int32_t *ci;    /* variants 1,2 (int16 stored widened),3 */
    unsigned char *hist; /* N-1 samples of In type, oldest first (dnsampling_filters.h:67) */
};

orc_decim *orc_decim_create(int variant, unsigned M, const void *coeffs, int ntaps, int abs_mode,
                            int fp_mode) {
    if (variant < 0 || variant > 3 || M == 0 || ntaps < 1) return NULL;
    orc_decim *d = (orc_decim *)calloc(1, sizeof(*d));
    d->variant = variant; d->M = M; d->ntaps = ntaps; d->fp_mode = fp_mode;
    if (variant == 0) {
        d->cf = (float *)malloc(sizeof(float) * ntaps);
        memcpy(d->cf, coeffs, sizeof(float) * ntaps);
        d->coeff_scaling = orc_coeff_scaling_f32(d->cf, ntaps, abs_mode);
    } else {
        d->ci = (int32_t *)malloc(sizeof(int32_t) * ntaps);
        if (variant == 2) {
            for (int i = 0; i < ntaps; ++i) d->ci[i] = ((const int16_t *)coeffs)[i];
            d->coeff_scaling = orc_coeff_scaling_i16((const int16_t *)coeffs, ntaps);
        } else {
            memcpy(d->ci, coeffs, sizeof(int32_t) * ntaps);
            d->coeff_scaling = orc_coeff_scaling_i32(d->ci, ntaps);
        }
    }
    /* history.resize(N-1), value-initialised (dnsampling_filters.h:90) */
    d->hist = (unsigned char *)calloc(ntaps > 1 ? ntaps - 1 : 1, decim_in_size(variant));
    d->left_shift = 0; /* :96 */
    return d;
}

void orc_decim_set_left_shift(orc_decim *d, int ls) { d->left_shift = ls; }  /* :63 */

/* setCoeffs (dsptl_dnsampling_filters.h:114-134): the history is RESIZED, not
 * cleared (std::vector::resize keeps the first min(old,new) entries, zero-fills
 * the rest); coeffScaling is recomputed and leftShift returns to 0. */
int orc_decim_set_coeffs(orc_decim *d, const void *coeffs, int ntaps, int abs_mode) {
    if (ntaps < 1) return -1;
    size_t es = decim_in_size(d->variant);
    long oldH = d->ntaps - 1, newH = ntaps - 1;
    unsigned char *nh = (unsigned char *)calloc(newH > 0 ? newH : 1, es);
    memcpy(nh, d->hist, (size_t)(oldH < newH ? oldH : newH) * es);
    free(d->hist); d->hist = nh;
    free(d->cf); free(d->ci); d->cf = NULL; d->ci = NULL;
    d->ntaps = ntaps;
    if (d->variant == 0) {
        d->cf = (float *)malloc(sizeof(float) * ntaps);
        memcpy(d->cf, coeffs, sizeof(float) * ntaps);
        d->coeff_scaling = orc_coeff_scaling_f32(d->cf, ntaps, abs_mode);
    } else {
        d->ci = (int32_t *)malloc(sizeof(int32_t) * ntaps);
        if (d->variant == 2) {
            for (int i = 0; i < ntaps; ++i) d->ci[i] = ((const int16_t *)coeffs)[i];
            d->coeff_scaling = orc_coeff_scaling_i16((const int16_t *)coeffs, ntaps);
        } else {
            memcpy(d->ci, coeffs, sizeof(int32_t) * ntaps);
            d->coeff_scaling = orc_coeff_scaling_i32(d->ci, ntaps);
        }
    }
    d->left_shift = 0;
    return 0;
}
void orc_decim_reset(orc_decim *d) {                                         /* :56-60 */
    memset(d->hist, 0, (size_t)(d->ntaps > 1 ? d->ntaps - 1 : 1) * decim_in_size(d->variant));
}
unsigned orc_decim_coeff_scaling(const orc_decim *d) { return d->coeff_scaling; }

/* fetch x[idx] (idx may be negative: history) as two int32 components */
static inline void decim_fetch_i(const orc_decim *d, const void *in, long idx, int32_t *re, int32_t *im) {
    const void *base = in;
    long i = idx;
    if (idx < 0) { base = d->hist; i = d->ntaps - 1 + idx; }
    if (d->variant == 3) {
        const int32_t *p = (const int32_t *)base;
        *re = p[2 * i]; *im = p[2 * i + 1];
    } else {
        const int16_t *p = (const int16_t *)base;
        *re = p[2 * i]; *im = p[2 * i + 1];
    }
}

/* step(): dnsampling_filters.h:129-172 (identical body dsptl_dnsampling_filters.h:172-220).
 * Output n = limitScale16(sum_{k=0}^{N-1} c[k] * x[nM-k], coeffScaling-leftShift),
 * taps accumulated strictly in ascending k, x[<0] taken from the history. */
void orc_decim_step(orc_decim *d, const void *in, long n_in, void *out) {
    const int N = d->ntaps;
    const unsigned shift = d->coeff_scaling - (unsigned)d->left_shift;
    long n_out = n_in / (long)d->M;
    for (long o = 0; o < n_out; ++o) {
        long j = o * (long)d->M;
        if (d->variant == 0) {
            const float *x = (const float *)in, *h = (const float *)d->hist;
            float yr = 0.f, yi = 0.f;
            for (int k = 0; k < N; ++k) {
                long idx = j - k;
                float xr, xi;
                if (idx >= 0) { xr = x[2 * idx]; xi = x[2 * idx + 1]; }
                else { long p = N - 1 + idx; xr = h[2 * p]; xi = h[2 * p + 1]; }
                cmac_f32(&yr, &yi, d->cf[k], xr, xi, d->fp_mode);
            }
            float *y = (float *)out;
            y[2 * o] = (float)orc_limit16(orc_cvt_f2i(yr), shift);
            y[2 * o + 1] = (float)orc_limit16(orc_cvt_f2i(yi), shift);
        } else {
            int32_t yr = 0, yi = 0;
            for (int k = 0; k < N; ++k) {
                int32_t xr, xi, c = d->ci[k];
                decim_fetch_i(d, in, j - k, &xr, &xi);
                if (d->variant == 2) {
                    /* std::operator*(const short&, const complex<short>&): each
                     * product wraps to int16 before the int32 accumulate. */
                    yr = wadd(yr, (int16_t)(uint16_t)(uint32_t)wmul(xr, c));
                    yi = wadd(yi, (int16_t)(uint16_t)(uint32_t)wmul(xi, c));
                } else {
                    /* variant 1: ::operator*(complex<int32_t>(c,0), complex<int16_t>)
                     * (dsp_complex.cpp:23-29); variant 3: std::operator*(int, complex<int>). */
                    yr = wadd(yr, wmul(c, xr));
                    yi = wadd(yi, wmul(c, xi));
                }
            }
            int16_t *y = (int16_t *)out;
            y[2 * o] = orc_limit16(yr, shift);
            y[2 * o + 1] = orc_limit16(yi, shift);
        }
    }
    /* history <- last N-1 samples (:170-171).  The reference indexes before
     * input[0] when n_in < N-1 (undefined); here the window simply slides over
     * the concatenation history ++ input, which equals the reference whenever
     * the reference is defined. */
    if (N > 1 && n_in > 0) {
        size_t es = decim_in_size(d->variant);
        long H = N - 1;
        unsigned char *nh = (unsigned char *)malloc(H * es);
        for (long k = 0; k < H; ++k) {
            long idx = n_in - H + k;
            const unsigned char *src = idx >= 0 ? (const unsigned char *)in + idx * es
                                                : d->hist + (H + idx) * es;
            memcpy(nh + k * es, src, es);
        }
        memcpy(d->hist, nh, H * es);
        free(nh);
    }
}

void orc_decim_destroy(orc_decim *d) {
    if (!d) return;
    free(d->cf); free(d->ci); free(d->hist); free(d);
}

/* ============================ FilterFir (filters.h) ============================ */

struct orc_fir {
    int variant, ntaps, fp_mode;
    unsigned coeff_scaling;  /* int in the reference (filters.h:62), passed as unsigned */
    float *cf; int32_t *ci;
    float *bf; int32_t *bi;  /* circular buffer of InternalType, N entries */
    unsigned top;
};

orc_fir *orc_fir_create(int variant, const void *coeffs, int ntaps, int abs_mode, int fp_mode) {
    if (variant < 0 || variant > 2 || ntaps < 1) return NULL;
    orc_fir *f = (orc_fir *)calloc(1, sizeof(*f));
    f->variant = variant; f->ntaps = ntaps; f->fp_mode = fp_mode; f->top = 0;
    if (variant == 2) {
        f->ci = (int32_t *)malloc(4 * ntaps); memcpy(f->ci, coeffs, 4 * ntaps);
        f->coeff_scaling = orc_coeff_scaling_i32(f->ci, ntaps);       /* filters.h:92-96 */
        f->bi = (int32_t *)calloc(2 * ntaps, 4);
    } else {
        f->cf = (float *)malloc(4 * ntaps); memcpy(f->cf, coeffs, 4 * ntaps);
        f->coeff_scaling = orc_coeff_scaling_f32(f->cf, ntaps, abs_mode);
        f->bf = (float *)calloc(2 * ntaps, 4);  /* variant 1 uses only the re slots */
    }
    return f;
}

/* setCoeffs (filters.h:86-97): new taps, coeffScaling recomputed, then reset()
 * clears the buffer.  `top` is kept (wrapped into range when N shrinks; the
 * reference would index out of bounds there). */
int orc_fir_set_coeffs(orc_fir *f, const void *coeffs, int ntaps, int abs_mode) {
    if (ntaps < 1) return -1;
    free(f->cf); free(f->ci); free(f->bf); free(f->bi);
    f->cf = NULL; f->ci = NULL; f->bf = NULL; f->bi = NULL;
    f->ntaps = ntaps;
    if (f->variant == 2) {
        f->ci = (int32_t *)malloc(4 * ntaps); memcpy(f->ci, coeffs, 4 * ntaps);
        f->coeff_scaling = orc_coeff_scaling_i32(f->ci, ntaps);
        f->bi = (int32_t *)calloc(2 * ntaps, 4);
    } else {
        f->cf = (float *)malloc(4 * ntaps); memcpy(f->cf, coeffs, 4 * ntaps);
        f->coeff_scaling = orc_coeff_scaling_f32(f->cf, ntaps, abs_mode);
        f->bf = (float *)calloc(2 * ntaps, 4);
    }
    if (f->top >= (unsigned)ntaps) f->top %= (unsigned)ntaps;
    return 0;
}

void orc_fir_reset(orc_fir *f) {  /* filters.h:107-113: clears the buffer, not `top` */
    if (f->bi) memset(f->bi, 0, 8 * (size_t)f->ntaps);
    if (f->bf) memset(f->bf, 0, 8 * (size_t)f->ntaps);
}

/* step(): filters.h:131-169.  buffer[top] = x[j]; y = sum_n c[n]*buffer[top-n mod N]
 * with n ascending (newest sample first); out = limitScale16(y, coeffScaling). */
void orc_fir_step(orc_fir *f, const void *in, long n, void *out) {
    const unsigned N = (unsigned)f->ntaps;
    for (long j = 0; j < n; ++j) {
        unsigned top = f->top;
        if (f->variant == 0) {
            const float *x = (const float *)in;
            f->bf[2 * top] = x[2 * j]; f->bf[2 * top + 1] = x[2 * j + 1];
            float yr = 0.f, yi = 0.f;
            for (unsigned t = 0; t < N; ++t) {
                unsigned k = (top + N - t) % N;
                cmac_f32(&yr, &yi, f->cf[t], f->bf[2 * k], f->bf[2 * k + 1], f->fp_mode);
            }
            float *y = (float *)out;
            y[2 * j] = (float)orc_limit16(orc_cvt_f2i(yr), f->coeff_scaling);
            y[2 * j + 1] = (float)orc_limit16(orc_cvt_f2i(yi), f->coeff_scaling);
        } else if (f->variant == 1) {
            const float *x = (const float *)in;
            f->bf[top] = x[j];
            float y = 0.f;
            for (unsigned t = 0; t < N; ++t) {
                unsigned k = (top + N - t) % N;
                y = (f->fp_mode == ORC_FP_FMA) ? fmaf(f->cf[t], f->bf[k], y) : y + f->cf[t] * f->bf[k];
            }
            /* float -> complex<int32_t>(int(y), 0) -> limitScale16 -> complex<float> */
            float *o = (float *)out;
            o[2 * j] = (float)orc_limit16(orc_cvt_f2i(y), f->coeff_scaling);
            o[2 * j + 1] = 0.f;
        } else {
            const int16_t *x = (const int16_t *)in;
            f->bi[2 * top] = x[2 * j]; f->bi[2 * top + 1] = x[2 * j + 1];
            int32_t yr = 0, yi = 0;
            for (unsigned t = 0; t < N; ++t) {
                unsigned k = (top + N - t) % N;
                yr = wadd(yr, wmul(f->ci[t], f->bi[2 * k]));
                yi = wadd(yi, wmul(f->ci[t], f->bi[2 * k + 1]));
            }
            int16_t *y = (int16_t *)out;
            y[2 * j] = orc_limit16(yr, f->coeff_scaling);
            y[2 * j + 1] = orc_limit16(yi, f->coeff_scaling);
        }
        f->top = (top + 1 >= N) ? 0 : top + 1;
    }
}

void orc_fir_destroy(orc_fir *f) {
    if (!f) return;
    free(f->cf); free(f->ci); free(f->bf); free(f->bi); free(f);
}

/* ================ FilterUpsamplingFir (upsampling_filters.h) ================ */

struct orc_up {
    int variant, ntaps;
    unsigned L, hsize, top, length;
    int left_shift_factor;
    int32_t *c;       /* int16 coefficients stored widened */
    int32_t *buf;     /* hsize samples, 2 components (variant 2: re only) */
};

orc_up *orc_up_create(int variant, unsigned L, const void *coeffs, int ntaps) {
    /* setCoefficients (upsampling_filters.h:107-126) asserts non-empty and N%L==0 */
    if (variant < 0 || variant > 2 || L == 0 || ntaps < 1 || ntaps % L) return NULL;
    orc_up *u = (orc_up *)calloc(1, sizeof(*u));
    u->variant = variant; u->L = L; u->ntaps = ntaps;
    u->c = (int32_t *)malloc(4 * ntaps);
    for (int i = 0; i < ntaps; ++i)
        u->c[i] = variant == 1 ? ((const int16_t *)coeffs)[i] : ((const int32_t *)coeffs)[i];
    u->hsize = ntaps / L;
    u->buf = (int32_t *)calloc(2 * u->hsize, 4);
    u->left_shift_factor = (int)round(log2((double)L));   /* :119 */
    u->length = ntaps;                                     /* :121-123 trailing zeros */
    while (u->length > 0 && u->c[u->length - 1] == 0) --u->length;
    return u;
}

void orc_up_reset(orc_up *u) { u->top = 0; memset(u->buf, 0, 8 * (size_t)u->hsize); }
int orc_up_get_length(const orc_up *u) { return (int)u->length; }

/* one input sample: push, then L polyphase outputs (upsampling_filters.h:163-194) */
static void up_push(orc_up *u, int32_t xr, int32_t xi, void *out, long base, unsigned shift) {
    const unsigned L = u->L, H = u->hsize, top = u->top;
    u->buf[2 * top] = xr; u->buf[2 * top + 1] = xi;
    for (unsigned o = 0; o < L; ++o) {
        int32_t yr = 0, yi = 0;
        for (unsigned i = 0; i < H; ++i) {
            unsigned k = (top + H - i) % H;
            int32_t c = u->c[o + i * L];
            if (u->variant == 1) {   /* std::operator*(short, complex<short>): int16 wrap */
                yr = wadd(yr, (int16_t)(uint16_t)(uint32_t)wmul(c, u->buf[2 * k]));
                yi = wadd(yi, (int16_t)(uint16_t)(uint32_t)wmul(c, u->buf[2 * k + 1]));
            } else {
                yr = wadd(yr, wmul(c, u->buf[2 * k]));
                yi = wadd(yi, wmul(c, u->buf[2 * k + 1]));
            }
        }
        int16_t *y = (int16_t *)out;
        if (u->variant == 2) {
            y[base + o] = limit_t16(yr, shift);
        } else {
            y[2 * (base + o)] = limit_t16(yr, shift);
            y[2 * (base + o) + 1] = limit_t16(yi, shift);
        }
    }
    u->top = (top + 1 >= H) ? 0 : top + 1;
}

/* step(vector) :149-233 uses shift 15-round(log2 L); step(iterator) :240-323
 * uses shift 0.  flush appends length/L zero inputs (:196, :281). */
void orc_up_step(orc_up *u, const void *in, long n_in, void *out, int flush, int iter) {
    unsigned shift = iter ? 0u : (unsigned)(15 - u->left_shift_factor);
    const int16_t *x = (const int16_t *)in;
    for (long j = 0; j < n_in; ++j) {
        if (u->variant == 2) up_push(u, x[j], 0, out, j * (long)u->L, shift);
        else up_push(u, x[2 * j], x[2 * j + 1], out, j * (long)u->L, shift);
    }
    if (flush) {
        long extra = (long)(u->length / u->L);
        for (long j = n_in; j < n_in + extra; ++j) up_push(u, 0, 0, out, j * (long)u->L, shift);
    }
}

void orc_up_destroy(orc_up *u) {
    if (!u) return;
    free(u->c); free(u->buf); free(u);
}

/* ===================== Mixer<ci16,ci16,int16_t,N> (mixers.h) ===================== */

struct orc_mixer {
    unsigned N;
    int16_t phi, freq;
    float nominal;
    int16_t *table;
};

orc_mixer *orc_mixer_create(unsigned N) {
    orc_mixer *m = (orc_mixer *)calloc(1, sizeof(*m));
    m->N = N;
    m->table = (int16_t *)malloc(2 * N);
    /* mixers.h:155-158: (int16_t)(16383 * sin(2*pi*k/N)), evaluated in double */
    const double pi = 3.141592653589793238462643383279502884;  /* constants.h:21 */
    for (unsigned k = 0; k < N; ++k)
        m->table[k] = (int16_t)(16383 * sin(2 * pi * (double)k / N));
    return m;
}

void orc_mixer_table(const orc_mixer *m, int16_t *t) { memcpy(t, m->table, 2 * m->N); }

/* _Mixer::setFrequency (mixers.h:51-67): products in float, rounding in double */
void orc_mixer_set_frequency(orc_mixer *m, float f) {
    m->nominal = f;
    float Nf = (float)m->N;
    if (f >= 0) {
        float v = f * Nf / 2;
        m->freq = (int16_t)round((double)v);
    } else {
        float v = -f * Nf / 2;
        m->freq = (int16_t)round((double)m->N - round((double)v));
        if (m->freq == (int16_t)m->N) m->freq = 0;
    }
}
void orc_mixer_reset(orc_mixer *m, float f) { m->phi = 0; orc_mixer_set_frequency(m, f); } /* :76-81 */
void orc_mixer_adjust_frequency(orc_mixer *m, float f) {                                  /* :91-98 */
    float nf = m->nominal + f;
    if (nf > 1) nf -= 2;
    if (nf < -1) nf += 2;
    orc_mixer_set_frequency(m, nf);
}
void orc_mixer_state(const orc_mixer *m, int *phi, int *freq, float *nom) {
    *phi = m->phi; *freq = m->freq; *nom = m->nominal;
}

/* step (mixers.h:169-188): out = limitScale16(x * (T[(phi+N/4)%N] + j T[phi]), 14)
 * with the product of dsp_complex.cpp:31-37; phi advances by freq mod N. */
void orc_mixer_step(orc_mixer *m, const int16_t *in, long n, int16_t *out) {
    const unsigned N = m->N;
    for (long k = 0; k < n; ++k) {
        int32_t lr = m->table[((unsigned)m->phi + N / 4) % N], li = m->table[(unsigned)m->phi];
        int32_t ar = in[2 * k], ai = in[2 * k + 1];
        int32_t r = wsub(wmul(ar, lr), wmul(ai, li));
        int32_t i = wadd(wmul(ai, lr), wmul(li, ar));
        out[2 * k] = orc_limit16(r, 14);
        out[2 * k + 1] = orc_limit16(i, 14);
        m->phi = (int16_t)(((unsigned)(m->phi + m->freq)) % N);
    }
}

void orc_mixer_destroy(orc_mixer *m) {
    if (!m) return;
    free(m->table); free(m);
}

/* ============ FixedPatternCorrelator<int16_t,int32_t,N,S> (correlators.h) ============ */

struct orc_corr {
    unsigned N, S, H;          /* H = N*S history ring */
    int32_t *hist;             /* ring of complex<int32_t> */
    int32_t *coef;             /* conjugated pattern */
    int16_t *bits;             /* bitSamples, N complex<int16_t> */
    size_t top;
    uint32_t energy[3], corr[3], coeffs_energy;
    int coeff_scaling;
    double threshold_factor;
};

orc_corr *orc_corr_create(unsigned N, unsigned S) {
    orc_corr *c = (orc_corr *)calloc(1, sizeof(*c));
    c->N = N; c->S = S; c->H = N * S;
    c->hist = (int32_t *)calloc(2 * c->H, 4);
    c->coef = (int32_t *)calloc(2 * N, 4);
    c->bits = (int16_t *)calloc(2 * N, 2);
    return c;
}

/* setPattern (correlators.h:167-194) */
void orc_corr_set_pattern(orc_corr *c, const int32_t *p, double th) {
    double tmp = 0;
    for (unsigned i = 0; i < c->N; ++i) {
        c->coef[2 * i] = p[2 * i];
        c->coef[2 * i + 1] = wsub(0, p[2 * i + 1]);              /* conjugate :173-176 */
        int32_t e = wadd(wmul(c->coef[2 * i], c->coef[2 * i]), wmul(c->coef[2 * i + 1], c->coef[2 * i + 1]));
        tmp += (double)e;                                         /* int sum, then double :183 */
    }
    /* static_cast<uint32_t>(double): x86-64 converts through int64 */
    c->coeffs_energy = (uint32_t)(uint64_t)(int64_t)tmp;
    c->threshold_factor = th * sqrt((double)c->coeffs_energy);
    c->coeff_scaling = orc_cvt_d2i(floor(log2(sqrt((double)c->coeffs_energy))));
}

void orc_corr_reset(orc_corr *c) {  /* :146-159 */
    c->top = 0;
    memset(c->energy, 0, sizeof c->energy);
    memset(c->corr, 0, sizeof c->corr);
    memset(c->hist, 0, 8 * (size_t)c->H);
    memset(c->bits, 0, 4 * (size_t)c->N);
}

/* step (correlators.h:209-303) */
/* detect = 0: stream the samples without the detection test (orc_corr_prime);
 * corr_out / energy_out (may be NULL): each sample's corrValue[0] and
 * energyValue[0] as computed at :244-250 */
static int corr_run(orc_corr *c, const int16_t *in, long n, int *corr_index, int detect, uint32_t *corr_out,
                    uint32_t *energy_out) {
    const long H = (long)c->H, S = (long)c->S, N = (long)c->N;
    for (long idx = 0; idx < n; ++idx) {
        long top = (long)c->top;
        c->hist[2 * top] = in[2 * idx];
        c->hist[2 * top + 1] = in[2 * idx + 1];
        int32_t tr = 0, ti = 0;
        uint32_t e0 = 0;
        c->energy[2] = c->energy[1];
        c->energy[1] = c->energy[0];
        /* taps: ring position top-k*S pairs with coef[N-1-k]; positions above top
         * (older samples, wrapped) pair with coef[k]  (:233-242) */
        for (long k = 0, h; (h = top - k * S) >= 0; ++k) {
            int32_t hr = c->hist[2 * h], hi = c->hist[2 * h + 1];
            int32_t cr = c->coef[2 * (N - 1 - k)], ci = c->coef[2 * (N - 1 - k) + 1];
            tr = wadd(tr, wsub(wmul(hr, cr), wmul(hi, ci)));
            ti = wadd(ti, wadd(wmul(hr, ci), wmul(hi, cr)));
            e0 += (uint32_t)wadd(wmul(hr, hr), wmul(hi, hi));
        }
        for (long k = 0, h; (h = top + (k + 1) * S) < H; ++k) {
            int32_t hr = c->hist[2 * h], hi = c->hist[2 * h + 1];
            int32_t cr = c->coef[2 * k], ci = c->coef[2 * k + 1];
            tr = wadd(tr, wsub(wmul(hr, cr), wmul(hi, ci)));
            ti = wadd(ti, wadd(wmul(hr, ci), wmul(hi, cr)));
            e0 += (uint32_t)wadd(wmul(hr, hr), wmul(hi, hi));
        }
        tr = sar32(tr, (unsigned)c->coeff_scaling);                 /* scale32 :244 */
        ti = sar32(ti, (unsigned)c->coeff_scaling);
        c->energy[0] = shr32(e0, (unsigned)(c->coeff_scaling / 2)); /* :245 */
        c->corr[2] = c->corr[1];
        c->corr[1] = c->corr[0];
        int32_t ar = tr >> 2, ai = ti >> 2;
        c->corr[0] = (uint32_t)wadd(wmul(ar, ar), wmul(ai, ai));   /* :250 */
        if (corr_out) corr_out[idx] = c->corr[0];
        if (energy_out) energy_out[idx] = c->energy[0];
        if (detect && c->corr[1] > c->corr[2] && c->corr[1] > c->corr[0]) {  /* :262 */
            double cm = sqrt((double)c->corr[1]);
            double em = sqrt((double)c->energy[1]);
            if (cm > em * 2.7 && em > 300) {                        /* :265-268 */
                *corr_index = (int)(idx - 1);
                long nt = top > 0 ? top - 1 : H - 1;                /* :278-288 */
                for (long k = 0, h; (h = nt - k * S) >= 0; ++k) {
                    c->bits[2 * (N - 1 - k)] = (int16_t)c->hist[2 * h];
                    c->bits[2 * (N - 1 - k) + 1] = (int16_t)c->hist[2 * h + 1];
                }
                for (long k = 0, h; (h = nt + (k + 1) * S) < H; ++k) {
                    c->bits[2 * k] = (int16_t)c->hist[2 * h];
                    c->bits[2 * k + 1] = (int16_t)c->hist[2 * h + 1];
                }
                return 1;  /* break: `top` NOT advanced (:291 vs :296) */
            }
        }
        c->top = (size_t)((top + 1) % H);
    }
    return 0;
}

int orc_corr_step(orc_corr *c, const int16_t *in, long n, int *corr_index) {
    return corr_run(c, in, n, corr_index, 1, NULL, NULL);
}

/* Not a reference call: the state the correlator has after streaming `in`
 * with no detection in it (used to seed a time segment with its halo, so a
 * buffer split over ranks finds the same first detection). */
void orc_corr_prime(orc_corr *c, const int16_t *in, long n) {
    int dummy = 0;
    (void)corr_run(c, in, n, &dummy, 0, NULL, NULL);
}

/* Not a reference call: stream `in` like orc_corr_prime (no detection test,
 * so no `break`) and record every sample's registers as the reference computes
 * them before its peak test (correlators.h:244-250): corr_out[i] =
 * corrValue[0], energy_out[i] = energyValue[0].  Test infrastructure for the
 * integer matrix-core probe (scripts/tune/corr_mfma.py), which computes the
 * same two values for every sample of the config-5 buffer. */
void orc_corr_registers(orc_corr *c, const int16_t *in, long n, uint32_t *corr_out, uint32_t *energy_out) {
    int dummy = 0;
    (void)corr_run(c, in, n, &dummy, 0, corr_out, energy_out);
}

void orc_corr_bit_samples(const orc_corr *c, int16_t *out) { memcpy(out, c->bits, 4 * (size_t)c->N); }
void orc_corr_status(const orc_corr *c, uint32_t *e3, uint32_t *c3, uint32_t *ce, int *cs, double *tf) {
    for (int i = 0; i < 3; ++i) { e3[i] = c->energy[i]; c3[i] = c->corr[i]; }
    *ce = c->coeffs_energy; *cs = c->coeff_scaling; *tf = c->threshold_factor;
}
void orc_corr_destroy(orc_corr *c) {
    if (!c) return;
    free(c->hist); free(c->coef); free(c->bits); free(c);
}

/* ============================ synthetic inputs ============================ */

uint64_t orc_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* component c of sample i: lo + (splitmix64((seed ^ ch<<40) + 2i + c) >> 32) mod (hi-lo+1) */
static inline int32_t gen_val(uint64_t key, uint64_t i, int lo, int hi) {
    uint64_t u = orc_splitmix64(key + i);
    return lo + (int32_t)((u >> 32) % (uint64_t)(hi - lo + 1));
}
void orc_gen_cf32(uint64_t seed, uint64_t ch, uint64_t off, long n, int lo, int hi, float *out) {
    uint64_t key = seed ^ (ch << 40);
    for (long i = 0; i < 2 * n; ++i) out[i] = (float)gen_val(key, 2 * off + (uint64_t)i, lo, hi);
}
void orc_gen_ci16(uint64_t seed, uint64_t ch, uint64_t off, long n, int lo, int hi, int16_t *out) {
    uint64_t key = seed ^ (ch << 40);
    for (long i = 0; i < 2 * n; ++i) out[i] = (int16_t)gen_val(key, 2 * off + (uint64_t)i, lo, hi);
}


/* ===================================================== FifoWithTimeTrack
 * buffers.h:58-459.  Bookkeeping restated with the reference's uint64/size_t
 * modular arithmetic, including its quirks: timeStart = 1 while the ring is
 * not full (:199-202), count() = timeEnd - timeStart + 1 (so 1 when empty,
 * :377-392), reset() clears the indices only (:245-258).                  */
struct orc_fifo {
    size_t es, N;
    unsigned char *storage;
    size_t write_ptr;
    uint64_t time_start, time_end;
    int rollover;
    double fs;
    uint64_t ref_tp;
    unsigned ref_sec;
    double ref_frac;
};

orc_fifo *orc_fifo_create(size_t elem_bytes, size_t N, double fs) {
    orc_fifo *f = (orc_fifo *)calloc(1, sizeof(orc_fifo));
    f->es = elem_bytes;
    f->N = N;
    f->storage = (unsigned char *)calloc(N, elem_bytes); /* storage(N): value-initialised */
    f->fs = fs;
    return f;
}

int orc_fifo_write(orc_fifo *f, const void *in, size_t n, unsigned seconds, double frac) {
    const size_t N = f->N, es = f->es;
    if (n >= N) return -1; /* assert(inSize < N) :145 */
    const size_t up = N - f->write_ptr;
    const unsigned char *src = (const unsigned char *)in;
    if (n <= up) {
        memcpy(f->storage + f->write_ptr * es, src, n * es);
    } else {
        memcpy(f->storage + f->write_ptr * es, src, up * es);
        memcpy(f->storage, src + up * es, (n - up) * es);
    }
    f->write_ptr = (f->write_ptr + n) % N; /* :162 */
    uint64_t diff = UINT64_MAX - f->time_end;
    f->ref_tp = f->time_end + 1; /* :171-173 */
    f->ref_sec = seconds;
    f->ref_frac = frac;
    if (diff >= n) {
        f->time_end += n;
    } else {
        f->time_end = n - diff;
        f->rollover = 1;
    }
    if (!f->rollover) { /* :192-202 */
        if ((f->time_end - f->time_start + 1) > N)
            f->time_start = f->time_end - N + 1;
        else
            f->time_start = 1;
    } else {
        uint64_t d2 = UINT64_MAX - f->time_start;
        if (d2 >= n)
            f->time_start += n;
        else
            f->time_start = n - d2;
        f->rollover = 0;
    }
    return 0;
}

int orc_fifo_read(orc_fifo *f, void *out, size_t n, uint64_t *start) {
    const size_t N = f->N, es = f->es;
    if (n == 0) return -1; /* assert(out.size() != 0) :286 */
    if (*start < f->time_start) *start = f->time_start; /* :299-305 (warning on stderr) */
    if ((*start + n - 1) > f->time_end) return 1;
    uint64_t end = *start + n - 1;
    size_t sp = (size_t)((f->write_ptr + N - (f->time_end - *start) - 1) % N); /* :313-314 */
    size_t ep = (size_t)((f->write_ptr + N - (f->time_end - end) - 1) % N);
    unsigned char *dst = (unsigned char *)out;
    if (ep >= sp) {
        memcpy(dst, f->storage + sp * es, (ep + 1 - sp) * es);
    } else {
        memcpy(dst, f->storage + sp * es, (N - sp) * es);
        memcpy(dst + (N - sp) * es, f->storage, (ep + 1) * es);
    }
    return 0;
}

size_t orc_fifo_count(const orc_fifo *f) {
    if (!f->rollover) return (size_t)((f->time_end - f->time_start) + 1);
    return (size_t)((UINT64_MAX - f->time_start) + f->time_end + 1);
}

void orc_fifo_reset(orc_fifo *f) {
    f->write_ptr = 0;
    f->time_start = 0;
    f->time_end = 0;
    f->rollover = 0;
}

/* buffers.h:413-459 */
void orc_fifo_absolute_time(const orc_fifo *f, uint64_t tp, double frac_tp, unsigned *seconds, double *frac_seconds) {
    int64_t sample_diff = (int64_t)(tp - f->ref_tp);
    double time_diff = sample_diff / f->fs;
    int32_t tdi = (int32_t)floor(time_diff);
    double tdf = time_diff - floor(time_diff);
    uint32_t sec = f->ref_sec + tdi;
    double fs = f->ref_frac + tdf + (frac_tp / f->fs);
    int32_t tmp = (int32_t)fs;
    fs -= tmp;
    sec += tmp;
    *seconds = sec;
    *frac_seconds = fs;
}

void orc_fifo_destroy(orc_fifo *f) {
    if (!f) return;
    free(f->storage);
    free(f);
}
