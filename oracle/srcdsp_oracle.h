/*
 * srcdsp_oracle.h -- CPU restatement of SrcDsp's sample-buffer hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this; the product path
 * (srcdsp_amd, libsrcdsp_hip.so) never links or calls it.
 *
 * Parity: PINNED.  Every operator is checked bit-exactly against golden vectors
 * produced by the real reference (oracle/refbuild -> oracle/_ref, fixtures in
 * tests/golden/) in both floating-point flavours:
 *   fp_mode 0 "strict": separate IEEE mul then add  == reference built -O2 (x86-64, no FMA)
 *   fp_mode 1 "fma"   : one fmaf per tap, k ascending == reference built -O2 -mfma
 * Integer instantiations are flavour independent.
 *
 * Variant codes match oracle/refbuild/ref_api.h and include/srcdsp_hip.h.
 */
#ifndef SRCDSP_ORACLE_H
#define SRCDSP_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_ABS_INT = 0, ORC_ABS_FABS = 1 };
enum { ORC_FP_STRICT = 0, ORC_FP_FMA = 1 };

/* ---- L0 helpers (dsp_complex.cpp / dsp_complex.h) ---- */
int32_t orc_cvt_f2i(float f);                  /* x86 cvttss2si */
int32_t orc_cvt_d2i(double d);                 /* x86 cvttsd2si */
int16_t orc_limit16(int32_t v, unsigned shift);/* one component of limitScale16 */
unsigned orc_coeff_scaling_f32(const float *c, int n, int abs_mode);
unsigned orc_coeff_scaling_i32(const int32_t *c, int n);
unsigned orc_coeff_scaling_i16(const int16_t *c, int n);

/* ---- FilterDnsamplingFir (dnsampling_filters.h / dsptl_dnsampling_filters.h) ---- */
typedef struct orc_decim orc_decim;
orc_decim *orc_decim_create(int variant, unsigned M, const void *coeffs, int ntaps, int abs_mode,
                            int fp_mode);
void orc_decim_set_left_shift(orc_decim *d, int ls);
int orc_decim_set_coeffs(orc_decim *d, const void *coeffs, int ntaps, int abs_mode);
void orc_decim_reset(orc_decim *d);
unsigned orc_decim_coeff_scaling(const orc_decim *d);
void orc_decim_step(orc_decim *d, const void *in, long n_in, void *out);
void orc_decim_destroy(orc_decim *d);

/* ---- FilterFir (filters.h) ---- */
typedef struct orc_fir orc_fir;
orc_fir *orc_fir_create(int variant, const void *coeffs, int ntaps, int abs_mode, int fp_mode);
int orc_fir_set_coeffs(orc_fir *f, const void *coeffs, int ntaps, int abs_mode);
void orc_fir_reset(orc_fir *f);
void orc_fir_step(orc_fir *f, const void *in, long n, void *out);
void orc_fir_destroy(orc_fir *f);

/* ---- FilterUpsamplingFir (upsampling_filters.h) ---- */
typedef struct orc_up orc_up;
orc_up *orc_up_create(int variant, unsigned L, const void *coeffs, int ntaps);
void orc_up_reset(orc_up *u);
int orc_up_get_length(const orc_up *u);
/* iter != 0: the iterator overload (output shift 0, upsampling_filters.h:244) */
void orc_up_step(orc_up *u, const void *in, long n_in, void *out, int flush, int iter);
void orc_up_destroy(orc_up *u);

/* ---- Mixer<ci16,ci16,int16_t,N> (mixers.h) ---- */
typedef struct orc_mixer orc_mixer;
orc_mixer *orc_mixer_create(unsigned N);
void orc_mixer_table(const orc_mixer *m, int16_t *table);
void orc_mixer_reset(orc_mixer *m, float f);
void orc_mixer_set_frequency(orc_mixer *m, float f);
void orc_mixer_adjust_frequency(orc_mixer *m, float f);
void orc_mixer_state(const orc_mixer *m, int *phi, int *freq, float *nominal);
void orc_mixer_step(orc_mixer *m, const int16_t *in, long n, int16_t *out);
void orc_mixer_destroy(orc_mixer *m);

/* ---- FixedPatternCorrelator<int16_t,int32_t,N,S> (correlators.h) ---- */
typedef struct orc_corr orc_corr;
orc_corr *orc_corr_create(unsigned N, unsigned S);
void orc_corr_set_pattern(orc_corr *c, const int32_t *pattern_ci32, double threshold_coeff);
void orc_corr_reset(orc_corr *c);
int orc_corr_step(orc_corr *c, const int16_t *in_ci16, long n, int *corr_index);
void orc_corr_prime(orc_corr *c, const int16_t *in_ci16, long n);
void orc_corr_registers(orc_corr *c, const int16_t *in_ci16, long n, uint32_t *corr_out, uint32_t *energy_out);
void orc_corr_bit_samples(const orc_corr *c, int16_t *out_ci16);
void orc_corr_status(const orc_corr *c, uint32_t *energy3, uint32_t *corr3, uint32_t *coeffs_energy,
                     int *coeff_scaling, double *threshold_factor);
void orc_corr_destroy(orc_corr *c);

/* ---- FifoWithTimeTrack<T, N> (buffers.h:58-459), element = elem_bytes ---- */
typedef struct orc_fifo orc_fifo;
orc_fifo *orc_fifo_create(size_t elem_bytes, size_t N, double sampling_frequency);
/* returns -1 where the reference asserts (n >= N) */
int orc_fifo_write(orc_fifo *f, const void *in, size_t n, unsigned seconds, double frac_seconds);
/* returns 1 for the reference's `true` (range not available), 0 otherwise,
 * -1 where the reference asserts (n == 0); *start may be raised to timeStart */
int orc_fifo_read(orc_fifo *f, void *out, size_t n, uint64_t *start);
size_t orc_fifo_count(const orc_fifo *f);
void orc_fifo_reset(orc_fifo *f);
void orc_fifo_absolute_time(const orc_fifo *f, uint64_t time_point, double frac_time_point, unsigned *seconds,
                            double *frac_seconds);
void orc_fifo_destroy(orc_fifo *f);

/* ---- counter-based synthetic inputs shared by tests and bench ---- */
uint64_t orc_splitmix64(uint64_t x);
void orc_gen_cf32(uint64_t seed, uint64_t channel, uint64_t offset, long n, int lo, int hi, float *out);
void orc_gen_ci16(uint64_t seed, uint64_t channel, uint64_t offset, long n, int lo, int hi, int16_t *out);

#ifdef __cplusplus
}
#endif
#endif
