/*
 * ref_api.h -- C entry points of the REFERENCE BUILD (test infrastructure only).
 *
 * The .cpp files next to this header instantiate the unmodified SrcDsp class
 * templates found under /root/reference (included via -I, never copied) and
 * expose them through a plain C ABI so that tests/golden/gen_golden.py and
 * bench.py's cpu_baseline leg can drive them through ctypes.  The build recipe
 * is oracle/refbuild/Makefile; outputs go to oracle/_ref/ only.
 *
 * Type-variant codes (shared with srcdsp_amd and include/srcdsp_hip.h):
 *   decimator  0: <cf32,cf32,cf32,float>      1: <ci16,ci16,ci32,int32_t>
 *              2: <ci16,ci16,ci32,int16_t>    3: <ci32,ci16,ci32,int32_t>
 *   fir        0: <cf32,cf32,cf32,float>      1: <float,cf32,float,float>
 *              2: <ci16,ci16,ci32,int32_t>
 *   upsampler  0: <ci16,ci16,ci32,int32_t>    1: <ci16,ci16,ci32,int16_t>
 *              2: <int16_t,int16_t,int32_t,int32_t>
 */
#ifndef SRCDSP_REF_API_H
#define SRCDSP_REF_API_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
#pragma GCC visibility push(default)

/* dnsampling_filters.h (obsolete header, no N%M assert) */
void *ref_decim_create(int variant, unsigned M, const void *coeffs, int ntaps);
void ref_decim_set_left_shift(void *h, int ls);
void ref_decim_reset(void *h);
void ref_decim_step(void *h, const void *in, long n_in, void *out);
void ref_decim_destroy(void *h);
double ref_decim_step_timed(void *h, const void *in, long n_in, void *out);

/* dsptl_dnsampling_filters.h (current header; setCoeffs asserts N%M==0) */
void *ref_decim2_create(int variant, unsigned M, const void *coeffs, int ntaps);
void ref_decim2_set_coeffs(void *h, const void *coeffs, int ntaps);
void ref_decim2_set_left_shift(void *h, int ls);
void ref_decim2_reset(void *h);
void ref_decim2_step(void *h, const void *in, long n_in, void *out);
void ref_decim2_destroy(void *h);

/* dnsampling_filters.h compiled with <math.h> included first (fabs binding) */
void *ref_decim_fabs_create(int variant, unsigned M, const void *coeffs, int ntaps);
void ref_decim_fabs_step(void *h, const void *in, long n_in, void *out);
void ref_decim_fabs_destroy(void *h);

/* filters.h */
void *ref_fir_create(int variant, const void *coeffs, int ntaps);
void ref_fir_set_coeffs(void *h, const void *coeffs, int ntaps);
void ref_fir_reset(void *h);
void ref_fir_step(void *h, const void *in, long n, void *out);
void ref_fir_destroy(void *h);

/* upsampling_filters.h */
void *ref_up_create(int variant, unsigned L, const void *coeffs, int ntaps);
void ref_up_reset(void *h);
int ref_up_get_length(void *h);
int ref_up_get_imp_length(void *h);
/* out must hold L*n_in (+ L*(length/L) when flush) elements */
void ref_up_step(void *h, const void *in, long n_in, void *out, int flush);
void ref_up_step_iter(void *h, const void *in, long n_in, void *out, int flush);
void ref_up_destroy(void *h);

/* mixers.h, Mixer<ci16,ci16,int16_t,N> */
void *ref_mixer_create(unsigned N);
void ref_mixer_reset(void *h, float f);
void ref_mixer_set_frequency(void *h, float f);
void ref_mixer_adjust_frequency(void *h, float f);
void ref_mixer_step(void *h, const int16_t *in, long n, int16_t *out);
void ref_mixer_state(void *h, int *phi, int *freq, float *nominal);
void ref_mixer_table(void *h, int16_t *table);
void ref_mixer_destroy(void *h);

/* correlators.h, FixedPatternCorrelator<int16_t,int32_t,N,S> */
void *ref_corr_create(unsigned N, unsigned S);
void ref_corr_set_pattern(void *h, const int32_t *pattern_ci32, double threshold_coeff);
void ref_corr_reset(void *h);
int ref_corr_step(void *h, const int16_t *in_ci16, long n, int *corr_index);
void ref_corr_bit_samples(void *h, int16_t *out_ci16);
/* energy[3], corr[3], coeffs_energy, coeff_scaling, threshold_factor */
void ref_corr_status(void *h, uint32_t *energy3, uint32_t *corr3, uint32_t *coeffs_energy,
                     int *coeff_scaling, double *threshold_factor);
void ref_corr_destroy(void *h);

#pragma GCC visibility pop
#ifdef __cplusplus
}
#endif
#endif
