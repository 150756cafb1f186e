/*
 * srcdsp_hip.h -- C ABI of libsrcdsp_hip.so, the MI355X (gfx950) implementation
 * of SrcDsp's sample-buffer hot path.
 *
 * Every entry point replaces one member function of a SrcDsp operator class;
 * the reference interface is cited next to each declaration as
 * <file>:<line> of the upstream tree (dogjin/SrcDsp).  Plain pointers and sizes
 * only: no C++ or framework types cross this boundary.  A `stream` argument is a
 * hipStream_t passed as void* (NULL = the default stream).
 *
 * Conventions shared by all operators
 *  - Handles own the operator state on the device (coefficients, history ring,
 *    NCO phase, correlator registers) exactly as the reference objects own it
 *    in member vectors; the caller owns input/output buffers.
 *  - `*_step` takes DEVICE pointers and is asynchronous on `stream`; successive
 *    calls on one handle are ordered even across streams (the handle keeps an
 *    event of its last step).  `*_step_host` takes HOST pointers, stages through
 *    pinned memory and returns when the result is in `out` (PCIe-bound;
 *    drop-in convenience).
 *  - Sizes are in samples (one complex sample = one element).  Where the
 *    reference asserts (e.g. dnsampling_filters.h:133 out.size()*M==in.size())
 *    the C ABI returns SRCDSP_ERR_SIZE instead of aborting.
 *  - Sample layouts are those of std::complex<T> (interleaved re, im).
 */
#ifndef SRCDSP_HIP_H
#define SRCDSP_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define SRCDSP_API __attribute__((visibility("default")))
#else
#define SRCDSP_API
#endif

/* ---------------------------------------------------------------- status */
enum {
    SRCDSP_OK = 0,
    SRCDSP_ERR_ARG = -1,         /* null handle/pointer, invalid parameter           */
    SRCDSP_ERR_UNSUPPORTED = -2, /* type combination / ratio the reference cannot build */
    SRCDSP_ERR_SIZE = -3,        /* a size the reference asserts on                 */
    SRCDSP_ERR_HIP = -4,         /* HIP runtime failure (see srcdsp_last_error)     */
    SRCDSP_ERR_NOMEM = -5
};

/* ---------------------------------------------------------------- flags */
enum {
    /* Coefficient magnitude for coeffScaling (dnsampling_filters.h:92-95,
     * filters.h:92-96).  Default: the binding of a canonical TU, where
     * unqualified abs(float) resolves to ::abs(int) (coefficient truncated).
     * With this flag: fabs(), the binding seen when <math.h> precedes the
     * header. */
    SRCDSP_FLAG_ABS_FABS = 1u << 0,
    /* Floating-point accumulation contract of the complex<float> paths.
     * Default: one fused multiply-add per tap, taps in ascending order --
     * bit-exact to the reference built with -mfma, and |d| <= 1 output LSB on
     * <= 1e-4 of outputs against the -O2 x86-64 build.  With this flag:
     * separately rounded multiply then add -- bit-exact to the -O2 build. */
    SRCDSP_FLAG_FP_STRICT = 1u << 1
};

/* ============================================================================
 * FilterDnsamplingFir<In,Out,Internal,Coef,M>   (dnsampling_filters.h:49-172,
 * dsptl_dnsampling_filters.h:47-220)
 * variant: 0 <complex<float>, complex<float>, complex<float>, float>
 *          1 <complex<int16_t>, complex<int16_t>, complex<int32_t>, int32_t>
 *          2 <complex<int16_t>, complex<int16_t>, complex<int32_t>, int16_t>
 *          3 <complex<int32_t>, complex<int16_t>, complex<int32_t>, int32_t>
 * coeffs points to ntaps values of the Coef type.
 * ==========================================================================*/
typedef struct srcdsp_decim *srcdsp_decim_t;

/* ctor FilterDnsamplingFir(const vector<Coef>&)  dnsampling_filters.h:84-97 */
SRCDSP_API int srcdsp_decim_create(srcdsp_decim_t *out, int variant, unsigned M, const void *coeffs,
                                   int ntaps, unsigned flags);
SRCDSP_API int srcdsp_decim_destroy(srcdsp_decim_t h);
/* copy construction / assignment (the reference class is a value type: its
 * implicit copy ctor copies coefficients, history and shifts,
 * dnsampling_filters.h:47-79): *out = a new handle with h's coefficients,
 * coeffScaling, leftShift and CURRENT history (after h's pending steps) */
SRCDSP_API int srcdsp_decim_clone(srcdsp_decim_t h, srcdsp_decim_t *out);
/* setCoeffs  dsptl_dnsampling_filters.h:114-134 (history resized, not cleared;
 * require_multiple != 0 reproduces its assert(N % M == 0) as SRCDSP_ERR_SIZE) */
SRCDSP_API int srcdsp_decim_set_coeffs(srcdsp_decim_t h, const void *coeffs, int ntaps,
                                       int require_multiple);
/* setLeftShiftBy2  dnsampling_filters.h:63 */
SRCDSP_API int srcdsp_decim_set_left_shift(srcdsp_decim_t h, int left_shift);
/* reset  dnsampling_filters.h:56-60 */
SRCDSP_API int srcdsp_decim_reset(srcdsp_decim_t h);
/* step  dnsampling_filters.h:129-172 ; requires n_out * M == n_in */
SRCDSP_API int srcdsp_decim_step(srcdsp_decim_t h, const void *d_in, size_t n_in, void *d_out,
                                 size_t n_out, void *stream);
SRCDSP_API int srcdsp_decim_step_host(srcdsp_decim_t h, const void *in, size_t n_in, void *out,
                                      size_t n_out);
/* C channels of one configuration in one launch (grid.y = channel).  Channel c
 * reads d_in + c*in_stride samples and writes d_out + c*out_stride samples;
 * each handle keeps its own history.  All handles must share variant, M, taps. */
SRCDSP_API int srcdsp_decim_step_batched(const srcdsp_decim_t *hs, int channels, const void *d_in,
                                         size_t in_stride, void *d_out, size_t out_stride,
                                         size_t n_in, void *stream);
/* state introspection (tests, checkpointing): coeffScaling as stored by the
 * reference (unsigned), leftShift, and the N-1 history samples (host copy). */
SRCDSP_API int srcdsp_decim_get_state(srcdsp_decim_t h, unsigned *coeff_scaling, int *left_shift,
                                      void *history_host);

/* ============================================================================
 * FilterFir<In,Out,Internal,Coef>   (filters.h:42-169, global namespace)
 * variant: 0 <complex<float>, complex<float>, complex<float>, float>
 *          1 <float, complex<float>, float, float>
 *          2 <complex<int16_t>, complex<int16_t>, complex<int32_t>, int32_t>
 * ==========================================================================*/
typedef struct srcdsp_fir *srcdsp_fir_t;
/* ctor / setCoeffs  filters.h:74-97 */
SRCDSP_API int srcdsp_fir_create(srcdsp_fir_t *out, int variant, const void *coeffs, int ntaps,
                                 unsigned flags);
SRCDSP_API int srcdsp_fir_destroy(srcdsp_fir_t h);
/* implicit copy of FilterFir (filters.h:42-70): coefficients, shift, history */
SRCDSP_API int srcdsp_fir_clone(srcdsp_fir_t h, srcdsp_fir_t *out);
SRCDSP_API int srcdsp_fir_set_coeffs(srcdsp_fir_t h, const void *coeffs, int ntaps);
/* reset  filters.h:107-113 */
SRCDSP_API int srcdsp_fir_reset(srcdsp_fir_t h);
/* step  filters.h:131-169 ; requires n_in == n_out */
SRCDSP_API int srcdsp_fir_step(srcdsp_fir_t h, const void *d_in, size_t n_in, void *d_out, size_t n_out,
                               void *stream);
SRCDSP_API int srcdsp_fir_step_host(srcdsp_fir_t h, const void *in, size_t n_in, void *out,
                                    size_t n_out);

/* ============================================================================
 * FilterUpsamplingFir<In,Out,Internal,Coef,L>   (upsampling_filters.h:36-326)
 * variant: 0 <complex<int16_t>, complex<int16_t>, complex<int32_t>, int32_t>
 *          1 <complex<int16_t>, complex<int16_t>, complex<int32_t>, int16_t>
 *          2 <int16_t, int16_t, int32_t, int32_t>
 * ==========================================================================*/
typedef struct srcdsp_up *srcdsp_up_t;
/* ctor / setCoefficients  upsampling_filters.h:86-126 (ntaps % L == 0) */
SRCDSP_API int srcdsp_up_create(srcdsp_up_t *out, int variant, unsigned L, const void *coeffs, int ntaps);
SRCDSP_API int srcdsp_up_destroy(srcdsp_up_t h);
/* implicit copy of FilterUpsamplingFir (upsampling_filters.h:36-87): taps,
 * length, shift and the current history ring */
SRCDSP_API int srcdsp_up_clone(srcdsp_up_t h, srcdsp_up_t *out);
SRCDSP_API int srcdsp_up_set_coeffs(srcdsp_up_t h, const void *coeffs, int ntaps);
/* reset  upsampling_filters.h:50-55 */
SRCDSP_API int srcdsp_up_reset(srcdsp_up_t h);
/* getLength / getImpLength / getUpsamplingRatio  upsampling_filters.h:57-67 */
SRCDSP_API int srcdsp_up_get_length(srcdsp_up_t h, int *length, int *imp_length, int *ratio);
/* step(vector, flush)  upsampling_filters.h:149-233 (iterator=0) and
 * step(iterator, flush)  :240-323 (iterator=1: output shift 0).
 * n_out must be L*n_in, or L*(n_in + length/L) when flush. */
SRCDSP_API int srcdsp_up_step(srcdsp_up_t h, const void *d_in, size_t n_in, void *d_out, size_t n_out,
                              int flush, int iterator, void *stream);
SRCDSP_API int srcdsp_up_step_host(srcdsp_up_t h, const void *in, size_t n_in, void *out, size_t n_out,
                                   int flush, int iterator);

/* ============================================================================
 * Mixer<complex<int16_t>, complex<int16_t>, int16_t, N>   (mixers.h:27-188)
 * ==========================================================================*/
typedef struct srcdsp_mixer *srcdsp_mixer_t;
/* ctor  mixers.h:149-159 (LUT of N points), _Mixer() phi = freq = 0 */
SRCDSP_API int srcdsp_mixer_create(srcdsp_mixer_t *out, unsigned N);
SRCDSP_API int srcdsp_mixer_destroy(srcdsp_mixer_t h);
/* implicit copy of Mixer (mixers.h:27-48, 134-160): table, phi, freq, nominal */
SRCDSP_API int srcdsp_mixer_clone(srcdsp_mixer_t h, srcdsp_mixer_t *out);
/* setFrequency / reset / adjustFrequency  mixers.h:51-98 */
SRCDSP_API int srcdsp_mixer_set_frequency(srcdsp_mixer_t h, float lo_freq);
SRCDSP_API int srcdsp_mixer_reset(srcdsp_mixer_t h, float lo_freq);
SRCDSP_API int srcdsp_mixer_adjust_frequency(srcdsp_mixer_t h, float adjust);
/* phase, frequency word, nominal frequency; and the N-entry LUT (host copy) */
SRCDSP_API int srcdsp_mixer_get_state(srcdsp_mixer_t h, int *phi, int *freq, float *nominal);
SRCDSP_API int srcdsp_mixer_get_table(srcdsp_mixer_t h, int16_t *table_host);
/* Extension (no reference call; SURVEY 8e time sharding): set the phase
 * accumulator phi (0 <= phi < N), the closed form (phi0 + k*freq) mod N of
 * mixers.h:177 at sample k, so a buffer segment starting at sample k mixes
 * exactly as the unsplit buffer. */
SRCDSP_API int srcdsp_mixer_set_phase(srcdsp_mixer_t h, int phi);
/* step  mixers.h:169-188 ; n_out == n_in */
SRCDSP_API int srcdsp_mixer_step(srcdsp_mixer_t h, const void *d_in, size_t n, void *d_out, void *stream);
SRCDSP_API int srcdsp_mixer_step_host(srcdsp_mixer_t h, const void *in, size_t n, void *out);

/* Mixer -> FilterDnsamplingFir (variant 1) fused: the two reference calls
 * mixer.step(in, tmp); decim.step(tmp, out) in one pass with no intermediate
 * buffer.  Both objects' state advances exactly as in the two calls. */
SRCDSP_API int srcdsp_mixdecim_step(srcdsp_mixer_t mixer, srcdsp_decim_t decim, const void *d_in,
                                    size_t n_in, void *d_out, size_t n_out, void *stream);

/* ============================================================================
 * FixedPatternCorrelator<int16_t, int32_t, N, S>   (correlators.h:54-316)
 * ==========================================================================*/
typedef struct srcdsp_corr *srcdsp_corr_t;
/* ctor  correlators.h:119-132 */
SRCDSP_API int srcdsp_corr_create(srcdsp_corr_t *out, unsigned N, unsigned S);
SRCDSP_API int srcdsp_corr_destroy(srcdsp_corr_t h);
/* implicit copy of FixedPatternCorrelator (correlators.h:54-118): pattern,
 * thresholds, history ring, the three corr/energy registers, bitSamples */
SRCDSP_API int srcdsp_corr_clone(srcdsp_corr_t h, srcdsp_corr_t *out);
/* setPattern(array<complex<int32_t>,N>, thresholdCoeff)  correlators.h:167-194;
 * pattern = N complex<int32_t> (2N int32).  The reference's
 * assert(energy <= 1073217600) is returned as SRCDSP_ERR_ARG. */
SRCDSP_API int srcdsp_corr_set_pattern(srcdsp_corr_t h, const int32_t *pattern, double threshold_coeff);
/* reset  correlators.h:146-159 */
SRCDSP_API int srcdsp_corr_reset(srcdsp_corr_t h);
/* step(in, corrIndex) -> bool  correlators.h:209-303.  *found = 0/1,
 * *corr_index written only when found (as the reference).  Synchronous: the
 * answer is needed on the host. */
SRCDSP_API int srcdsp_corr_step(srcdsp_corr_t h, const void *d_in, size_t n, int *found, int *corr_index,
                                void *stream);
SRCDSP_API int srcdsp_corr_step_host(srcdsp_corr_t h, const void *in, size_t n, int *found,
                                     int *corr_index);
/* Extension (no reference call; SURVEY 8e time sharding): the state step()
 * leaves after streaming these n samples with NO detection test
 * (correlators.h:221-250 without :262-291): history ring and the
 * energy/correlation registers.  Seeds a time segment with its halo. */
SRCDSP_API int srcdsp_corr_prime(srcdsp_corr_t h, const void *d_in, size_t n, void *stream);
/* step() as built with CREATE_DEBUG_FILES (correlators.h:107-132, 253-257):
 * also returns, for every sample the call processed, the registers the
 * reference writes to its debug files -- corr_out[k] = corrValue[0] and
 * energy_out[k] = energyValue[0] after input sample k (host arrays of n
 * entries; *count = corrIndex + 2 on a detection, else n).  Runs the
 * segmented kernels (they keep per-sample values); same results as step(). */
SRCDSP_API int srcdsp_corr_step_trace(srcdsp_corr_t h, const void *d_in, size_t n, int *found, int *corr_index,
                                      uint32_t *corr_out, uint32_t *energy_out, size_t *count, void *stream);
SRCDSP_API int srcdsp_corr_step_host_trace(srcdsp_corr_t h, const void *in, size_t n, int *found, int *corr_index,
                                           uint32_t *corr_out, uint32_t *energy_out, size_t *count);
/* getRefBitSamples  correlators.h:311-316 (N complex<int16_t>, host copy) */
SRCDSP_API int srcdsp_corr_get_bit_samples(srcdsp_corr_t h, int16_t *bits_host);
/* getStatus  correlators.h:90 (CorrState fields) */
SRCDSP_API int srcdsp_corr_get_status(srcdsp_corr_t h, uint32_t *energy3, uint32_t *corr3,
                                      uint32_t *coeffs_energy, int *coeff_scaling,
                                      double *threshold_factor);

/* ============================================================================
 * FifoWithTimeTrack<T, N>   (buffers.h:58-459), the ring in HBM
 * One producer thread writes, one consumer thread reads (as the reference).
 * Element type T is opaque: elem_bytes per element.
 * ==========================================================================*/
typedef struct srcdsp_fifo *srcdsp_fifo_t;
/* ctor FifoWithTimeTrack(samplingFrequency)  buffers.h:62-66 (storage(N) zeroed) */
SRCDSP_API int srcdsp_fifo_create(srcdsp_fifo_t *out, size_t elem_bytes, size_t N, double sampling_frequency);
SRCDSP_API int srcdsp_fifo_destroy(srcdsp_fifo_t h);
/* write(in, seconds, fracSeconds)  buffers.h:140-224.  Host input, staged
 * through two pinned buffers; returns before its H2D copy completes (readers
 * are ordered after it on the device).  assert(inSize < N) -> SRCDSP_ERR_SIZE. */
SRCDSP_API int srcdsp_fifo_write(srcdsp_fifo_t h, const void *in, size_t n, unsigned seconds,
                                 double frac_seconds);
/* the same for device-resident input, copied D2D on `stream` */
SRCDSP_API int srcdsp_fifo_write_device(srcdsp_fifo_t h, const void *d_in, size_t n, unsigned seconds,
                                        double frac_seconds, void *stream);
/* read(out, start) -> bool  buffers.h:282-349.  *error = the reference's return
 * value (1: range not available); *start is raised to timeStart as the
 * reference does (with its stderr warning).  Output in device memory, copied
 * on `stream`; assert(out.size() != 0) -> SRCDSP_ERR_SIZE. */
SRCDSP_API int srcdsp_fifo_read(srcdsp_fifo_t h, void *d_out, size_t n, uint64_t *start, int *error,
                                void *stream);
SRCDSP_API int srcdsp_fifo_read_host(srcdsp_fifo_t h, void *out, size_t n, uint64_t *start, int *error);
/* count()  buffers.h:377-392 ; reset()  buffers.h:245-258 (indices only) */
SRCDSP_API int srcdsp_fifo_count(srcdsp_fifo_t h, size_t *count);
SRCDSP_API int srcdsp_fifo_reset(srcdsp_fifo_t h);
/* the fields dumpInfo() prints  buffers.h:229-240 */
SRCDSP_API int srcdsp_fifo_get_state(srcdsp_fifo_t h, size_t *write_ptr, uint64_t *time_start,
                                     uint64_t *time_end, int *rollover);
/* getAbsoluteTime(timePoint, fracTimePoint)  buffers.h:413-459 */
SRCDSP_API int srcdsp_fifo_get_absolute_time(srcdsp_fifo_t h, uint64_t time_point, double frac_time_point,
                                             unsigned *seconds, double *frac_seconds);

/* ============================================================================
 * Binary I/Q captures   (dsptl_files.h:101-109 saveBinarySamples,
 * :250-262 readBinarySamples).  Interleaved I,Q components of
 * component_bytes each.  Reading returns whole samples only and replaces the
 * output (the reference's out.empty() / trailing-sample bugs fixed).
 * ==========================================================================*/
SRCDSP_API int srcdsp_iq_save(const char *path, const void *d_samples, size_t n, size_t component_bytes,
                              int append, void *stream);
SRCDSP_API int srcdsp_iq_save_host(const char *path, const void *samples, size_t n, size_t component_bytes,
                                   int append);
/* number of whole samples in the file */
SRCDSP_API int srcdsp_iq_count(const char *path, size_t component_bytes, size_t *n);
SRCDSP_API int srcdsp_iq_load(const char *path, size_t component_bytes, void *d_out, size_t cap, size_t *n,
                              void *stream);
SRCDSP_API int srcdsp_iq_load_host(const char *path, size_t component_bytes, void *out, size_t cap, size_t *n);

/* ============================================================================
 * Multi-GPU (BASELINE configs[2]): one host process drives
 * several GPUs of one node.  The reference has no multi-device code; these
 * entries shard what its users do with one FilterDnsamplingFir object per
 * channel (dnsampling_filters.h:49-172) across devices, and bring the results
 * back with RCCL over xGMI.
 *
 * srcdsp_comm_t: one RCCL communicator per device, made together in this
 * process by ncclCommInitAll (rccl.h:236), plus one non-blocking HIP stream
 * per device on which the sharded operators run.  `rank` below = index into
 * the device list.
 * RCCL is loaded at the first srcdsp_comm_create (dlopen of librccl): without
 * it that call returns SRCDSP_ERR_UNSUPPORTED, and nothing else needs RCCL.
 * A sharded operator holds a reference to its comm: srcdsp_comm_destroy may
 * come before srcdsp_decim_sharded_destroy.
 * Verified on one GPU (contiguous and strided gathers); the N > 1 paths are
 * unverified on hardware until a multi-GPU node runs them.
 * ==========================================================================*/
typedef struct srcdsp_comm *srcdsp_comm_t;
/* devs may be NULL (devices 0..ndev-1) */
SRCDSP_API int srcdsp_comm_create(srcdsp_comm_t *out, int ndev, const int *devs);
SRCDSP_API int srcdsp_comm_destroy(srcdsp_comm_t c);
/* ndev, and the HIP device id of each rank (devs may be NULL) */
SRCDSP_API int srcdsp_comm_info(srcdsp_comm_t c, int *ndev, int *devs);
/* the hipStream_t (as void*) the sharded operators use on rank's device */
SRCDSP_API int srcdsp_comm_stream(srcdsp_comm_t c, int rank, void **stream);
/* wait for every rank's stream */
SRCDSP_API int srcdsp_comm_synchronize(srcdsp_comm_t c);
/* ORDERING RULE.  The comm streams are non-blocking: they do not wait for the
 * null stream or for any stream of the caller, and the caller's streams do
 * not wait for them.  Caller work that writes a rank's d_in, or touches its
 * d_out / the gather target d_root, must run on comm stream(rank), or after
 * srcdsp_comm_synchronize, or be ordered by these two calls (no host block):
 *   srcdsp_comm_wait_stream(c, r, s):   work queued later on rank r's comm
 *       stream (steps, gathers) waits for everything queued on `s` so far;
 *   srcdsp_comm_signal_stream(c, r, s): work queued later on `s` waits for
 *       everything queued on rank r's comm stream so far.
 * `s` is a hipStream_t (as void*) on rank r's device; NULL = its null stream. */
SRCDSP_API int srcdsp_comm_wait_stream(srcdsp_comm_t c, int rank, void *stream);
SRCDSP_API int srcdsp_comm_signal_stream(srcdsp_comm_t c, int rank, void *stream);

/* `channels` independent FilterDnsamplingFir objects of one configuration
 * (same variant/M/taps/flags as srcdsp_decim_create), block-partitioned over
 * the comm's devices: rank r owns channels [first_r, first_r + count_r), the
 * first channels % ndev ranks one more.  Each channel keeps its own history
 * on its own device; a step is one batched launch per device (no collective). */
typedef struct srcdsp_decim_sharded *srcdsp_decim_sharded_t;
SRCDSP_API int srcdsp_decim_sharded_create(srcdsp_decim_sharded_t *out, srcdsp_comm_t comm, int channels,
                                           int variant, unsigned M, const void *coeffs, int ntaps,
                                           unsigned flags);
SRCDSP_API int srcdsp_decim_sharded_destroy(srcdsp_decim_sharded_t h);
SRCDSP_API int srcdsp_decim_sharded_partition(srcdsp_decim_sharded_t h, int rank, int *first_channel,
                                              int *count);
/* the per-channel handle of global channel ch (for reset / setCoeffs /
 * setLeftShiftBy2 / get_state on its own device) */
SRCDSP_API int srcdsp_decim_sharded_channel(srcdsp_decim_sharded_t h, int ch, srcdsp_decim_t *handle);
/* one step() of every channel: d_in[r] / d_out[r] are device pointers on
 * rank r's device holding its count_r channels as rows in_stride / out_stride
 * samples apart; n_in samples per channel (n_in % M == 0).  Asynchronous on
 * the comm streams (ORDERING RULE above). */
SRCDSP_API int srcdsp_decim_sharded_step(srcdsp_decim_sharded_t h, const void *const *d_in, size_t in_stride,
                                         void *const *d_out, size_t out_stride, size_t n_in);
/* reset every channel (dnsampling_filters.h:56-60), each on its own device */
SRCDSP_API int srcdsp_decim_sharded_reset(srcdsp_decim_sharded_t h);
/* host std::vector convenience (reference-style: one vector per channel):
 * in[ch] -> out[ch] for every channel, n_in samples each; each device's
 * channels staged through pinned memory by one host thread per device;
 * returns when every output is on the host. */
SRCDSP_API int srcdsp_decim_sharded_step_host(srcdsp_decim_sharded_t h, const void *const *in, void *const *out,
                                              size_t n_in);
/* result gather to one device: channel ch's n_out outputs land at
 * d_root + ch*n_out samples (d_root on rank `root`'s device, room for
 * channels*n_out samples).  ncclGather (rccl.h:745) when every rank holds the
 * same number of contiguous rows, else grouped ncclSend/ncclRecv
 * (rccl.h:700,720) with the root's own rows copied on its device.
 * Asynchronous on the comm streams (ORDERING RULE above). */
SRCDSP_API int srcdsp_decim_sharded_gather(srcdsp_decim_sharded_t h, void *const *d_out, size_t out_stride,
                                           size_t n_out, void *d_root, int root);

/* ---------------------------------------------------------------- misc */
/* Last error text of the calling thread (HIP error string or argument check). */
SRCDSP_API const char *srcdsp_last_error(void);
/* Library version "major.minor.patch" and the offload target it was built for. */
SRCDSP_API const char *srcdsp_version(void);
/* Test switches this library was built with, read back from a kernel of this
 * library: 0 for the shipped build; SRCDSP_BUILD_CORR_ALWAYS_EXACT for the
 * test-only always-exact correlator build (tests/_build/). */
#define SRCDSP_BUILD_CORR_ALWAYS_EXACT 1u
SRCDSP_API int srcdsp_build_flags(unsigned *flags);
/* Fill d_out with the counter-based synthetic samples the benchmarks use
 * (SURVEY.md §8d): component c of sample i (global index off+i) is
 * lo + (splitmix64((seed ^ channel<<40) + 2(off+i) + c) >> 32) mod (hi-lo+1).
 * kind 0 = complex<float>, 1 = complex<int16_t>. */
SRCDSP_API int srcdsp_fill_synthetic(void *d_out, int kind, size_t n, uint64_t seed, uint64_t channel,
                                     uint64_t offset, int lo, int hi, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* SRCDSP_HIP_H */
