// ops.h -- handle layouts shared between the operator translation units.
#pragma once
#include "common.h"

namespace srcdsp {

// Kernel-level sample/coefficient combinations.  Decimator variants 0-3 map
// 1:1; FilterFir variant 1 (float in, float taps, complex<float> out with a
// zero imaginary part) is KV_F32_REAL.
enum KernelVariant { KV_CF32 = 0, KV_CI16_I32 = 1, KV_CI16_I16 = 2, KV_CI32_I32 = 3, KV_F32_REAL = 4 };

inline int kv_in_bytes(int kv) { return kv == KV_CF32 || kv == KV_CI32_I32 ? 8 : 4; }
inline int kv_out_bytes(int kv) { return kv == KV_CF32 || kv == KV_F32_REAL ? 8 : 4; }
inline int kv_coef_bytes(int kv) { return kv == KV_CI16_I16 ? 2 : 4; }

// The FIR core behind FilterDnsamplingFir and FilterFir: N taps, decimation M,
// history = the last N-1 input samples (ping-pong device buffers so a step can
// read the old history while writing the new one).
struct FirCore {
    int kv = 0;
    unsigned M = 1;
    int ntaps = 0;
    unsigned flags = 0;
    unsigned coeff_scaling = 0;  // as the reference stores it (unsigned)
    int left_shift = 0;
    bool coef_fits_i24 = false;   // integer taps usable by v_mad_i32_i24
    bool coef_fits_i16 = false;   // int32 taps all in int16 range: v_dot2 tap pairs
    void *d_coef = nullptr;       // float[N] or int32[N] (int16 taps widened)
    uint32_t *d_cpair = nullptr;  // N/2+1 packed tap pairs (lo c[2j], hi c[2j-1]) when coef_fits_i16
    std::string h_coef;           // host copy of the taps as given (batch compatibility)
    void *d_hist[2] = {nullptr, nullptr};
    size_t hist_cap = 0;          // bytes per history buffer
    int cur = 0;
    Ordering order;
    HostStage stage;

    int init(int kv, unsigned M, const void *coeffs, int ntaps, unsigned flags);
    int set_coeffs(const void *coeffs, int ntaps, bool keep_history);
    int clear_history();
    int clone_from(FirCore &src);
    void destroy();
    unsigned shift() const { return coeff_scaling - (unsigned)left_shift; }
    int H() const { return ntaps - 1; }
};

// Per-launch description of one channel for the batched kernels.
constexpr int kMaxBatch = 64;

struct DecimLaunch {
    const void *in;
    void *out;
    const void *coef;
    long n_in, n_out;
    long in_stride, out_stride;   // samples, between channels (grid.y)
    int ntaps;
    unsigned shift;
    long ntiles;
    // fused NCO mixer (mixers.h) ahead of the filter
    const int16_t *mix_table;
    unsigned mix_N;
    unsigned mix_phase0, mix_freq;
    // host-precomputed phases (no 64-bit modulo on the device):
    unsigned mix_phase_tile0;  // phase of tile 0's first staged sample (index -4*NQ)
    unsigned mix_dtile;        // phase advance per tile (4*TO samples)
    unsigned mix_phase_hist;   // phase of input sample n_in - H (history write-back)
    // sequence-table mixer (decim_dot2_ci16 TABM = 2): the table holds the
    // (cos, sin) word of input sample s at s mod mix_pe, mix_pe = lcm(period of
    // s*freq mod N, 4); per-tile / per-granule-row advances of that index
    unsigned mix_pe, mix_pe_dtile, mix_pe_drow;
    const void *hist_in[kMaxBatch];
    void *hist_out[kMaxBatch];
};

int decim_launch(FirCore &f, const DecimLaunch &L, int channels, hipStream_t s, bool mixed);
// the complex<float> headline kernel (decim_cf32_ct.hip / decim_cf32_rt.hip):
// with the tap count compiled in (SRCDSP_ERR_UNSUPPORTED for a shape it is not
// compiled for), or at run time (M in 1/2/3/4/8/16, N <= kCfMaxTaps)
int launch_cf32_compiled(DecimLaunch L, int channels, unsigned M, int N, bool fma, hipStream_t s);
int launch_cf32_rt(DecimLaunch L, int channels, unsigned M, bool fma, hipStream_t s);

struct MixerState {
    unsigned N = 4096;
    int16_t phi = 0, freq = 0;
    float nominal = 0.f;
    int16_t *d_table = nullptr;
    int16_t *h_table = nullptr;
    // grow-only scratch of the unfused mixer -> decimator chain (the mixed
    // samples between the two launches)
    void *d_scratch = nullptr;
    size_t scratch_cap = 0;
    Ordering order;
    HostStage stage;
};

}  // namespace srcdsp

struct srcdsp_decim { srcdsp::FirCore core; };
struct srcdsp_fir { srcdsp::FirCore core; };
struct srcdsp_mixer { srcdsp::MixerState m; };
