// common.h -- shared device arithmetic and host runtime plumbing of
// libsrcdsp_hip.so (gfx950).  Device helpers restate, in the GPU's own
// instructions, the x86 behaviour the reference's quantisers compile to
// (dsp_complex.cpp:43-73, dsp_complex.h:45-108); host helpers hold the
// per-handle stream ordering and pinned staging used by the *_step_host calls.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <type_traits>

#include "../../include/srcdsp_hip.h"

namespace srcdsp {

// ----------------------------------------------------------------- errors
void set_error(const std::string &msg);
const char *get_error();

#define SRCDSP_HIP_TRY(expr)                                                              \
    do {                                                                                  \
        hipError_t _e = (expr);                                                           \
        if (_e != hipSuccess) {                                                           \
            ::srcdsp::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));       \
            return SRCDSP_ERR_HIP;                                                        \
        }                                                                                 \
    } while (0)

#define SRCDSP_ARG_CHECK(cond, msg)                                                       \
    do {                                                                                  \
        if (!(cond)) {                                                                    \
            ::srcdsp::set_error(msg);                                                     \
            return SRCDSP_ERR_ARG;                                                        \
        }                                                                                 \
    } while (0)

// ------------------------------------------------- x86 semantics on device
// float -> int32 the way x86 cvttss2si does it: truncate, INT_MIN when out of
// range or NaN (v_cvt_i32_f32 saturates instead, so the range is tested).
__device__ __forceinline__ int32_t cvt_f2i_x86(float f) {
    int32_t i = __float2int_rz(f);
    return (f >= -2147483648.0f && f < 2147483648.0f) ? i : INT32_MIN;
}

// limitScale16 (dsp_complex.cpp:63-73), one component: sar by (shift & 31),
// symmetric clamp to +-32767 via abs(); abs(INT_MIN) is negative so INT_MIN is
// left alone and truncates to 0.
__device__ __forceinline__ int32_t limit16(int32_t v, unsigned shift) {
    int32_t a = v >> (shift & 31u);
    int32_t c = a > 32767 ? 32767 : (a < -32767 ? -32767 : a);
    return (int16_t)(a == INT32_MIN ? a : c);
}

// limitScale<int16-type, int32-type> (dsp_complex.h:45-63 / :83-108):
// asymmetric clamp to [-32768, 32767].
__device__ __forceinline__ int32_t limit_t16(int32_t v, unsigned shift) {
    int32_t a = v >> (shift & 31u);
    return a > 32767 ? 32767 : (a < -32768 ? -32768 : a);
}

// pack16(limit_t16(re, shift), limit_t16(im, shift)) in 3 VALU ops: the
// saturating v_cvt_pk_i16_i32 clamps to exactly [-32768, 32767]
__device__ __forceinline__ uint32_t limit_t16_pair(int32_t re, int32_t im, unsigned shift) {
    typedef short s2_t __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, (s2_t)__builtin_amdgcn_cvt_pk_i16(re >> (shift & 31u), im >> (shift & 31u)));
}

__device__ __forceinline__ int32_t sext16(uint32_t w) { return (int32_t)(int16_t)(w & 0xffffu); }
__device__ __forceinline__ int32_t sext16_hi(uint32_t w) { return ((int32_t)w) >> 16; }
__device__ __forceinline__ uint32_t pack16(int32_t re, int32_t im) {
    return ((uint32_t)re & 0xffffu) | ((uint32_t)im << 16);
}

// Bijective XCD-aware block -> tile map: blocks b and b+8 share an XCD
// (MI355X dispatch observation, speed only), so XCD k is handed a contiguous
// run of tiles and a tile's halo (the previous tile's tail) is an L2 hit.
__device__ __forceinline__ long xcd_tile(long bid, long nb) {
    long q = nb >> 3, r = nb & 7, x = bid & 7, i = bid >> 3;
    return x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
}

// Taps of the tile kernels are read through a CONSTANT-address-space view of
// the device coefficient buffer: wave-uniform s_load into SGPRs, consumed as
// the scalar operand of each FMA.  (Through a plain pointer the compiler must
// assume the taps may alias the outputs and uses vector loads into VGPRs.)
// The view is made opaque every 16 taps so the scalar loads are not all
// hoisted to the top of the tile (127 live SGPRs would spill).
template <typename T>
using ConstPtr = const __attribute__((address_space(4))) T *;

template <typename T>
__device__ __forceinline__ ConstPtr<T> const_view(const void *p) {
    return (ConstPtr<T>)p;
}

constexpr int floordiv(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }
constexpr int ceildiv(int a, int b) { return (a + b - 1) / b; }

// ------------------------------------------------------------ host copies
// host memcpy into / out of pinned staging buffers, split over a persistent
// pool of host threads for large copies (one thread cannot fill the host link)
void host_copy(void *dst, const void *src, size_t bytes);
// fn(part, parts) on the caller and the pool's threads (runtime.hip)
void host_parallel(const std::function<void(int, int)> &fn);
void host_piece(size_t n, int part, int parts, size_t *lo, size_t *hi);
int host_threads();

// --------------------------------------------------------- host semantics
// coeffScaling = static_cast<int>(floor(log2(sum |c|)))  (dnsampling_filters.h:92-95,
// filters.h:92-96) with the x86 double->int conversion (INT_MIN when not finite).
int32_t cvt_d2i_x86(double d);
int32_t cvt_f2i_x86_host(float f);
unsigned coeff_scaling_f32(const float *c, int n, bool fabs_binding);
unsigned coeff_scaling_i32(const int32_t *c, int n);
unsigned coeff_scaling_i16(const int16_t *c, int n);

// ------------------------------------------------------ stream ordering
// Each handle records an event after its last enqueued work; the next call
// on any stream waits for it, so one handle's steps stay ordered.
struct Ordering {
    hipEvent_t ev = nullptr;
    bool pending = false;
    int init();
    int before(hipStream_t s);   // make s wait for the previous step
    int after(hipStream_t s);    // record this step
    int sync();                  // host waits for the last step
    void destroy();
};

// Pinned host staging + an owned stream for the *_step_host entry points.
struct HostStage {
    hipStream_t stream = nullptr;
    void *h_buf = nullptr;
    size_t h_cap = 0;
    void *d_buf = nullptr;
    size_t d_cap = 0;
    int init();
    int reserve(size_t host_bytes, size_t dev_bytes);
    void destroy();
};

int sample_bytes(int kind);  // 0 cf32, 1 ci16, 2 ci32, 3 f32, 4 i16, 5 i32

}  // namespace srcdsp
