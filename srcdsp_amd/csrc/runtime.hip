// runtime.hip -- host-side runtime pieces shared by every operator of
// libsrcdsp_hip.so: error reporting, the coefficient-scaling semantics of the
// reference constructors, stream ordering, pinned staging, and the synthetic
// sample generator used by benchmarks.
#include "common.h"

#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>

namespace srcdsp {

static thread_local std::string g_err;
void set_error(const std::string &m) { g_err = m; }
const char *get_error() { return g_err.c_str(); }

// ------------------------------------------------------------ host copies
// host_parallel(fn): fn(part, parts) on the caller and parts-1 pool threads,
// returns when all are done.  The staging copies and capture reads use it to
// cut one large transfer into `parts` cache-line-aligned pieces (one host
// thread cannot fill the host link).  parts = SRCDSP_HOST_COPY_THREADS
// (default 8), capped by the machine.  Calls from different caller threads
// are serialized (one pool).  The pool is created on first use and lives until
// exit (detached threads parked on a condvar).
namespace {
class HostPool {
  public:
    static HostPool &get() {
        static HostPool *p = new HostPool();
        return *p;
    }
    int threads() const { return T; }
    void run(const std::function<void(int, int)> &fn) {
        std::lock_guard<std::mutex> call(call_mx);
        {
            std::lock_guard<std::mutex> g(mx);
            job = &fn;
            remaining = T - 1;
            ++gen;
        }
        cv_work.notify_all();
        fn(0, T);
        std::unique_lock<std::mutex> g(mx);
        cv_done.wait(g, [&] { return remaining == 0; });
    }

  private:
    HostPool() {
        const char *e = std::getenv("SRCDSP_HOST_COPY_THREADS");
        int want = e ? std::atoi(e) : 8;
        const int hw = (int)std::thread::hardware_concurrency();
        T = std::max(1, std::min(want, hw > 0 ? hw : 1));
        for (int i = 1; i < T; ++i) std::thread([this, i] { worker(i); }).detach();
    }
    void worker(int id) {
        unsigned seen = 0;
        for (;;) {
            const std::function<void(int, int)> *fn;
            {
                std::unique_lock<std::mutex> g(mx);
                cv_work.wait(g, [&] { return gen != seen; });
                seen = gen;
                fn = job;
            }
            (*fn)(id, T);
            std::lock_guard<std::mutex> g(mx);
            if (--remaining == 0) cv_done.notify_one();
        }
    }
    int T = 1;
    std::mutex call_mx, mx;
    std::condition_variable cv_work, cv_done;
    const std::function<void(int, int)> *job = nullptr;
    unsigned gen = 0;
    int remaining = 0;
};
constexpr size_t kParMin = 2u << 20;
}  // namespace

int host_threads() { return HostPool::get().threads(); }

void host_parallel(const std::function<void(int, int)> &fn) {
    if (HostPool::get().threads() == 1) return fn(0, 1);
    HostPool::get().run(fn);
}

// [lo, hi) of piece `part` of `parts` over n bytes, 64-B aligned cuts
void host_piece(size_t n, int part, int parts, size_t *lo, size_t *hi) {
    const size_t step = (n / (size_t)parts + 63) & ~(size_t)63;
    *lo = std::min(n, step * (size_t)part);
    *hi = part == parts - 1 ? n : std::min(n, *lo + step);
}

void host_copy(void *dst, const void *src, size_t bytes) {
    if (bytes < kParMin || HostPool::get().threads() == 1) {
        std::memcpy(dst, src, bytes);
        return;
    }
    host_parallel([&](int part, int parts) {
        size_t lo, hi;
        host_piece(bytes, part, parts, &lo, &hi);
        if (hi > lo) std::memcpy((char *)dst + lo, (const char *)src + lo, hi - lo);
    });
}

int32_t cvt_d2i_x86(double d) {
    if (!(d > -2147483649.0 && d < 2147483648.0)) return INT32_MIN;
    return (int32_t)d;
}
int32_t cvt_f2i_x86_host(float f) {
    if (!(f >= -2147483648.0f && f < 2147483648.0f)) return INT32_MIN;
    return (int32_t)f;
}

// sumMagnitude loop of dnsampling_filters.h:92-94 / filters.h:92-94.
// Canonical binding: abs(float) -> ::abs(int) (the float is truncated first);
// abs(INT_MIN) stays INT_MIN.  fabs binding: |c| in float.
unsigned coeff_scaling_f32(const float *c, int n, bool fabs_binding) {
    double s = 0;
    for (int i = 0; i < n; ++i) {
        if (fabs_binding) {
            s += (double)std::fabs(c[i]);
        } else {
            int32_t v = cvt_f2i_x86_host(c[i]);
            s += (double)(v == INT32_MIN ? INT32_MIN : (v < 0 ? -v : v));
        }
    }
    return (unsigned)cvt_d2i_x86(std::floor(std::log2(s)));
}
unsigned coeff_scaling_i32(const int32_t *c, int n) {
    double s = 0;
    for (int i = 0; i < n; ++i) s += (double)(c[i] == INT32_MIN ? INT32_MIN : (c[i] < 0 ? -c[i] : c[i]));
    return (unsigned)cvt_d2i_x86(std::floor(std::log2(s)));
}
unsigned coeff_scaling_i16(const int16_t *c, int n) {
    double s = 0;
    for (int i = 0; i < n; ++i) s += (double)std::abs((int)c[i]);
    return (unsigned)cvt_d2i_x86(std::floor(std::log2(s)));
}

int Ordering::init() {
    SRCDSP_HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    return SRCDSP_OK;
}
int Ordering::before(hipStream_t s) {
    if (pending) SRCDSP_HIP_TRY(hipStreamWaitEvent(s, ev, 0));
    return SRCDSP_OK;
}
int Ordering::after(hipStream_t s) {
    SRCDSP_HIP_TRY(hipEventRecord(ev, s));
    pending = true;
    return SRCDSP_OK;
}
int Ordering::sync() {
    if (pending) SRCDSP_HIP_TRY(hipEventSynchronize(ev));
    return SRCDSP_OK;
}
void Ordering::destroy() {
    if (ev) (void)hipEventDestroy(ev);
    ev = nullptr;
}

int HostStage::init() {
    SRCDSP_HIP_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    return SRCDSP_OK;
}
int HostStage::reserve(size_t hb, size_t db) {
    if (hb > h_cap) {
        if (h_buf) (void)hipHostFree(h_buf);
        h_buf = nullptr;
        SRCDSP_HIP_TRY(hipHostMalloc(&h_buf, hb, hipHostMallocDefault));
        h_cap = hb;
    }
    if (db > d_cap) {
        if (d_buf) (void)hipFree(d_buf);
        d_buf = nullptr;
        SRCDSP_HIP_TRY(hipMalloc(&d_buf, db));
        d_cap = db;
    }
    return SRCDSP_OK;
}
void HostStage::destroy() {
    if (h_buf) (void)hipHostFree(h_buf);
    if (d_buf) (void)hipFree(d_buf);
    if (stream) (void)hipStreamDestroy(stream);
    h_buf = d_buf = nullptr;
    stream = nullptr;
    h_cap = d_cap = 0;
}

int sample_bytes(int kind) {
    switch (kind) {
    case 0: return 8;
    case 1: return 4;
    case 2: return 8;
    case 3: return 4;
    case 4: return 2;
    case 5: return 4;
    default: return 0;
    }
}

// --------------------------------------------------------- synthetic data
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <typename T>
__global__ void fill_synthetic_kernel(T *out, size_t ncomp, uint64_t key, uint64_t off2, int lo,
                                      uint64_t span) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t stride = (size_t)gridDim.x * blockDim.x;
    for (; i < ncomp; i += stride) {
        uint64_t u = splitmix64(key + off2 + i);
        out[i] = (T)(lo + (int32_t)((u >> 32) % span));
    }
}

}  // namespace srcdsp

using namespace srcdsp;

extern "C" {

SRCDSP_API const char *srcdsp_last_error(void) { return get_error(); }
SRCDSP_API const char *srcdsp_version(void) { return "0.1.0 gfx950"; }

SRCDSP_API int srcdsp_fill_synthetic(void *d_out, int kind, size_t n, uint64_t seed, uint64_t channel,
                                     uint64_t offset, int lo, int hi, void *stream) {
    SRCDSP_ARG_CHECK(d_out != nullptr || n == 0, "fill_synthetic: null output");
    SRCDSP_ARG_CHECK(hi >= lo, "fill_synthetic: hi < lo");
    SRCDSP_ARG_CHECK(kind == 0 || kind == 1, "fill_synthetic: kind must be 0 (cf32) or 1 (ci16)");
    if (n == 0) return SRCDSP_OK;
    uint64_t key = seed ^ (channel << 40);
    size_t ncomp = 2 * n;
    int blocks = (int)std::min<size_t>((ncomp + 255) / 256, 256 * 64);
    hipStream_t s = (hipStream_t)stream;
    uint64_t span = (uint64_t)((int64_t)hi - (int64_t)lo + 1);
    if (kind == 0)
        hipLaunchKernelGGL(fill_synthetic_kernel<float>, dim3(blocks), dim3(256), 0, s, (float *)d_out,
                           ncomp, key, 2 * offset, lo, span);
    else
        hipLaunchKernelGGL(fill_synthetic_kernel<int16_t>, dim3(blocks), dim3(256), 0, s,
                           (int16_t *)d_out, ncomp, key, 2 * offset, lo, span);
    SRCDSP_HIP_TRY(hipGetLastError());
    return SRCDSP_OK;
}

}  // extern "C"
