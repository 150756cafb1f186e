// fifo.hip -- dsptl::FifoWithTimeTrack<T, N> (buffers.h:58-459) as a
// device-staging ring, and the dsptl_files.h binary I/Q capture format.
//
// FIFO.  The N-element ring lives in HBM, so step() operators consume what a
// producer thread wrote without a host round trip.  Host writes are staged
// through two pinned buffers: write() copies the caller's vector into one
// while the other's H2D copy is still in flight, and returns without waiting
// for its own copy (double-buffered, PCIe overlapped with the consumer's
// compute).  Ordering on the device: every write records an event on its copy
// stream and every read makes its stream wait for it; every read records an
// event that the next write's copies wait for.  The bookkeeping (writePtr,
// timeStart, timeEnd, rolloverFlag, the time reference) is the reference's,
// line for line in meaning: uint64/size_t modular arithmetic, timeStart = 1
// while the ring is not full, count() = timeEnd - timeStart + 1, reset() of
// the indices only, the start adjustment with its stderr warning, and the
// assert()s returned as SRCDSP_ERR_SIZE.
//
// I/Q files.  saveBinarySamples (dsptl_files.h:101-109) writes the samples'
// bytes, interleaved I,Q.  readBinarySamples (:250-262) is fixed as SURVEY 8f
// asks: the output is cleared first (the reference calls out.empty()) and
// only whole samples are returned (the reference's while(is) loop appends one
// indeterminate sample at EOF).  Device loads overlap a parallel pread of one
// pinned chunk with the H2D copy of the other.
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <iostream>
#include <mutex>

#include "common.h"

namespace srcdsp {

constexpr size_t kStageBytes = 8u << 20;  // per pinned staging buffer

struct srcdsp_fifo_state {
    size_t es = 0, N = 0;
    char *d_ring = nullptr;
    // reference state (buffers.h:84-115)
    size_t write_ptr = 0;
    uint64_t time_start = 0, time_end = 0;
    bool rollover = false;
    double fs = 0;
    uint64_t ref_tp = 0;
    unsigned ref_sec = 0;
    double ref_frac = 0;
    std::mutex mx;
    // device staging
    hipStream_t cs = nullptr;               // copy stream of host writes
    void *pin[2] = {nullptr, nullptr};      // pinned staging buffers
    hipEvent_t ev_pin[2] = {nullptr, nullptr};
    bool pin_busy[2] = {false, false};
    int k = 0;
    hipEvent_t ev_written = nullptr, ev_read = nullptr;
    std::atomic<bool> any_write{false}, any_read{false};  // writer and reader may be different threads
    void *h_rd = nullptr;                   // pinned buffer of read_host
    size_t h_rd_cap = 0;
};

// copy n elements into the ring at position p (wrapping), on stream s
static int ring_put(srcdsp_fifo_state &f, size_t p, const char *src, size_t n, hipMemcpyKind kind, hipStream_t s) {
    const size_t up = f.N - p;
    if (n <= up) {
        SRCDSP_HIP_TRY(hipMemcpyAsync(f.d_ring + p * f.es, src, n * f.es, kind, s));
    } else {
        SRCDSP_HIP_TRY(hipMemcpyAsync(f.d_ring + p * f.es, src, up * f.es, kind, s));
        SRCDSP_HIP_TRY(hipMemcpyAsync(f.d_ring, src + up * f.es, (n - up) * f.es, kind, s));
    }
    return SRCDSP_OK;
}

// buffers.h:162-221 (the critical section of write())
static void publish(srcdsp_fifo_state &f, size_t n, unsigned seconds, double frac) {
    std::lock_guard<std::mutex> g(f.mx);
    f.write_ptr = (f.write_ptr + n) % f.N;
    const uint64_t diff = UINT64_MAX - f.time_end;
    f.ref_tp = f.time_end + 1;
    f.ref_sec = seconds;
    f.ref_frac = frac;
    if (diff >= n) {
        f.time_end += n;
    } else {
        f.time_end = n - diff;
        f.rollover = true;
    }
    if (!f.rollover) {
        if ((f.time_end - f.time_start + 1) > f.N)
            f.time_start = f.time_end - f.N + 1;
        else
            f.time_start = 1;
    } else {
        const uint64_t d2 = UINT64_MAX - f.time_start;
        if (d2 >= n)
            f.time_start += n;
        else
            f.time_start = n - d2;
        f.rollover = false;
    }
}

// buffers.h:290-315: range check and ring positions; 1 = the reference's `true`
static int locate(srcdsp_fifo_state &f, size_t n, uint64_t *start, size_t *sp, size_t *ep) {
    std::lock_guard<std::mutex> g(f.mx);
    if (*start < f.time_start) {
        std::cerr << "******* REQUESTED START BEFORE FIRST AVAILABLE SAMPLE *****";
        *start = f.time_start;
    }
    if ((*start + n - 1) > f.time_end) return 1;
    const uint64_t end = *start + n - 1;
    *sp = (size_t)((f.write_ptr + f.N - (f.time_end - *start) - 1) % f.N);
    *ep = (size_t)((f.write_ptr + f.N - (f.time_end - end) - 1) % f.N);
    return 0;
}

// copy ring [sp..ep] (closed, wrapping) to dst on stream s
static int ring_get(srcdsp_fifo_state &f, size_t sp, size_t ep, char *dst, hipMemcpyKind kind, hipStream_t s) {
    if (ep >= sp) {
        SRCDSP_HIP_TRY(hipMemcpyAsync(dst, f.d_ring + sp * f.es, (ep + 1 - sp) * f.es, kind, s));
    } else {
        SRCDSP_HIP_TRY(hipMemcpyAsync(dst, f.d_ring + sp * f.es, (f.N - sp) * f.es, kind, s));
        SRCDSP_HIP_TRY(hipMemcpyAsync(dst + (f.N - sp) * f.es, f.d_ring, (ep + 1) * f.es, kind, s));
    }
    return SRCDSP_OK;
}

}  // namespace srcdsp

using namespace srcdsp;
struct srcdsp_fifo { srcdsp_fifo_state f; };

extern "C" {

SRCDSP_API int srcdsp_fifo_destroy(srcdsp_fifo_t h);

SRCDSP_API int srcdsp_fifo_create(srcdsp_fifo_t *out, size_t elem_bytes, size_t N, double sampling_frequency) {
    SRCDSP_ARG_CHECK(out != nullptr, "fifo_create: null out");
    *out = nullptr;
    SRCDSP_ARG_CHECK(elem_bytes >= 1 && N >= 2, "fifo_create: need elem_bytes >= 1 and N >= 2");
    auto *h = new srcdsp_fifo();
    srcdsp_fifo_state &f = h->f;
    f.es = elem_bytes;
    f.N = N;
    f.fs = sampling_frequency;
    const size_t stage = std::min(kStageBytes, N * elem_bytes);
    bool ok = hipMalloc(&f.d_ring, N * elem_bytes) == hipSuccess &&
              hipMemset(f.d_ring, 0, N * elem_bytes) == hipSuccess &&  // storage(N): value-initialised
              hipStreamCreateWithFlags(&f.cs, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&f.ev_written, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&f.ev_read, hipEventDisableTiming) == hipSuccess;
    for (int b = 0; ok && b < 2; ++b)
        ok = hipHostMalloc(&f.pin[b], stage, hipHostMallocDefault) == hipSuccess &&
             hipEventCreateWithFlags(&f.ev_pin[b], hipEventDisableTiming) == hipSuccess;
    if (!ok || hipDeviceSynchronize() != hipSuccess) {
        set_error("fifo_create: device allocation failed");
        srcdsp_fifo_destroy(h);
        return SRCDSP_ERR_HIP;
    }
    *out = h;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_fifo_destroy(srcdsp_fifo_t h) {
    if (!h) return SRCDSP_OK;
    srcdsp_fifo_state &f = h->f;
    if (f.cs) (void)hipStreamSynchronize(f.cs);
    (void)hipDeviceSynchronize();
    if (f.d_ring) (void)hipFree(f.d_ring);
    for (int b = 0; b < 2; ++b) {
        if (f.pin[b]) (void)hipHostFree(f.pin[b]);
        if (f.ev_pin[b]) (void)hipEventDestroy(f.ev_pin[b]);
    }
    if (f.h_rd) (void)hipHostFree(f.h_rd);
    if (f.ev_written) (void)hipEventDestroy(f.ev_written);
    if (f.ev_read) (void)hipEventDestroy(f.ev_read);
    if (f.cs) (void)hipStreamDestroy(f.cs);
    delete h;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_fifo_write(srcdsp_fifo_t h, const void *in, size_t n, unsigned seconds, double frac_seconds) {
    SRCDSP_ARG_CHECK(h != nullptr && (in != nullptr || n == 0), "fifo_write: null argument");
    srcdsp_fifo_state &f = h->f;
    if (n >= f.N) {
        set_error("fifo_write: the input must be shorter than the FIFO (assert(inSize < N), buffers.h:145)");
        return SRCDSP_ERR_SIZE;
    }
    if (f.any_read) SRCDSP_HIP_TRY(hipStreamWaitEvent(f.cs, f.ev_read, 0));
    const size_t stage = std::min(kStageBytes, f.N * f.es);
    size_t p;
    {
        std::lock_guard<std::mutex> g(f.mx);
        p = f.write_ptr;
    }
    const char *src = (const char *)in;
    for (size_t done = 0; done < n;) {
        const size_t m = std::min(n - done, stage / f.es);
        const int k = f.k;
        if (f.pin_busy[k]) SRCDSP_HIP_TRY(hipEventSynchronize(f.ev_pin[k]));  // its previous copy has landed
        host_copy(f.pin[k], src + done * f.es, m * f.es);
        int rc = ring_put(f, (p + done) % f.N, (const char *)f.pin[k], m, hipMemcpyHostToDevice, f.cs);
        if (rc) return rc;
        SRCDSP_HIP_TRY(hipEventRecord(f.ev_pin[k], f.cs));
        f.pin_busy[k] = true;
        f.k ^= 1;
        done += m;
    }
    SRCDSP_HIP_TRY(hipEventRecord(f.ev_written, f.cs));
    f.any_write = true;
    publish(f, n, seconds, frac_seconds);
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_fifo_write_device(srcdsp_fifo_t h, const void *d_in, size_t n, unsigned seconds,
                                        double frac_seconds, void *stream) {
    SRCDSP_ARG_CHECK(h != nullptr && (d_in != nullptr || n == 0), "fifo_write_device: null argument");
    srcdsp_fifo_state &f = h->f;
    if (n >= f.N) {
        set_error("fifo_write_device: the input must be shorter than the FIFO (buffers.h:145)");
        return SRCDSP_ERR_SIZE;
    }
    hipStream_t s = (hipStream_t)stream;
    if (f.any_read) SRCDSP_HIP_TRY(hipStreamWaitEvent(s, f.ev_read, 0));
    if (f.any_write) SRCDSP_HIP_TRY(hipStreamWaitEvent(s, f.ev_written, 0));  // writes stay in order
    size_t p;
    {
        std::lock_guard<std::mutex> g(f.mx);
        p = f.write_ptr;
    }
    int rc = ring_put(f, p, (const char *)d_in, n, hipMemcpyDeviceToDevice, s);
    if (rc) return rc;
    SRCDSP_HIP_TRY(hipEventRecord(f.ev_written, s));
    f.any_write = true;
    publish(f, n, seconds, frac_seconds);
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_fifo_read(srcdsp_fifo_t h, void *d_out, size_t n, uint64_t *start, int *error,
                                void *stream) {
    SRCDSP_ARG_CHECK(h != nullptr && start != nullptr && error != nullptr, "fifo_read: null argument");
    if (n == 0) {
        set_error("fifo_read: empty output (assert(out.size() != 0), buffers.h:286)");
        return SRCDSP_ERR_SIZE;
    }
    SRCDSP_ARG_CHECK(d_out != nullptr, "fifo_read: null output");
    srcdsp_fifo_state &f = h->f;
    size_t sp = 0, ep = 0;
    *error = locate(f, n, start, &sp, &ep);
    if (*error) return SRCDSP_OK;
    hipStream_t s = (hipStream_t)stream;
    if (f.any_write) SRCDSP_HIP_TRY(hipStreamWaitEvent(s, f.ev_written, 0));
    int rc = ring_get(f, sp, ep, (char *)d_out, hipMemcpyDeviceToDevice, s);
    if (rc) return rc;
    SRCDSP_HIP_TRY(hipEventRecord(f.ev_read, s));
    f.any_read = true;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_fifo_read_host(srcdsp_fifo_t h, void *out, size_t n, uint64_t *start, int *error) {
    SRCDSP_ARG_CHECK(h != nullptr && start != nullptr && error != nullptr, "fifo_read_host: null argument");
    if (n == 0) {
        set_error("fifo_read_host: empty output (assert(out.size() != 0), buffers.h:286)");
        return SRCDSP_ERR_SIZE;
    }
    SRCDSP_ARG_CHECK(out != nullptr, "fifo_read_host: null output");
    srcdsp_fifo_state &f = h->f;
    size_t sp = 0, ep = 0;
    *error = locate(f, n, start, &sp, &ep);
    if (*error) return SRCDSP_OK;
    if (n * f.es > f.h_rd_cap) {
        if (f.h_rd) (void)hipHostFree(f.h_rd);
        f.h_rd = nullptr;
        f.h_rd_cap = 0;
        SRCDSP_HIP_TRY(hipHostMalloc(&f.h_rd, n * f.es, hipHostMallocDefault));
        f.h_rd_cap = n * f.es;
    }
    if (f.any_write) SRCDSP_HIP_TRY(hipStreamWaitEvent(f.cs, f.ev_written, 0));
    int rc = ring_get(f, sp, ep, (char *)f.h_rd, hipMemcpyDeviceToHost, f.cs);
    if (rc) return rc;
    SRCDSP_HIP_TRY(hipStreamSynchronize(f.cs));
    host_copy(out, f.h_rd, n * f.es);
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_fifo_count(srcdsp_fifo_t h, size_t *count) {
    SRCDSP_ARG_CHECK(h != nullptr && count != nullptr, "fifo_count: null argument");
    srcdsp_fifo_state &f = h->f;
    std::lock_guard<std::mutex> g(f.mx);
    *count = !f.rollover ? (size_t)((f.time_end - f.time_start) + 1)  // buffers.h:377-392
                         : (size_t)((UINT64_MAX - f.time_start) + f.time_end + 1);
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_fifo_reset(srcdsp_fifo_t h) {
    SRCDSP_ARG_CHECK(h != nullptr, "fifo_reset: null handle");
    srcdsp_fifo_state &f = h->f;
    std::lock_guard<std::mutex> g(f.mx);  // buffers.h:245-258: indices only
    f.write_ptr = 0;
    f.time_start = 0;
    f.time_end = 0;
    f.rollover = false;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_fifo_get_state(srcdsp_fifo_t h, size_t *write_ptr, uint64_t *time_start, uint64_t *time_end,
                                     int *rollover) {
    SRCDSP_ARG_CHECK(h != nullptr, "fifo_get_state: null handle");
    srcdsp_fifo_state &f = h->f;
    std::lock_guard<std::mutex> g(f.mx);
    if (write_ptr) *write_ptr = f.write_ptr;
    if (time_start) *time_start = f.time_start;
    if (time_end) *time_end = f.time_end;
    if (rollover) *rollover = f.rollover ? 1 : 0;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_fifo_get_absolute_time(srcdsp_fifo_t h, uint64_t time_point, double frac_time_point,
                                             unsigned *seconds, double *frac_seconds) {
    SRCDSP_ARG_CHECK(h != nullptr && seconds != nullptr && frac_seconds != nullptr,
                     "fifo_get_absolute_time: null argument");
    srcdsp_fifo_state &f = h->f;
    std::lock_guard<std::mutex> g(f.mx);  // buffers.h:413-459
    const int64_t sample_diff = (int64_t)(time_point - f.ref_tp);
    const double time_diff = sample_diff / f.fs;
    const int32_t tdi = cvt_d2i_x86(std::floor(time_diff));
    const double tdf = time_diff - std::floor(time_diff);
    uint32_t sec = f.ref_sec + tdi;
    double fs = f.ref_frac + tdf + (frac_time_point / f.fs);
    const int32_t tmp = cvt_d2i_x86(fs);
    fs -= tmp;
    sec += tmp;
    *seconds = sec;
    *frac_seconds = fs;
    return SRCDSP_OK;
}

// -------------------------------------------------------------- I/Q files
static FILE *open_or_err(const char *path, const char *mode) {
    FILE *fp = path ? std::fopen(path, mode) : nullptr;
    if (!fp) set_error(std::string("cannot open ") + (path ? path : "(null)"));
    return fp;
}

SRCDSP_API int srcdsp_iq_save_host(const char *path, const void *samples, size_t n, size_t component_bytes,
                                   int append) {
    SRCDSP_ARG_CHECK(component_bytes >= 1 && (samples != nullptr || n == 0), "iq_save_host: bad argument");
    FILE *fp = open_or_err(path, append ? "ab" : "wb");
    if (!fp) return SRCDSP_ERR_ARG;
    const size_t bytes = n * 2 * component_bytes;
    const bool ok = bytes == 0 || std::fwrite(samples, 1, bytes, fp) == bytes;
    std::fclose(fp);
    if (!ok) {
        set_error("iq_save_host: short write");
        return SRCDSP_ERR_ARG;
    }
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_iq_count(const char *path, size_t component_bytes, size_t *n) {
    SRCDSP_ARG_CHECK(component_bytes >= 1 && n != nullptr, "iq_count: bad argument");
    FILE *fp = open_or_err(path, "rb");
    if (!fp) return SRCDSP_ERR_ARG;
    std::fseek(fp, 0, SEEK_END);
    const long len = std::ftell(fp);
    std::fclose(fp);
    *n = len > 0 ? (size_t)len / (2 * component_bytes) : 0;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_iq_load_host(const char *path, size_t component_bytes, void *out, size_t cap, size_t *n) {
    int rc = srcdsp_iq_count(path, component_bytes, n);
    if (rc) return rc;
    SRCDSP_ARG_CHECK(out != nullptr || *n == 0, "iq_load_host: null output");
    if (*n > cap) {
        set_error("iq_load_host: output too small for the file's samples");
        return SRCDSP_ERR_SIZE;
    }
    FILE *fp = open_or_err(path, "rb");
    if (!fp) return SRCDSP_ERR_ARG;
    const size_t bytes = *n * 2 * component_bytes;
    const bool ok = bytes == 0 || std::fread(out, 1, bytes, fp) == bytes;
    std::fclose(fp);
    if (!ok) {
        set_error("iq_load_host: short read");
        return SRCDSP_ERR_ARG;
    }
    return SRCDSP_OK;
}

// Pinned staging of the capture loads, kept across calls (allocating 2 pinned
// chunks per call cost more than the copy of a small capture); one load at a
// time uses it.
namespace {
struct IqStage {
    std::mutex mx;
    void *pin[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    size_t cap = 0;
    int reserve(size_t bytes) {
        if (cap >= bytes) return SRCDSP_OK;
        for (int b = 0; b < 2; ++b) {
            if (pin[b]) (void)hipHostFree(pin[b]);
            pin[b] = nullptr;
        }
        cap = 0;
        for (int b = 0; b < 2; ++b) {
            SRCDSP_HIP_TRY(hipHostMalloc(&pin[b], bytes, hipHostMallocDefault));
            if (!ev[b]) SRCDSP_HIP_TRY(hipEventCreateWithFlags(&ev[b], hipEventDisableTiming));
        }
        cap = bytes;
        return SRCDSP_OK;
    }
};
IqStage &iq_stage() {
    static IqStage *s = new IqStage();  // lives until exit
    return *s;
}
constexpr size_t kIqChunk = 32u << 20;
}  // namespace

// file -> device: the pread of chunk i+1 (split over the host pool's threads)
// overlaps the H2D copy of chunk i
SRCDSP_API int srcdsp_iq_load(const char *path, size_t component_bytes, void *d_out, size_t cap, size_t *n,
                              void *stream) {
    int rc = srcdsp_iq_count(path, component_bytes, n);
    if (rc) return rc;
    SRCDSP_ARG_CHECK(d_out != nullptr || *n == 0, "iq_load: null output");
    if (*n > cap) {
        set_error("iq_load: output too small for the file's samples");
        return SRCDSP_ERR_SIZE;
    }
    const size_t bytes = *n * 2 * component_bytes;
    if (bytes == 0) return SRCDSP_OK;
    const int fd = ::open(path, O_RDONLY);
    if (fd < 0) {
        set_error(std::string("cannot open ") + path);
        return SRCDSP_ERR_ARG;
    }
    hipStream_t s = (hipStream_t)stream;
    IqStage &st = iq_stage();
    std::lock_guard<std::mutex> lock(st.mx);
    const size_t chunk = std::min(kIqChunk, bytes);
    int err = st.reserve(chunk);
    bool used[2] = {false, false};
    for (size_t done = 0, k = 0; !err && done < bytes; done += chunk, k ^= 1) {
        const size_t m = std::min(chunk, bytes - done);
        if (used[k] && hipEventSynchronize(st.ev[k]) != hipSuccess) err = SRCDSP_ERR_HIP;
        if (err) break;
        std::atomic<bool> short_read{false};
        char *dst = (char *)st.pin[k];
        host_parallel([&](int part, int parts) {
            size_t lo, hi;
            host_piece(m, part, parts, &lo, &hi);
            while (lo < hi) {
                const ssize_t r = ::pread(fd, dst + lo, hi - lo, (off_t)(done + lo));
                if (r <= 0) {
                    short_read = true;
                    return;
                }
                lo += (size_t)r;
            }
        });
        if (short_read) {
            set_error("iq_load: short read");
            err = SRCDSP_ERR_ARG;
        }
        if (!err && (hipMemcpyAsync((char *)d_out + done, st.pin[k], m, hipMemcpyHostToDevice, s) != hipSuccess ||
                     hipEventRecord(st.ev[k], s) != hipSuccess))
            err = SRCDSP_ERR_HIP;
        used[k] = true;
    }
    // the staging is reused by the next load: its copies must have landed
    for (int b = 0; b < 2; ++b)
        if (used[b] && hipEventSynchronize(st.ev[b]) != hipSuccess && !err) err = SRCDSP_ERR_HIP;
    ::close(fd);
    if (err == SRCDSP_ERR_HIP) set_error("iq_load: HIP staging failed");
    return err;
}

// device -> file: D2H of chunk i+1 overlaps the fwrite of chunk i
SRCDSP_API int srcdsp_iq_save(const char *path, const void *d_samples, size_t n, size_t component_bytes, int append,
                              void *stream) {
    SRCDSP_ARG_CHECK(component_bytes >= 1 && (d_samples != nullptr || n == 0), "iq_save: bad argument");
    FILE *fp = open_or_err(path, append ? "ab" : "wb");
    if (!fp) return SRCDSP_ERR_ARG;
    const size_t bytes = n * 2 * component_bytes;
    hipStream_t s = (hipStream_t)stream;
    void *pin[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    const size_t chunk = std::max<size_t>(1, std::min(kStageBytes, bytes));
    int err = SRCDSP_OK;
    for (int b = 0; b < 2 && !err && bytes; ++b)
        if (hipHostMalloc(&pin[b], chunk, hipHostMallocDefault) != hipSuccess ||
            hipEventCreateWithFlags(&ev[b], hipEventDisableTiming) != hipSuccess)
            err = SRCDSP_ERR_HIP;
    // issue chunk 0, then: issue chunk i+1, wait chunk i, write chunk i
    auto issue = [&](size_t off, int k) {
        const size_t m = std::min(chunk, bytes - off);
        return hipMemcpyAsync(pin[k], (const char *)d_samples + off, m, hipMemcpyDeviceToHost, s) == hipSuccess &&
               hipEventRecord(ev[k], s) == hipSuccess;
    };
    if (!err && bytes && !issue(0, 0)) err = SRCDSP_ERR_HIP;
    for (size_t off = 0, k = 0; !err && off < bytes; off += chunk, k ^= 1) {
        const size_t m = std::min(chunk, bytes - off);
        if (off + chunk < bytes && !issue(off + chunk, (int)(k ^ 1))) err = SRCDSP_ERR_HIP;
        if (!err && hipEventSynchronize(ev[k]) != hipSuccess) err = SRCDSP_ERR_HIP;
        if (!err && std::fwrite(pin[k], 1, m, fp) != m) {
            set_error("iq_save: short write");
            err = SRCDSP_ERR_ARG;
        }
    }
    if (hipStreamSynchronize(s) != hipSuccess && !err) err = SRCDSP_ERR_HIP;
    std::fclose(fp);
    for (int b = 0; b < 2; ++b) {
        if (pin[b]) (void)hipHostFree(pin[b]);
        if (ev[b]) (void)hipEventDestroy(ev[b]);
    }
    if (err == SRCDSP_ERR_HIP) set_error("iq_save: HIP staging failed");
    return err;
}

}  // extern "C"
