// multi.hip -- one host process driving several MI355X GPUs (SURVEY.md §8e,
// BASELINE configs[2]): RCCL communicators made together by ncclCommInitAll,
// independent decimator channels block-partitioned over the devices, and the
// result gather to one device over xGMI.
//
// The data path has no collective: each device steps its own channels with
// one batched launch (srcdsp_decim_step_batched) on its own stream.  The only
// exchange is the optional gather of the decimated outputs, which the caller
// issues (and times) separately.
//
// RCCL is loaded lazily (dlopen at the first srcdsp_comm_create): the
// single-GPU entries of libsrcdsp_hip.so neither link nor load librccl, and
// without it srcdsp_comm_create returns SRCDSP_ERR_UNSUPPORTED.  The header
// gives the types only.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "ops.h"

using namespace srcdsp;

struct srcdsp_comm {
    std::vector<int> devs;
    std::vector<ncclComm_t> comms;
    std::vector<hipStream_t> streams;
    // per rank: the events of srcdsp_comm_wait_stream / srcdsp_comm_signal_stream
    // (record + wait pairs, serialised by order_mu)
    std::vector<hipEvent_t> wait_ev, signal_ev;
    std::mutex order_mu;
    // the caller's reference plus one per sharded handle built on it: the
    // communicator is released when the last of them goes, whatever the order
    // of srcdsp_comm_destroy and srcdsp_decim_sharded_destroy (atomic: handles
    // built on one comm may be destroyed from different threads)
    std::atomic<int> refs{1};
};

struct srcdsp_decim_sharded {
    srcdsp_comm *comm = nullptr;
    int channels = 0;
    std::vector<int> first, count;          // per rank
    std::vector<srcdsp_decim_t> handles;    // per global channel, on its rank's device
};

namespace {

// the RCCL entry points this file uses, resolved from librccl at run time
struct Rccl {
    bool ok = false;
    std::string why;
    ncclResult_t (*CommInitAll)(ncclComm_t *, int, const int *) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    const char *(*GetErrorString)(ncclResult_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*Gather)(const void *, void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
};

const Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *lib = nullptr;
        for (const char *name : {"librccl.so.1", "librccl.so"})
            if ((lib = dlopen(name, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
        if (!lib) {
            r.why = std::string("librccl not loadable: ") + dlerror();
            return;
        }
        auto sym = [&](auto &fn, const char *name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(lib, name));
            return fn != nullptr;
        };
        r.ok = sym(r.CommInitAll, "ncclCommInitAll") && sym(r.CommDestroy, "ncclCommDestroy") &&
               sym(r.GetErrorString, "ncclGetErrorString") && sym(r.GroupStart, "ncclGroupStart") &&
               sym(r.GroupEnd, "ncclGroupEnd") && sym(r.Gather, "ncclGather") && sym(r.Send, "ncclSend") &&
               sym(r.Recv, "ncclRecv");
        if (!r.ok) r.why = "librccl lacks ncclCommInitAll / ncclGather / ncclSend / ncclRecv";
    });
    return r;
}

#define SRCDSP_NCCL_TRY(expr)                                                              \
    do {                                                                                   \
        ncclResult_t _r = (expr);                                                          \
        if (_r != ncclSuccess) {                                                           \
            ::srcdsp::set_error(std::string(#expr) + ": " + rccl().GetErrorString(_r));    \
            return SRCDSP_ERR_HIP;                                                         \
        }                                                                                  \
    } while (0)

void comm_release(srcdsp_comm *c) {
    if (c->refs.fetch_sub(1) > 1) return;
    int saved = -1;
    (void)hipGetDevice(&saved);
    for (size_t r = 0; r < c->devs.size(); ++r) {
        if (r < c->streams.size() && c->streams[r]) {
            (void)hipSetDevice(c->devs[r]);
            (void)hipStreamSynchronize(c->streams[r]);
            (void)hipStreamDestroy(c->streams[r]);
        }
        if (r < c->wait_ev.size() && c->wait_ev[r]) (void)hipEventDestroy(c->wait_ev[r]);
        if (r < c->signal_ev.size() && c->signal_ev[r]) (void)hipEventDestroy(c->signal_ev[r]);
        if (r < c->comms.size() && c->comms[r]) (void)rccl().CommDestroy(c->comms[r]);
    }
    if (saved >= 0) (void)hipSetDevice(saved);
    delete c;
}

// A communicator whose ranks share a device is refused, as RCCL refuses it.
// Only a TEST build of this file (-DSRCDSP_TEST_SHARED_DEVICES, built by
// srcdsp_amd.build.build_test_probes into tests/_build/, never shipped)
// lets tests/test_sharded_stub.py rehearse ndev > 1 on one GPU through the
// test-only communicator library tests/rccl_stub, opting in with the
// environment variable SRCDSP_COMM_SHARED_DEVICES=1.
bool shared_devices_allowed() {
#ifdef SRCDSP_TEST_SHARED_DEVICES
    const char *v = std::getenv("SRCDSP_COMM_SHARED_DEVICES");
    return v && std::strcmp(v, "1") == 0;
#else
    return false;
#endif
}

// restores the caller's current device on scope exit
struct DeviceGuard {
    int saved = -1;
    DeviceGuard() { (void)hipGetDevice(&saved); }
    ~DeviceGuard() {
        if (saved >= 0) (void)hipSetDevice(saved);
    }
};

}  // namespace

SRCDSP_API int srcdsp_comm_create(srcdsp_comm_t *out, int ndev, const int *devs) {
    SRCDSP_ARG_CHECK(out != nullptr, "comm_create: null out");
    *out = nullptr;
    SRCDSP_ARG_CHECK(ndev >= 1, "comm_create: ndev must be >= 1");
    int have = 0;
    SRCDSP_HIP_TRY(hipGetDeviceCount(&have));
    std::vector<int> d(ndev);
    for (int r = 0; r < ndev; ++r) {
        d[r] = devs ? devs[r] : r;
        SRCDSP_ARG_CHECK(d[r] >= 0 && d[r] < have, "comm_create: device id out of range");
        // RCCL refuses a communicator whose ranks share a device (see
        // shared_devices_allowed for the test build that rehearses it)
        if (!shared_devices_allowed())
            for (int q = 0; q < r; ++q) SRCDSP_ARG_CHECK(d[q] != d[r], "comm_create: a device listed twice");
    }
    const Rccl &R = rccl();
    if (!R.ok) {
        set_error("comm_create: " + R.why);
        return SRCDSP_ERR_UNSUPPORTED;
    }
    DeviceGuard g;
    auto *c = new srcdsp_comm();
    c->devs = d;
    c->comms.assign(ndev, nullptr);
    ncclResult_t nr = R.CommInitAll(c->comms.data(), ndev, c->devs.data());
    if (nr != ncclSuccess) {
        set_error(std::string("ncclCommInitAll: ") + R.GetErrorString(nr));
        delete c;
        return SRCDSP_ERR_HIP;
    }
    c->streams.assign(ndev, nullptr);
    c->wait_ev.assign(ndev, nullptr);
    c->signal_ev.assign(ndev, nullptr);
    for (int r = 0; r < ndev; ++r) {
        hipError_t e = hipSetDevice(c->devs[r]);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->streams[r], hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->wait_ev[r], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->signal_ev[r], hipEventDisableTiming);
        if (e != hipSuccess) {
            set_error(std::string("comm_create: stream on device: ") + hipGetErrorString(e));
            srcdsp_comm_destroy(c);
            return SRCDSP_ERR_HIP;
        }
    }
    *out = c;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_comm_destroy(srcdsp_comm_t c) {
    if (!c) return SRCDSP_OK;
    comm_release(c);  // freed now, or with the last sharded handle built on it
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_comm_info(srcdsp_comm_t c, int *ndev, int *devs) {
    SRCDSP_ARG_CHECK(c != nullptr, "comm_info: null comm");
    if (ndev) *ndev = (int)c->devs.size();
    if (devs) std::copy(c->devs.begin(), c->devs.end(), devs);
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_comm_stream(srcdsp_comm_t c, int rank, void **stream) {
    SRCDSP_ARG_CHECK(c != nullptr && stream != nullptr, "comm_stream: null argument");
    SRCDSP_ARG_CHECK(rank >= 0 && rank < (int)c->devs.size(), "comm_stream: rank out of range");
    *stream = (void *)c->streams[rank];
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_comm_synchronize(srcdsp_comm_t c) {
    SRCDSP_ARG_CHECK(c != nullptr, "comm_synchronize: null comm");
    DeviceGuard g;
    for (size_t r = 0; r < c->devs.size(); ++r) {
        SRCDSP_HIP_TRY(hipSetDevice(c->devs[r]));
        SRCDSP_HIP_TRY(hipStreamSynchronize(c->streams[r]));
    }
    return SRCDSP_OK;
}

// Ordering with caller streams.  The comm streams are non-blocking: they do
// not wait for the null stream or any stream of the caller, so caller work on
// d_in / d_out / d_root is ordered only through these two calls (or
// srcdsp_comm_synchronize).  Each is one event record on one stream and one
// wait on the other, on rank's device; nothing blocks the host.
SRCDSP_API int srcdsp_comm_wait_stream(srcdsp_comm_t c, int rank, void *stream) {
    SRCDSP_ARG_CHECK(c != nullptr, "comm_wait_stream: null comm");
    SRCDSP_ARG_CHECK(rank >= 0 && rank < (int)c->devs.size(), "comm_wait_stream: rank out of range");
    DeviceGuard g;
    std::lock_guard<std::mutex> lk(c->order_mu);
    SRCDSP_HIP_TRY(hipSetDevice(c->devs[rank]));
    SRCDSP_HIP_TRY(hipEventRecord(c->wait_ev[rank], (hipStream_t)stream));
    SRCDSP_HIP_TRY(hipStreamWaitEvent(c->streams[rank], c->wait_ev[rank], 0));
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_comm_signal_stream(srcdsp_comm_t c, int rank, void *stream) {
    SRCDSP_ARG_CHECK(c != nullptr, "comm_signal_stream: null comm");
    SRCDSP_ARG_CHECK(rank >= 0 && rank < (int)c->devs.size(), "comm_signal_stream: rank out of range");
    DeviceGuard g;
    std::lock_guard<std::mutex> lk(c->order_mu);
    SRCDSP_HIP_TRY(hipSetDevice(c->devs[rank]));
    SRCDSP_HIP_TRY(hipEventRecord(c->signal_ev[rank], c->streams[rank]));
    SRCDSP_HIP_TRY(hipStreamWaitEvent((hipStream_t)stream, c->signal_ev[rank], 0));
    return SRCDSP_OK;
}

// ----------------------------------------------------------- sharded decim
SRCDSP_API int srcdsp_decim_sharded_create(srcdsp_decim_sharded_t *out, srcdsp_comm_t comm, int channels,
                                           int variant, unsigned M, const void *coeffs, int ntaps,
                                           unsigned flags) {
    SRCDSP_ARG_CHECK(out != nullptr, "decim_sharded_create: null out");
    *out = nullptr;
    SRCDSP_ARG_CHECK(comm != nullptr, "decim_sharded_create: null comm");
    SRCDSP_ARG_CHECK(channels >= 1, "decim_sharded_create: channels must be >= 1");
    const int nr = (int)comm->devs.size();
    DeviceGuard g;
    auto *h = new srcdsp_decim_sharded();
    h->comm = comm;
    comm->refs.fetch_add(1);
    h->channels = channels;
    h->first.resize(nr);
    h->count.resize(nr);
    h->handles.assign(channels, nullptr);
    const int q = channels / nr, rem = channels % nr;  // block partition (srcdsp_amd/dist.py channels_for_rank)
    for (int r = 0; r < nr; ++r) {
        h->first[r] = r * q + std::min(r, rem);
        h->count[r] = q + (r < rem ? 1 : 0);
    }
    for (int r = 0; r < nr; ++r) {
        hipError_t e = hipSetDevice(comm->devs[r]);
        if (e != hipSuccess) {
            set_error(std::string("decim_sharded_create: hipSetDevice: ") + hipGetErrorString(e));
            srcdsp_decim_sharded_destroy(h);
            return SRCDSP_ERR_HIP;
        }
        for (int k = 0; k < h->count[r]; ++k) {
            int rc = srcdsp_decim_create(&h->handles[h->first[r] + k], variant, M, coeffs, ntaps, flags);
            if (rc) {
                srcdsp_decim_sharded_destroy(h);
                return rc;
            }
        }
    }
    *out = h;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_decim_sharded_destroy(srcdsp_decim_sharded_t h) {
    if (!h) return SRCDSP_OK;
    DeviceGuard g;
    for (int r = 0; r < (int)h->first.size(); ++r) {
        (void)hipSetDevice(h->comm->devs[r]);
        for (int k = 0; k < h->count[r]; ++k) srcdsp_decim_destroy(h->handles[h->first[r] + k]);
    }
    comm_release(h->comm);
    delete h;
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_decim_sharded_partition(srcdsp_decim_sharded_t h, int rank, int *first, int *count) {
    SRCDSP_ARG_CHECK(h != nullptr, "decim_sharded_partition: null handle");
    SRCDSP_ARG_CHECK(rank >= 0 && rank < (int)h->first.size(), "decim_sharded_partition: rank out of range");
    if (first) *first = h->first[rank];
    if (count) *count = h->count[rank];
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_decim_sharded_channel(srcdsp_decim_sharded_t h, int ch, srcdsp_decim_t *handle) {
    SRCDSP_ARG_CHECK(h != nullptr && handle != nullptr, "decim_sharded_channel: null argument");
    SRCDSP_ARG_CHECK(ch >= 0 && ch < h->channels, "decim_sharded_channel: channel out of range");
    *handle = h->handles[ch];
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_decim_sharded_step(srcdsp_decim_sharded_t h, const void *const *d_in, size_t in_stride,
                                         void *const *d_out, size_t out_stride, size_t n_in) {
    SRCDSP_ARG_CHECK(h != nullptr && d_in != nullptr && d_out != nullptr, "decim_sharded_step: null argument");
    DeviceGuard g;
    for (int r = 0; r < (int)h->first.size(); ++r) {
        if (h->count[r] == 0) continue;
        SRCDSP_ARG_CHECK(d_in[r] != nullptr && d_out[r] != nullptr, "decim_sharded_step: null rank buffer");
        SRCDSP_HIP_TRY(hipSetDevice(h->comm->devs[r]));
        int rc = srcdsp_decim_step_batched(h->handles.data() + h->first[r], h->count[r], d_in[r], in_stride,
                                           d_out[r], out_stride, n_in, (void *)h->comm->streams[r]);
        if (rc) return rc;
    }
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_decim_sharded_reset(srcdsp_decim_sharded_t h) {
    SRCDSP_ARG_CHECK(h != nullptr, "decim_sharded_reset: null handle");
    DeviceGuard g;
    for (int r = 0; r < (int)h->first.size(); ++r) {
        SRCDSP_HIP_TRY(hipSetDevice(h->comm->devs[r]));
        for (int k = 0; k < h->count[r]; ++k) {
            int rc = srcdsp_decim_reset(h->handles[h->first[r] + k]);
            if (rc) return rc;
        }
    }
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_decim_sharded_step_host(srcdsp_decim_sharded_t h, const void *const *in, void *const *out,
                                              size_t n_in) {
    SRCDSP_ARG_CHECK(h != nullptr && in != nullptr && out != nullptr, "decim_sharded_step_host: null argument");
    const int nr = (int)h->first.size();
    const unsigned M = h->handles[0]->core.M;
    SRCDSP_ARG_CHECK(n_in % M == 0, "decim_sharded_step_host: n_in must be a multiple of M");
    std::vector<int> rcs(nr, SRCDSP_OK);
    std::vector<std::string> errs(nr);
    auto run = [&](int r) {
        if (hipSetDevice(h->comm->devs[r]) != hipSuccess) {
            rcs[r] = SRCDSP_ERR_HIP;
            errs[r] = "decim_sharded_step_host: hipSetDevice failed";
            return;
        }
        for (int k = 0; k < h->count[r] && rcs[r] == SRCDSP_OK; ++k) {
            const int ch = h->first[r] + k;
            rcs[r] = srcdsp_decim_step_host(h->handles[ch], in[ch], n_in, out[ch], n_in / M);
            if (rcs[r]) errs[r] = get_error();  // the error text is per thread
        }
    };
    std::vector<std::thread> th;
    for (int r = 1; r < nr; ++r) th.emplace_back(run, r);
    {
        DeviceGuard g;
        run(0);
    }
    for (auto &t : th) t.join();
    for (int r = 0; r < nr; ++r)
        if (rcs[r]) {
            set_error(errs[r]);
            return rcs[r];
        }
    return SRCDSP_OK;
}

SRCDSP_API int srcdsp_decim_sharded_gather(srcdsp_decim_sharded_t h, void *const *d_out, size_t out_stride,
                                           size_t n_out, void *d_root, int root) {
    SRCDSP_ARG_CHECK(h != nullptr && d_out != nullptr && d_root != nullptr, "decim_sharded_gather: null argument");
    const int nr = (int)h->first.size();
    SRCDSP_ARG_CHECK(root >= 0 && root < nr, "decim_sharded_gather: root out of range");
    SRCDSP_ARG_CHECK(out_stride >= n_out, "decim_sharded_gather: out_stride < n_out");
    if (n_out == 0) return SRCDSP_OK;
    const size_t ob = (size_t)kv_out_bytes(h->handles[0]->core.kv);
    const size_t row = n_out * ob;
    srcdsp_comm *c = h->comm;
    DeviceGuard g;
    const bool even = std::all_of(h->count.begin(), h->count.end(), [&](int k) { return k == h->count[0]; });
    if (even && out_stride == n_out) {
        // every rank's rows are one contiguous block of the same size: ncclGather (rccl.h:745)
        SRCDSP_NCCL_TRY(rccl().GroupStart());
        for (int r = 0; r < nr; ++r) {
            ncclResult_t e = rccl().Gather(d_out[r], r == root ? d_root : nullptr, (size_t)h->count[r] * row,
                                           ncclUint8, root, c->comms[r], c->streams[r]);
            if (e != ncclSuccess) {
                (void)rccl().GroupEnd();
                set_error(std::string("ncclGather: ") + rccl().GetErrorString(e));
                return SRCDSP_ERR_HIP;
            }
        }
        SRCDSP_NCCL_TRY(rccl().GroupEnd());
        return SRCDSP_OK;
    }
    // uneven partition or strided rows: the root copies its own rows on its
    // device; every other row travels by ncclSend/ncclRecv (rccl.h:700,720)
    SRCDSP_HIP_TRY(hipSetDevice(c->devs[root]));
    if (h->count[root] > 0)
        SRCDSP_HIP_TRY(hipMemcpy2DAsync((char *)d_root + (size_t)h->first[root] * row, row, d_out[root],
                                        out_stride * ob, row, (size_t)h->count[root], hipMemcpyDeviceToDevice,
                                        c->streams[root]));
    SRCDSP_NCCL_TRY(rccl().GroupStart());
    for (int r = 0; r < nr; ++r) {
        if (r == root) continue;
        const bool contiguous = out_stride == n_out;
        const int pieces = contiguous ? (h->count[r] > 0 ? 1 : 0) : h->count[r];
        const size_t bytes = contiguous ? (size_t)h->count[r] * row : row;
        for (int k = 0; k < pieces; ++k) {
            const char *src = (const char *)d_out[r] + (size_t)k * out_stride * ob;
            char *dst = (char *)d_root + ((size_t)h->first[r] + k) * row;
            ncclResult_t e = rccl().Send(src, bytes, ncclUint8, root, c->comms[r], c->streams[r]);
            if (e == ncclSuccess) e = rccl().Recv(dst, bytes, ncclUint8, r, c->comms[root], c->streams[root]);
            if (e != ncclSuccess) {
                (void)rccl().GroupEnd();
                set_error(std::string("ncclSend/ncclRecv: ") + rccl().GetErrorString(e));
                return SRCDSP_ERR_HIP;
            }
        }
    }
    SRCDSP_NCCL_TRY(rccl().GroupEnd());
    return SRCDSP_OK;
}
