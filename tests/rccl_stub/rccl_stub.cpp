// rccl_stub.cpp -- TEST-ONLY stand-in for librccl.so.1 (never shipped with
// libsrcdsp_hip.so, never on the product's library path).
//
// Purpose (VERDICT r3 Next #2): run the multi-device logic of
// srcdsp_amd/csrc/multi.hip -- the per-rank host threads, the ncclGather of
// an even partition, the uneven / strided ncclSend/ncclRecv loop with its
// destination offsets and the root's own hipMemcpy2DAsync -- at ndev > 1 on a
// box with ONE GPU.  Real RCCL cannot make a communicator whose ranks share a
// device, so this library implements the few entry points multi.hip resolves
// (multi.hip rccl()) with stream-ordered hipMemcpyAsync on whatever devices
// the ranks name (all the same device here):
//
//   ncclCommInitAll  any device list, repeats allowed (one comm per entry)
//   ncclGroupStart/End  per-thread nesting; operations queue and run at the
//                    outermost ncclGroupEnd; an operation outside a group is
//                    ncclInvalidUsage (multi.hip always groups)
//   ncclGather       at GroupEnd every rank of the communicator must have
//                    queued one gather with the same root and count; rank r's
//                    sendbuf lands at recvbuf + r*count (the root's recvbuf)
//   ncclSend/Recv    paired at GroupEnd in issue order per (src, dst) pair;
//                    counts and types must match
//
// Stream semantics follow NCCL's: the copy for rank r's contribution starts
// after the work queued on rank r's stream and on the root's (receiver's)
// stream before the call, and both streams' later work waits for it.
//
// Built by tests/test_sharded_stub.py with g++ against libamdhip64; loaded by
// dlopen("librccl.so.1") through LD_LIBRARY_PATH in the test's child process.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>
#include <utility>
#include <vector>

struct ncclComm {
    int rank, nranks, dev;
    std::shared_ptr<int> clique;  // shared by the comms of one ncclCommInitAll
};

namespace {

struct Op {
    enum Kind { GATHER, SEND, RECV } kind;
    ncclComm *comm;
    const void *sbuf;
    void *rbuf;
    size_t bytes;
    int peer;  // gather: root; send: destination rank; recv: source rank
    hipStream_t stream;
};

thread_local int g_depth = 0;
thread_local std::vector<Op> g_ops;
std::mutex g_log_mu;

size_t type_bytes(ncclDataType_t t) {
    switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 0;
    }
}

// dst stream waits for src stream's queued work
hipError_t order(hipStream_t src, int src_dev, hipStream_t dst, int dst_dev) {
    hipEvent_t e;
    hipError_t rc = hipSetDevice(src_dev);
    if (rc == hipSuccess) rc = hipEventCreateWithFlags(&e, hipEventDisableTiming);
    if (rc == hipSuccess) rc = hipEventRecord(e, src);
    if (rc == hipSuccess) rc = hipSetDevice(dst_dev);
    if (rc == hipSuccess) rc = hipStreamWaitEvent(dst, e, 0);
    if (rc == hipSuccess) rc = hipEventDestroy(e);  // released once the wait resolves
    return rc;
}

// one transfer: src rank's buffer on its stream -> dst rank's buffer; issued
// on the receiver's stream after both streams' earlier work, and the
// sender's stream waits for it
ncclResult_t transfer(const Op &s, const Op &r, const void *src, void *dst, size_t bytes) {
    if (bytes == 0) return ncclSuccess;
    if (order(s.stream, s.comm->dev, r.stream, r.comm->dev) != hipSuccess) return ncclUnhandledCudaError;
    if (hipSetDevice(r.comm->dev) != hipSuccess) return ncclUnhandledCudaError;
    if (hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, r.stream) != hipSuccess)
        return ncclUnhandledCudaError;
    if (order(r.stream, r.comm->dev, s.stream, s.comm->dev) != hipSuccess) return ncclUnhandledCudaError;
    if (std::getenv("RCCL_STUB_LOG")) {
        std::lock_guard<std::mutex> g(g_log_mu);
        std::fprintf(stderr, "rccl_stub: rank %d -> rank %d, %zu bytes, dst %p\n", s.comm->rank, r.comm->rank, bytes,
                     dst);
    }
    return ncclSuccess;
}

ncclResult_t run_group(std::vector<Op> &ops) {
    int saved = 0;
    (void)hipGetDevice(&saved);
    ncclResult_t res = ncclSuccess;
    // gathers: one per rank of each clique, same root and size
    std::map<int *, std::vector<const Op *>> gathers;
    for (const Op &o : ops)
        if (o.kind == Op::GATHER) gathers[o.comm->clique.get()].push_back(&o);
    for (auto &kv : gathers) {
        auto &g = kv.second;
        const int n = g[0]->comm->nranks;
        std::vector<const Op *> by_rank(n, nullptr);
        for (const Op *o : g) {
            if (by_rank[o->comm->rank] || o->peer != g[0]->peer || o->bytes != g[0]->bytes) return ncclInvalidUsage;
            by_rank[o->comm->rank] = o;
        }
        if ((int)g.size() != n) return ncclInvalidUsage;  // a rank did not take part
        const Op *root = by_rank[g[0]->peer];
        if (!root || !root->rbuf) return ncclInvalidArgument;
        for (int r = 0; r < n && res == ncclSuccess; ++r)
            res = transfer(*by_rank[r], *root, by_rank[r]->sbuf, (char *)root->rbuf + (size_t)r * root->bytes,
                           root->bytes);
    }
    // send/recv: FIFO per (clique, src rank, dst rank)
    std::map<std::tuple<int *, int, int>, std::vector<const Op *>> sends, recvs;
    for (const Op &o : ops) {
        if (o.kind == Op::SEND) sends[std::make_tuple(o.comm->clique.get(), o.comm->rank, o.peer)].push_back(&o);
        if (o.kind == Op::RECV) recvs[std::make_tuple(o.comm->clique.get(), o.peer, o.comm->rank)].push_back(&o);
    }
    if (sends.size() != recvs.size()) res = ncclInvalidUsage;
    for (auto &kv : sends) {
        if (res != ncclSuccess) break;
        auto it = recvs.find(kv.first);
        if (it == recvs.end() || it->second.size() != kv.second.size()) {
            res = ncclInvalidUsage;
            break;
        }
        for (size_t k = 0; k < kv.second.size() && res == ncclSuccess; ++k) {
            const Op *s = kv.second[k], *r = it->second[k];
            if (s->bytes != r->bytes) {
                res = ncclInvalidUsage;
                break;
            }
            res = transfer(*s, *r, s->sbuf, r->rbuf, s->bytes);
        }
    }
    (void)hipSetDevice(saved);
    return res;
}

ncclResult_t enqueue(Op o) {
    if (g_depth == 0) return ncclInvalidUsage;
    if (!o.comm) return ncclInvalidArgument;
    g_ops.push_back(o);
    return ncclSuccess;
}

}  // namespace

extern "C" {

ncclResult_t ncclCommInitAll(ncclComm_t *comms, int ndev, const int *devlist) {
    if (!comms || ndev < 1) return ncclInvalidArgument;
    int have = 0;
    if (hipGetDeviceCount(&have) != hipSuccess) return ncclUnhandledCudaError;
    auto clique = std::make_shared<int>(ndev);
    for (int r = 0; r < ndev; ++r) {
        int d = devlist ? devlist[r] : r;
        if (d < 0 || d >= have) return ncclInvalidArgument;
        comms[r] = new ncclComm{r, ndev, d, clique};
    }
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    delete comm;
    return ncclSuccess;
}

const char *ncclGetErrorString(ncclResult_t r) {
    switch (r) {
    case ncclSuccess: return "no error (rccl_stub)";
    case ncclUnhandledCudaError: return "HIP call failed (rccl_stub)";
    case ncclInvalidArgument: return "invalid argument (rccl_stub)";
    case ncclInvalidUsage: return "invalid usage: unmatched or ungrouped operation (rccl_stub)";
    default: return "error (rccl_stub)";
    }
}

ncclResult_t ncclGroupStart() {
    ++g_depth;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    if (g_depth == 0) return ncclInvalidUsage;
    if (--g_depth > 0) return ncclSuccess;
    std::vector<Op> ops;
    ops.swap(g_ops);
    return run_group(ops);
}

ncclResult_t ncclGather(const void *sendbuff, void *recvbuff, size_t sendcount, ncclDataType_t datatype, int root,
                        ncclComm_t comm, hipStream_t stream) {
    size_t tb = type_bytes(datatype);
    if (!tb || !comm || root < 0 || root >= comm->nranks) return ncclInvalidArgument;
    return enqueue({Op::GATHER, comm, sendbuff, comm->rank == root ? recvbuff : nullptr, sendcount * tb, root, stream});
}

ncclResult_t ncclSend(const void *sendbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
    size_t tb = type_bytes(datatype);
    if (!tb || !comm || peer < 0 || peer >= comm->nranks) return ncclInvalidArgument;
    return enqueue({Op::SEND, comm, sendbuff, nullptr, count * tb, peer, stream});
}

ncclResult_t ncclRecv(void *recvbuff, size_t count, ncclDataType_t datatype, int peer, ncclComm_t comm,
                      hipStream_t stream) {
    size_t tb = type_bytes(datatype);
    if (!tb || !comm || peer < 0 || peer >= comm->nranks) return ncclInvalidArgument;
    return enqueue({Op::RECV, comm, nullptr, recvbuff, count * tb, peer, stream});
}

}  // extern "C"
