/*
 * Multi-GPU extension of the drop-in (BASELINE configs[2]).
 * The reference has no multi-device code: a reference user filtering C
 * independent channels owns C dsptl::FilterDnsamplingFir objects
 * (dnsampling_filters.h:49-172) and calls step() on each.  Here one object
 * owns all C channels, block-partitions them over the GPUs of a GpuComm and
 * steps every GPU's share with one batched launch; gather() brings the
 * decimated channels to one GPU with RCCL over xGMI (ncclGather,
 * rccl.h:745, or grouped ncclSend/ncclRecv for uneven shares).
 *
 *   dsptl::GpuComm comm({0, 1, 2, 3, 4, 5, 6, 7});              // ncclCommInitAll
 *   dsptl::ShardedDnsamplingFir<cf32, cf32, cf32, float, 4> f(comm, 64, taps);
 *   f.step(inputs, outputs);          // std::vector per channel, as 64 step() calls
 *   f.step(d_in, in_stride, d_out, out_stride, n_in);   // device-resident, per GPU
 *   f.gather(d_out, out_stride, n_out, d_root, 0);     // all channels to GPU 0
 *
 * Results are those of C separate FilterDnsamplingFir objects, bit for bit.
 *
 * Ordering: step() and gather() run on the comm streams, which are
 * non-blocking -- they wait neither for the null stream nor for the caller's
 * streams, and the caller's streams do not wait for them.  Caller work that
 * fills d_in or reads d_out / d_root must run on comm.stream(r), or after
 * comm.synchronize(), or be ordered with
 *   comm.waitFor(r, s);  // comm stream r waits for what `s` queued so far
 *   comm.signal(r, s);   // `s` waits for what comm stream r queued so far
 *   e.g. fill d_in[r] on s; comm.waitFor(r, s); f.step(...); f.gather(...);
 *        comm.signal(root, s); copy d_root out on s; hipStreamSynchronize(s);
 *
 * Lifetime: a ShardedDnsamplingFir holds its own reference to the
 * communicator (srcdsp_decim_sharded_create), so the GpuComm may be destroyed
 * before the operators built on it.
 * Verification: run on a 1-GPU communicator only (tests/cpp/sharded_main.cpp,
 * contiguous and strided gathers); the N > 1 step and gather paths (threaded
 * host step, ncclGather across devices, the uneven-share ncclSend/ncclRecv
 * loop) are unverified on hardware until a multi-GPU node runs them.
 */
#ifndef SRCDSP_DROPIN_SHARDED_FILTERS_H
#define SRCDSP_DROPIN_SHARDED_FILTERS_H

#include "dnsampling_filters.h"

namespace dsptl {

/// One host process driving several GPUs: one RCCL communicator and one HIP
/// stream per device (srcdsp_comm_create over ncclCommInitAll, rccl.h:236).
class GpuComm {
public:
    explicit GpuComm(const std::vector<int> &devices) : c_(nullptr) {
        srcdsp_detail::check(srcdsp_comm_create(&c_, (int)devices.size(), devices.data()), "GpuComm");
    }
    ~GpuComm() { srcdsp_comm_destroy(c_); }
    GpuComm(const GpuComm &) = delete;
    GpuComm &operator=(const GpuComm &) = delete;
    int size() const {
        int n = 0;
        srcdsp_detail::check(srcdsp_comm_info(c_, &n, nullptr), "GpuComm::size");
        return n;
    }
    /// hipStream_t (as void*) the sharded operators use on rank's device
    void *stream(int rank) const {
        void *s = nullptr;
        srcdsp_detail::check(srcdsp_comm_stream(c_, rank, &s), "GpuComm::stream");
        return s;
    }
    void synchronize() { srcdsp_detail::check(srcdsp_comm_synchronize(c_), "GpuComm::synchronize"); }
    /// work queued later on rank's comm stream waits for everything queued on
    /// `stream` (a hipStream_t on rank's device, as void*) so far
    void waitFor(int rank, void *stream) {
        srcdsp_detail::check(srcdsp_comm_wait_stream(c_, rank, stream), "GpuComm::waitFor");
    }
    /// work queued later on `stream` waits for everything queued on rank's comm stream so far
    void signal(int rank, void *stream) {
        srcdsp_detail::check(srcdsp_comm_signal_stream(c_, rank, stream), "GpuComm::signal");
    }
    srcdsp_comm_t handle() const { return c_; }

private:
    srcdsp_comm_t c_;
};

template <class InType, class OutType, class InternalType, class CoefType, unsigned M>
class ShardedDnsamplingFir {
    static constexpr int kVariant = srcdsp_detail::decim_variant<InType, OutType, InternalType, CoefType>();
    static_assert(kVariant >= 0,
                  "ShardedDnsamplingFir: this type combination does not compile in the reference "
                  "(limitScale16 returns complex<int16_t>, dsptl_dnsampling_filters.h:215)");
    static_assert(M >= 1, "decimation ratio");

public:
    /// `channels` FilterDnsamplingFir(firCoeff) objects (dnsampling_filters.h:84-97)
    ShardedDnsamplingFir(GpuComm &comm, int channels, const std::vector<CoefType> &firCoeff,
                         unsigned flags = SRCDSP_DEFAULT_FLAGS)
        : h_(nullptr), ranks_(comm.size()), channels_(channels) {
        srcdsp_detail::check(srcdsp_decim_sharded_create(&h_, comm.handle(), channels, kVariant, M, firCoeff.data(),
                                                         (int)firCoeff.size(), flags),
                             "ShardedDnsamplingFir");
    }
    ~ShardedDnsamplingFir() { srcdsp_decim_sharded_destroy(h_); }
    ShardedDnsamplingFir(const ShardedDnsamplingFir &) = delete;
    ShardedDnsamplingFir &operator=(const ShardedDnsamplingFir &) = delete;

    int channels() const { return channels_; }
    /// channels [first, first + count) live on rank's GPU
    void partition(int rank, int &first, int &count) const {
        srcdsp_detail::check(srcdsp_decim_sharded_partition(h_, rank, &first, &count), "partition");
    }
    /// dnsampling_filters.h:129-172 for every channel: input[ch] -> filteredSignal[ch],
    /// each output vector pre-sized to input[ch].size()/M (all channels the same length)
    void step(const std::vector<std::vector<InType>> &input, std::vector<std::vector<OutType>> &filteredSignal) {
        // the C ABI takes one length for every channel and no output sizes:
        // every vector is checked here (throws under NDEBUG) before any is touched
        srcdsp_detail::check_shape((int)input.size() == channels_ && (int)filteredSignal.size() == channels_,
                                  "ShardedDnsamplingFir::step: one input and one output vector per channel");
        std::vector<const void *> in(channels_);
        std::vector<void *> out(channels_);
        for (int ch = 0; ch < channels_; ++ch) {
            srcdsp_detail::check_shape(input[ch].size() == input[0].size(),
                                      "ShardedDnsamplingFir::step: channels of different lengths");
            srcdsp_detail::check_shape(filteredSignal[ch].size() * M == input[ch].size(),
                                      "ShardedDnsamplingFir::step: output vector != input size / M");
            in[ch] = input[ch].data();
            out[ch] = filteredSignal[ch].data();
        }
        srcdsp_detail::check(srcdsp_decim_sharded_step_host(h_, in.data(), out.data(), input[0].size()),
                             "ShardedDnsamplingFir::step");
    }
    /// device-resident: d_in[r] / d_out[r] on rank r's GPU hold its channels as
    /// rows in_stride / out_stride samples apart; asynchronous on the comm streams
    void step(const std::vector<const InType *> &d_in, size_t in_stride, const std::vector<OutType *> &d_out,
              size_t out_stride, size_t n_in) {
        srcdsp_detail::check_shape((int)d_in.size() == ranks_ && (int)d_out.size() == ranks_,
                                  "ShardedDnsamplingFir::step(device): one input and one output pointer per rank");
        std::vector<const void *> i(d_in.begin(), d_in.end());
        std::vector<void *> o(d_out.begin(), d_out.end());
        srcdsp_detail::check(srcdsp_decim_sharded_step(h_, i.data(), in_stride, o.data(), out_stride, n_in),
                             "ShardedDnsamplingFir::step(device)");
    }
    /// every channel's n_out outputs to d_root (rank root's GPU), channel-major
    void gather(const std::vector<OutType *> &d_out, size_t out_stride, size_t n_out, OutType *d_root, int root = 0) {
        srcdsp_detail::check_shape((int)d_out.size() == ranks_, "ShardedDnsamplingFir::gather: one pointer per rank");
        std::vector<void *> o(d_out.begin(), d_out.end());
        srcdsp_detail::check(srcdsp_decim_sharded_gather(h_, o.data(), out_stride, n_out, d_root, root),
                             "ShardedDnsamplingFir::gather");
    }
    /// dnsampling_filters.h:56-60 for every channel
    void reset() { srcdsp_detail::check(srcdsp_decim_sharded_reset(h_), "reset"); }
    /// the FilterDnsamplingFir state of one channel (C ABI handle, on its GPU)
    srcdsp_decim_t channel(int ch) const {
        srcdsp_decim_t c = nullptr;
        srcdsp_detail::check(srcdsp_decim_sharded_channel(h_, ch, &c), "channel");
        return c;
    }
    srcdsp_decim_sharded_t handle() const { return h_; }

private:
    srcdsp_decim_sharded_t h_;
    int ranks_;
    int channels_;
};

}  // namespace dsptl
#endif
