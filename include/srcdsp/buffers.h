/*
 * Drop-in for SrcDsp's buffers.h: dsptl::FifoWithTimeTrack<T, N>
 * (reference buffers.h:58-459) with its ring in HBM, executed by
 * libsrcdsp_hip.so.  Same members and semantics; write() of a host vector
 * returns before its H2D copy completes (double-buffered pinned staging), and
 * reads are ordered after it on the device.  Added: device overloads of
 * write()/read() (DeviceSpan + stream), so a step() can consume the FIFO
 * without a host round trip.  T must be trivially copyable.
 */
#ifndef SRCDSP_DROPIN_BUFFERS_H
#define SRCDSP_DROPIN_BUFFERS_H

#include <iostream>
#include <utility>

#include "srcdsp_dropin_common.h"

namespace dsptl {

template <class T, size_t N>
class FifoWithTimeTrack {
    static_assert(std::is_trivially_copyable<T>::value, "FIFO elements are copied as bytes");

public:
    /// buffers.h:62-66
    FifoWithTimeTrack(double samplingFrequencyArg = 0) : h_(nullptr) {
        srcdsp_detail::check(srcdsp_fifo_create(&h_, sizeof(T), N, samplingFrequencyArg), "FifoWithTimeTrack");
    }
    ~FifoWithTimeTrack() { srcdsp_fifo_destroy(h_); }
    FifoWithTimeTrack(const FifoWithTimeTrack &) = delete;
    FifoWithTimeTrack &operator=(const FifoWithTimeTrack &) = delete;

    /// buffers.h:140-224 (assert(inSize < N))
    void write(std::vector<T> &in, unsigned int seconds = 0, double fracSeconds = 0) {
        assert(in.size() < N);
        srcdsp_detail::check(srcdsp_fifo_write(h_, in.data(), in.size(), seconds, fracSeconds), "write");
    }
    void write(const DeviceSpan<const T> &in, unsigned int seconds = 0, double fracSeconds = 0,
               void *stream = nullptr) {
        assert(in.size < N);
        srcdsp_detail::check(srcdsp_fifo_write_device(h_, in.data, in.size, seconds, fracSeconds, stream),
                             "write(device)");
    }
    /// buffers.h:282-349: true = the requested range is not available
    bool read(std::vector<T> &out, uint64_t &start) {
        assert(out.size() != 0);
        int err = 0;
        srcdsp_detail::check(srcdsp_fifo_read_host(h_, out.data(), out.size(), &start, &err), "read");
        return err != 0;
    }
    bool read(DeviceSpan<T> out, uint64_t &start, void *stream = nullptr) {
        assert(out.size != 0);
        int err = 0;
        srcdsp_detail::check(srcdsp_fifo_read(h_, out.data, out.size, &start, &err, stream), "read(device)");
        return err != 0;
    }
    /// buffers.h:377-392
    size_t count() {
        size_t c = 0;
        srcdsp_detail::check(srcdsp_fifo_count(h_, &c), "count");
        return c;
    }
    /// buffers.h:245-258
    void reset() { srcdsp_detail::check(srcdsp_fifo_reset(h_), "reset"); }
    /// buffers.h:229-240 (the ring contents are printed from a host copy)
    void dumpInfo(bool dumpData = false) {
        size_t wp = 0;
        uint64_t ts = 0, te = 0;
        int ro = 0;
        srcdsp_detail::check(srcdsp_fifo_get_state(h_, &wp, &ts, &te, &ro), "dumpInfo");
        std::cout << "writePtr: " << wp << '\n';
        std::cout << "timeStart : " << ts << '\n';
        std::cout << "timeEnd : " << te << '\n';
        std::cout << "rolloverFlag : " << ro << '\n';
        (void)dumpData;  // element dump needs operator<< of T on host: not provided for device rings
    }
    /// buffers.h:413-459
    std::pair<unsigned int, double> getAbsoluteTime(uint64_t timePoint, double fracTimePoint) {
        unsigned s = 0;
        double f = 0;
        srcdsp_detail::check(srcdsp_fifo_get_absolute_time(h_, timePoint, fracTimePoint, &s, &f), "getAbsoluteTime");
        return std::make_pair(s, f);
    }
    srcdsp_fifo_t handle() const { return h_; }

private:
    srcdsp_fifo_t h_;
};

}  // namespace dsptl
#endif
