// Multi-GPU drop-in test program: C independent complex<float> decim-4
// channels through dsptl::ShardedDnsamplingFir over the GPUs listed on the
// command line (include/srcdsp/sharded_filters.h, RCCL via libsrcdsp_hip.so).
// tests/test_dropin_cpp.py writes the inputs, runs this on the GPU box and
// compares every output with the oracle.
//
//   sharded_main <in.bin> <out.bin> <dev> [<dev> ...]
// in.bin: tag 1 = taps (float), tag 2 = channel count (int32),
//         tag 10+ch = channel ch's input (complex<float>), all the same length.
// out.bin: tag 100+ch = channel ch by the host-vector step() in two chained
//          calls; tag 200 = all channels by the device step() after reset(),
//          gathered to rank ROOT's device (channel-major; ROOT from the
//          environment variable SHARDED_ROOT, default 0); 201 = strided
//          rows; 202 = an operator outliving its communicator; 203 = inputs
//          filled and the gather target cleared and read back on the CALLER's
//          own streams, ordered with comm.waitFor / comm.signal only (no
//          synchronize() of the comm).
#include <hip/hip_runtime.h>

#include <complex>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <vector>

#include "sharded_filters.h"

using cf32 = std::complex<float>;

static std::map<int, std::vector<char>> read_records(const char *path) {
    std::map<int, std::vector<char>> m;
    std::ifstream f(path, std::ios::binary);
    int32_t tag;
    int64_t nb;
    while (f.read((char *)&tag, 4) && f.read((char *)&nb, 8)) {
        std::vector<char> b(nb);
        f.read(b.data(), nb);
        m[tag] = std::move(b);
    }
    return m;
}

template <class T>
static std::vector<T> as(const std::vector<char> &b) {
    return std::vector<T>((const T *)b.data(), (const T *)(b.data() + b.size()));
}

static void put(std::ofstream &f, int32_t tag, const void *p, int64_t nb) {
    f.write((const char *)&tag, 4);
    f.write((const char *)&nb, 8);
    f.write((const char *)p, nb);
}

#define HIP_OK(x)                                                                  \
    do {                                                                           \
        if ((x) != hipSuccess) {                                                   \
            std::fprintf(stderr, "%s failed at %s:%d\n", #x, __FILE__, __LINE__);  \
            return 1;                                                              \
        }                                                                          \
    } while (0)

int main(int argc, char **argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s in.bin out.bin dev...\n", argv[0]);
        return 2;
    }
    std::vector<int> devs;
    for (int i = 3; i < argc; ++i) devs.push_back(std::atoi(argv[i]));
    auto rec = read_records(argv[1]);
    const std::vector<float> taps = as<float>(rec[1]);
    const int C = as<int32_t>(rec[2])[0];
    std::vector<std::vector<cf32>> in(C);
    for (int ch = 0; ch < C; ++ch) in[ch] = as<cf32>(rec[10 + ch]);
    const size_t n = in[0].size(), n_out = n / 4, half = (n / 2) & ~(size_t)3;
    const int root = std::getenv("SHARDED_ROOT") ? std::atoi(std::getenv("SHARDED_ROOT")) : 0;
    if (root < 0 || root >= (int)devs.size()) {
        std::fprintf(stderr, "SHARDED_ROOT out of range\n");
        return 2;
    }
    std::ofstream out(argv[2], std::ios::binary);

    dsptl::GpuComm comm(devs);
    dsptl::ShardedDnsamplingFir<cf32, cf32, cf32, float, 4> f(comm, C, taps);

    // reference-style host vectors, two chained step() calls per channel
    std::vector<std::vector<cf32>> a(C), b(C), y1(C, std::vector<cf32>(half / 4)),
        y2(C, std::vector<cf32>((n - half) / 4));
    for (int ch = 0; ch < C; ++ch) {
        a[ch].assign(in[ch].begin(), in[ch].begin() + half);
        b[ch].assign(in[ch].begin() + half, in[ch].end());
    }
    f.step(a, y1);
    f.step(b, y2);
    for (int ch = 0; ch < C; ++ch) {
        std::vector<cf32> y = y1[ch];
        y.insert(y.end(), y2[ch].begin(), y2[ch].end());
        put(out, 100 + ch, y.data(), (int64_t)(y.size() * sizeof(cf32)));
    }

    // device-resident: each rank's channels as rows of one buffer on its GPU,
    // then every channel gathered to the first GPU
    f.reset();
    const int R = comm.size();
    std::vector<const cf32 *> d_in(R);
    std::vector<cf32 *> d_out(R);
    cf32 *d_root = nullptr;
    for (int r = 0; r < R; ++r) {
        int first, count;
        f.partition(r, first, count);
        HIP_OK(hipSetDevice(devs[r]));
        cf32 *x = nullptr, *y = nullptr;
        HIP_OK(hipMalloc(&x, std::max<size_t>(1, count * n) * sizeof(cf32)));
        HIP_OK(hipMalloc(&y, std::max<size_t>(1, count * n_out) * sizeof(cf32)));
        for (int k = 0; k < count; ++k)
            HIP_OK(hipMemcpy(x + k * n, in[first + k].data(), n * sizeof(cf32), hipMemcpyHostToDevice));
        d_in[r] = x;
        d_out[r] = y;
        if (r == root) HIP_OK(hipMalloc(&d_root, (size_t)C * n_out * sizeof(cf32)));
    }
    f.step(d_in, n, d_out, n_out, n);
    f.gather(d_out, n_out, n_out, d_root, root);
    comm.synchronize();
    std::vector<cf32> all((size_t)C * n_out);
    HIP_OK(hipSetDevice(devs[root]));
    HIP_OK(hipMemcpy(all.data(), d_root, all.size() * sizeof(cf32), hipMemcpyDeviceToHost));
    put(out, 200, all.data(), (int64_t)(all.size() * sizeof(cf32)));

    // strided rows (out_stride > n_out): the gather's Memcpy2D / send-recv branch
    f.reset();
    const size_t ostr = n_out + 37;
    std::vector<cf32 *> d_out2(R);
    for (int r = 0; r < R; ++r) {
        int first, count;
        f.partition(r, first, count);
        HIP_OK(hipSetDevice(devs[r]));
        HIP_OK(hipMalloc(&d_out2[r], std::max<size_t>(1, count * ostr) * sizeof(cf32)));
    }
    f.step(d_in, n, d_out2, ostr, n);
    HIP_OK(hipSetDevice(devs[root]));
    // on the root's comm stream: the gather's copies into d_root are ordered
    // after it there (a plain hipMemset on the null stream is not ordered
    // with the comm streams, which are non-blocking)
    HIP_OK(hipMemsetAsync(d_root, 0, (size_t)C * n_out * sizeof(cf32), (hipStream_t)comm.stream(root)));
    f.gather(d_out2, ostr, n_out, d_root, root);
    comm.synchronize();
    HIP_OK(hipSetDevice(devs[root]));
    HIP_OK(hipMemcpy(all.data(), d_root, all.size() * sizeof(cf32), hipMemcpyDeviceToHost));
    put(out, 201, all.data(), (int64_t)(all.size() * sizeof(cf32)));
    for (int r = 0; r < R; ++r) {
        HIP_OK(hipSetDevice(devs[r]));
        HIP_OK(hipFree(d_out2[r]));
    }

    // a communicator destroyed before the operator built on it: the operator
    // keeps its own reference and still steps and gathers
    {
        auto *c2 = new dsptl::GpuComm(devs);
        auto *g2 = new dsptl::ShardedDnsamplingFir<cf32, cf32, cf32, float, 4>(*c2, C, taps);
        delete c2;
        g2->step(d_in, n, d_out, n_out, n);
        g2->gather(d_out, n_out, n_out, d_root, root);
        HIP_OK(hipSetDevice(devs[root]));
        HIP_OK(hipDeviceSynchronize());
        HIP_OK(hipMemcpy(all.data(), d_root, all.size() * sizeof(cf32), hipMemcpyDeviceToHost));
        put(out, 202, all.data(), (int64_t)(all.size() * sizeof(cf32)));
        delete g2;
    }
    // caller streams (the ordering rule of sharded_filters.h): the caller fills
    // fresh input buffers and clears the gather target on streams of its own,
    // hands them to the comm streams with waitFor, and reads the gathered rows
    // back on its root stream after signal -- no comm.synchronize()
    {
        f.reset();
        std::vector<hipStream_t> cs(R);
        std::vector<const cf32 *> d_in3(R);
        for (int r = 0; r < R; ++r) {
            int first, count;
            f.partition(r, first, count);
            HIP_OK(hipSetDevice(devs[r]));
            HIP_OK(hipStreamCreateWithFlags(&cs[r], hipStreamNonBlocking));
            cf32 *x = nullptr;
            HIP_OK(hipMalloc(&x, std::max<size_t>(1, count * n) * sizeof(cf32)));
            HIP_OK(hipMemsetAsync(x, 0x7f, std::max<size_t>(1, count * n) * sizeof(cf32), cs[r]));
            if (count > 0)
                HIP_OK(hipMemcpyAsync(x, d_in[r], count * n * sizeof(cf32), hipMemcpyDeviceToDevice, cs[r]));
            d_in3[r] = x;
        }
        HIP_OK(hipSetDevice(devs[root]));
        HIP_OK(hipMemsetAsync(d_root, 0x55, (size_t)C * n_out * sizeof(cf32), cs[root]));
        for (int r = 0; r < R; ++r) comm.waitFor(r, (void *)cs[r]);
        f.step(d_in3, n, d_out, n_out, n);
        f.gather(d_out, n_out, n_out, d_root, root);
        comm.signal(root, (void *)cs[root]);
        cf32 *h_all = nullptr;
        HIP_OK(hipSetDevice(devs[root]));
        HIP_OK(hipHostMalloc((void **)&h_all, all.size() * sizeof(cf32), 0));
        HIP_OK(hipMemcpyAsync(h_all, d_root, all.size() * sizeof(cf32), hipMemcpyDeviceToHost, cs[root]));
        HIP_OK(hipStreamSynchronize(cs[root]));
        put(out, 203, h_all, (int64_t)(all.size() * sizeof(cf32)));
        HIP_OK(hipHostFree(h_all));
        comm.synchronize();  // before the buffers go
        for (int r = 0; r < R; ++r) {
            HIP_OK(hipSetDevice(devs[r]));
            HIP_OK(hipStreamDestroy(cs[r]));
            HIP_OK(hipFree((void *)d_in3[r]));
        }
    }
    for (int r = 0; r < R; ++r) {
        HIP_OK(hipSetDevice(devs[r]));
        HIP_OK(hipFree((void *)d_in[r]));
        HIP_OK(hipFree(d_out[r]));
    }
    HIP_OK(hipSetDevice(devs[root]));
    HIP_OK(hipFree(d_root));
    std::printf("sharded_main: %d channels x %zu samples over %d GPU(s) ok\n", C, n, R);
    return 0;
}
