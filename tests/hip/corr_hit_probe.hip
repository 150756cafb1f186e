// corr_hit_probe.hip -- TEST-ONLY probe of the correlator's detection test
// (srcdsp_amd/csrc/corr_hit.h, restating correlators.h:262-268).
//
// Built by srcdsp_amd.build.build_test_probes() into tests/_build/ (never part
// of libsrcdsp_hip.so).  tests/test_gpu_corr_hit.py feeds it crafted register
// values -- exact ties c * 100 == 729 * e, their +-1 neighbours, energies
// 90000 / 90001, c / e = 7.29 (1 +- 2e-9), the uint32 maxima -- and compares
// every decision with the host's IEEE double evaluation of the reference's
// expression.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../srcdsp_amd/csrc/corr_hit.h"

using namespace srcdsp;

// q[4 i .. 4 i + 3] = (c2, c1, c0, e1) of case i;
// out[2 i] = corr_hit as the kernels use it (fast sign test + band),
// out[2 i + 1] = the same test with the exact square roots for every peak
__global__ void corr_hit_probe_kernel(const uint32_t *__restrict__ q, long n, uint8_t *__restrict__ out) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const uint32_t c2 = q[4 * i], c1 = q[4 * i + 1], c0 = q[4 * i + 2], e1 = q[4 * i + 3];
        out[2 * i] = corr_hit(c2, c1, c0, e1) ? 1 : 0;
        out[2 * i + 1] = (c1 > c2 && c1 > c0 && e1 > 90000u && corr_hit_exact(c1, e1)) ? 1 : 0;
    }
}

// out[i] = crsqrt_u32(v[i]), to be compared with the host's correctly rounded sqrt
__global__ void crsqrt_probe_kernel(const uint32_t *__restrict__ v, long n, double *__restrict__ out) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        out[i] = crsqrt_u32(v[i]);
}

static unsigned grid_for(long n) {
    long b = (n + 255) / 256;
    return (unsigned)(b < 4096 ? (b > 0 ? b : 1) : 4096);
}

extern "C" __attribute__((visibility("default"))) int corr_hit_probe(const void *d_q, long n, void *d_out,
                                                                      void *stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(corr_hit_probe_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                       (const uint32_t *)d_q, n, (uint8_t *)d_out);
    return hipGetLastError() == hipSuccess ? 0 : -4;
}

extern "C" __attribute__((visibility("default"))) int crsqrt_probe(const void *d_v, long n, void *d_out,
                                                                    void *stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(crsqrt_probe_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                       (const uint32_t *)d_v, n, (double *)d_out);
    return hipGetLastError() == hipSuccess ? 0 : -4;
}
