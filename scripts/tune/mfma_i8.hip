// Integer matrix-core probes (tuning only, not the product).
//
// Layout/numerics check of the gfx950 i8 MFMAs: one wave, every lane loads its
// raw 16-byte A and B fragments and its C registers from host-prepared arrays
// and writes D back, so the host can test a lane map and the accumulator's
// overflow behaviour (wrap modulo 2^32 or saturate) with exact integer data.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void __launch_bounds__(64) i8_32x32x32_raw(const v4i* a, const v4i* b, const v16i* c, v16i* d, int reps)
{
    const int l = threadIdx.x;
    v16i acc = c[l];
    for (int i = 0; i < reps; ++i)
        acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[l], b[l], acc, 0, 0, 0);
    d[l] = acc;
}

__global__ void __launch_bounds__(64) i8_16x16x64_raw(const v4i* a, const v4i* b, const v4i* c, v4i* d, int reps)
{
    const int l = threadIdx.x;
    v4i acc = c[l];
    for (int i = 0; i < reps; ++i)
        acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[l], b[l], acc, 0, 0, 0);
    d[l] = acc;
}

extern "C" int tune_i8_mfma_raw(int shape, const void* a, const void* b, const void* c, void* d, int reps, hipStream_t s)
{
    if (shape == 32)
        hipLaunchKernelGGL(i8_32x32x32_raw, dim3(1), dim3(64), 0, s, (const v4i*)a, (const v4i*)b, (const v16i*)c,
                           (v16i*)d, reps);
    else
        hipLaunchKernelGGL(i8_16x16x64_raw, dim3(1), dim3(64), 0, s, (const v4i*)a, (const v4i*)b, (const v4i*)c,
                           (v4i*)d, reps);
    return (int)hipGetLastError();
}
