// Tuning harness (not part of the product): per-instruction VALU issue cost on
// gfx950, in shader cycles (s_memtime), for the instructions the kernels'
// rooflines are priced on.  Each lane runs 16 independent accumulator chains
// of one instruction; every wave stamps s_memtime around its loop.  With W
// waves per SIMD, the SIMD's throughput is W / (cycles per instruction per wave).
#include <hip/hip_runtime.h>

template <int MODE>
__global__ __launch_bounds__(256) void issue_rate(unsigned long long *cyc, int *sink, int iters) {
    // cyc[4 per wave]: s_memtime and s_memrealtime (100 MHz) at loop start and end
    int a[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) a[j] = threadIdx.x * 3 + j;
    float f[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) f[j] = threadIdx.x * 0.001f + j;
    const int x = 0x00030005 + threadIdx.x, y = 0x00070002;
    const float fx = 1.0001f, fy = 0.9999f;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) {
        if constexpr (MODE == 0) {  // v_fmac_f32 (VOP2)
#pragma unroll
            for (int j = 0; j < 16; ++j) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(f[j]) : "v"(fx), "v"(fy));
        } else if constexpr (MODE == 1) {  // v_pk_fma_f32 (8 pairs = 16 FMAs)
#pragma unroll
            for (int j = 0; j < 16; j += 2) {
                float2 p = make_float2(f[j], f[j + 1]);
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p) : "v"(make_float2(fx, fx)), "v"(make_float2(fy, fy)));
                f[j] = p.x; f[j + 1] = p.y;
            }
        } else if constexpr (MODE == 2) {  // v_dot2c_i32_i16 (VOP2, accumulating)
#pragma unroll
            for (int j = 0; j < 16; ++j) asm volatile("v_dot2c_i32_i16 %0, %1, %2" : "+v"(a[j]) : "v"(x), "v"(y));
        } else if constexpr (MODE == 3) {  // v_dot2_i32_i16 (VOP3P)
#pragma unroll
            for (int j = 0; j < 16; ++j) asm volatile("v_dot2_i32_i16 %0, %1, %2, %0" : "+v"(a[j]) : "v"(x), "v"(y));
        } else if constexpr (MODE == 4) {  // v_mad_i32_i24 (VOP3)
#pragma unroll
            for (int j = 0; j < 16; ++j) asm volatile("v_mad_i32_i24 %0, %1, %2, %0" : "+v"(a[j]) : "v"(x), "v"(y));
        } else if constexpr (MODE == 5) {  // v_fma_f32 (VOP3)
#pragma unroll
            for (int j = 0; j < 16; ++j) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(f[j]) : "v"(fx), "v"(fy));
        } else if constexpr (MODE == 6) {  // v_add_u32 (plain integer VALU)
#pragma unroll
            for (int j = 0; j < 16; ++j) asm volatile("v_add_u32 %0, %1, %0" : "+v"(a[j]) : "v"(x));
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    int s = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) s += a[j] + (int)f[j];
    sink[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) {
        unsigned long long *c = cyc + 4 * (blockIdx.x * 4 + threadIdx.x / 64);
        c[0] = t0; c[1] = t1; c[2] = r0; c[3] = r1;
    }
}

extern "C" int tune_issue_rate(int mode, int blocks, int iters, unsigned long long *cyc, int *sink, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    switch (mode) {
    case 0: hipLaunchKernelGGL(issue_rate<0>, dim3(blocks), dim3(256), 0, s, cyc, sink, iters); break;
    case 1: hipLaunchKernelGGL(issue_rate<1>, dim3(blocks), dim3(256), 0, s, cyc, sink, iters); break;
    case 2: hipLaunchKernelGGL(issue_rate<2>, dim3(blocks), dim3(256), 0, s, cyc, sink, iters); break;
    case 3: hipLaunchKernelGGL(issue_rate<3>, dim3(blocks), dim3(256), 0, s, cyc, sink, iters); break;
    case 4: hipLaunchKernelGGL(issue_rate<4>, dim3(blocks), dim3(256), 0, s, cyc, sink, iters); break;
    case 5: hipLaunchKernelGGL(issue_rate<5>, dim3(blocks), dim3(256), 0, s, cyc, sink, iters); break;
    case 6: hipLaunchKernelGGL(issue_rate<6>, dim3(blocks), dim3(256), 0, s, cyc, sink, iters); break;
    default: return -1;
    }
    return hipGetLastError();
}
