#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const unsigned *in, unsigned *out, unsigned nrec) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)in, 0, nrec, 0x00020000);
    auto w = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * threadIdx.x, 0, 2);
    out[4 * threadIdx.x + 0] = w[0]; out[4 * threadIdx.x + 1] = w[1];
    out[4 * threadIdx.x + 2] = w[2]; out[4 * threadIdx.x + 3] = w[3];
    unsigned d = __builtin_amdgcn_raw_buffer_load_b32(rs, 16 * threadIdx.x + 4, 0, 2);
    out[64 + threadIdx.x] = d;
}
int main() {
    unsigned h[64], *din, *dout, ho[80];
    for (int i = 0; i < 64; ++i) h[i] = 1000 + i;
    hipMalloc(&din, 256); hipMalloc(&dout, 320);
    hipMemcpy(din, h, 256, hipMemcpyHostToDevice);
    for (unsigned nrec : {40u, 44u, 36u}) {
        hipMemset(dout, 0xff, 320);
        hipLaunchKernelGGL(k, dim3(1), dim3(4), 0, 0, din, dout, nrec);
        hipMemcpy(ho, dout, 320, hipMemcpyDeviceToHost);
        printf("nrec=%u b128:", nrec);
        for (int i = 0; i < 16; ++i) printf(" %u", ho[i]);
        printf(" | b32@+4:");
        for (int i = 0; i < 4; ++i) printf(" %u", ho[64 + i]);
        printf("\n");
    }
    return 0;
}
