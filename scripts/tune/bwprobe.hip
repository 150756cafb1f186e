// HBM streaming probes (not part of the product): what read:write mixes,
// store/load policies and work distributions reach on MI355X, to set the
// practical ceiling of the 4:1 decimator stream (8 B read + 2 B written per
// input sample).
#include <hip/hip_runtime.h>

typedef float float4_t __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ float4_t ld(const float4_t *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(float4_t *p, float4_t v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// RATIO input granules (16 B) per output granule; RATIO 0 = read only.
// U output granules per lane per iteration (U*RATIO loads in flight).
// CONTIG: block b owns a contiguous range (else grid-stride interleave).
template <int RATIO, int U, bool NTL, bool NTS, bool CONTIG>
__global__ __launch_bounds__(256) void rw_probe(const float4_t *in, float4_t *out, long n_out) {
    const long nth = (long)gridDim.x * 256;
    const int t = threadIdx.x;
    long begin, end, step, lane0;
    if constexpr (CONTIG) {
        const long per = (n_out + gridDim.x - 1) / gridDim.x;
        begin = blockIdx.x * per;
        end = begin + per < n_out ? begin + per : n_out;
        step = 256L * U;
        lane0 = t;
    } else {
        begin = 0;
        end = n_out;
        step = nth * U;
        lane0 = (long)blockIdx.x * 256 + t;
    }
    const long sub = CONTIG ? 256 : nth;  // distance between a lane's U outputs
    float4_t acc = {0, 0, 0, 0};
    for (long base = begin; base + step <= end; base += step) {
        float4_t v[U * (RATIO > 0 ? RATIO : 4)];
        constexpr int R = RATIO > 0 ? RATIO : 4;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long o = base + lane0 + u * sub;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                // a wave reads R contiguous KiB runs: granule (o - lane) * R + r * 64... keep coalesced:
                // input granule index = R*(o - lane0_wave) + r*64 + lane_in_wave
                const long ow = o - (t & 63);
                v[u * R + r] = ld<NTL>(in + R * ow + r * 64 + (t & 63));
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float4_t s = v[u * R];
#pragma unroll
            for (int r = 1; r < R; ++r) s += v[u * R + r];
            if constexpr (RATIO > 0) st<NTS>(out + base + lane0 + u * sub, s);
            else acc += s;
        }
    }
    if constexpr (RATIO == 0)
        if (acc.x == 1234.5f) out[0] = acc;
}

// 4:1 contiguous-per-block stream through buffer intrinsics with explicit
// cache-policy bits (gfx950 aux: bit0 sc0, bit1 nt, bit4 sc1) on loads / stores
template <int LA, int SA>
__global__ __launch_bounds__(256) void aux_probe(const float4_t *in, float4_t *out, long n_out) {
    const int t = threadIdx.x;
    const long per = (n_out + gridDim.x - 1) / gridDim.x;
    const long begin = blockIdx.x * per;
    const long end = begin + per < n_out ? begin + per : n_out;
    __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc((void *)(in + 4 * begin), 0, 0x7ffffff0, 0x00020000);
    __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void *)(out + begin), 0, 0x7ffffff0, 0x00020000);
    for (long base = 0; begin + base + 512 <= end; base += 512) {
        float4_t v[8];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const long ow = base + u * 256 + (t & ~63);
                auto w = __builtin_amdgcn_raw_buffer_load_b128(ri, (int)(16 * (4 * ow + r * 64 + (t & 63))), 0, LA);
                v[u * 4 + r] = __builtin_bit_cast(float4_t, w);
            }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            float4_t s = v[u * 4] + v[u * 4 + 1] + v[u * 4 + 2] + v[u * 4 + 3];
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b128(ri, 0, 0, 0)), s),
                                                   ro, (int)(16 * (base + u * 256 + t)), 0, SA);
        }
    }
}

// Output bursts: each block reduces K chunks (64 KiB in -> 16 KiB out each)
// into LDS, then writes the K*16 KiB as one contiguous burst.  Chunks are
// taken in grid-stride order of K-chunk super tiles.  Tests whether fewer,
// larger write bursts ease the HBM read/write turnaround of the 4:1 mix.
template <int K, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void burst_probe(const float4_t *in, float4_t *out, long n_out) {
    __shared__ float4_t ob[K * 1024];
    const int t = threadIdx.x;
    const long nsuper = n_out / (K * 1024);
    for (long s = blockIdx.x; s < nsuper; s += gridDim.x) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const long o0 = (s * K + k) * 1024;  // first output granule of the chunk
            float4_t v[16];
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int r = 0; r < 4; ++r) v[4 * u + r] = ld<NTL>(in + 4 * o0 + u * 1024 + r * 256 + t);
#pragma unroll
            for (int u = 0; u < 4; ++u) ob[k * 1024 + u * 256 + t] = v[4 * u] + v[4 * u + 1] + v[4 * u + 2] + v[4 * u + 3];
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 4 * K; ++i) st<NTS>(out + s * K * 1024 + i * 256 + t, ob[i * 256 + t]);
        __syncthreads();
    }
}

// 1:2 expansion (the float -> complex<float> FilterFir stream: 4 B read, 8 B
// written per sample): each lane reads one granule and writes two; a wave's
// stores cover 2 KiB contiguous.  n_in = input granules.
template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void expand_probe(const float4_t *in, float4_t *out, long n_in) {
    const long nth = (long)gridDim.x * 256;
    const int t = threadIdx.x;
    for (long base = (long)blockIdx.x * 256; base < n_in; base += nth) {
        const float4_t v = ld<NTL>(in + base + t);
        // the wave's input granules base + (t & ~63) .. +63 -> its output granules
        // 2 (base + (t & ~63)) .. +127; lane l writes l and 64 + l of them
        const long w0 = 2 * (base + (t & ~63)) + (t & 63);
        st<NTS>(out + w0, v);
        st<NTS>(out + w0 + 64, v * 2.f);
    }
}

__global__ __launch_bounds__(256) void fill_probe(float4_t *out, long n) {
    const long nth = (long)gridDim.x * 256;
    const float4_t z = {1, 2, 3, 4};
    for (long k = (long)blockIdx.x * 256 + threadIdx.x; k < n; k += nth) out[k] = z;
}

#define CASE(id, R, U, NL, NS, C)                                                                  \
    case id:                                                                                       \
        hipLaunchKernelGGL((rw_probe<R, U, NL, NS, C>), dim3(blocks), dim3(256), 0, s, in, out,    \
                           (R) > 0 ? n_in16 / (R) : n_in16 / 4);                                    \
        break;

extern "C" int bw_probe(int id, int blocks, const void *in_, void *out_, long n_in16, void *stream) {
    const float4_t *in = (const float4_t *)in_;
    float4_t *out = (float4_t *)out_;
    hipStream_t s = (hipStream_t)stream;
    switch (id) {
        CASE(0, 1, 2, false, false, false)  // copy 1:1
        CASE(1, 4, 1, false, false, false)  // 4:1 grid-stride, 4 loads in flight
        CASE(2, 4, 2, false, false, false)  // 4:1, 8 loads in flight
        CASE(3, 4, 2, false, true, false)   // 4:1 nt stores
        CASE(4, 4, 2, true, false, false)   // 4:1 nt loads
        CASE(5, 4, 2, true, true, false)    // 4:1 nt both
        CASE(6, 4, 1, false, false, true)   // 4:1 contiguous per block
        CASE(7, 4, 2, false, false, true)   // 4:1 contiguous, 8 in flight
        CASE(8, 4, 2, false, true, true)    // 4:1 contiguous, nt stores
        CASE(9, 0, 2, false, false, false)  // read only
        CASE(10, 0, 2, true, false, false)  // read only nt
        CASE(11, 4, 4, false, false, false) // 4:1, 16 loads in flight
        CASE(12, 1, 2, false, true, false)  // copy nt stores
#define ACASE(id, LA, SA)                                                                          \
    case id:                                                                                        \
        hipLaunchKernelGGL((aux_probe<LA, SA>), dim3(blocks), dim3(256), 0, s, in, out, n_in16 / 4); \
        break;
        ACASE(100, 0, 0) ACASE(101, 0, 1) ACASE(102, 0, 2) ACASE(103, 0, 3) ACASE(104, 0, 16) ACASE(105, 0, 17)
        ACASE(106, 0, 18) ACASE(107, 0, 19)
        ACASE(110, 2, 0) ACASE(111, 2, 1) ACASE(112, 2, 2) ACASE(113, 2, 3) ACASE(114, 2, 16) ACASE(115, 2, 17)
        ACASE(116, 2, 18) ACASE(117, 2, 19)
        ACASE(120, 1, 2) ACASE(121, 3, 2) ACASE(122, 16, 2) ACASE(123, 17, 2) ACASE(124, 18, 2) ACASE(125, 19, 2)
    case 20:
        hipLaunchKernelGGL(fill_probe, dim3(blocks), dim3(256), 0, s, out, n_in16 / 4);
        break;
    case 30:  // 1:2 expansion over n_in16 / 2 input granules (output = n_in16 granules)
        hipLaunchKernelGGL((expand_probe<false, false>), dim3(blocks), dim3(256), 0, s, in, out, n_in16 / 2);
        break;
    case 31:
        hipLaunchKernelGGL((expand_probe<true, true>), dim3(blocks), dim3(256), 0, s, in, out, n_in16 / 2);
        break;
    case 32:
        hipLaunchKernelGGL((expand_probe<false, true>), dim3(blocks), dim3(256), 0, s, in, out, n_in16 / 2);
        break;
        CASE(13, 4, 2, true, true, true)    // 4:1 contiguous, nt both
#define BCASE(id, K, NL, NS)                                                                          \
    case id:                                                                                         \
        hipLaunchKernelGGL((burst_probe<K, NL, NS>), dim3(blocks), dim3(256), 0, s, in, out, n_in16 / 4); \
        break;
        BCASE(40, 1, true, true) BCASE(41, 2, true, true) BCASE(42, 4, true, true) BCASE(43, 8, true, true)
        BCASE(44, 4, true, false)
    default:
        return -1;
    }
    return hipGetLastError();
}
