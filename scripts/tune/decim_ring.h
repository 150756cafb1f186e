// decim_ring.h -- tuning experiment (not part of the product): the headline
// decimator (complex<float>, M = 4, 127 taps, FMA contract) with a
// loader/consumer split inside one workgroup per CU, as VERDICT round 1 asked:
// one loader wave streams wave tiles into an LDS ring by LDS-DMA
// (global_load_lds_dwordx4: no VGPR round trip, no ds_write) and NCONS
// consumer waves run the tap loop, synchronised by per-slot FULL / FREE words
// in LDS instead of workgroup barriers.
//
// Slot = one wave tile: 64 lanes x 4 outputs = 1024 input samples plus the
// 128-sample halo = 576 16-B granules, stored padded (granule G at G + G/8:
// one pad after every 8, so the lanes' ds_read_b128 land on 16 distinct
// slots) = 648 slots = 10,368 B.  LDS-DMA writes 64 consecutive slots per
// wave instruction (base + lane x 16), so lane i of DMA instruction j fills
// position P = 64 j + i: granule P - P/9, or (pad) a duplicate of its left
// neighbour; 11 instructions per slot, the last masked to 8 lanes.
// The loader keeps NPF slots in flight (counted vmcnt), publishes FULL[k] =
// generation + 1 once a slot has landed, and reuses a slot when its consumer
// has stored FREE[k] = generation.  Every wait is a bounded spin (s_sleep), so
// a protocol bug ends the kernel with wrong outputs instead of a hang.
// Wave tile order: chunks of CH consecutive wave tiles per workgroup, the
// chunks grid-strided over the (XCD-mapped) workgroups.
#pragma once
#include "../../srcdsp_amd/csrc/decim_kernels.h"

namespace srcdsp {

constexpr int kRingSlotG = 648;              // LDS granules per slot (576 data + 72 pads)
constexpr int kRingSlotB = kRingSlotG * 16;  // bytes per slot

__device__ __forceinline__ unsigned ring_ld(unsigned addr) {
    unsigned v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    return v;
}
__device__ __forceinline__ void ring_st(unsigned addr, unsigned v) {
    asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(addr), "v"(v) : "memory");
}
// bounded spin until the LDS word at addr >= want; returns false on timeout
__device__ __forceinline__ bool ring_wait(unsigned addr, unsigned want) {
    for (unsigned n = 0; n < (1u << 22); ++n) {
        if (ring_ld(addr) >= want) return true;
        __builtin_amdgcn_s_sleep(1);
    }
    return false;
}
// one 16-B LDS-DMA: lds_dst wave-uniform (M0), src per lane
__device__ __forceinline__ void ring_dma16(const void *src, unsigned lds_dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds_dst)
                 : "memory");
}

template <int NCONS, int NSLOT, int NPF, int CH, int AUX = 2>
__global__ __launch_bounds__(64 * (NCONS + 1), 1) void decim_ring_cf32(DecimLaunch a) {
    constexpr int NT = 127, NQ = 32, R = 4;
    static_assert(NSLOT > NPF && (NPF - 1) * 11 <= 63, "ring geometry");
    __shared__ __attribute__((aligned(16))) float4 ring[NSLOT * kRingSlotG];
    __shared__ unsigned flags[2 * NSLOT];  // FULL[k], FREE[k]
    const int t = threadIdx.x, lane = t & 63;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
    const float2 *in = (const float2 *)a.in;
    const float2 *hist = (const float2 *)a.hist_in[0];
    float2 *out = (float2 *)a.out;
    const long n_in = a.n_in;
    const long nwg = gridDim.x;
    const long b = xcd_tile(blockIdx.x, nwg);
    const long NW = a.ntiles;  // wave tiles of 256 outputs (host: divisible by nwg * CH)
    const int n_it = (int)(NW / nwg);
    auto gw_of = [&](int it) { return ((long)(it / CH) * nwg + b) * CH + it % CH; };
    const unsigned ring_b = (unsigned)(uintptr_t)ring;
    const unsigned full_b = (unsigned)(uintptr_t)flags, free_b = full_b + 4 * NSLOT;
    for (int i = t; i < 2 * NSLOT; i += blockDim.x) flags[i] = 0;
    if (b == 0) write_history(in, n_in, hist, (float2 *)a.hist_out[0], NT - 1);
    __syncthreads();

    if (wv == NCONS) {
        // ------------------------------------------------------------ loader
        auto issue = [&](int it) {
            const int k = it % NSLOT;
            const long gw = gw_of(it);
            const unsigned dst = ring_b + k * kRingSlotB;
            if (gw == 0) {  // the halo is the history: plain loads and LDS stores
                for (int G = lane; G < 576; G += 64) {
                    const long s = -128 + 2L * G;
                    const float2 lo = fetch(in, hist, s, n_in, NT - 1), hi = fetch(in, hist, s + 1, n_in, NT - 1);
                    ring[k * kRingSlotG + G + G / 8] = make_float4(lo.x, lo.y, hi.x, hi.y);
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                return;
            }
            const float2 *base = in + 1024 * gw - 128;
#pragma unroll
            for (int j = 0; j < 11; ++j) {
                const int P = 64 * j + lane;
                const int m = P / 9, r = P - 9 * m;
                const int G = 8 * m + (r == 8 ? 7 : r);
                if (P < kRingSlotG) ring_dma16(base + 2 * G, dst + 1024 * j);
            }
        };
        auto publish = [&](int it) { if (lane == 0) ring_st(full_b + 4 * (it % NSLOT), it / NSLOT + 1); };
        const int pro = n_it < NPF - 1 ? n_it : NPF - 1;
        for (int it = 0; it < pro; ++it) issue(it);
        for (int it = pro; it < n_it; ++it) {
            if (!ring_wait(free_b + 4 * (it % NSLOT), it / NSLOT)) break;
            issue(it);
            if constexpr (NPF == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if constexpr (NPF == 2) asm volatile("s_waitcnt vmcnt(11)" ::: "memory");
            if constexpr (NPF == 3) asm volatile("s_waitcnt vmcnt(22)" ::: "memory");
            if constexpr (NPF == 4) asm volatile("s_waitcnt vmcnt(33)" ::: "memory");
            if constexpr (NPF == 5) asm volatile("s_waitcnt vmcnt(44)" ::: "memory");
            publish(it - (NPF - 1));
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        for (int it = n_it - (NPF - 1) < 0 ? 0 : n_it - (NPF - 1); it < n_it; ++it) publish(it);
        return;
    }

    // -------------------------------------------------------------- consumers
    ConstPtr<unsigned long long> tp2 = const_view<unsigned long long>(a.coef);
    for (int it = wv; it < n_it; it += NCONS) {
        const int k = it % NSLOT;
        if (!ring_wait(full_b + 4 * k, it / NSLOT + 1)) break;
        asm volatile("" : "+s"(tp2));
        // lane chunk of this wave tile: granule 64 + 8 lane -> slot 72 + 9 lane
        const float4 *img = ring + k * kRingSlotG + 72 + 9 * lane;
        float2 X[4 * (NQ + R)];
        auto load_group = [&](int e) {
            const float4 g0 = img[2 * e + floordiv(2 * e, 8)];
            const float4 g1 = img[2 * e + 1 + floordiv(2 * e + 1, 8)];
            X[4 * e + 4 * NQ + 0] = make_float2(g0.x, g0.y);
            X[4 * e + 4 * NQ + 1] = make_float2(g0.z, g0.w);
            X[4 * e + 4 * NQ + 2] = make_float2(g1.x, g1.y);
            X[4 * e + 4 * NQ + 3] = make_float2(g1.z, g1.w);
        };
#pragma unroll
        for (int e = -1; e < R; ++e) load_group(e);
        f2_t acc[R];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            if (q + 1 < NQ) load_group(-q - 2);
            if ((q & 3) == 0) asm volatile("" : "+s"(tp2));
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const int kk = 4 * q + p;
                if (kk < NT) {
                    const unsigned long long cp = tp2[kk >> 1];
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const float2 x = X[4 * (r - q) - p + 4 * NQ];
                        const f2_t xv = {x.x, x.y};
                        if (kk == 0) pk_fma_tap<false, true>(acc[r], cp, xv);
                        else if (kk & 1) pk_fma_tap<true, false>(acc[r], cp, xv);
                        else pk_fma_tap<false, false>(acc[r], cp, xv);
                    }
                }
            }
        }
        // every read of the slot has returned (the FMAs consumed them): release it
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) ring_st(free_b + 4 * k, it / NSLOT + 1);
        float2 o[R];
#pragma unroll
        for (int r = 0; r < R; ++r) o[r] = make_float2(q16f_shift0(acc[r].x), q16f_shift0(acc[r].y));
        store_wave_lines<R, true>(out + 256 * gw_of(it), o, lane);
    }
}

}  // namespace srcdsp
