// cf32_launch.h -- host launcher of the complex<float> headline kernel
// (decim_stream_cf32), shared by the two translation units that instantiate
// it: decim_cf32_ct.hip (tap counts compiled in) and decim_cf32_rt.hip (tap
// count at run time).  Split from decim.hip so the instantiations compile in
// parallel.
#pragma once
#include <algorithm>
#include <map>
#include <mutex>

#include "ops.h"

#include "decim_kernels.h"

namespace srcdsp {

// 4 outputs per lane, 512 lanes -> 8192 input samples per tile, 75 KB LDS and
// <= 128 VGPRs = 2 resident workgroups (16 waves) per CU; the persistent grid
// is 2x the resident capacity (measured best on MI355X: scripts/tune, profiles/).
constexpr int kCfBlock = 512, kCfGrid = 1024;

// M = 4 is the headline; M = 8 uses the same kernel with R = 2 outputs per
// lane (the same 16-sample lane chunks, LDS image and memory schedule), M = 2
// with R = 4 and M = 1 (complex<float> FilterFir) with R = 8, both on 8-sample
// lane chunks (R = 8 at M = 2 spills at the 128-VGPR budget of 16 waves per CU).
// NT = 0: the tap count at run time (any N <= kCfMaxTaps), dynamic LDS.
template <int M>
constexpr int cf32_r() { return M == 1 ? 8 : (M <= 3 ? 4 : 16 / M); }

// allow a kernel's dynamic LDS beyond the default limit (once per kernel and size)
inline int raise_lds_limit(const void *kern, size_t bytes) {
    static std::mutex mu;
    static std::map<const void *, size_t> set;
    std::lock_guard<std::mutex> g(mu);
    size_t &cur = set[kern];
    if (bytes > cur) {
        hipError_t e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
        if (e != hipSuccess) {  // not cached: the next call tries again
            set_error(std::string("hipFuncSetAttribute(MaxDynamicSharedMemorySize): ") + hipGetErrorString(e));
            return SRCDSP_ERR_HIP;
        }
        cur = bytes;
    }
    return SRCDSP_OK;
}

template <int NT, int M = 4>
int launch_cf32(DecimLaunch L, int channels, bool fma, hipStream_t s) {
    constexpr int R = cf32_r<M>(), TO = kCfBlock * R;
    L.ntiles = (L.n_out + TO - 1) / TO;
    dim3 grid((unsigned)std::min<long>(L.ntiles, kCfGrid), channels);
    const bool q0 = (L.shift & 31u) == 0;  // limitScale16 shift 0: the 4-op float quantiser
    const size_t smem = NT == 0 ? 16 * (size_t)cf32_lds_granules(M, R, kCfBlock, L.ntaps) : 0;
    // measured best (scripts/tune, sustained back-to-back): 512-lane tiles
    // (8192 samples: half the halo re-read of 256), grid-stride tile order,
    // non-temporal input loads, outputs paired across half-waves by
    // v_permlane32_swap into whole-line non-temporal stores (no LDS round
    // trip: 2 barriers per tile, not 4); 2 workgroups (16 waves) per CU;
    // taps issued tap-major through inline asm (FMA: 0.88 M instead of
    // 1.08 M cycles per launch, -8.6 % time on one box,
    // profiles/tuning/r02_ramp_ab.txt)
    auto go = [&](auto kern) -> int {
        if (NT == 0) {
            int rc = raise_lds_limit((const void *)kern, smem);
            if (rc) return rc;
        }
        hipLaunchKernelGGL(kern, grid, dim3(kCfBlock), smem, s, L);
        return SRCDSP_OK;
    };
    if (fma && q0)
        return go(decim_stream_cf32<NT, R, kCfBlock, true, 4, true, M>);
    if (fma)
        return go(decim_stream_cf32<NT, R, kCfBlock, true, 4, false, M>);
    if (q0)
        return go(decim_stream_cf32<NT, R, kCfBlock, false, 4, true, M>);
    return go(decim_stream_cf32<NT, R, kCfBlock, false, 4, false, M>);
}

}  // namespace srcdsp
