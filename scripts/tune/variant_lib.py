#!/usr/bin/env python3
"""Tuning variants of the library (never product): a patched COPY of
srcdsp_amd/csrc built into scripts/tune/ab/libsrcdsp_hip_<name>.so (the
product sources are not touched), for same-box A/Bs with
scripts/tune/ab_libs.sh (LIBS="<name> new").

  halflds  the headline kernel with HALF its tap-loop LDS window reads
           (VERDICT r4 item 4): in decim_stream_cf32's compiled-tap path every
           odd window group takes two opaque registers instead of its two
           ds_read_b128 -- same v_pk_fma_f32 work and memory schedule, wrong
           outputs.  Its time and energy per launch (window_power.py) price the
           LDS reads of the 127-tap loop: the ceiling of any LDS-lighter variant.
  r4mix    config 4 as round 4 left it: the single-copy two-word mixer table
           with per-granule index arithmetic (form 4, no rotated form 5) and
           zero-initialised accumulators (a v_mov each) in the compiled-tap loop.

  r8       the headline at 8 outputs per lane (32-sample lane chunks: 160-sample
           windows for 8 outputs, 44 % fewer LDS window reads per output) in
           256-lane workgroups (the same 8192-sample tiles and LDS image), 2
           waves per SIMD (the wider window and the doubled per-lane prefetch
           need up to 256 VGPRs)
  corrmfma the correlator's fused scan (srcdsp_corr_step, N = 1024, S = 1)
           on the i8 matrix cores behind the product's C ABI
           (scripts/tune/corr_mfma_scan.h; SRCDSP_CORR_MFMA=0 turns it off at
           run time, SRCDSP_CORR_MFMA_PL=2 forces two pattern limbs,
           SRCDSP_CORR_MFMA_RB=1 one row block per wave with one limb)
  mixmfma  config 4's mixer -> decimator chain with the tap loop on the i8
           matrix cores behind srcdsp_mixdecim_step
           (scripts/tune/mixdecim_mfma_step.h; SRCDSP_MIXDECIM_MFMA=0: off)
  rev:<REV> the product sources of git revision REV, unpatched (e.g. rev:HEAD
           before a kernel change is committed); built as libsrcdsp_hip_<REV>.so

    python scripts/tune/variant_lib.py halflds|r8|corrmfma|rev:<REV>
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from srcdsp_amd import build as B  # noqa: E402

PATCHES = {
    "halflds": [("decim_kernels.h", """            auto load_group = [&](int e) {
                const float4 g0 = rd(Bt + 2 * e + floordiv(2 * e, PR));
                const float4 g1 = rd(Bt + 2 * e + 1 + floordiv(2 * e + 1, PR));""",
                 """            auto load_group = [&](int e) {
                float4 g0, g1;
                if ((e & 1) == 0) {
                    g0 = rd(Bt + 2 * e + floordiv(2 * e, PR));
                    g1 = rd(Bt + 2 * e + 1 + floordiv(2 * e + 1, PR));
                } else {  // PROBE: no LDS read, two opaque registers
                    asm volatile("" : "=v"(g0.x), "=v"(g0.y), "=v"(g0.z), "=v"(g0.w));
                    asm volatile("" : "=v"(g1.x), "=v"(g1.y), "=v"(g1.z), "=v"(g1.w));
                }""")],
    "r8": [("decim_kernels.h", """    static_assert((M * R) % 4 == 0 && M * R <= 16, "a lane chunk is 4, 8, 12 or 16 input samples");""",
            """    static_assert((M * R) % 4 == 0 && M * R <= 32, "a lane chunk is 4 to 32 input samples");"""),
           ("cf32_launch.h", """template <int NT, int M = 4>
int launch_cf32(DecimLaunch L, int channels, bool fma, hipStream_t s) {
    constexpr int R = cf32_r<M>(), TO = kCfBlock * R;""", """template <int NT, int M = 4>
int launch_cf32(DecimLaunch L, int channels, bool fma, hipStream_t s) {
    if constexpr (M == 4 && NT != 0) return launch_cf32_r8<NT>(L, channels, fma, s);
    constexpr int R = cf32_r<M>(), TO = kCfBlock * R;"""),
           ("cf32_launch.h", """template <int NT, int M = 4>
int launch_cf32(""", """template <int NT>
int launch_cf32_r8(DecimLaunch L, int channels, bool fma, hipStream_t s) {
    constexpr int R = 8, B = 256, TO = B * R;
    L.ntiles = (L.n_out + TO - 1) / TO;
    dim3 grid((unsigned)std::min<long>(L.ntiles, kCfGrid), channels);
    const bool q0 = (L.shift & 31u) == 0;
    if (fma && q0) hipLaunchKernelGGL((decim_stream_cf32<NT, R, B, true, 2, true, 4>), grid, dim3(B), 0, s, L);
    else if (fma) hipLaunchKernelGGL((decim_stream_cf32<NT, R, B, true, 2, false, 4>), grid, dim3(B), 0, s, L);
    else if (q0) hipLaunchKernelGGL((decim_stream_cf32<NT, R, B, false, 2, true, 4>), grid, dim3(B), 0, s, L);
    else hipLaunchKernelGGL((decim_stream_cf32<NT, R, B, false, 2, false, 4>), grid, dim3(B), 0, s, L);
    return SRCDSP_OK;
}
template <int NT, int M = 4>
int launch_cf32(""")
           # the compiled-tap window in EH + 3 rotating group slots (as the
           # runtime-tap path): the flat 4 (NQ + GPC) array is not promoted to
           # registers at GPC = 8
           , ("decim_kernels.h", """            float2 X[4 * (NQC + GPC)];
            auto load_group = [&](int e) {
                const float4 g0 = rd(Bt + 2 * e + floordiv(2 * e, PR));
                const float4 g1 = rd(Bt + 2 * e + 1 + floordiv(2 * e + 1, PR));
                X[4 * e + 4 * NQC + 0] = make_float2(g0.x, g0.y);
                X[4 * e + 4 * NQC + 1] = make_float2(g0.z, g0.w);
                X[4 * e + 4 * NQC + 2] = make_float2(g1.x, g1.y);
                X[4 * e + 4 * NQC + 3] = make_float2(g1.z, g1.w);
            };""", """            constexpr int SL = (M * (R - 1)) / 4 + 3;
            float2 X[SL][4];
            auto slot = [](int e) { return ((e % SL) + SL) % SL; };
            auto load_group = [&](int e) {
                const float4 g0 = rd(Bt + 2 * e + floordiv(2 * e, PR));
                const float4 g1 = rd(Bt + 2 * e + 1 + floordiv(2 * e + 1, PR));
                X[slot(e)][0] = make_float2(g0.x, g0.y);
                X[slot(e)][1] = make_float2(g0.z, g0.w);
                X[slot(e)][2] = make_float2(g1.x, g1.y);
                X[slot(e)][3] = make_float2(g1.z, g1.w);
            };"""),
           ("decim_kernels.h", """                auto xs = [&](int r, int p) { return X[M * r - 4 * q - p + 4 * NQC]; };""",
            """                auto xs = [&](int r, int p) {
                    const int s = M * r - 4 * q - p;
                    return X[slot(floordiv(s, 4))][s - 4 * floordiv(s, 4)];
                };""")],
    "r4mix": [("decim.hip", """    if constexpr (BLOCK == 512)
        if ((16u * BLOCK) % pe == 0) return""", """    if constexpr (false)
        if ((16u * BLOCK) % pe == 0) return"""),
              ("decim_kernels.h", """                    if (j == 0) {
                        yr[r] = sdot2_0(Dr[OFF + 2 * r], P);
                        yi[r] = sdot2_0(Di[OFF + 2 * r], P);
                    } else {""", """                    if (j == 0) {
                        int32_t z0 = 0, z1 = 0;
                        asm volatile("v_mov_b32 %0, 0" : "=v"(z0));
                        asm volatile("v_mov_b32 %0, 0" : "=v"(z1));
                        yr[r] = sdot2(Dr[OFF + 2 * r], P, z0);
                        yi[r] = sdot2(Di[OFF + 2 * r], P, z1);
                    } else {""")],
}

# the correlator's fused scan on the i8 matrix cores (scripts/tune/corr_mfma_scan.h)
PATCHES["corrmfma"] = [
    ("corr.hip", "    unsigned *d_best = nullptr;\n",
     "    unsigned *d_best = nullptr;\n"
     "    int mfma_pl = 0;             // tuning variant: 1 or 2 pattern limbs, 0 = the product path\n"
     "    uint32_t mfma_scale = 1, mfma_bias[2] = {0u, 0u};\n"
     "    unsigned char *d_mfma_b = nullptr;\n"
     "    uint32_t *d_seams = nullptr;\n"
     "    size_t seams_cap = 0;\n"),
    ("corr.hip", "// ---------------------------------------------------------------- host side\n",
     "#include \"corr_mfma_scan.h\"\n\n// ---------------------------------------------------------------- host side\n"),
    ("corr.hip", """        hipLaunchKernelGGL(corr_scan_s1, dim3((unsigned)blocks), dim3(kCBlock), smem, s, d_in, n, hist, c.d_ptaps,
                           (int)c.N, (int)c.NP, cs, c.corr[0], c.corr[1], c.energy[0], c.d_best);
        SRCDSP_HIP_TRY(hipGetLastError());
""", """        if (corr_mfma_usable(c, d_in, n)) {
            rc = corr_mfma_launch(c, d_in, n, hist, s);
            if (rc) return rc;
        } else {
            hipLaunchKernelGGL(corr_scan_s1, dim3((unsigned)blocks), dim3(kCBlock), smem, s, d_in, n, hist, c.d_ptaps,
                               (int)c.N, (int)c.NP, cs, c.corr[0], c.corr[1], c.energy[0], c.d_best);
            SRCDSP_HIP_TRY(hipGetLastError());
        }
"""),
    ("corr.hip", "hipMemcpyHostToDevice));\n    return SRCDSP_OK;\n}\n\n// reset",
     "hipMemcpyHostToDevice));\n    return corr_mfma_prepare(c);\n}\n\n// reset"),
    ("corr.hip", "    c.cur = 0;\n    *out = n;\n",
     "    c.cur = 0;\n    rc = corr_mfma_prepare(c);\n    if (rc) {\n        srcdsp_corr_destroy(n);\n"
     "        return rc;\n    }\n    *out = n;\n"),
    ("corr.hip", "(void *)c.d_best})", "(void *)c.d_best, (void *)c.d_mfma_b, (void *)c.d_seams})"),
]

# variants whose patch sites the product sources have since moved past (the
# A/B they were built for is recorded; rebuild such a baseline with rev:<REV>)
STALE = {"r4mix": "round 6 moved config 4's mixer table into registers (ccc91a7): build rev:ccc91a7~1 for round 5's "
                  "side of that A/B"}

# config 4's mixer -> decimator chain with the tap loop on the i8 matrix cores
# (scripts/tune/mixdecim_mfma_step.h)
PATCHES["mixmfma"] = [
    ("decim.hip", "static int core_step(FirCore &f, const void *d_in, size_t n_in, void *d_out, size_t n_out, hipStream_t s,\n"
                  "                     const MixerState *mix) {\n"
                  "    SRCDSP_ARG_CHECK(n_out * f.M == n_in, \"step: output size * M must equal input size\");\n"
                  "    if (n_in == 0) return SRCDSP_OK;\n"
                  "    SRCDSP_ARG_CHECK(d_in && d_out, \"step: null buffer\");\n",
     "#include \"mixdecim_mfma_step.h\"\n\n"
     "static int core_step(FirCore &f, const void *d_in, size_t n_in, void *d_out, size_t n_out, hipStream_t s,\n"
     "                     const MixerState *mix) {\n"
     "    SRCDSP_ARG_CHECK(n_out * f.M == n_in, \"step: output size * M must equal input size\");\n"
     "    if (n_in == 0) return SRCDSP_OK;\n"
     "    SRCDSP_ARG_CHECK(d_in && d_out, \"step: null buffer\");\n"
     "    if (!mix && plainmfma_usable(f, d_in, n_in, d_out)) {  // tuning variant: row a2 on the matrix cores\n"
     "        const int r = mfma_decim_step<false>(f, nullptr, d_in, n_in, d_out, s);\n"
     "        if (r != SRCDSP_ERR_UNSUPPORTED) return r;\n"
     "    }\n"),
    ("decim.hip", "    rc = core_step(f, d_in, n_in, d_out, n_out, s, &m);\n",
     "    rc = mixmfma_usable(f, m, d_in, n_in, d_out) ? mixmfma_step(f, m, d_in, n_in, d_out, s)\n"
     "                                                 : SRCDSP_ERR_UNSUPPORTED;\n"
     "    if (rc == SRCDSP_ERR_UNSUPPORTED) rc = core_step(f, d_in, n_in, d_out, n_out, s, &m);\n"),
]

# files a variant adds to its csrc copy (from scripts/tune/)
EXTRA = {"corrmfma": ["corr_mfma_scan.h"], "mixmfma": ["mixdecim_mfma_step.h"]}


# extra compiler flags of a variant (the whole library)
FLAGS = {
    # the R = 8 tap loop (32 steps x 32 pk_fma) is past the default
    # pragma-unroll threshold: not unrolled, its window goes to scratch
    "r8": ["-mllvm", "-pragma-unroll-threshold=1000000"],
}


def main():
    name = sys.argv[1]
    rev = name[4:] if name.startswith("rev:") else None
    if name in STALE:
        sys.exit(f"{name}: stale ({STALE[name]})")
    out = os.path.join(HERE, "ab", f"libsrcdsp_hip_{rev or name}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "srcdsp_amd", "csrc")  # csrc includes ../../include/srcdsp_hip.h
        if rev:
            tar = subprocess.run(["git", "-C", ROOT, "archive", rev, "srcdsp_amd/csrc", "include"],
                                 check=True, capture_output=True).stdout
            subprocess.run(["tar", "-x", "-C", d], input=tar, check=True)
        else:
            shutil.copytree(B.CSRC, src)
            shutil.copytree(os.path.join(ROOT, "include"), os.path.join(d, "include"))
        for fname in ([] if rev else EXTRA.get(name, [])):
            shutil.copy(os.path.join(HERE, fname), src)
        for fname, old, new in ([] if rev else PATCHES[name]):
            k = os.path.join(src, fname)
            text = open(k).read()
            assert text.count(old) == 1, f"patch site not found in {fname}"
            open(k, "w").write(text.replace(old, new))
        hipcc = B._hipcc()
        srcs = sorted(glob.glob(os.path.join(src, "*.hip")))
        objs = [s + ".o" for s in srcs]

        def cc(s):
            subprocess.run([hipcc, *B.CXXFLAGS, *FLAGS.get(name, []), "-c", s, "-o", s + ".o"], check=True)

        with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
            list(ex.map(cc, srcs))
        subprocess.run([hipcc, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", out, *objs, "-ldl",
                        f"-Wl,-rpath,{B.ROCM_LIB}"], check=True)
    print(out)


if __name__ == "__main__":
    main()
