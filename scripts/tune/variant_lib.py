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

  rev:<REV> the product sources of git revision REV, unpatched (e.g. rev:HEAD
           before a kernel change is committed); built as libsrcdsp_hip_<REV>.so

    python scripts/tune/variant_lib.py halflds|r4mix|rev:<REV>
"""
from __future__ import annotations

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


def main():
    name = sys.argv[1]
    rev = name[4:] if name.startswith("rev:") else None
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
        for fname, old, new in ([] if rev else PATCHES[name]):
            k = os.path.join(src, fname)
            text = open(k).read()
            assert text.count(old) == 1, f"patch site not found in {fname}"
            open(k, "w").write(text.replace(old, new))
        hipcc = B._hipcc()
        objs = []
        for s in sorted(glob.glob(os.path.join(src, "*.hip"))):
            o = s + ".o"
            subprocess.run([hipcc, *B.CXXFLAGS, "-c", s, "-o", o], check=True)
            objs.append(o)
        subprocess.run([hipcc, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", out, *objs, "-ldl",
                        f"-Wl,-rpath,{B.ROCM_LIB}"], check=True)
    print(out)


if __name__ == "__main__":
    main()
