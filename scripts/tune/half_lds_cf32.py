#!/usr/bin/env python3
"""Tuning probe (never product): the headline kernel with HALF its tap-loop
LDS window reads.

Builds scripts/tune/ab/libsrcdsp_hip_halflds.so from a patched COPY of
srcdsp_amd/csrc (the product sources are not touched): in the compiled-tap
path of decim_stream_cf32 (decim_kernels.h, `load_group`), every odd window
group takes two opaque registers instead of its two ds_read_b128 -- the same
v_pk_fma_f32 work and the same memory schedule, wrong outputs.  Timed against
the product with scripts/tune/ab_libs.sh (LIBS="halflds new", WORKLOADS=decim)
under the driver's protocol, with scripts/tune/window_power.py's energy per
launch, it prices the LDS-read energy of the 127-tap loop: the ceiling of any
LDS-lighter variant (e.g. sharing the overlapping windows of neighbouring
lanes by DPP / permlane instead of re-reading them).

    python scripts/tune/half_lds_cf32.py
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

OLD = """            auto load_group = [&](int e) {
                const float4 g0 = rd(Bt + 2 * e + floordiv(2 * e, PR));
                const float4 g1 = rd(Bt + 2 * e + 1 + floordiv(2 * e + 1, PR));"""
NEW = """            auto load_group = [&](int e) {
                float4 g0, g1;
                if ((e & 1) == 0) {
                    g0 = rd(Bt + 2 * e + floordiv(2 * e, PR));
                    g1 = rd(Bt + 2 * e + 1 + floordiv(2 * e + 1, PR));
                } else {  // PROBE: no LDS read, two opaque registers
                    asm volatile("" : "=v"(g0.x), "=v"(g0.y), "=v"(g0.z), "=v"(g0.w));
                    asm volatile("" : "=v"(g1.x), "=v"(g1.y), "=v"(g1.z), "=v"(g1.w));
                }"""


def main():
    out = os.path.join(HERE, "ab", "libsrcdsp_hip_halflds.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "srcdsp_amd", "csrc")  # csrc includes ../../include/srcdsp_hip.h
        shutil.copytree(B.CSRC, src)
        shutil.copytree(os.path.join(ROOT, "include"), os.path.join(d, "include"))
        k = os.path.join(src, "decim_kernels.h")
        text = open(k).read()
        assert text.count(OLD) == 1, "probe patch site not found"
        open(k, "w").write(text.replace(OLD, NEW))
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
