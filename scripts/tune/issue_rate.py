#!/usr/bin/env python3
"""Per-instruction VALU issue cost on gfx950 (scripts/tune/libissue.so; tuning
only, not part of the product).  Prints, per instruction and waves per SIMD,
the cycles one wave spends per instruction (s_memtime) and the SIMD throughput
in lanes per cycle, i.e. the per-clock peak a roofline should be priced on."""
import ctypes as C
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = C.CDLL(os.path.join(HERE, "libissue.so"))
lib.tune_issue_rate.argtypes = [C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
NAMES = ["v_fmac_f32", "v_pk_fma_f32", "v_dot2c_i32_i16", "v_dot2_i32_i16", "v_mad_i32_i24", "v_fma_f32",
         "v_add_u32"]
CUS = 256


def main():
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for mode, name in enumerate(NAMES):
        for wps in (1, 2, 4, 8):
            iters = 40000 // wps  # ~the same kernel length at every occupancy
            blocks = CUS * wps  # 256-thread blocks: one wave per SIMD each
            cyc = torch.zeros(blocks * 16, dtype=torch.int64, device="cuda")
            sink = torch.zeros(blocks * 256, dtype=torch.int32, device="cuda")
            for _ in range(3):
                rc = lib.tune_issue_rate(mode, blocks, iters, C.c_void_p(cyc.data_ptr()), C.c_void_p(sink.data_ptr()),
                                         st)
                assert rc == 0, rc
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            lib.tune_issue_rate(mode, blocks, iters, C.c_void_p(cyc.data_ptr()), C.c_void_p(sink.data_ptr()), st)
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b)
            c = cyc.cpu().numpy().astype(np.float64).reshape(-1, 4)
            ghz = np.median((c[:, 1] - c[:, 0]) / (c[:, 3] - c[:, 2])) * 0.1
            span_ns = (c[:, 3].max() - c[:, 2].min()) * 10.0  # realtime ticks are 10 ns
            n_instr = iters * (8 if mode == 1 else 16)  # per wave
            simd_cyc = span_ns * ghz  # shader cycles of the whole loop span
            per_simd = wps * n_instr / simd_cyc  # wave-instructions per cycle per SIMD
            ops = blocks * 256 * iters * 16
            print(f"{name:16s} waves/SIMD={wps}: {1 / per_simd:5.2f} cyc per wave-instr per SIMD "
                  f"({64 * per_simd:5.1f} lanes/cyc), clock {ghz:.2f} GHz, "
                  f"{ops / (ms * 1e-3) / 1e12:6.2f} T ops/s ({ms:.3f} ms)", flush=True)


if __name__ == "__main__":
    main()
