#!/usr/bin/env python3
"""Per-phase shader cycles of the fused mixer -> decimator kernel
(decim_dot2_ci16<MIX>, config 4) from the tuning build with
-DSRCDSP_PHASE_CLOCK (tuning only).

  SRCDSP_HIP_LIB=scripts/tune/ab/libsrcdsp_hip_phase.so \\
      python scripts/tune/phase_clock.py [WORKLOAD] [LAUNCHES]

Runs bench.py's workload (default mixdecim) warm for 100 launches, then
LAUNCHES (default 100) launches with the phase sums cleared before, and
prints one JSON line: cycles per wave-tile in each phase, their shares, and
the mean launch time (instrumented, so somewhat slower than the product).
Build the library with `python -m srcdsp_amd.build phase SRCDSP_TUNING
SRCDSP_PHASE_CLOCK`."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import srcdsp_amd as S  # noqa: E402

NAMES = ["prologue", "wait_pre_stage", "stage_mix", "wait_post_stage", "taps_quant", "store"]


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "mixdecim"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    lib = S.lib()
    fn = lib.srcdsp_tune_phase_clock
    fn.argtypes = [C.c_void_p]
    work = bench.WORKLOADS[wl](S, torch, 1 << 28, 1, 0, "fma")
    for _ in range(100):
        work.step()
    buf = (C.c_ulonglong * 8)()
    assert fn(buf) == 0
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        work.step()
        b.record()
    torch.cuda.synchronize()
    assert fn(buf) == 0
    v = list(buf)
    waves, tiles = v[6], v[7]  # tiles: wave-tiles (each wave counts its tiles)
    per = {NAMES[k]: round(v[k] / max(tiles, 1), 1) for k in range(1, 6)}
    per["prologue_per_wave"] = round(v[0] / max(waves, 1), 1)
    tot = sum(v[1:6]) + v[0]
    share = {NAMES[k]: round(v[k] / tot, 4) for k in range(6)}
    ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    print(json.dumps({"workload": work.name, "launches": n, "waves": waves, "wave_tiles": tiles,
                      "cycles_per_wave_tile": per, "share": share, "ms_instrumented": round(ms, 4),
                      "cycles_per_wave_per_launch": round(tot / max(waves, 1), 1)}), flush=True)


if __name__ == "__main__":
    main()
