#!/usr/bin/env python3
"""Config 3's per-GPU share two ways on one box (tuning only): one batched
launch of C channels (srcdsp_decim_step_batched, grid.y = channel) against C
single-channel step() calls on the same stream, and one channel alone; the
per-channel kernel time of each, steady state (warm-up launches first), in
interleaved rounds.

  python scripts/tune/batched_ab.py [C] [rounds]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import srcdsp_amd as S  # noqa: E402
from srcdsp_amd.design import hamming_sinc  # noqa: E402


def timed(fn, warm, n):
    for _ in range(warm):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.mean([a.elapsed_time(b) for a, b in ev]))


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    L = 1 << 28
    c = hamming_sinc(127)
    x = torch.empty((C, L), dtype=torch.complex64, device="cuda")
    for k in range(C):
        S.fill_synthetic(x[k], "cf32", seed=0x5EED, channel=k)
    y = torch.empty((C, L // 4), dtype=torch.complex64, device="cuda")
    fs = [S.FilterDnsamplingFir(c, 4, fp="fma") for _ in range(C)]
    ways = {
        "batched": lambda: S.decim_step_batched(fs, x, y),
        "separate": lambda: [fs[k].step(x[k], y[k]) for k in range(C)],
        "one": lambda: fs[0].step(x[0], y[0]),
    }
    per = {"batched": C, "separate": C, "one": 1}
    for r in range(rounds):
        for name, fn in ways.items():
            n = 200 if name == "one" else 30
            ms = timed(fn, n // 2, n)
            print(json.dumps({"round": r, "way": name, "ms_per_step": round(ms, 4),
                              "ms_per_channel": round(ms / per[name], 4)}), flush=True)


if __name__ == "__main__":
    main()
