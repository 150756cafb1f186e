#!/usr/bin/env python3
"""Interleaved A/B timing of decimator kernel variants and the FMA issue rate
(scripts/tune/libtune.so; not part of the product).  Prints a table."""
import ctypes as C
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from srcdsp_amd.design import hamming_sinc  # noqa: E402
import srcdsp_amd as S  # noqa: E402

lib = C.CDLL(os.path.join(HERE, "libtune.so"))
lib.tune_fma_rate.argtypes = [C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
lib.tune_decim.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_long, C.c_void_p,
                           C.c_void_p, C.c_void_p]


def timeit(fn, reps=10):
    st = torch.cuda.current_stream()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        fn()
        b.record(st)
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return np.median(ts), np.min(ts)


def main():
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    out = torch.empty(256 * 256 * 16, device="cuda")
    iters = 4000
    print("FMA issue rate (16 chains/lane):")
    for mode in (0, 1):
        for wps in (1, 2, 4, 8):
            blocks = 256 * wps  # 256-thread blocks: 4 waves = 1 per SIMD
            fn = lambda: lib.tune_fma_rate(mode, blocks, iters, C.c_void_p(out.data_ptr()), stream)
            fn()
            med, mn = timeit(fn, 5)
            fmas = blocks * 256 * iters * 16
            print(f"  {'v_fmac_f32' if mode == 0 else 'v_pk_fma_f32'} waves/SIMD={wps}: "
                  f"{fmas / (mn * 1e-3) / 1e12:7.2f} TFMA/s  ({med:.3f} ms)")

    L = 1 << 28
    x = torch.empty(L, dtype=torch.complex64, device="cuda")
    S.fill_synthetic(x, "cf32")
    y = torch.empty(L // 4, dtype=torch.complex64, device="cuda")
    ref = torch.empty_like(y)
    h0 = torch.zeros(126, dtype=torch.complex64, device="cuda")
    h1 = torch.zeros(126, dtype=torch.complex64, device="cuda")
    c = hamming_sinc(127)
    cdev = torch.from_numpy(c).cuda()
    S.FilterDnsamplingFir(c, 4).step(x, ref)
    variants = [(0, 0, "tile R8 B256"), (1, 0, "tile R4 B256"), (2, 0, "tile R8 B128"),
                (3, 256, "stream R8 B256 g256"), (3, 512, "stream R8 B256 g512"),
                (4, 512, "stream R4 B256 g512"), (4, 1024, "stream R4 B256 g1024"), (4, 2048, "stream R4 B256 g2048"),
                (5, 512, "stream R8 B128 g512"), (5, 1024, "stream R8 B128 g1024"),
                (6, 1024, "stream R8 B64 g1024"), (6, 2048, "stream R8 B64 g2048"),
                (7, 512, "stream R6 B256 g512"), (7, 768, "stream R6 B256 g768")]
    res = {v: [] for v in variants}
    for rnd in range(5):
        for v in variants:
            fn = lambda: lib.tune_decim(v[0], v[1], C.c_void_p(cdev.data_ptr()), C.c_void_p(x.data_ptr()),
                                        C.c_void_p(y.data_ptr()), L, C.c_void_p(h0.data_ptr()),
                                        C.c_void_p(h1.data_ptr()), stream)
            if rnd == 0:
                print("checking", v[2], flush=True)
                y.zero_()
                fn()
                torch.cuda.synchronize()
                ok = torch.equal(y.view(torch.float32), ref.view(torch.float32))
                res[v].append(("ok" if ok else "MISMATCH"))
            med, mn = timeit(fn, 5)
            res[v].append(mn)
    print(f"decimator cf32 M=4 127 taps, 2^28 samples (min over rounds):")
    for v in variants:
        tmin = min(t for t in res[v][1:])
        gbs = 10 * L / (tmin * 1e-3) / 1e9
        print(f"  {v[2]:24s} {res[v][0]:8s} {tmin:.4f} ms  {L / tmin / 1e6:8.1f} Gsamp/s  {gbs:7.1f} GB/s "
              f"({gbs / 8000 * 100:.1f}% of 8 TB/s)")


if __name__ == "__main__":
    main()
