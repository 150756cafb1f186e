#!/usr/bin/env python3
"""Interleaved A/B timing of decimator kernel variants and the FMA issue rate
(scripts/tune/libtune.so; not part of the product).  Prints a table."""
import ctypes as C
import os
import time
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from srcdsp_amd.design import hamming_sinc  # noqa: E402
import srcdsp_amd as S  # noqa: E402

lib = C.CDLL(os.path.join(HERE, "libtune.so"))
_old = os.path.join(HERE, "libtune_old.so")  # optional A/B baseline: the previous headline kernel
lib_old = C.CDLL(_old) if os.path.exists(_old) else None


def tune_decim(variant, grid, *args):
    """variant < 0: the previous headline kernel from libtune_old.so"""
    if variant < 0:
        return lib_old.tune_decim_old(grid, *args)
    return lib.tune_decim(variant, grid, *args)
lib.tune_fma_rate.argtypes = [C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
if lib_old is not None:
    lib_old.tune_decim_old.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_long, C.c_void_p,
                                       C.c_void_p, C.c_void_p]
lib.tune_mfma4x4_probe.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
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
    for mode in ((0, 1) if os.environ.get("TUNE_FMA") else ()):
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
    lib.tune_stream_probe.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_long, C.c_void_p]
    for blocks in (() if not os.environ.get("TUNE_PROBES") else (1024, 2048, 4096, 8192)):
        fn = lambda: lib.tune_stream_probe(blocks, C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), L, stream)
        fn()
        med, mn = timeit(fn, 10)
        print(f"  streaming ceiling probe (8 B in / 2 B out per sample), {blocks} blocks: {mn:.4f} ms "
              f"-> {10 * L / (mn * 1e-3) / 1e9:.1f} GB/s")
    lib.tune_stream_probe2.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_long, C.c_void_p]
    for mode, label, bps in (((0, "coalesced 4:1 stream (10 B/sample)", 10), (1, "read-only stream (8 B/sample)", 8))
                             if os.environ.get("TUNE_PROBES") else ()):
        for blocks in (2048, 4096, 8192, 16384):
            fn = lambda: lib.tune_stream_probe2(mode, blocks, C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), L,
                                                stream)
            fn()
            med, mn = timeit(fn, 10)
            print(f"  {label}, {blocks} blocks: {mn:.4f} ms -> {bps * L / (mn * 1e-3) / 1e9:.1f} GB/s")
    variants = [(48, 1024, "product (nt/nt builtin)"), (60, 1024, "ld 2 st 2 (buffer)"), (61, 1024, "ld 2 st 3"),
                (62, 1024, "ld 3 st 2"), (63, 1024, "ld 3 st 3"), (64, 1024, "ld 18 st 18"), (65, 1024, "ld 2 st 19"),
                (66, 1024, "ld 19 st 2")]
    if os.environ.get("TUNE_OCC"):  # workgroups per CU; PROBE1 = memory path only (no correctness check)
        variants = [(-1, 1024, "previous head g1024"), (48, 1024, "head g1024"), (48, 512, "head g512"),
                    (80, 1024, "PROBE1 512 g1024"), (80, 512, "PROBE1 512 g512"), (90, 256, "PROBE1 512 mw2 g256"),
                    (84, 1024, "PROBE1 256 g1024"), (88, 1024, "256 lanes g1024"), (48, 1024, "head g1024 (again)"),
                    (-1, 1024, "previous head g1024 (again)")]
    if os.environ.get("TUNE_COMPUTE"):  # PROBE2 = compute path only (L2-resident input)
        variants = [(48, 1024, "head g1024"), (110, 1024, "PROBE2 512 mw4 g1024"), (114, 1024, "PROBE3 (no tap loads) g1024"),
                    (110, 512, "PROBE2 512 mw4 g512"),
                    (111, 256, "PROBE2 512 mw2 g256"), (112, 256, "PROBE2 1024 mw4 g256"),
                    (113, 256, "1024 mw4 g256"), (90, 256, "PROBE1 512 mw2 g256"), (80, 1024, "PROBE1 512 g1024")]
    if os.environ.get("TUNE_R8"):  # 8 outputs per lane (half the LDS reads per output), 2 waves/SIMD
        variants = [(48, 1024, "head g1024"), (120, 512, "R8 256 g512"), (120, 1024, "R8 256 g1024"),
                    (121, 512, "PROBE2 R8 256 g512"), (122, 256, "R8 512 g256"), (123, 1024, "R8 128 g1024"),
                    (123, 2048, "R8 128 g2048"), (110, 1024, "PROBE2 head g1024"), (48, 1024, "head g1024 (again)")]
    if os.environ.get("TUNE_OST"):  # output store shapes: LDS staging (product) vs permlane32 pairing vs none
        variants = [(48, 1024, "head g1024"), (70, 1024, "OST2 g1024"), (70, 512, "OST2 g512"),
                    (72, 256, "OST2 mw2 g256"), (72, 512, "OST2 mw2 g512"), (74, 1024, "OST2 256 g1024"),
                    (74, 2048, "OST2 256 g2048"), (75, 1024, "OST0 g1024"),
                    (71, 1024, "PROBE1 OST2 g1024"), (73, 1024, "PROBE2 OST2 g1024"), (110, 1024, "PROBE2 head g1024"),
                    (48, 1024, "head g1024 (again)"), (70, 1024, "OST2 g1024 (again)")]
    if os.environ.get("TUNE_W12"):  # 12 waves per CU (2 x 384 or 1 x 768 lanes); PROBE1 = memory path only
        variants = [(70, 1024, "head (OST2) g1024"), (92, 512, "384 mw3 g512"), (92, 1024, "384 mw3 g1024"),
                    (96, 512, "384 mw4 g512"), (93, 256, "768 mw3 g256"), (93, 512, "768 mw3 g512"),
                    (94, 512, "PROBE1 384 mw3 g512"), (95, 256, "PROBE1 768 mw3 g256"), (71, 1024, "PROBE1 head g1024"),
                    (70, 1024, "head (again)")]
    if os.environ.get("TUNE_ILV"):  # tap-major pk_fma issue order (inline asm) vs the compiler's order
        variants = [(70, 1024, "head g1024"), (200, 1024, "ILV g1024"), (73, 1024, "PROBE2 head g1024"),
                    (201, 1024, "PROBE2 ILV g1024"), (202, 512, "ILV mw2 g512"), (202, 256, "ILV mw2 g256"),
                    (203, 2048, "ILV 256 g2048"), (204, 512, "ILV R8 mw2 g512"), (204, 256, "ILV R8 mw2 g256"),
                    (71, 1024, "PROBE1 head g1024"), (70, 1024, "head (again)"), (200, 1024, "ILV (again)")]
    if os.environ.get("TUNE_MFMA"):  # matrix-core decimator (decim_mfma.h) vs the VALU headline
        variants = [(70, 1024, "head g1024"), (300, 512, "MFMA mw2 g512"), (73, 1024, "PROBE2 head g1024"),
                    (301, 512, "PROBE2 MFMA g512"), (302, 512, "PROBE1 MFMA g512"), (71, 1024, "PROBE1 head g1024"),
                    (300, 1024, "MFMA mw2 g1024"), (303, 768, "MFMA mw3 g768"), (304, 768, "PROBE2 MFMA mw3 g768"),
                    (70, 1024, "head (again)"),
                    (300, 512, "MFMA (again)")]
    if os.environ.get("TUNE_FIR"):
        fir_ab()
        return
    if os.environ.get("TUNE_SUSTAINED_ONLY"):
        sustained_rounds(variants, x, y, cdev, h0, h1, stream, L, ref)
        return
    res = {v: [] for v in variants}
    for rnd in range(int(os.environ.get('TUNE_ROUNDS', '6'))):
        for v in variants:
            fn = lambda: tune_decim(v[0], v[1], C.c_void_p(cdev.data_ptr()), C.c_void_p(x.data_ptr()),
                                        C.c_void_p(y.data_ptr()), L, C.c_void_p(h0.data_ptr()),
                                        C.c_void_p(h1.data_ptr()), stream)
            if rnd == 0:
                print("checking", v[2], flush=True)
                y.zero_()
                fn()
                torch.cuda.synchronize()
                ok = torch.equal(y.view(torch.int32), ref.view(torch.int32))  # bytes, not float ==
                res[v].append(("ok" if ok else ("n/a" if "PROBE" in v[2] else "MISMATCH")))
            med, mn = timeit(fn, 5)
            res[v].append(mn)
    print(f"decimator cf32 M=4 127 taps, 2^28 samples (min over rounds):")
    for v in variants:
        tmin = min(t for t in res[v][1:])
        gbs = 10 * L / (tmin * 1e-3) / 1e9
        print(f"  {v[2]:28s} {res[v][0]:8s} {tmin:.4f} ms  {L / tmin / 1e6:8.1f} Gsamp/s  {gbs:7.1f} GB/s "
              f"({gbs / 8000 * 100:.1f}% of 8 TB/s)")
    sustained(variants, x, y, cdev, h0, h1, stream, L)


def fir_ab(rounds=4, reps=30):
    """FilterFir stream kernel (31 taps, 2^28 samples): LDS-staged vs lane-transposed output stores."""
    lib.tune_fir.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_long, C.c_int, C.c_uint,
                             C.c_void_p, C.c_void_p, C.c_void_p]
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    L = 1 << 28
    c = hamming_sinc(31, 0.2)
    cdev = torch.from_numpy(c.astype(np.float32)).cuda()
    h0 = torch.zeros(64, dtype=torch.complex64, device="cuda")
    h1 = torch.zeros(64, dtype=torch.complex64, device="cuda")
    cases = []
    for kin, var0 in (("float", 0),):  # the complex<float> variants left fir_stream_f32 (tune.hip)
        if kin == "float":
            x = torch.randint(-2048, 2048, (L,), device="cuda").float()
        else:
            x = torch.randint(-2048, 2048, (L, 2), device="cuda").float().view(torch.complex64).view(-1)
        ref = S.FilterFir(c, kin, "complex<float>", kin, "float").step(x)
        y = torch.empty(L, dtype=torch.complex64, device="cuda")
        shift = None
        for sh in range(0, 8):
            y.zero_()
            lib.tune_fir(var0, 2048, cdev.data_ptr(), x.data_ptr(), y.data_ptr(), L, 31, sh, h0.data_ptr(),
                         h1.data_ptr(), stream)
            torch.cuda.synchronize()
            if torch.equal(y.view(torch.int32), ref.view(torch.int32)):
                shift = sh
                break
        assert shift is not None, "no shift reproduces the product FIR"
        for v in (var0, var0 + 1):
            y.zero_()
            lib.tune_fir(v, 2048, cdev.data_ptr(), x.data_ptr(), y.data_ptr(), L, 31, shift, h0.data_ptr(),
                         h1.data_ptr(), stream)
            torch.cuda.synchronize()
            assert torch.equal(y.view(torch.int32), ref.view(torch.int32)), (kin, v)
            cases.append((kin, v, x, y, shift))
    st = torch.cuda.current_stream()
    res = {(k, v): [] for k, v, *_ in cases}
    for rnd in range(rounds):
        for kin, v, x, y, shift in cases:
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
            for i in range(reps):
                ev[i][0].record(st)
                lib.tune_fir(v, 2048, cdev.data_ptr(), x.data_ptr(), y.data_ptr(), L, 31, shift, h0.data_ptr(),
                             h1.data_ptr(), stream)
                ev[i][1].record(st)
            torch.cuda.synchronize()
            res[(kin, v)].append(float(np.median([a.elapsed_time(b) for a, b in ev][-20:])))
    print("FilterFir stream kernel, 31 taps, 2^28 samples (bit-exact vs the product checked); "
          f"{rounds} interleaved rounds x {reps} launches, median of last 20:")
    for (kin, v), r in res.items():
        bps = 12 if kin == "float" else 16
        print(f"  {kin:15s} {'LDS-staged stores' if v % 2 == 0 else 'lane-transposed stores':24s} "
              f"min {min(r):.4f} median {np.median(r):.4f} ms -> {bps * L / (np.median(r) * 1e-3) / 1e9:7.1f} GB/s "
              f"rounds {' '.join(f'{t:.4f}' for t in r)}", flush=True)


def sustained_rounds(variants, x, y, cdev, h0, h1, stream, L, ref, rounds=4, reps=30):
    """Interleaved rounds of back-to-back launches (the bench's pattern): per
    round and variant the median of the last 20 launches; min/median over rounds."""
    res = {v: [] for v in variants}
    for v in variants:  # correctness first
        if "PROBE" in v[2]:
            continue
        y.zero_()
        tune_decim(v[0], v[1], C.c_void_p(cdev.data_ptr()), C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()),
                       L, C.c_void_p(h0.data_ptr()), C.c_void_p(h1.data_ptr()), stream)
        torch.cuda.synchronize()
        eq = y.view(torch.int32) == ref.view(torch.int32)
        if not bool(eq.all()):
            bad = (~eq).nonzero().flatten()
            print(f"MISMATCH {v[2]}: {bad.numel()} words differ, first {bad[:8].tolist()}", flush=True)
        else:
            print(f"bit-exact {v[2]}", flush=True)
    st = torch.cuda.current_stream()
    for rnd in range(rounds):
        for v in variants:
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
            for i in range(reps):
                ev[i][0].record(st)
                tune_decim(v[0], v[1], C.c_void_p(cdev.data_ptr()), C.c_void_p(x.data_ptr()),
                               C.c_void_p(y.data_ptr()), L, C.c_void_p(h0.data_ptr()), C.c_void_p(h1.data_ptr()),
                               stream)
                ev[i][1].record(st)
            torch.cuda.synchronize()
            res[v].append(float(np.median([a.elapsed_time(b) for a, b in ev][-20:])))
    print(f"sustained, {rounds} interleaved rounds x {reps} launches (median of last 20 per round):", flush=True)
    for v in variants:
        r = res[v]
        print(f"  {v[2]:32s} min {min(r):.4f}  median {np.median(r):.4f} ms -> {10 * L / (np.median(r) * 1e-3) / 1e9:7.1f} GB/s"
              f"  rounds {' '.join(f'{t:.4f}' for t in r)}", flush=True)


def sustained(variants, x, y, cdev, h0, h1, stream, L, reps=60):
    print("sustained back-to-back (60 launches each; median of last 20, first 5):")
    for v in variants:
        st = torch.cuda.current_stream()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for i in range(reps):
            ev[i][0].record(st)
            tune_decim(v[0], v[1], C.c_void_p(cdev.data_ptr()), C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()),
                           L, C.c_void_p(h0.data_ptr()), C.c_void_p(h1.data_ptr()), stream)
            ev[i][1].record(st)
        torch.cuda.synchronize()
        t = [a.elapsed_time(b) for a, b in ev]
        print(f"  {v[2]:28s} first5 {np.median(t[:5]):.4f} ms  last20 {np.median(t[-20:]):.4f} ms "
              f"-> {10 * L / (np.median(t[-20:]) * 1e-3) / 1e9:7.1f} GB/s")
        time.sleep(2)


if __name__ == "__main__":
    main()
