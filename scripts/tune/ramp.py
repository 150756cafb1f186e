#!/usr/bin/env python3
"""Cold-start ramp of one kernel variant, with the shader clock beside it
(tuning only, not part of the product).

  python scripts/tune/ramp.py VARIANT [LAUNCHES]

VARIANT: a tune_decim id (70 = the product headline shape, 71 = its memory
path only, 73 = its compute path only on L2-resident input), "prod" (the
product library's FilterDnsamplingFir.step), "prodT<n>" (the same at M = 4
with an n-tap filter: the tap loop's share of the energy varies, the bytes do
not), "w:<workload>" (one step of a
bench.py workload: w:mixdecim, w:ci16decim, w:up, w:corr, w:fir), "read"
(read-only stream) or "copy" (4:1 coalesced stream).  A one-lane clock probe runs on a second
stream for the whole run; every launch's kernel time is printed with the mean
shader clock over its span.  Run each variant in a fresh process.
"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
import srcdsp_amd as S  # noqa: E402
from srcdsp_amd.design import hamming_sinc  # noqa: E402

lib = C.CDLL(os.path.join(HERE, "libtune.so"))
lib.tune_decim.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_long, C.c_void_p,
                           C.c_void_p, C.c_void_p]
lib.tune_stream_probe2.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_long, C.c_void_p]
lib.tune_clock_probe.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
lib.tune_realtime_stamp.argtypes = [C.c_void_p, C.c_void_p]


def main():
    var = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    L = 1 << 28
    x = torch.empty(L, dtype=torch.complex64, device="cuda")
    S.fill_synthetic(x, "cf32")
    y = torch.empty(L // 4, dtype=torch.complex64, device="cuda")
    h0 = torch.zeros(126, dtype=torch.complex64, device="cuda")
    h1 = torch.zeros(126, dtype=torch.complex64, device="cuda")
    c = hamming_sinc(127)
    cdev = torch.from_numpy(c).cuda()
    f = S.FilterDnsamplingFir(c, 4)
    main_s = torch.cuda.current_stream()
    st = C.c_void_p(main_s.cuda_stream)
    side = torch.cuda.Stream()
    nst = 20000
    gap = 2000  # 20 us at 100 MHz -> 400 ms of coverage
    stamps = torch.zeros(2 * nst, dtype=torch.int64, device="cuda")
    t0buf = torch.zeros(1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()

    # VARIANT may be a sequence "A*n,B*m,...": n launches of A, then m of B
    # (e.g. "70*8,71*40": the memory path timed at the clock the product left)
    seq = []
    for part in var.split(","):
        v, _, k = part.partition("*")
        seq += [v] * (int(k) if k else n)
    n = len(seq)

    # bench.py workloads (the product path), built before anything is timed
    works = {}
    for v in set(seq):
        if v.startswith("w:"):
            import importlib.util
            spec = importlib.util.spec_from_file_location("bench", os.path.join(HERE, "..", "..", "bench.py"))
            bench = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(bench)
            n_w = (1 << 26) if v[2:] in ("corr", "up") else (1 << 28)
            works[v] = bench.WORKLOADS[v[2:]](S, torch, n_w, 1, 0, "fma")
    fT = {v: S.FilterDnsamplingFir(hamming_sinc(int(v[5:])), 4) for v in set(seq) if v.startswith("prodT")}
    torch.cuda.synchronize()

    def launch(var):
        if var.startswith("w:"):  # one step of a bench.py workload, e.g. w:mixdecim
            works[var].step()
        elif var == "prod":
            f.step(x, y)
        elif var in fT:
            fT[var].step(x, y)
        elif var == "read":
            lib.tune_stream_probe2(1, 8192, C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), L, st)
        elif var == "copy":
            lib.tune_stream_probe2(0, 8192, C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), L, st)
        else:
            lib.tune_decim(int(var), int(os.environ.get("RAMP_GRID", "1024")), C.c_void_p(cdev.data_ptr()), C.c_void_p(x.data_ptr()),
                           C.c_void_p(y.data_ptr()), L, C.c_void_p(h0.data_ptr()), C.c_void_p(h1.data_ptr()), st)

    lib.tune_clock_probe(C.c_void_p(stamps.data_ptr()), nst, gap, C.c_void_p(side.cuda_stream))
    # let the probe record the idle clock for ~10 ms first
    lib.tune_realtime_stamp(C.c_void_p(t0buf.data_ptr()), st)
    torch.cuda._sleep(int(10e6))  # busy-wait kernel on the main stream (cycles, approximate)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    lib.tune_realtime_stamp(C.c_void_p(t0buf.data_ptr()), st)
    for i in range(n):
        ev[i][0].record(main_s)
        launch(seq[i])
        ev[i][1].record(main_s)
    torch.cuda.synchronize()
    # the last launch's output against a fresh product filter (zero history,
    # like the tuning launches): every variant must stay bit-exact
    bitexact = None
    if seq[-1].isdigit():
        ref = S.FilterDnsamplingFir(c, 4).step(x)
        torch.cuda.synchronize()
        bitexact = bool(torch.equal(torch.view_as_real(ref).view(torch.int32), torch.view_as_real(y).view(torch.int32)))
    ms = np.array([a.elapsed_time(b) for a, b in ev])
    start_ms = np.array([ev[0][0].elapsed_time(a) for a, _ in ev])
    s = stamps.view(-1, 2).cpu().numpy().astype(np.float64)
    r0 = float(t0buf.item())
    s = s[s[:, 1] > 0]
    rt_ms = (s[:, 1] - r0) / 1e5  # 100 MHz ticks -> ms since the stamp before launch 0
    clk = np.diff(s[:, 0]) / np.diff(s[:, 1]) * 0.1  # GHz
    mid = 0.5 * (rt_ms[1:] + rt_ms[:-1])
    ghz = []
    for a, d in zip(start_ms, ms):
        sel = (mid >= a) & (mid < a + d)
        ghz.append(float(np.mean(clk[sel])) if sel.any() else float("nan"))
    idle = clk[mid < -1.0]
    out = {"variant": var, "launches": n, "bitexact_vs_product": bitexact, "idle_ghz": round(float(np.median(idle)), 3) if idle.size else None,
           "ms": [round(float(v), 4) for v in ms], "ghz": [round(v, 3) for v in ghz],
           "ms_6_25": round(float(np.mean(ms[5:25])), 4), "ms_last100": round(float(np.mean(ms[-100:])), 4),
           "ghz_6_25": round(float(np.nanmean(ghz[5:25])), 3), "ghz_last100": round(float(np.nanmean(ghz[-100:])), 3)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
