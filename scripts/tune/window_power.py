#!/usr/bin/env python3
"""Socket power, shader clock and the firmware's limiter residency counters
through the driver's window (launches 6-25 of a cold start) of the headline
(tuning only; read-only amdsmi queries, no setting touched).

  python scripts/tune/window_power.py [LAUNCHES] [IDLE_S] [TAPS | w:WORKLOAD]

TAPS: the headline at M = 4 with an n-tap filter (default 127); w:WORKLOAD: one
step of a bench.py workload instead (w:mixdecim, w:ci16decim, w:up, w:corr,
w:fir, w:decim).

One fresh process: build the headline operator, idle IDLE_S seconds (default
8), then LAUNCHES (default 300) back-to-back FilterDnsamplingFir.step() calls
on 2^28 samples with HIP events around each.  A sampler thread polls
amdsmi_get_gpu_metrics_info as fast as it returns for the whole run (the
launches queue behind a one-thread spin of ~0.1 s, so the GIL the sampler
holds cannot open gaps between them); every
sample is placed on the launch timeline (the events' offsets from a start
event recorded on an idle queue, i.e. host time ~= device time), so each
launch gets the power/clock samples that fall inside it.  The violation /
throttle accumulators (PPT, thermal, ...) are read before and after, and per
sample, so the limiter that engages in the window is named by the counter
that moves there.

Prints one JSON line (per-phase means: launches 1-5, 6-25, 26-100, 101-end)
and writes the full sample series to gpurun_out/window_power_<taps>.jsonl."""
import json
import os
import sys
import threading
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..", "..")
sys.path.insert(0, ROOT)
import srcdsp_amd as S  # noqa: E402
from srcdsp_amd.design import hamming_sinc  # noqa: E402
import amdsmi  # noqa: E402

KEEP = ("power", "clk", "throttle", "residency", "acc", "temperature_hotspot", "activity", "violation", "ppt",
        "thm", "prochot", "voltage", "curr")


def flat(m):
    out = {}
    for k, v in m.items():
        if not any(s in k for s in KEEP):
            continue
        if isinstance(v, (int, float)):
            out[k] = v
        elif isinstance(v, list) and "clk" in k:
            out[k] = v[:8]
    return out


def sampler(h, out, stop):
    while not stop.is_set():
        t0 = time.perf_counter()
        try:
            m = flat(amdsmi.amdsmi_get_gpu_metrics_info(h))
        except Exception as e:  # noqa: BLE001
            m = {"err": str(e)[:80]}
        t1 = time.perf_counter()
        m["t"] = 0.5 * (t0 + t1)
        m["dt_call"] = t1 - t0
        out.append(m)


def num(x):
    try:
        v = float(x)
        return v if v < 1e15 else float("nan")  # 0xFFFF.. = not supported
    except (TypeError, ValueError):
        return float("nan")


def violation(h):
    try:
        v = amdsmi.amdsmi_get_violation_status(h)
        return {k: (x if isinstance(x, (int, float, str)) else str(x)) for k, x in v.items()}
    except Exception as e:  # noqa: BLE001
        return {"err": str(e)[:120]}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    idle_s = float(sys.argv[2]) if len(sys.argv) > 2 else 8.0
    arg = sys.argv[3] if len(sys.argv) > 3 else "127"
    amdsmi.amdsmi_init()
    h = amdsmi.amdsmi_get_processor_handles()[0]
    if arg.startswith("w:"):
        import bench
        wl = arg[2:]
        L = (1 << 26) if wl == "corr" else (1 << 28)
        work = bench.WORKLOADS[wl](S, torch, L, 1, 0, "fma")
        step = work.step
        step()  # code objects loaded before the idle pause
        taps = wl
    else:
        taps = int(arg)
        L = 1 << 28
        x = torch.empty(L, dtype=torch.complex64, device="cuda")
        S.fill_synthetic(x, "cf32")
        y = torch.empty(L // 4, dtype=torch.complex64, device="cuda")
        f = S.FilterDnsamplingFir(hamming_sinc(taps), 4)
        f.step(x[: 1 << 16], y[: 1 << 14])  # load the code object; negligible work
        step = lambda: f.step(x, y)  # noqa: E731
    torch.cuda.synchronize()
    recs, stop = [], threading.Event()
    th = threading.Thread(target=sampler, args=(h, recs, stop), daemon=True)
    th.start()
    time.sleep(idle_s)
    v0 = violation(h)
    e0 = torch.cuda.Event(enable_timing=True)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    t_host0 = time.perf_counter()
    e0.record()
    # one thread spinning ~0.1 s holds the queue while the host enqueues every
    # launch (the sampler thread competes for the GIL), so the launches run
    # back to back; it draws idle power
    torch.cuda._sleep(int(2e8))
    for a, b in ev:
        a.record()
        step()
        b.record()
    torch.cuda.synchronize()
    t_end = time.perf_counter()
    time.sleep(0.3)
    stop.set()
    th.join()
    v1 = violation(h)
    amdsmi.amdsmi_shut_down()
    # launch spans on the host clock
    spans = [(t_host0 + e0.elapsed_time(a) * 1e-3, t_host0 + e0.elapsed_time(b) * 1e-3) for a, b in ev]
    ms = np.array([a.elapsed_time(b) for a, b in ev])
    for r in recs:
        r["launch"] = next((i + 1 for i, (s0, s1) in enumerate(spans) if s0 <= r["t"] <= s1), None)
        r["rel_ms"] = (r["t"] - t_host0) * 1e3
    keys = sorted({k for r in recs for k in r if k not in ("t", "launch", "rel_ms", "err")})

    def phase(lo, hi):
        rs = [r for r in recs if r["launch"] is not None and lo <= r["launch"] <= hi]
        d = {"launches": f"{lo}-{hi}", "ms": round(float(ms[lo - 1:hi].mean()), 4), "samples": len(rs)}
        for k in keys:
            vals = [num(r.get(k)) for r in rs if not isinstance(r.get(k), (list, str))]
            vals = [v for v in vals if v == v]
            if vals:
                d[k] = round(float(np.mean(vals)), 2)
        return d

    idle = [r for r in recs if r["t"] < t_host0 - 0.5]
    idle_d = {k: round(float(np.nanmean([num(r.get(k)) for r in idle])), 2) for k in keys
              if any(num(r.get(k)) == num(r.get(k)) for r in idle)}
    out = {"taps": taps, "launches": n, "idle_s": idle_s, "samples": len(recs),
           "sample_period_ms": round(1e3 * float(np.median(np.diff([r["t"] for r in recs]))), 3),
           "idle": idle_d, "phases": [phase(1, 5), phase(6, 25), phase(26, 100), phase(101, n)],
           "violation_before": v0, "violation_after": v1, "run_s": round(t_end - t_host0, 4)}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"window_power_{taps}.jsonl"), "w") as fo:
        for r in recs:
            if r["t"] >= t_host0 - 0.05 and r["t"] <= t_end + 0.05:
                fo.write(json.dumps(r) + "\n")
        fo.write(json.dumps({"launch_ms": [round(v, 4) for v in ms.tolist()],
                             "launch_start_rel_ms": [round((s0 - t_host0) * 1e3, 4) for s0, _ in spans]}) + "\n")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
