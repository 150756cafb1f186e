#!/usr/bin/env python3
"""Socket power and shader clock while one decimator variant runs back to back
(tuning only; read-only amdsmi queries, no settings touched).

  python scripts/tune/power.py VARIANT [SECONDS]

Prints one JSON line: idle power before the run, and the mean socket power /
gfx clock / activity over the second half of the run (steady state), with the
mean kernel time over the same span."""
import ctypes as C
import json
import os
import sys
import threading
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
import srcdsp_amd as S  # noqa: E402
from srcdsp_amd.design import hamming_sinc  # noqa: E402
import amdsmi  # noqa: E402

lib = C.CDLL(os.path.join(HERE, "libtune.so"))
lib.tune_decim.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_long, C.c_void_p,
                           C.c_void_p, C.c_void_p]
lib.tune_stream_probe2.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_long, C.c_void_p]


def sampler(h, out, stop):
    while not stop.is_set():
        t = time.perf_counter()
        rec = {"t": t}
        try:
            p = amdsmi.amdsmi_get_power_info(h)
            rec["socket_w"] = p.get("current_socket_power", p.get("average_socket_power"))
            rec["avg_w"] = p.get("average_socket_power")
        except Exception as e:  # noqa: BLE001
            rec["err"] = str(e)[:80]
        try:
            m = amdsmi.amdsmi_get_gpu_metrics_info(h)
            rec["gfxclk"] = m.get("current_gfxclk") or m.get("average_gfxclk_frequency")
            rec["act"] = m.get("average_gfx_activity")
            rec["temp"] = m.get("temperature_hotspot")
        except Exception as e:  # noqa: BLE001
            rec["err2"] = str(e)[:80]
        out.append(rec)
        time.sleep(0.01)


def num(x):
    try:
        return float(x)
    except (TypeError, ValueError):
        return float("nan")


def main():
    var = sys.argv[1]
    secs = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
    amdsmi.amdsmi_init()
    h = amdsmi.amdsmi_get_processor_handles()[0]
    L = 1 << 28
    x = torch.empty(L, dtype=torch.complex64, device="cuda")
    S.fill_synthetic(x, "cf32")
    y = torch.empty(L // 4, dtype=torch.complex64, device="cuda")
    h0 = torch.zeros(126, dtype=torch.complex64, device="cuda")
    h1 = torch.zeros(126, dtype=torch.complex64, device="cuda")
    c = hamming_sinc(127)
    cdev = torch.from_numpy(c).cuda()
    f = S.FilterDnsamplingFir(c, 4)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)

    def launch():
        if var == "prod":
            f.step(x, y)
        elif var == "read":
            lib.tune_stream_probe2(1, 8192, C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), L, st)
        else:
            lib.tune_decim(int(var), int(os.environ.get("RAMP_GRID", "1024")), C.c_void_p(cdev.data_ptr()),
                           C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), L, C.c_void_p(h0.data_ptr()),
                           C.c_void_p(h1.data_ptr()), st)

    torch.cuda.synchronize()
    recs, stop = [], threading.Event()
    th = threading.Thread(target=sampler, args=(h, recs, stop), daemon=True)
    th.start()
    time.sleep(1.0)  # idle
    t_start = time.perf_counter()
    ev, n = [], 0
    while time.perf_counter() - t_start < secs:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        launch()
        b.record()
        ev.append((time.perf_counter(), a, b))
        n += 1
        if n % 20 == 0:
            b.synchronize()
    torch.cuda.synchronize()
    t_end = time.perf_counter()
    stop.set()
    th.join()
    mid = t_start + 0.5 * (t_end - t_start)
    ms = [a.elapsed_time(b) for t, a, b in ev if t >= mid]
    idle = [r for r in recs if r["t"] < t_start - 0.2]
    run = [r for r in recs if mid <= r["t"] <= t_end]
    out = {"variant": var, "launches": n, "ms_second_half": round(float(np.mean(ms)), 4),
           "idle_w": round(float(np.nanmedian([num(r.get("socket_w")) for r in idle])), 1) if idle else None,
           "run_w": round(float(np.nanmean([num(r.get("socket_w")) for r in run])), 1) if run else None,
           "run_avg_w": round(float(np.nanmean([num(r.get("avg_w")) for r in run])), 1) if run else None,
           "run_gfxclk": round(float(np.nanmean([num(r.get("gfxclk")) for r in run])), 1) if run else None,
           "run_act": round(float(np.nanmean([num(r.get("act")) for r in run])), 1) if run else None,
           "run_temp": round(float(np.nanmean([num(r.get("temp")) for r in run])), 1) if run else None,
           "samples": len(run), "errors": [r.get("err") or r.get("err2") for r in recs if "err" in r or "err2" in r][:2]}
    print(json.dumps(out), flush=True)
    amdsmi.amdsmi_shut_down()


if __name__ == "__main__":
    main()
