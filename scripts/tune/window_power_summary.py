#!/usr/bin/env python3
"""Summarise window_power.py's sample series (tuning only).

  python scripts/tune/window_power_summary.py gpurun_out/window_power_127.jsonl [...]

The metrics table the SMU publishes updates every ~20 ms (accumulation_counter
advances by 1 per ms).  current_socket_power is a slow moving average, so the
real power of an interval is taken from the energy accumulator instead:
dE x 15.259 uJ over the interval's accumulation-counter ticks (1 ms each).
ppt_residency_acc advances by 1 per ms while the firmware's package power
tracking (PPT) limiter is active, so dPPT / dAcc is the fraction of the
interval spent PPT-limited.  Each interval is listed with the launches that
ran in it and their mean kernel time."""
import json
import sys

ENERGY_UJ = 15.259  # uJ per energy_accumulator count (SMU energy unit)


def summarise(path):
    rows = [json.loads(l) for l in open(path)]
    tail, rows = rows[-1], rows[:-1]
    ms, st = tail["launch_ms"], tail["launch_start_rel_ms"]
    upd, prev = [], None
    for r in rows:
        k = r.get("accumulation_counter")
        if k is not None and k != prev:
            upd.append(r)
            prev = k
    out = [f"# {path}: {len(ms)} launches, first at {st[0]:.1f} ms, last ends at {st[-1] + ms[-1]:.1f} ms",
           "# launches 1-25 ms: " + " ".join(f"{v:.3f}" for v in ms[:25]),
           "interval_ms        launches  mean_ms  power_W  mJ/launch  ppt_active  gfxclk_MHz  avg_pwr_reported_W"]
    for a, b in zip(upd, upd[1:]):
        t0, t1 = a["rel_ms"], b["rel_ms"]
        dacc = b["accumulation_counter"] - a["accumulation_counter"]
        if dacc <= 0:
            continue
        p = (b["energy_accumulator"] - a["energy_accumulator"]) * ENERGY_UJ * 1e-6 / (dacc * 1e-3)
        ppt = (b["ppt_residency_acc"] - a["ppt_residency_acc"]) / dacc
        ls = [i for i, s in enumerate(st) if t0 <= s < t1]
        lr = f"{ls[0] + 1}-{ls[-1] + 1}" if ls else "-"
        mm = f"{sum(ms[i] for i in ls) / len(ls):.4f}" if ls else "-"
        # energy per launch where launches fill the interval back to back
        full = ls and st[ls[0]] - t0 < 1.0 and st[ls[-1]] + ms[ls[-1]] > t1 - 1.0
        mj = f"{p * sum(ms[i] for i in ls) / len(ls) * 1e-3 * 1e3:.1f}" if full else "-"
        out.append(f"{t0:7.1f}-{t1:7.1f}  {lr:>9}  {mm:>7}  {p:7.0f}  {mj:>9}  {ppt:10.2f}  {b['current_gfxclk']:10.0f}"
                   f"  {b['current_socket_power']:8.0f}")
    return "\n".join(out)


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(summarise(p))
        print()
