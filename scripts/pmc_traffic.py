#!/usr/bin/env python3
"""Collect per-launch HBM traffic of the dominant kernel with rocprofv3 PMC
counters, corrected as /opt/skills/guides/MI355X_MICROARCH.md §HBM prescribes:
  * FETCH_SIZE and WRITE_SIZE in SEPARATE passes (TCC slots: 3 + 2 > 4),
    each with --kernel-trace only (no sys/runtime traces beside --pmc);
  * units of KiB (x1024);
  * gfx950: FETCH_SIZE reads exactly 1/2 of a wide (16 B/lane) coalesced
    streaming read -> doubled; WRITE_SIZE exact for 16 B/lane stores.
A third pass records SQ/GRBM counters for diagnosis.  Writes
gpurun_out/pmc_<workload>_<tag>.json; merged into profiles/pmc_traffic.json
(which bench.py reports as roofline.traffic) after review.

usage: python scripts/pmc_traffic.py [--workload decim] [--tag r01]
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from srcdsp_amd.build import source_digest  # noqa: E402
KERNEL_KEYS = {"decim": "decim_stream_cf32", "mixdecim": "decim_dot2_ci16", "ci16decim": "decim_dot2_ci16", "corr": "corr_scan_s1",
               "fir": "fir_stream_f32", "up": "up_tile"}
BYTES_PER_SAMPLE = {"decim": 10.0, "mixdecim": 5.0, "ci16decim": 5.0, "corr": 4.0, "fir": 12.0, "up": 20.0}
NAMES = {"decim": "decim_cf32_m4_t127", "mixdecim": "mixer4096_f0.1_to_decim_ci16_q14_m4_t127",
         "ci16decim": "decim_ci16_q14_m4_t127",
         "corr": "corr_1024x1", "fir": "fir_f32_t31", "up": "up_ci16_q14_l4_t128"}
PASSES = [["FETCH_SIZE"], ["WRITE_SIZE"],
          ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
           "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "GRBM_GUI_ACTIVE"],
          ["SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
           "SQ_INSTS_SALU", "SQ_INSTS_SMEM"]]


def run_pass(counters, out_dir, bench_args):
    os.makedirs(out_dir, exist_ok=True)
    cmd = ["rocprofv3", "--pmc", *counters, "--kernel-trace", "--output-format", "csv", "-d", out_dir, "-o", "p",
           "--", sys.executable, os.path.join(ROOT, "bench.py"), *bench_args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise RuntimeError(f"rocprofv3 failed ({r.returncode}):\n{r.stderr[-3000:]}")
    files = glob.glob(os.path.join(out_dir, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise RuntimeError(f"no counter_collection.csv under {out_dir}")
    per = {}
    with open(files[0]) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "")
            disp = row.get("Dispatch_Id") or row.get("Correlation_Id")
            per.setdefault((name, disp), {})
            c = row["Counter_Name"]
            per[(name, disp)][c] = per[(name, disp)].get(c, 0.0) + float(row["Counter_Value"])
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="decim")
    ap.add_argument("--tag", default="latest")
    ap.add_argument("--samples", type=int, default=None, help="default: bench.py's (2^28; corr: 2^26, config 5)")
    ap.add_argument("--channels", type=int, default=1, help="decim only: channels per launch (config 3's share: 8)")
    a = ap.parse_args()
    if a.samples is None:
        a.samples = (1 << 26) if a.workload == "corr" else (1 << 28)
    key = KERNEL_KEYS[a.workload]
    steps_run = 6  # bench.py --warmup 1 --steps 5: every step's dispatches are counted
    # --no-parity: the decim line's post-timing parity step is one more launch of
    # the same kernel; counters are summed over dispatches and divided by the
    # steps run, so it must not run here (round 6: it read as 7/6 x the traffic)
    bench_args = ["--workload", a.workload, "--steps", "5", "--warmup", "1", "--no-cpu-baseline", "--no-pcie",
                  "--no-parity", "--samples", str(a.samples)]
    if a.channels > 1:
        bench_args += ["--channels-per-gpu", str(a.channels)]
    res = {}
    for i, counters in enumerate(PASSES):
        per = run_pass(counters, os.path.join(ROOT, "gpurun_out", f"pmc_{a.workload}_{i}"), bench_args)
        rows = [v for (n, d), v in per.items() if key in n]
        if not rows:
            raise RuntimeError(f"kernel {key} not found among {sorted({n for n, _ in per})}")
        # per step: a step may be several dispatches (the batched complex<float>
        # decimator launches once per channel)
        for c in counters:
            res[c] = sum(r[c] for r in rows if c in r) / steps_run
        res["dispatches"] = len(rows)
        res["dispatches_per_step"] = len(rows) / steps_run
    L = (a.samples - a.samples % 4) * a.channels
    if a.workload == "up":
        L //= 4  # bench.py's up workload takes samples/4 inputs (4x as many outputs)
    read_b = 2.0 * res["FETCH_SIZE"] * 1024.0      # gfx950 FETCH_SIZE half-count correction
    write_b = res["WRITE_SIZE"] * 1024.0
    alg = BYTES_PER_SAMPLE[a.workload] * L
    entry = {"kernel": key, "samples_per_launch": L, "hbm_bytes_per_launch": int(read_b + write_b),
             "read_bytes_per_launch": int(read_b), "write_bytes_per_launch": int(write_b),
             "algorithmic_bytes_per_launch": int(alg), "traffic_over_algorithmic": (read_b + write_b) / alg,
             "raw_counters_per_launch": res,
             "correction": "read = 2*FETCH_SIZE*1024 (gfx950 half-count), write = WRITE_SIZE*1024",
             "kernel_sources_sha": source_digest(a.workload)}
    if "SQ_WAVE_CYCLES" in res and res.get("SQ_WAVE_CYCLES"):
        entry["valu_active_frac_of_wave_cycles"] = res["SQ_ACTIVE_INST_VALU"] / res["SQ_WAVE_CYCLES"]
        entry["wait_any_frac"] = res["SQ_WAIT_ANY"] / res["SQ_WAVE_CYCLES"]
    # written under gpurun_out/ (what the GPU box hands back); copied into
    # profiles/ (tracked) by hand after review
    out = os.path.join(ROOT, "gpurun_out")
    key = NAMES[a.workload] + (f"x{a.channels}" if a.channels > 1 else "")
    with open(os.path.join(out, f"pmc_{a.workload}{'x%d' % a.channels if a.channels > 1 else ''}_{a.tag}.json"), "w") as f:
        json.dump({key: entry}, f, indent=1)
    print(json.dumps(entry, indent=1))


if __name__ == "__main__":
    main()
