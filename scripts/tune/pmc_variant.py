#!/usr/bin/env python3
"""SQ/LDS counters of tune_decim variants, one rocprofv3 --pmc pass per
counter group (kernel trace only), averaged over the variant's launches
(tuning only).  usage: pmc_variant.py OUT.json VARIANT:GRID [VARIANT:GRID ...]"""
import csv
import glob
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PASSES = [["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
           "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE"],
          ["SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_WAIT_INST_LDS",
           "SQ_LDS_IDX_ACTIVE", "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS"]]


def one(var, grid, counters, tag):
    out = os.path.join("gpurun_out", "pmcv", f"{tag}_{var}_{grid}")
    cmd = ["timeout", "-s", "KILL", "90", "rocprofv3", "--pmc", *counters, "--kernel-trace", "--output-format",
           "csv", "-d", out, "-o", "p", "--", sys.executable, os.path.join(HERE, "launch_variant.py"), str(var),
           str(grid), "12"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise SystemExit(f"pass failed rc={r.returncode}: {r.stderr[-2000:]}")
    f = glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)[0]
    per = {}
    for row in csv.DictReader(open(f)):
        if "decim" not in row.get("Kernel_Name", ""):
            continue
        d = row.get("Dispatch_Id") or row.get("Correlation_Id")
        per.setdefault(d, {}).setdefault(row["Counter_Name"], 0.0)
        per[d][row["Counter_Name"]] += float(row["Counter_Value"])
    ds = sorted(per, key=lambda k: int(k))[2:]  # skip the first two launches
    return {c: sum(per[d].get(c, 0.0) for d in ds) / len(ds) for c in counters}


def main():
    res = {}
    for spec in sys.argv[2:]:
        var, grid = map(int, spec.split(":"))
        r = {}
        for i, p in enumerate(PASSES):
            r.update(one(var, grid, p, f"p{i}"))
        res[spec] = r
        print(spec, json.dumps(r), flush=True)
    json.dump(res, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
