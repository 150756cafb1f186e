#!/usr/bin/env python3
"""SQ/LDS counters of one bench.py workload's kernel (tuning only): one
rocprofv3 --pmc pass per counter group (kernel trace only), averaged over the
launches after the first two.

  pmc_workload.py OUT.json WORKLOAD KERNEL_SUBSTRING [extra bench.py args]"""
import csv
import glob
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
PASSES = [["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
           "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE"],
          ["SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_WAIT_INST_LDS",
           "SQ_LDS_IDX_ACTIVE", "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS"],
          ["SQ_INSTS_VMEM_WR", "SQ_INSTS_VMEM_RD", "SQ_INST_CYCLES_VMEM_WR", "SQ_INST_CYCLES_VMEM_RD",
           "SQ_ACTIVE_INST_MISC", "SQ_ACTIVE_INST_SCA", "SQ_INSTS_BRANCH", "SQ_INSTS_SENDMSG"]]


def one(workload, ksub, counters, tag, extra):
    out = os.path.join(ROOT, "gpurun_out", "pmcw", f"{tag}_{workload}")
    cmd = ["timeout", "-s", "KILL", "90", "rocprofv3", "--pmc", *counters, "--kernel-trace", "--output-format",
           "csv", "-d", out, "-o", "p", "--", sys.executable, os.path.join(ROOT, "bench.py"), "--workload", workload,
           "--steps", "10", "--warmup", "2", "--no-cpu-baseline", "--no-pcie", *extra]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise SystemExit(f"pass failed rc={r.returncode}: {r.stderr[-2000:]}")
    f = glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)[0]
    per = {}
    for row in csv.DictReader(open(f)):
        if ksub not in row.get("Kernel_Name", ""):
            continue
        d = row.get("Dispatch_Id") or row.get("Correlation_Id")
        per.setdefault(d, {}).setdefault(row["Counter_Name"], 0.0)
        per[d][row["Counter_Name"]] += float(row["Counter_Value"])
    ds = sorted(per, key=lambda k: int(k))[2:]
    return {c: sum(per[d].get(c, 0.0) for d in ds) / max(1, len(ds)) for c in counters}


def main():
    outp, workload, ksub, extra = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4:]
    r = {}
    for i, p in enumerate(PASSES):
        r.update(one(workload, ksub, p, f"p{i}", extra))
        print(workload, i, json.dumps(r), flush=True)
    json.dump({workload: r}, open(outp, "w"), indent=1)


if __name__ == "__main__":
    main()
