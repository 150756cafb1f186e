#!/usr/bin/env python3
"""SQ counters of one kernel of an arbitrary command (tuning only): the passes
of pmc_workload.py plus an MFMA pass, one rocprofv3 --pmc run per pass
(kernel trace only, each under its own `timeout -s KILL`), averaged over the
matching dispatches after the first two.

  pmc_cmd.py OUT.json KERNEL_SUBSTRING -- COMMAND..."""
import csv
import glob
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
from pmc_workload import PASSES  # noqa: E402

MFMA_PASS = ["SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_MFMA", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"]
# HBM traffic, one derived counter per pass (FETCH_SIZE takes 3 TCC counters, WRITE_SIZE 2;
# scripts/pmc_traffic.py applies the gfx950 corrections: read = 2 x FETCH_SIZE x 1024 B,
# write = WRITE_SIZE x 1024 B)
TRAFFIC_PASSES = [["FETCH_SIZE"], ["WRITE_SIZE"]]


def one(cmd, ksub, counters, tag):
    out = os.path.join(ROOT, "gpurun_out", "pmcc", tag)
    full = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc", *counters, "--kernel-trace", "--output-format",
            "csv", "-d", out, "-o", "p", "--", *cmd]
    r = subprocess.run(full, capture_output=True, text=True)
    if r.returncode != 0:
        return {"error": f"rc={r.returncode}: {r.stderr[-1500:]}"}
    f = glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)[0]
    per = {}
    for row in csv.DictReader(open(f)):
        if ksub not in row.get("Kernel_Name", ""):
            continue
        d = row.get("Dispatch_Id") or row.get("Correlation_Id")
        per.setdefault(d, {}).setdefault(row["Counter_Name"], 0.0)
        per[d][row["Counter_Name"]] += float(row["Counter_Value"])
    ds = sorted(per, key=lambda k: int(k))[2:]
    res = {c: sum(per[d].get(c, 0.0) for d in ds) / max(1, len(ds)) for c in counters} | {"dispatches": len(ds)}
    # the same dispatches' durations from the kernel trace of this pass: the
    # clock the kernel held (GRBM_GUI_ACTIVE sums the 8 XCDs) and, with
    # SQ_VALU_MFMA_BUSY_CYCLES (summed over the 1024 SIMDs), the MFMA busy share
    tr = glob.glob(os.path.join(out, "**", "*kernel_trace.csv"), recursive=True)
    if tr:
        dur = {}
        for row in csv.DictReader(open(tr[0])):
            d = row.get("Dispatch_Id") or row.get("Correlation_Id")
            if d in per:
                dur[d] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
        if all(d in dur for d in ds) and ds:
            t = sum(dur[d] for d in ds) / len(ds)
            res["mean_s"] = t
            if "GRBM_GUI_ACTIVE" in res:
                res["clock_ghz"] = res["GRBM_GUI_ACTIVE"] / 8 / t / 1e9
                if "SQ_VALU_MFMA_BUSY_CYCLES" in res:
                    res["mfma_busy_frac"] = res["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (res["GRBM_GUI_ACTIVE"] / 8)
    return res


def main():
    sep = sys.argv.index("--")
    outp, ksub = sys.argv[1], sys.argv[2]
    cmd = sys.argv[sep + 1:]
    r = {}
    passes = [MFMA_PASS] + PASSES + TRAFFIC_PASSES  # indices 0 (MFMA), 1-3 (SQ), 4-5 (traffic)
    if os.environ.get("PMC_PASSES"):  # e.g. "0": the MFMA pass only; "0,4,5": and the traffic
        passes = [passes[int(i)] for i in os.environ["PMC_PASSES"].split(",")]
    for i, p in enumerate(passes):
        res = one(cmd, ksub, p, f"p{i}")
        r[f"pass{i}"] = res
        print(i, json.dumps(res), flush=True)
    json.dump({"kernel": ksub, "cmd": cmd, "passes": r}, open(outp, "w"), indent=1)


if __name__ == "__main__":
    main()
