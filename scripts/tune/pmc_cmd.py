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
    return {c: sum(per[d].get(c, 0.0) for d in ds) / max(1, len(ds)) for c in counters} | {"dispatches": len(ds)}


def main():
    sep = sys.argv.index("--")
    outp, ksub = sys.argv[1], sys.argv[2]
    cmd = sys.argv[sep + 1:]
    r = {}
    for i, p in enumerate([MFMA_PASS] + PASSES):
        res = one(cmd, ksub, p, f"p{i}")
        r[f"pass{i}"] = res
        print(i, json.dumps(res), flush=True)
    json.dump({"kernel": ksub, "cmd": cmd, "passes": r}, open(outp, "w"), indent=1)


if __name__ == "__main__":
    main()
