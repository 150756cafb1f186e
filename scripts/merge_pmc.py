#!/usr/bin/env python3
"""Merge the PMC traffic entries a GPU session wrote (gpurun_out/pmc_*_<TAG>.json,
scripts/pmc_traffic.py) into profiles/pmc_traffic.json, which bench.py reports
as roofline.traffic.  Refuses an entry whose kernel_sources_sha no longer
matches the tree (measured on other kernel sources).

  python scripts/merge_pmc.py TAG"""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from srcdsp_amd.build import source_digest  # noqa: E402

WORKLOAD_OF = {"decim_cf32": "decim", "mixer4096": "mixdecim", "decim_ci16": "ci16decim", "fir_f32": "fir",
               "up_ci16": "up", "corr_1024": "corr"}


def main():
    tag = sys.argv[1]
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    cur = json.load(open(path))
    n = 0
    for f in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", f"pmc_*_{tag}.json"))):
        for k, e in json.load(open(f)).items():
            w = next(v for p, v in WORKLOAD_OF.items() if k.startswith(p))
            if e.get("kernel_sources_sha") != source_digest(w):
                raise SystemExit(f"{f}: {k} was measured on other kernel sources; not merged")
            cur[k] = e
            n += 1
            print(f"{k}: {e['traffic_over_algorithmic']:.4f} x algorithmic ({os.path.basename(f)})")
    json.dump(cur, open(path, "w"), indent=1)
    print(f"merged {n} entries into {path}")


if __name__ == "__main__":
    main()
