#!/bin/bash
# PMC traffic of config 3's per-GPU share (8 x 2^28 channels, one batched launch), then its bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 500 python3 scripts/pmc_traffic.py --workload decim --channels 8 --tag r02final > gpurun_out/final/pmc_decim8ch.log 2>&1 || { tail -20 gpurun_out/final/pmc_decim8ch.log; exit 1; }
grep traffic_over gpurun_out/pmc_decimx8_r02final.json
