#!/bin/bash
# after compiling the ci16 tuning variants out of the product: ci16 / mixer / chain / fuzz /
# golden parity, then the PMC refresh of the decimator translation unit
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
  -k "ci16 or mix or config4 or pipeline or fuzz or golden or time_split" > gpurun_out/final/g_tests.log 2>&1 || { tail -30 gpurun_out/final/g_tests.log; exit 1; }
tail -1 gpurun_out/final/g_tests.log
WORKLOADS="decim mixdecim ci16decim fir" WITH8CH=1 bash scripts/gpu_r02_final_pmc.sh
