#!/bin/bash
# interpolator swizzled output staging: parity, same-box A/B vs HEAD, then its PMC traffic
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_r02_up_ab.sh || exit $?
timeout -k 10 400 python3 scripts/pmc_traffic.py --workload up --tag r02final > gpurun_out/pmc_up_final.log 2>&1 || { tail -20 gpurun_out/pmc_up_final.log; exit 1; }
grep -E '"SQ_LDS_BANK_CONFLICT"|traffic_over' gpurun_out/pmc_up_r02final.json
