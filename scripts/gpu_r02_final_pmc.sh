#!/bin/bash
# Final round-2 PMC traffic of every bench workload's dominant kernel (separate
# FETCH_SIZE / WRITE_SIZE / SQ passes, scripts/pmc_traffic.py), stamped with the
# kernel's translation-unit digest
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
export TMPDIR=/tmp
for w in decim mixdecim ci16decim fir up; do
  timeout -k 10 400 python3 scripts/pmc_traffic.py --workload $w --tag r02final > gpurun_out/final/pmc_$w.log 2>&1 || { tail -20 gpurun_out/final/pmc_$w.log; exit 1; }
done
ls gpurun_out/ | grep pmc_
