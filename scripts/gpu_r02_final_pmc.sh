#!/bin/bash
# Final round-2 PMC traffic of every bench workload's dominant kernel (separate
# FETCH_SIZE / WRITE_SIZE / SQ passes, scripts/pmc_traffic.py), stamped with the
# kernel's translation-unit digest.  WORKLOADS overrides the list.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
export TMPDIR=/tmp
for w in ${WORKLOADS:-decim mixdecim ci16decim fir up}; do
  timeout -k 10 400 python3 scripts/pmc_traffic.py --workload $w --tag r02final > gpurun_out/final/pmc_$w.log 2>&1 || { tail -20 gpurun_out/final/pmc_$w.log; exit 1; }
done
if [ -z "$WORKLOADS" ] || [ -n "$WITH8CH" ]; then
  timeout -k 10 500 python3 scripts/pmc_traffic.py --workload decim --channels 8 --tag r02final > gpurun_out/final/pmc_decim8ch.log 2>&1 || { tail -20 gpurun_out/final/pmc_decim8ch.log; exit 1; }
fi
ls gpurun_out/ | grep "r02final.json"
