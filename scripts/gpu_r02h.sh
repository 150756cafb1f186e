#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "ci16 or mix or config4 or pipeline or time_split or fuzz or golden" > gpurun_out/pytest_mix.log 2>&1 || exit $?
for w in ci16decim mixdecim; do
timeout -k 10 200 python3 bench.py --workload $w --steps 200 --warmup 100 > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || exit $?
timeout -k 10 400 python3 scripts/pmc_traffic.py --workload $w --tag r02 > gpurun_out/pmc_$w.log 2>&1 || exit $?
done
