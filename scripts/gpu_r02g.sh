#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 bench.py --workload ci16decim --steps 200 --warmup 100 > gpurun_out/bench_ci16decim.json 2> gpurun_out/bench_ci16decim.err || exit $?
timeout -k 10 400 python3 scripts/pmc_traffic.py --workload ci16decim --tag r02 > gpurun_out/pmc_ci16decim.log 2>&1 || exit $?
