#!/bin/bash
# sequence-table mixer: parity, bench, PMC (bank conflicts)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mix or config4 or pipeline or time_split or fuzz" > gpurun_out/pytest_mix.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --workload mixdecim --steps 200 --warmup 100 --no-cpu-baseline > gpurun_out/bench_mixdecim.json 2> gpurun_out/bench_mixdecim.err || exit $?
timeout -k 10 400 python3 scripts/pmc_traffic.py --workload mixdecim --tag r02 > gpurun_out/pmc_mixdecim.log 2>&1 || exit $?
