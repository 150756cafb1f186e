#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "up or ci16 or mix or config4 or pipeline or time_split or fuzz or golden" > gpurun_out/pytest_sel.log 2>&1 || exit $?
for w in up ci16decim mixdecim; do
timeout -k 10 200 python3 bench.py --workload $w --steps 200 --warmup 100 --no-cpu-baseline > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || exit $?
done
