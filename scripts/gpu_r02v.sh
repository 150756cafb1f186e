#!/bin/bash
# column-major dot2 planes: ci16 / mixer / chain parity, then the ci16decim and mixdecim bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "ci16 or mix or config4 or pipeline or time_split or fuzz or golden or dropin or sharded" > gpurun_out/v_pytest.log 2>&1 || exit $?
for w in ci16decim mixdecim; do
timeout -k 10 200 python3 bench.py --workload $w --no-cpu-baseline > gpurun_out/v_bench_$w.json 2> gpurun_out/v_bench_$w.err || exit $?
done
