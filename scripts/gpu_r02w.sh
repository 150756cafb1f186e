#!/bin/bash
# interpolator: (c[2p+1], c[2p]) tap pairs + compile-time 16-pair shape
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "up or fuzz or golden or pipeline" > gpurun_out/w_pytest.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --workload up --no-cpu-baseline > gpurun_out/w_bench_up.json 2> gpurun_out/w_bench_up.err || exit $?
