#!/bin/bash
# round 2 session 3: baseline of this session -- issue rates, driver-style bench, full GPU suite
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python3 scripts/tune/issue_rate.py > gpurun_out/issue_rate.txt 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || exit $?
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --channels-per-gpu 8 --no-cpu-baseline --no-pcie --dump-steps > gpurun_out/bench_ch8.json 2> gpurun_out/bench_ch8.err || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
