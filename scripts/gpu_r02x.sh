#!/bin/bash
# round-2 evidence, part 1: full GPU suite, driver-style headline (with the CPU
# baselines), steady lines of every workload
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/x
export TMPDIR=/tmp
O=gpurun_out/x
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-pcie > $O/bench_decim.json 2> $O/bench_decim.err || exit $?
timeout -k 10 200 python3 bench.py --fp strict --no-cpu-baseline --no-pcie > $O/bench_strict.json 2> $O/bench_strict.err || exit $?
timeout -k 10 200 python3 bench.py --channels-per-gpu 8 --steps 20 --warmup 5 --no-cpu-baseline --no-pcie > $O/bench_decim8ch.json 2> $O/bench_decim8ch.err || exit $?
for w in mixdecim ci16decim fir up fifo iq; do
  timeout -k 10 300 python3 bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || exit $?
done
timeout -k 10 300 python3 bench.py --workload corr --samples 67108864 --steps 3 --warmup 1 > $O/bench_corr.json 2> $O/bench_corr.err || exit $?
