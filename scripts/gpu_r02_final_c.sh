#!/bin/bash
# Final round-2 evidence, part C (after the late FIR / interpolator LDS-read fixes):
# full GPU suite, then the bench lines of the kernels that changed or whose
# accounting changed, then their rocprof kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/pytest_gpu_c.log 2>&1 || { tail -30 $O/pytest_gpu_c.log; exit 1; }
tail -2 $O/pytest_gpu_c.log
for w in mixdecim ci16decim fir up; do
  timeout -k 10 300 python3 bench.py --workload $w > $O/bench_${w}_c.json 2> $O/bench_${w}_c.err || exit $?
done
for w in fir up; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${w}_c -o run --output-format csv \
      -- python3 bench.py --workload $w --no-cpu-baseline --no-pcie > $O/prof_${w}_c.log 2>&1 || exit $?
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_c.json 2> $O/bench_driver_c.err || exit $?
ls $O
