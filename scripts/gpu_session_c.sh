#!/bin/bash
# dot2 ci16 decimator + correlator queueing: GPU tests, benches, profiles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-d}
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${name}.log" 2>&1
  local rc=$?
  echo "[$name] exit $rc" >> gpurun_out/steps.log
  if [ "$rc" -ne 0 ]; then echo "stopping after $name"; exit "$rc"; fi
}
step tests_$TAG 900 python -m pytest tests -m gpu -q -x
step bench_mixdecim_$TAG 300 python bench.py --workload mixdecim --no-cpu-baseline
step bench_corr_$TAG 300 python bench.py --workload corr --samples 67108864 --steps 3 --warmup 1 --no-cpu-baseline
step prof_mixdecim_$TAG 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mixdecim_$TAG -o run --output-format csv -- python bench.py --workload mixdecim --no-cpu-baseline
step prof_corr_$TAG 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_corr_$TAG -o run --output-format csv -- python bench.py --workload corr --samples 67108864 --steps 3 --warmup 1 --no-cpu-baseline
