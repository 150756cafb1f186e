#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-f}
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${name}.log" 2>&1
  local rc=$?
  echo "[$name] exit $rc" >> gpurun_out/steps.log
  if [ "$rc" -ne 0 ]; then echo "stopping after $name"; exit "$rc"; fi
}
step tests_$TAG 900 python -m pytest tests -m gpu -q -x
step bench_decim_$TAG 300 python bench.py
step bench_up_$TAG 300 python bench.py --workload up --no-cpu-baseline
step prof_decim_$TAG 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_decim_$TAG -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline
step prof_up_$TAG 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_up_$TAG -o run --output-format csv -- python bench.py --workload up --steps 10 --warmup 2 --no-cpu-baseline
step prof_fir_$TAG 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fir_$TAG -o run --output-format csv -- python bench.py --workload fir --steps 10 --warmup 2 --no-cpu-baseline
step pmc_decim_$TAG 600 python scripts/pmc_traffic.py --workload decim --tag $TAG
