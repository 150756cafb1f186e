#!/bin/bash
# Perf session: bench (default + variants) -> rocprofv3 kernel stats -> PMC traffic.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-latest}
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${name}.log" 2>&1
  local rc=$?
  echo "[$name] exit $rc" | tee -a gpurun_out/steps.log
  if [ "$rc" -ne 0 ]; then echo "stopping after $name"; exit "$rc"; fi
}
for s in ${STEPS:-bench prof pmc}; do
  case $s in
    bench) step bench_$TAG 300 python bench.py ${BENCH_ARGS} ;;
    prof) step prof_$TAG 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
            -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} ;;
    pmc) step pmc_$TAG 600 python scripts/pmc_traffic.py --tag $TAG ${PMC_ARGS} ;;
    tests) step tests_$TAG 900 python -m pytest tests -m gpu -q --maxfail=30 ;;
    tune) step tune_$TAG 300 python scripts/tune/tune.py ;;
  esac
done
