#!/bin/bash
# Evidence session: rocprofv3 kernel stats of every bench workload + PMC traffic
# of the two streaming decimators.  Outputs under gpurun_out/<name>_$TAG; the
# reviewed summaries are copied into profiles/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${name}.log" 2>&1
  local rc=$?
  echo "[$name] exit $rc" >> gpurun_out/steps.log
  if [ "$rc" -ne 0 ]; then echo "stopping after $name"; exit "$rc"; fi
}
prof() {  # workload, extra bench args...
  local w=$1; shift
  step prof_${w}_$TAG 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${w}_$TAG -o run --output-format csv \
      -- python bench.py --workload $w --no-cpu-baseline "$@"
}
for s in ${STEPS:-prof_decim prof_mixdecim prof_corr prof_fir pmc_decim pmc_mixdecim bench_mixdecim bench_corr}; do
  case $s in
    prof_decim) prof decim --steps 20 --warmup 3 ;;
    prof_mixdecim) prof mixdecim --steps 20 --warmup 3 ;;
    prof_corr) prof corr --samples 67108864 --steps 3 --warmup 1 ;;
    prof_fir) prof fir --steps 10 --warmup 2 ;;
    pmc_decim) step pmc_decim_$TAG 600 python scripts/pmc_traffic.py --workload decim --tag $TAG ;;
    pmc_mixdecim) step pmc_mixdecim_$TAG 600 python scripts/pmc_traffic.py --workload mixdecim --tag $TAG ;;
    bench) step bench_$TAG 300 python bench.py ;;
    bench_mixdecim) step bench_mixdecim_$TAG 300 python bench.py --workload mixdecim ;;
    bench_corr) step bench_corr_$TAG 300 python bench.py --workload corr --samples 67108864 --steps 3 --warmup 1 ;;
    tests) step tests_$TAG 900 python -m pytest tests -m gpu -q --maxfail=30 ;;
  esac
done
