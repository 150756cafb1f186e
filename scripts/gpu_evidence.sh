#!/bin/bash
# Full evidence session: GPU tests, every bench line (with its CPU baseline),
# rocprofv3 kernel stats of every workload, PMC traffic of the two streaming
# decimators.  Outputs gpurun_out/*_$TAG*; reviewed copies go to profiles/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-ev}
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${name}.log" 2>&1
  local rc=$?
  echo "[$name] exit $rc" >> gpurun_out/steps.log
  if [ "$rc" -ne 0 ]; then echo "stopping after $name"; exit "$rc"; fi
}
prof() {
  local w=$1; shift
  step prof_${w}_$TAG 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${w}_$TAG -o run --output-format csv \
      -- python bench.py --workload $w --no-cpu-baseline "$@"
}
for s in ${STEPS:-tests bench prof pmc}; do
  case $s in
    tests) step tests_$TAG 900 python -m pytest tests -m gpu -q -x ;;
    bench)
      step bench_decim_$TAG 300 python bench.py
      step bench_mixdecim_$TAG 300 python bench.py --workload mixdecim
      step bench_corr_$TAG 300 python bench.py --workload corr --samples 67108864
      step bench_fir_$TAG 300 python bench.py --workload fir
      step bench_up_$TAG 300 python bench.py --workload up ;;
    prof)
      prof decim
      prof mixdecim
      prof corr --samples 67108864 --steps 50 --warmup 20
      prof fir
      prof up ;;
    pmc)
      step pmc_decim_$TAG 600 python scripts/pmc_traffic.py --workload decim --tag $TAG
      step pmc_mixdecim_$TAG 600 python scripts/pmc_traffic.py --workload mixdecim --tag $TAG ;;
  esac
done
