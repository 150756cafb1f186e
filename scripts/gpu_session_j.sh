#!/bin/bash
# Same-box comparison: tune (sustained) vs bench for the headline; mixdecim
# kernel variants (SRCDSP_CI16_VARIANT) tested and benched.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${name}.log" 2>&1
  local rc=$?
  echo "[$name] exit $rc" >> gpurun_out/steps.log
  if [ "$rc" -ne 0 ]; then echo "stopping after $name"; exit "$rc"; fi
}
step tune_j 300 env TUNE_SUSTAINED_ONLY=1 python scripts/tune/tune.py
step bench_decim_j1 300 python bench.py --no-cpu-baseline
step bench_decim_j2 300 python bench.py --no-cpu-baseline --steps 60 --warmup 5
for v in 0 1 2 3; do
  step tests_ci16_v$v 600 env SRCDSP_CI16_VARIANT=$v python -m pytest tests/test_gpu_parity.py -q -x -m gpu -k "ci16 or mixdecim or time_split or golden"
done
for r in 1 2; do
  for v in 0 1 2 3; do
    step bench_mix_v${v}_r$r 300 env SRCDSP_CI16_VARIANT=$v python bench.py --workload mixdecim --no-cpu-baseline
  done
done
