#!/bin/bash
# One GPU session: smoke -> GPU parity tests -> bench -> rocprofv3 kernel trace.
# Each GPU step has its own time limit; a fault/abort/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() {  # continue on success (0) or plain test failures (1); stop on anything else
  local rc=$1 step=$2
  echo "[$step] exit $rc" | tee -a gpurun_out/steps.log
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $step"; exit "$rc"; fi
}
STEPS="${STEPS:-smoke tests bench prof}"
for s in $STEPS; do
  case $s in
    smoke) timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; ok $? smoke ;;
    tests) timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=30 ${PYTEST_K:+-k "$PYTEST_K"} \
             > gpurun_out/pytest_gpu.log 2>&1; ok $? tests ;;
    bench) timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err; ok $? bench ;;
    prof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv \
             -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/prof.log 2>&1; ok $? prof ;;
  esac
done
