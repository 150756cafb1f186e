#!/bin/bash
# Round-2 first session: smoke, the whole GPU suite, the driver-style bench
# (cold box, --warmup 5 --steps 20), then the cold-start ramp of the product
# kernel beside its memory-only (71) and compute-only (73) variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || exit $?
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
IDLE=10 TAG=r02a VARIANTS="prod 71 73" LAUNCHES=120 bash scripts/gpu_ramp.sh || exit $?
