#!/bin/bash
# long-run (300 launches, ~150 ms) same-box A/B: old compiler-order headline (70) vs ILV (200)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
IDLE=8 TAG=r02u VARIANTS="70*300 200*300 70*300 200*300" LAUNCHES=300 bash scripts/gpu_ramp.sh || exit $?
