#!/bin/bash
# matrix-core decimator (16x16x4 f32): A/B against the VALU headline, ramp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TUNE_MFMA=1 TUNE_SUSTAINED_ONLY=1 timeout -k 10 300 python3 -u scripts/tune/tune.py > gpurun_out/tune_mfma.txt 2>&1 || exit $?
RAMP_GRID=768 IDLE=10 TAG=r02d VARIANTS="303 304" LAUNCHES=120 bash scripts/gpu_ramp.sh || exit $?
