#!/bin/bash
# A/B of the tap-major (ILV) headline kernel against the product one
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TUNE_ILV=1 TUNE_SUSTAINED_ONLY=1 timeout -k 10 300 python3 -u scripts/tune/tune.py > gpurun_out/tune_ilv.txt 2>&1 || exit $?
IDLE=10 TAG=r02b VARIANTS="200 201" LAUNCHES=120 bash scripts/gpu_ramp.sh || exit $?
