#!/bin/bash
# decim_wave_cf32 memory path: default cache policy (404), no halo load (405),
# full kernel with default policy (406), 256-lane blocks memory path (407)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
IDLE=3 TAG=r02q VARIANTS="404 405 406 407 402" LAUNCHES=60 bash scripts/gpu_ramp.sh || exit $?
RAMP_GRID=2048 IDLE=3 TAG=r02q_g2048 VARIANTS="402 407" LAUNCHES=60 bash scripts/gpu_ramp.sh || exit $?
