#!/bin/bash
# decim_wave_cf32 with one barrier per tile before the loads: memory path (408), full (409)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
IDLE=3 TAG=r02r VARIANTS="408 409 402" LAUNCHES=60 bash scripts/gpu_ramp.sh || exit $?
