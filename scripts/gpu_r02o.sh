#!/bin/bash
# wave-private barrier-free headline kernel (decim_wave_cf32): bit-exact check
# against the product, then cold ramps beside the product shape (70)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/tune/wave_check.py 400 401 > gpurun_out/wave_check.log 2>&1 || exit $?
IDLE=5 TAG=r02o VARIANTS="400 401 70" LAUNCHES=80 bash scripts/gpu_ramp.sh || exit $?
RAMP_GRID=512 IDLE=5 TAG=r02o_g512 VARIANTS="400" LAUNCHES=80 bash scripts/gpu_ramp.sh || exit $?
RAMP_GRID=2048 IDLE=5 TAG=r02o_g2048 VARIANTS="401" LAUNCHES=80 bash scripts/gpu_ramp.sh || exit $?
