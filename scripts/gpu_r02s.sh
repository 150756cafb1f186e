#!/bin/bash
# same-box cold ramps: product, ILV (200, g1024), ILV MINW2 (202, g512),
# wave-private + per-tile barrier (409), product again
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
IDLE=8 TAG=r02s VARIANTS="prod 200 409" LAUNCHES=100 bash scripts/gpu_ramp.sh || exit $?
RAMP_GRID=512 IDLE=8 TAG=r02s_g512 VARIANTS="202" LAUNCHES=100 bash scripts/gpu_ramp.sh || exit $?
IDLE=8 TAG=r02s_b VARIANTS="prod 200 409" LAUNCHES=100 bash scripts/gpu_ramp.sh || exit $?
