#!/bin/bash
# Where does the headline's tap loop lose VALU issue?  Cold ramps (clock beside)
# of the compute-only (73), no-staging (76), no-staging-no-store (77) probes
# and their ILV (inline-asm tap-major) counterparts (201, 205, 206).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
IDLE=5 TAG=r02m VARIANTS="73 76 77 201 205 206 70 200" LAUNCHES=80 bash scripts/gpu_ramp.sh || exit $?
