#!/bin/bash
# decim_wave_cf32 split: memory path only (402) and compute path only (403)
# beside the product-shape memory (71) / compute (73) probes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
IDLE=5 TAG=r02p VARIANTS="402 403 71 73" LAUNCHES=80 bash scripts/gpu_ramp.sh || exit $?
