#!/bin/bash
# Is the headline's memory path core-clock bound?  Time the memory-only path
# (71) and a read-only stream right after 8 product launches have pulled the
# clock down, against the same from idle.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
make -C scripts/tune -q libtune.so || make -C scripts/tune libtune.so > /dev/null || exit 1
IDLE=10 TAG=r02l VARIANTS="prod*8,71*60 prod*8,read*60 71*68 read*68 prod*68" LAUNCHES=68 bash scripts/gpu_ramp.sh || exit $?
