#!/bin/bash
# A/B (tuning): decim_tile with non-temporal body loads / output stores vs HEAD's library, same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/tile_nt_ab.txt
for round in 1 2; do
  for lib in srcdsp_amd/lib_ab/libsrcdsp_hip_head.so srcdsp_amd/lib/libsrcdsp_hip.so; do
    echo "## $lib" >> gpurun_out/tile_nt_ab.txt
    SRCDSP_HIP_LIB=$PWD/$lib timeout -k 10 200 python3 -u scripts/shape_envelope.py >> gpurun_out/tile_nt_ab.txt 2>&1 || exit $?
  done
done
cat gpurun_out/tile_nt_ab.txt
