#!/bin/bash
# interpolator compile-time shapes for 8 / 16 / 32 tap pairs per phase: parity, then same-box A/B vs HEAD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "upsampler or golden" \
  > gpurun_out/uppp_tests.log 2>&1 || { tail -30 gpurun_out/uppp_tests.log; exit 1; }
tail -2 gpurun_out/uppp_tests.log
: > gpurun_out/uppp_ab.txt
for round in 1 2; do
  for lib in srcdsp_amd/lib_ab/libsrcdsp_hip_head.so srcdsp_amd/lib/libsrcdsp_hip.so; do
    echo "## $lib" >> gpurun_out/uppp_ab.txt
    SRCDSP_HIP_LIB=$PWD/$lib timeout -k 10 200 python3 -u scripts/up_envelope.py >> gpurun_out/uppp_ab.txt 2>&1 || exit $?
  done
done
grep -E "^##|L=" gpurun_out/uppp_ab.txt
