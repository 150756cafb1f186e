#!/bin/bash
# headline kernel compiled for 63/64/255/256 taps too: parity, then the shape envelope vs HEAD (decim_tile for those)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 240 --timeout-method thread \
  -k "decim or golden or fuzz or fir" > gpurun_out/nt_tests.log 2>&1 || { tail -30 gpurun_out/nt_tests.log; exit 1; }
tail -2 gpurun_out/nt_tests.log
: > gpurun_out/nt_ab.txt
for round in 1 2; do
  for lib in srcdsp_amd/lib_ab/libsrcdsp_hip_head.so srcdsp_amd/lib/libsrcdsp_hip.so; do
    echo "## $lib" >> gpurun_out/nt_ab.txt
    SRCDSP_HIP_LIB=$PWD/$lib timeout -k 10 200 python3 -u scripts/shape_envelope.py >> gpurun_out/nt_ab.txt 2>&1 || exit $?
  done
done
grep -E "^##|M=" gpurun_out/nt_ab.txt
