#!/bin/bash
# A/B (tuning): interpolator with whole-b128 window reads vs the HEAD library, same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "upsampler" \
  > gpurun_out/up_tests.log 2>&1 || { tail -30 gpurun_out/up_tests.log; exit 1; }
tail -2 gpurun_out/up_tests.log
: > gpurun_out/up_ab.txt
for round in 1 2 3; do
  for lib in srcdsp_amd/lib_ab/libsrcdsp_hip_head.so srcdsp_amd/lib/libsrcdsp_hip.so; do
    echo "## $lib" >> gpurun_out/up_ab.txt
    SRCDSP_HIP_LIB=$PWD/$lib timeout -k 10 120 python3 -u bench.py --workload up --steps 100 --warmup 50 --no-cpu-baseline >> gpurun_out/up_ab.txt 2>/dev/null || exit $?
  done
done
python3 - <<'P'
import json
lib=None
for l in open('gpurun_out/up_ab.txt'):
    if l.startswith('##'): lib=l.split('/')[-1].strip(); continue
    d=json.loads(l); print(f"{lib:28s} kernel_ms {d['roofline']['kernel_ms']:.4f}  ms/step {d['ms_per_step']:.4f}")
P
