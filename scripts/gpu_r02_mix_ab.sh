#!/bin/bash
# A/B (tuning): config-4 two-word mixer table vs the HEAD library, same box; mixer/chain parity first
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 200 --timeout-method thread \
  -k "mix or config4 or pipeline or fuzz or ci16" > gpurun_out/mix_tests.log 2>&1 || { tail -30 gpurun_out/mix_tests.log; exit 1; }
tail -2 gpurun_out/mix_tests.log
: > gpurun_out/mix_ab.txt
for round in 1 2 3; do
  for lib in srcdsp_amd/lib_ab/libsrcdsp_hip_head.so srcdsp_amd/lib/libsrcdsp_hip.so; do
    echo "## $lib" >> gpurun_out/mix_ab.txt
    SRCDSP_HIP_LIB=$PWD/$lib timeout -k 10 120 python3 -u bench.py --workload mixdecim --steps 100 --warmup 50 --no-cpu-baseline >> gpurun_out/mix_ab.txt 2>/dev/null || exit $?
  done
done
python3 - <<'P'
import json
lib=None
for l in open('gpurun_out/mix_ab.txt'):
    if l.startswith('##'): lib=l.split('/')[-1].strip(); continue
    d=json.loads(l); print(f"{lib:28s} kernel_ms {d['roofline']['kernel_ms']:.4f}  ms/step {d['ms_per_step']:.4f}")
P
