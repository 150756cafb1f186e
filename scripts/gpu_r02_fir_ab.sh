#!/bin/bash
# FIR window reads kept whole ds_read_b128: parity, same-box A/B vs HEAD, then PMC traffic
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "fir or golden" \
  > gpurun_out/fir_tests.log 2>&1 || { tail -30 gpurun_out/fir_tests.log; exit 1; }
tail -2 gpurun_out/fir_tests.log
: > gpurun_out/fir_ab.txt
for round in 1 2 3; do
  for lib in srcdsp_amd/lib_ab/libsrcdsp_hip_head.so srcdsp_amd/lib/libsrcdsp_hip.so; do
    echo "## $lib" >> gpurun_out/fir_ab.txt
    SRCDSP_HIP_LIB=$PWD/$lib timeout -k 10 120 python3 -u bench.py --workload fir --steps 100 --warmup 50 --no-cpu-baseline >> gpurun_out/fir_ab.txt 2>/dev/null || exit $?
  done
done
python3 - <<'P'
import json
lib=None
for l in open('gpurun_out/fir_ab.txt'):
    if l.startswith('##'): lib=l.split('/')[-1].strip(); continue
    d=json.loads(l); print(f"{lib:28s} kernel_ms {d['roofline']['kernel_ms']:.4f}  ms/step {d['ms_per_step']:.4f}")
P
timeout -k 10 400 python3 scripts/pmc_traffic.py --workload fir --tag r02final > gpurun_out/pmc_fir_final.log 2>&1 || { tail -20 gpurun_out/pmc_fir_final.log; exit 1; }
grep -E '"SQ_LDS_BANK_CONFLICT"|traffic_over' gpurun_out/pmc_fir_r02final.json
