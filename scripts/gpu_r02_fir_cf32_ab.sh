#!/bin/bash
# A/B of the cf32 FIR at 31 taps: runtime tap loop (srcdsp_amd/lib/ab/base.so) against
# the tap count compiled in (in-tree library), 3 interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fircf
for r in 1 2 3; do
  for v in base new; do
    lib=srcdsp_amd/lib/libsrcdsp_hip.so
    [ $v = base ] && lib=srcdsp_amd/lib/ab/base.so
    echo -n "$v: " >> gpurun_out/fircf/ab.txt
    SRCDSP_HIP_LIB=$lib timeout -k 10 120 python3 scripts/fir_cf32_time.py 31 >> gpurun_out/fircf/ab.txt 2> gpurun_out/fircf/err_$v$r.txt || exit $?
  done
done
cat gpurun_out/fircf/ab.txt
