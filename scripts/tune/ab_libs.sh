#!/bin/bash
# Same-box A/B of builds of the product library (tuning only): LIBS names
# scripts/tune/ab/libsrcdsp_hip_<name>.so builds ("new" = the working tree's
# srcdsp_amd/lib/libsrcdsp_hip.so; default "base new"), interleaved ROUNDS
# times, each run a fresh process after IDLE s (scripts/tune/ramp.py on each
# bench workload in WORKLOADS).
# Output: gpurun_out/ab_${TAG}.jsonl (one line per run, "lib" = the name).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/ab_${TAG:-x}.jsonl
: > $OUT
for r in $(seq ${ROUNDS:-3}); do
  for lib in ${LIBS:-base new}; do
    for w in ${WORKLOADS:-mixdecim}; do
      sleep ${IDLE:-5}
      if [ $lib != new ]; then export SRCDSP_HIP_LIB=$PWD/scripts/tune/ab/libsrcdsp_hip_$lib.so; else unset SRCDSP_HIP_LIB; fi
      timeout -k 10 150 python3 -u scripts/tune/ramp.py w:$w ${LAUNCHES:-200} > gpurun_out/ab_last.log 2>&1 || { echo "ramp failed rc=$?"; tail -5 gpurun_out/ab_last.log; exit 1; }
      tail -n 1 gpurun_out/ab_last.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d.pop('ms'); d.pop('ghz'); d['lib']='$lib'; d['round']=$r; print(json.dumps(d))" >> $OUT
      echo "round $r $lib $w done"
    done
  done
done
