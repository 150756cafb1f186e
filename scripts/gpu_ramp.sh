#!/bin/bash
# Cold-start ramp of the headline kernel and of its memory-only / compute-only
# variants, each in a fresh process after an idle pause, with the shader clock
# (scripts/tune/ramp.py).  Output: gpurun_out/ramp_<tag>.jsonl
set -o pipefail
TAG=${TAG:-a}
OUT=gpurun_out/ramp_$TAG.jsonl
: > $OUT
for v in ${VARIANTS:-prod 71 73 read prod}; do
  sleep ${IDLE:-15}
  timeout -k 10 120 python3 -u scripts/tune/ramp.py $v ${LAUNCHES:-300} >> $OUT 2> gpurun_out/ramp_$TAG.err || exit $?
  echo "done $v" 
done
