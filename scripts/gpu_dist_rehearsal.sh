#!/bin/bash
# Rehearse bench.py's N>1 path on ONE GPU: 2 ranks over gloo (collectives on
# host copies), torchrun on 127.0.0.1.  Checks that the code path runs end to
# end; the numbers are not scaling numbers (both ranks share one GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export SRCDSP_BENCH_BACKEND=gloo
for w in decim corr; do
  extra=""
  [ $w = corr ] && extra="--samples 16777216 --steps 2 --warmup 1"
  [ $w = decim ] && extra="--samples 67108864 --steps 3 --warmup 1"
  # bench.py --gpus 2 starts its own 2 ranks (a child torch.distributed.run)
  timeout -k 10 400 python bench.py --gpus 2 --workload $w --no-cpu-baseline $extra \
      > gpurun_out/dist_${w}.log 2>&1 || { echo "[dist_$w] failed"; exit 1; }
  echo "[dist_$w] ok"
done
