#!/bin/bash
# Evidence for the caller-side rows: FIFO ring and I/Q capture
# replay feeding the mixer->decimator chain.  Bench lines + rocprofv3 kernel
# and memory-copy stats (no PMC counters here).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for w in fifo iq; do
  timeout -k 10 300 python bench.py --workload $w --steps 40 --warmup 10 > gpurun_out/ev_${w}_bench.json 2> gpurun_out/ev_${w}_bench.err || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_${w} -o run --output-format csv \
      -- python bench.py --workload $w --steps 40 --warmup 10 --no-cpu-baseline > gpurun_out/ev_${w}_under_rocprof.json 2> gpurun_out/ev_${w}_prof.err || exit $?
done
