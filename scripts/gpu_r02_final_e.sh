#!/bin/bash
# Final round-2 evidence on the final kernels: rocprofv3 kernel stats of every bench workload
# (the driver's --steps 20 --warmup 5 protocol for the headline)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/final2
mkdir -p $O
export TMPDIR=/tmp
prof() {  # workload, extra bench args...
  local w=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv \
      -- python3 bench.py --workload $w --no-cpu-baseline --no-pcie "$@" > $O/prof_$w.log 2>&1
}
prof decim --steps 20 --warmup 5 || exit $?
prof mixdecim || exit $?
prof ci16decim || exit $?
prof fir || exit $?
prof up || exit $?
prof corr --samples 67108864 --steps 3 --warmup 1 || exit $?
find $O -name "*kernel_stats.csv" | sort
