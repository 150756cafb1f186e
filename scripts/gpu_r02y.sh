#!/bin/bash
# round-2 evidence, part 2: rocprofv3 kernel stats of every workload, PMC HBM traffic
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/y
export TMPDIR=/tmp
O=gpurun_out/y
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
for w in decim mixdecim ci16decim fir up; do
  timeout -k 10 400 python3 scripts/pmc_traffic.py --workload $w --tag r02 > $O/pmc_$w.log 2>&1 || exit $?
done
