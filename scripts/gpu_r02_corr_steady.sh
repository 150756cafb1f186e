#!/bin/bash
# The correlator line at round 1's steady-state protocol (--steps 200 --warmup 100; the
# round-2 evidence scripts ran it cold, --steps 3 --warmup 1), with its rocprofv3 stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/corr
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --workload corr --samples 67108864 --steps 200 --warmup 100 > $O/bench_corr.json 2> $O/bench_corr.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_corr -o run --output-format csv \
    -- python3 bench.py --workload corr --samples 67108864 --steps 200 --warmup 100 --no-cpu-baseline --no-pcie > $O/prof_corr.log 2>&1 || exit $?
find $O -name "*kernel_stats.csv"
