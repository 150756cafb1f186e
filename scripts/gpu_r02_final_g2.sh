#!/bin/bash
# After the 31-tap FIR specialisation: the closing check (driver-protocol headline line
# first, full suite, smoke, envelope: gpu_r02_final_f.sh), then the fir bench line and its
# rocprofv3 kernel stats.  Outputs under gpurun_out/final3/ and gpurun_out/final6/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_r02_final_f.sh || exit $?
O=gpurun_out/final6
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --workload fir > $O/fir_bench.json 2> $O/fir_bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fir -o run --output-format csv \
    -- python3 bench.py --workload fir --no-cpu-baseline --no-pcie > $O/prof_fir.log 2>&1 || exit $?
find $O -name "*kernel_stats.csv" | sort
