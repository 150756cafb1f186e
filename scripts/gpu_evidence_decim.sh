#!/bin/bash
# Headline-only evidence: bench line, rocprofv3 kernel stats, PMC traffic (outputs gpurun_out/ev3_*).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/ev3_decim_bench.json 2> gpurun_out/ev3_decim_bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_decim_ev3 -o run --output-format csv -- python bench.py --no-cpu-baseline --no-pcie > gpurun_out/ev3_decim_under_rocprof.json 2> gpurun_out/ev3_prof.err || exit $?
timeout -k 10 600 python scripts/pmc_traffic.py --workload decim --tag ev3 > gpurun_out/ev3_pmc.log 2>&1 || exit $?
