#!/bin/bash
# ILV headline in the product: full GPU suite, driver-style and steady bench
# lines (fma and strict), config 3's 8-channel share, rocprof stats + PMC
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/t_bench_driver.json 2> gpurun_out/t_bench_driver.err || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-pcie > gpurun_out/t_bench_steady.json 2> gpurun_out/t_bench_steady.err || exit $?
timeout -k 10 200 python3 bench.py --fp strict --no-cpu-baseline --no-pcie > gpurun_out/t_bench_strict.json 2> gpurun_out/t_bench_strict.err || exit $?
timeout -k 10 200 python3 bench.py --channels-per-gpu 8 --steps 20 --warmup 5 --no-cpu-baseline --no-pcie > gpurun_out/t_bench_ch8.json 2> gpurun_out/t_bench_ch8.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/t_prof_decim -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pcie > gpurun_out/t_prof_decim.log 2>&1 || exit $?
timeout -k 10 600 python3 scripts/pmc_traffic.py --workload decim --tag r02t > gpurun_out/t_pmc_decim.log 2>&1 || exit $?
