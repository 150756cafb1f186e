#!/bin/bash
# Permlane whole-line stores (OST=2) in the headline and FIR kernels: full GPU
# parity suite, then headline evidence and the FIR bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${name}.log" 2>&1
  local rc=$?
  echo "[$name] exit $rc" >> gpurun_out/steps.log
  if [ "$rc" -ne 0 ]; then echo "stopping after $name"; exit "$rc"; fi
}
step tests_k 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench_decim_k 300 python bench.py
step bench_fir_k 300 python bench.py --workload fir --no-pcie
step prof_decim_k 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_decim_k -o run --output-format csv -- python bench.py --no-cpu-baseline --no-pcie
step prof_fir_k 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fir_k -o run --output-format csv -- python bench.py --workload fir --no-cpu-baseline --no-pcie
step pmc_k 600 python scripts/pmc_traffic.py --workload decim --tag k
