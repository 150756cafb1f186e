set -o pipefail
mkdir -p gpurun_out
for l in libcorrmfma.so libcorrmfma_dpp.so; do
  timeout -k 10 400 python -u scripts/tune/corr_mfma.py --lib $l > gpurun_out/dpp_${l%.so}.log 2>&1 || exit $?
done
A=$PWD/scripts/tune/ab/libsrcdsp_hip_corrmfma.so
D=$PWD/scripts/tune/ab/libsrcdsp_hip_corrmfmadpp.so
SRCDSP_HIP_LIB=$D timeout -k 10 300 python -u scripts/tune/corr_mfma_lib.py > gpurun_out/dpp_libcheck.log 2>&1 || exit $?
for rep in 1 2; do
  for v in A D; do
    sleep 8
    L=${!v}
    SRCDSP_HIP_LIB=$L timeout -k 10 300 python -u bench.py --workload corr --no-cpu-baseline --no-pcie --warmup 5 --steps 20 > gpurun_out/dpp_bench_${v}${rep}.log 2>&1 || exit $?
  done
done
