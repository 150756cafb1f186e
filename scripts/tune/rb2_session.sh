# the two-row-block correlator probe (CORR_ROWB=2, one limb) beside the base probe, twice, interleaved
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for l in libcorrmfma.so libcorrmfma_rb2.so; do
    timeout -k 10 400 python -u scripts/tune/corr_mfma.py --lib $l --pattern-limbs 1 $( [ $rep = 2 ] && echo --no-check ) \
      > gpurun_out/rb2_${l%.so}_$rep.log 2>&1 || exit $?
  done
done
