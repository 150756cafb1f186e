#!/bin/bash
# One GPU session (the single session script; earlier rounds' one-off scripts
# are folded into these steps).  STEPS is a space-separated list, run in
# order; every GPU step has its own time limit, and a fault / abort / timeout
# ends the script (no retries).  Outputs go to gpurun_out/, tagged ${TAG}.
#
#   smoke            __graft_entry__.py smoke
#   tests            pytest -m gpu (PYTEST_K: -k filter)
#   bench            bench.py ${BENCH_ARGS} (default: the headline, driver protocol --steps 20 --warmup 5)
#   bench_all        every workload's bench line (steady protocol)
#   bench_cold       every workload's line under the driver's protocol (--warmup 5 --steps 20), IDLE s apart
#   bench8           config 3's per-GPU share (--channels-per-gpu 8), driver protocol and steady
#   prof             rocprofv3 --kernel-trace --stats of bench.py ${BENCH_ARGS} (per-dispatch CSV kept)
#   pmc              FETCH_SIZE / WRITE_SIZE passes (scripts/pmc_traffic.py) for each of ${PMC_WORKLOADS}
#                    (decimx8 = the headline's 8-channel batched step, config 3's per-GPU share);
#                    merge into profiles/pmc_traffic.json with scripts/merge_pmc.py TAG
#   ramp             cold ramps of tune variants ${VARIANTS} (scripts/tune/ramp.py), IDLE s apart
#   wpower           socket power / clock / limiter counters through a cold start (scripts/tune/window_power.py)
#                    for each tap count of ${WP_TAPS} (default 127)
#   phase            per-phase cycles of the config-4 kernel (scripts/tune/phase_clock.py; tuning build
#                    scripts/tune/ab/libsrcdsp_hip_phase.so)
#   pmcw             SQ/LDS counter passes (scripts/tune/pmc_workload.py) for each WORKLOAD:KERNEL of ${PMCW}
#   envelope         scripts/shape_envelope.py ${ENV_M}
#   census           workgroup placement census (scripts/tune/census.py)
#   ab               same-box A/B of scripts/tune/ab/libsrcdsp_hip_base.so vs the tree's library
#                    (scripts/tune/ab_libs.sh; WORKLOADS, ROUNDS, LAUNCHES)
#   dist             the 2-rank GPU test of the N > 1 path (tests/test_gpu_dist.py)
#   cpp              the drop-in C++ tests (tests/test_dropin_cpp.py -m gpu)
#   merge            scripts/merge_pmc.py ${TAG} on the box, so a later bench step in the same session reports the
#                    traffic just measured (merge locally too: gpurun_out/ comes back, profiles/ does not)
#   mfma             the integer matrix-core probes (tuning only, never shipped): config 5's correlator
#                    (scripts/tune/corr_mfma.py ${CORR_ARGS}, for each of ${CORR_LIBS}) and config 4's tap loop
#                    (scripts/tune/mixdecim_mfma.py ${MIX_ARGS}), each checked against the oracle and timed
#                    beside the product on the same box
#   mixlib           config 4's chain with its tap loop on the i8 matrix cores behind the product's C ABI (tuning
#                    library scripts/tune/ab/libsrcdsp_hip_mixmfma.so, never shipped): parity, tests, bench
#   pg1              bench.py's N > 1 path at one rank on RCCL (SRCDSP_BENCH_PG=1, launched by torchrun)
#   corrlib          the correlator's fused scan on the i8 matrix cores behind the product's C ABI (tuning
#                    library scripts/tune/ab/libsrcdsp_hip_corrmfma.so, never shipped): parity, tests, bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-s}
step() {  # step NAME SECONDS cmd...: stdout+stderr to gpurun_out/NAME.log
  local name=$1 t=$2; shift 2
  echo "[$name] start $(date +%T)"
  timeout -k 10 "$t" "$@" > "gpurun_out/${name}.log" 2>&1
  local rc=$?
  echo "[$name] exit $rc" | tee -a gpurun_out/steps_$TAG.log
  # 1 = test failures (keep going); anything else (fault, abort, timeout) ends the session
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $name"; exit "$rc"; fi
  return 0
}
for s in ${STEPS:-smoke tests bench}; do
  case $s in
    smoke) step smoke_$TAG 300 python -u __graft_entry__.py smoke ;;
    tests) step tests_$TAG 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
             --maxfail=30 --durations=25 ${PYTEST_K:+-k "$PYTEST_K"} ;;
    bench) step bench_$TAG 300 python -u bench.py ${BENCH_ARGS:---steps 20 --warmup 5} ;;
    bench_all)
      for w in decim mixdecim ci16decim corr fir up; do
        step bench_${w}_$TAG 300 python -u bench.py --workload $w --no-cpu-baseline --no-pcie
      done ;;
    bench8)  # config 3's per-GPU share (8 x 2^28 channels per step): driver protocol, then steady
      step bench8cold_$TAG 300 python -u bench.py --channels-per-gpu 8 --warmup 5 --steps 20 --no-cpu-baseline --no-pcie
      step bench8_$TAG 300 python -u bench.py --channels-per-gpu 8 --warmup 20 --steps 50 --no-cpu-baseline --no-pcie ;;
    bench_cold)  # the driver's protocol for every workload, each a fresh process after ${IDLE:-8} s idle
      for w in decim mixdecim ci16decim corr fir up; do
        sleep ${IDLE:-8}
        step benchcold_${w}_$TAG 300 python -u bench.py --workload $w --no-cpu-baseline --no-pcie --warmup 5 --steps 20
      done ;;
    prof) step prof_$TAG 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv \
            -- python3 bench.py --no-cpu-baseline --no-pcie ${BENCH_ARGS:---steps 20 --warmup 5} ;;
    pmc)
      for w in ${PMC_WORKLOADS:-decim}; do
        if [ "$w" = decimx8 ]; then
          step pmc_${w}_$TAG 600 python -u scripts/pmc_traffic.py --workload decim --channels 8 --tag $TAG
        else
          step pmc_${w}_$TAG 600 python -u scripts/pmc_traffic.py --workload $w --tag $TAG
        fi
      done ;;
    ramp)
      : > gpurun_out/ramp_$TAG.jsonl
      for v in ${VARIANTS:-prod}; do
        sleep ${IDLE:-8}
        step ramp_${TAG}_$v 150 python3 -u scripts/tune/ramp.py $v ${LAUNCHES:-300}
        tail -n 1 gpurun_out/ramp_${TAG}_$v.log >> gpurun_out/ramp_$TAG.jsonl
      done ;;
    wpower)
      for tp in ${WP_TAPS:-127}; do
        step wpower_${TAG}_$tp 120 python3 -u scripts/tune/window_power.py ${LAUNCHES:-300} ${IDLE:-8} $tp
      done ;;
    phase) SRCDSP_HIP_LIB=$PWD/scripts/tune/ab/libsrcdsp_hip_phase.so \
             step phase_$TAG 120 python3 -u scripts/tune/phase_clock.py ${PHASE_WL:-mixdecim} ;;
    pmcw)
      for wk in ${PMCW:-mixdecim:decim_dot2_ci16}; do
        w=${wk%%:*}; k=${wk#*:}
        step pmcw_${w}_$TAG 300 python -u scripts/tune/pmc_workload.py gpurun_out/pmcw_${w}_$TAG.json $w $k
      done ;;
    envelope) step envelope_$TAG 600 python -u scripts/shape_envelope.py ${ENV_M} ;;
    census) step census_$TAG 120 python -u scripts/tune/census.py ;;
    ab) step ab_$TAG 1000 bash scripts/tune/ab_libs.sh ;;
    dist) step dist_$TAG 300 python -u -m pytest tests/test_gpu_dist.py -m gpu -v --timeout 240 --timeout-method thread ;;
    merge)  # this session's PMC entries into profiles/pmc_traffic.json (on the box: a later bench step reports them)
      step merge_$TAG 60 python -u scripts/merge_pmc.py $TAG ;;
    mfma)
      for lib in ${CORR_LIBS:-libcorrmfma.so}; do
        step corrmfma_${lib%.so}_$TAG 400 python -u scripts/tune/corr_mfma.py --lib $lib ${CORR_ARGS}
      done
      step mixmfma_$TAG 400 python -u scripts/tune/mixdecim_mfma.py ${MIX_ARGS} ;;
    mfmapmc)  # SQ / MFMA counter passes of the two probes' kernels
      for lib in ${CORR_LIBS:-libcorrmfma.so}; do
        step corrmfmapmc_${lib%.so}_$TAG 600 python -u scripts/tune/pmc_cmd.py gpurun_out/corrmfma_pmc_${lib%.so}_$TAG.json \
          corr_mfma_i8 -- python3 scripts/tune/corr_mfma.py --only-probe --reps 8 --lib $lib
      done
      step mixmfmapmc_$TAG 600 python -u scripts/tune/pmc_cmd.py gpurun_out/mixmfma_pmc_$TAG.json mixdecim_mfma_i8 \
        -- python3 scripts/tune/mixdecim_mfma.py --only-probe --reps 8 ;;
    corrlib)  # the corrmfma tuning library behind the product's C ABI: its own seam / history / limb
              # cases, the correlator GPU tests, then config 5's bench line beside the product's
      L=$PWD/scripts/tune/ab/libsrcdsp_hip_corrmfma.so
      SRCDSP_HIP_LIB=$L step corrlib_check_$TAG 300 python -u scripts/tune/corr_mfma_lib.py
      SRCDSP_HIP_LIB=$L SRCDSP_CORR_MFMA_RB=1 step corrlib_checkrb1_$TAG 300 python -u scripts/tune/corr_mfma_lib.py
      SRCDSP_HIP_LIB=$L step corrlib_tests_$TAG 900 python -u -m pytest tests -m gpu -q --timeout 120 \
        --timeout-method thread --maxfail=30 -k "corr or config5 or time_split"
      SRCDSP_HIP_LIB=$L SRCDSP_CORR_MFMA_PL=2 step corrlib_tests2_$TAG 600 python -u -m pytest \
        tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -k "config5 or time_split"
      for rep in 1 2; do
        sleep ${IDLE:-8}
        step corrlib_benchprod${rep}_$TAG 300 python -u bench.py --workload corr --no-cpu-baseline --no-pcie --warmup 5 --steps 20
        sleep ${IDLE:-8}
        SRCDSP_HIP_LIB=$L step corrlib_bench${rep}_$TAG 300 python -u bench.py --workload corr --no-cpu-baseline --no-pcie \
          --warmup 5 --steps 20
        sleep ${IDLE:-8}
        SRCDSP_HIP_LIB=$L SRCDSP_CORR_MFMA_PL=2 step corrlib_bench2l${rep}_$TAG 300 python -u bench.py --workload corr \
          --no-cpu-baseline --no-pcie --warmup 5 --steps 20
        sleep ${IDLE:-8}
        SRCDSP_HIP_LIB=$L SRCDSP_CORR_MFMA_RB=1 step corrlib_benchrb1${rep}_$TAG 300 python -u bench.py --workload corr \
          --no-cpu-baseline --no-pcie --warmup 5 --steps 20
      done
      SRCDSP_HIP_LIB=$L step corrlib_prof_$TAG 300 rocprofv3 --kernel-trace --stats -d gpurun_out/corrlib_prof_$TAG -o run \
        --output-format csv -- python3 bench.py --workload corr --no-cpu-baseline --no-pcie --warmup 5 --steps 20 ;;
    mixlib)  # the mixmfma tuning library behind the product's C ABI: its own cases, the chain GPU tests,
             # then config 4's bench line beside the product's
      L=$PWD/scripts/tune/ab/libsrcdsp_hip_mixmfma.so
      SRCDSP_HIP_LIB=$L step mixlib_check_$TAG 300 python -u scripts/tune/mixdecim_mfma_lib.py
      SRCDSP_HIP_LIB=$L step mixlib_tests_$TAG 900 python -u -m pytest tests -m gpu -q --timeout 120 \
        --timeout-method thread --maxfail=30 -k "chain or mixdecim or config4 or mixer or pipeline or streams or decim"
      for rep in 1 2; do
        sleep ${IDLE:-8}
        step mixlib_benchprod${rep}_$TAG 300 python -u bench.py --workload mixdecim --no-cpu-baseline --no-pcie \
          --warmup 5 --steps 20
        sleep ${IDLE:-8}
        SRCDSP_HIP_LIB=$L step mixlib_bench${rep}_$TAG 300 python -u bench.py --workload mixdecim --no-cpu-baseline \
          --no-pcie --warmup 5 --steps 20
      done
      for rep in 1 2; do  # row a2 (the plain decimator) through the same kernel
        sleep ${IDLE:-8}
        step mixlib_a2prod${rep}_$TAG 300 python -u bench.py --workload ci16decim --no-cpu-baseline --no-pcie \
          --warmup 5 --steps 20
        sleep ${IDLE:-8}
        SRCDSP_HIP_LIB=$L step mixlib_a2${rep}_$TAG 300 python -u bench.py --workload ci16decim --no-cpu-baseline \
          --no-pcie --warmup 5 --steps 20
      done
      SRCDSP_HIP_LIB=$L step mixlib_steady_$TAG 300 python -u bench.py --workload mixdecim --no-cpu-baseline --no-pcie \
        --warmup 100 --steps 50
      step mixlib_steadyprod_$TAG 300 python -u bench.py --workload mixdecim --no-cpu-baseline --no-pcie \
        --warmup 100 --steps 50
      SRCDSP_HIP_LIB=$L step mixlib_prof_$TAG 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mixlib_prof_$TAG -o run \
        --output-format csv -- python3 bench.py --workload mixdecim --no-cpu-baseline --no-pcie --warmup 5 --steps 20 ;;
    libpmc)  # MFMA-busy / clock counters of the two C-ABI matrix-core builds' kernels (PMC_PASSES, default MFMA + traffic)
      SRCDSP_HIP_LIB=$PWD/scripts/tune/ab/libsrcdsp_hip_corrmfma.so PMC_PASSES=${PMC_PASSES:-0,4,5} step libpmc_corr_$TAG 400 \
        python -u scripts/tune/pmc_cmd.py gpurun_out/libpmc_corr_$TAG.json corr_scan_mfma \
        -- python3 bench.py --workload corr --no-cpu-baseline --no-parity --warmup 2 --steps 8
      SRCDSP_HIP_LIB=$PWD/scripts/tune/ab/libsrcdsp_hip_mixmfma.so PMC_PASSES=${PMC_PASSES:-0,4,5} step libpmc_mix_$TAG 400 \
        python -u scripts/tune/pmc_cmd.py gpurun_out/libpmc_mix_$TAG.json mixdecim_mfma_step_i8 \
        -- python3 bench.py --workload mixdecim --no-cpu-baseline --no-pcie --no-parity --warmup 2 --steps 8 ;;
    pg1)  # the N > 1 path on the real backend at one rank (torchrun, RCCL process group, device collectives,
          # the share's gather and its digests; bench.py SRCDSP_BENCH_PG=1)
      SRCDSP_BENCH_PG=1 step pg1_decim_$TAG 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --share --steps 5 --warmup 2 --no-cpu-baseline --no-pcie
      SRCDSP_BENCH_PG=1 step pg1_corr_$TAG 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 1 --workload corr --steps 5 --warmup 2 --no-cpu-baseline ;;
    cpp) step cpp_$TAG 600 python -u -m pytest tests/test_dropin_cpp.py -m gpu -v --timeout 240 --timeout-method thread ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "session $TAG done"
