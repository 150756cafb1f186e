cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
run() { local n=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "[$n] $rc" >> gpurun_out/steps.log; return $rc; }
run tests_b 900 python -m pytest tests -m gpu -q --maxfail=20 ; rc=$?; [ $rc -gt 1 ] && exit $rc
run bench_decim 300 python bench.py || exit 1
run bench_mixdecim 300 python bench.py --workload mixdecim --no-cpu-baseline || exit 1
run bench_corr 600 python bench.py --workload corr --samples 67108864 --steps 3 --warmup 1 --no-cpu-baseline || exit 1
run prof_mix 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mix -o run --output-format csv -- python bench.py --workload mixdecim --steps 10 --warmup 2 --no-cpu-baseline
