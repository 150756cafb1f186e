#!/bin/bash
# Final round-2 evidence on the final kernels (after PMC refresh): the driver-protocol
# headline line first on the fresh box, the full GPU suite, smoke, every bench line,
# the decimator shape envelope and the interpolator envelope.  Outputs under gpurun_out/final2/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/final2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit $?
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python3 __graft_entry__.py smoke > $O/smoke.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-pcie > $O/bench_decim_steady.json 2> $O/bench_decim_steady.err || exit $?
timeout -k 10 200 python3 bench.py --fp strict --steps 200 --warmup 100 --no-cpu-baseline --no-pcie > $O/bench_strict.json 2> $O/bench_strict.err || exit $?
timeout -k 10 200 python3 bench.py --channels-per-gpu 8 --steps 20 --warmup 5 --no-cpu-baseline --no-pcie > $O/bench_decim8ch.json 2> $O/bench_decim8ch.err || exit $?
for w in mixdecim ci16decim fir up fifo iq; do
  timeout -k 10 300 python3 bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || exit $?
done
timeout -k 10 300 python3 bench.py --workload corr --samples 67108864 --steps 3 --warmup 1 > $O/bench_corr.json 2> $O/bench_corr.err || exit $?
timeout -k 10 300 python3 -u scripts/shape_envelope.py > $O/shape_envelope.txt 2>&1 || exit $?
timeout -k 10 300 python3 -u scripts/up_envelope.py > $O/up_envelope.txt 2>&1 || exit $?
ls $O
