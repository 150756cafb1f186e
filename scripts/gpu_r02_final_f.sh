#!/bin/bash
# Closing check on the final tree: the driver-protocol headline line first on the box,
# the full GPU suite, smoke, and the decimator shape envelope.  Outputs under gpurun_out/final3/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/final3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit $?
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python3 __graft_entry__.py smoke > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python3 -u scripts/shape_envelope.py > $O/shape_envelope.txt 2>&1 || exit $?
cat $O/bench_driver.json
