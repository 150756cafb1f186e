#!/bin/bash
# persistent decim_tile: parity of every tile case, then the shape envelope
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread \
  -k "any_taps or persistent or ci16_tile or fir_ci16 or batched or generic or errors" \
  > gpurun_out/tile_tests.log 2>&1 || { tail -30 gpurun_out/tile_tests.log; exit 1; }
tail -3 gpurun_out/tile_tests.log
timeout -k 10 300 python3 -u scripts/shape_envelope.py > gpurun_out/tile_envelope.txt 2>&1 || { cat gpurun_out/tile_envelope.txt; exit 1; }
cat gpurun_out/tile_envelope.txt
