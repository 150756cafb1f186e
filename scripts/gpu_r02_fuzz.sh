#!/bin/bash
# the widened differential fuzz (new tuned shapes, special input values) on the GPU
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fuzz.py -q --timeout 240 --timeout-method thread > gpurun_out/fuzz.log 2>&1
rc=$?; tail -15 gpurun_out/fuzz.log; exit $rc
