#!/bin/bash
# SQ/LDS counters: product headline (70), its compute path (73), memory path (71), ILV (200/201)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u scripts/tune/pmc_variant.py gpurun_out/pmcv_r02e.json 70:1024 73:1024 71:1024 201:1024 > gpurun_out/pmcv_r02e.txt 2>&1
