#!/bin/bash
# LDS-DMA loader/consumer ring (scripts/tune/decim_ring.h, tuning only): bit-exact
# check against the product on 2^28 samples, then same-box cold ramps (300
# launches each after an 8 s idle) beside the product and the ILV variant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python3 -u scripts/tune/wave_check.py 500 501 502 503 504 505 > gpurun_out/ring_check.log 2>&1
rc=$?; grep -v "skipped" gpurun_out/ring_check.log | tail -12; [ $rc -eq 0 ] || exit $rc
IDLE=8 TAG=r02ring VARIANTS="prod 500 501 502 503 504 505 200 prod" LAUNCHES=300 bash scripts/gpu_ramp.sh || exit $?
python3 - <<'P'
import json
for l in open('gpurun_out/ramp_r02ring.jsonl'):
    d=json.loads(l); print(f"{d['variant']:>5s} ms_6_25 {d['ms_6_25']:.4f} @ {d['ghz_6_25']} GHz | last100 {d['ms_last100']:.4f} @ {d['ghz_last100']} GHz")
P
