#!/bin/bash
# cold ramps: ILV 512-lane tiles (200, the product shape) vs ILV 256-lane tiles (203) at grids 1024 / 2048
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
IDLE=8 TAG=r02r256a VARIANTS="200 203 200" LAUNCHES=300 bash scripts/gpu_ramp.sh || exit $?
RAMP_GRID=2048 IDLE=8 TAG=r02r256b VARIANTS="203" LAUNCHES=300 bash scripts/gpu_ramp.sh || exit $?
RAMP_GRID=4096 IDLE=8 TAG=r02r256c VARIANTS="203" LAUNCHES=300 bash scripts/gpu_ramp.sh || exit $?
python3 - <<'P'
import json
for tag in ("r02r256a","r02r256b","r02r256c"):
    for l in open(f'gpurun_out/ramp_{tag}.jsonl'):
        d=json.loads(l); print(f"{tag} {d['variant']:>5s} ms_6_25 {d['ms_6_25']:.4f} @ {d['ghz_6_25']} GHz | last100 {d['ms_last100']:.4f} @ {d['ghz_last100']} GHz")
P
