#!/bin/bash
# A/B of the FIR stream kernel: runtime tap loop (srcdsp_amd/lib/ab/base.so) against
# the tap count compiled in (the in-tree library), 3 interleaved rounds of the fir
# workload at steady state.  Output: gpurun_out/firab/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/firab
mkdir -p $O
for r in 1 2 3; do
  for v in base new; do
    lib=srcdsp_amd/lib/libsrcdsp_hip.so
    [ $v = base ] && lib=srcdsp_amd/lib/ab/base.so
    SRCDSP_HIP_LIB=$lib timeout -k 10 200 python3 bench.py --workload fir --steps 50 --warmup 100 --no-cpu-baseline > $O/${v}_$r.json 2> $O/${v}_$r.err || exit $?
  done
done
python3 - <<'PY'
import json, glob
for v in ("base", "new"):
    ms = [json.load(open(f))["roofline"]["kernel_ms"] for f in sorted(glob.glob(f"gpurun_out/firab/{v}_*.json"))]
    print(v, ms)
PY
