#!/bin/bash
# socket power / gfx clock per headline variant (read-only amdsmi), 3 s each
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/power_r02z.jsonl
for v in read 71 201 200 70 73 303 prod; do
  sleep 3
  timeout -k 10 60 python3 -u scripts/tune/power.py $v 3 >> gpurun_out/power_r02z.jsonl 2> gpurun_out/power_r02z.err || exit $?
done
