#!/bin/bash
# Submit one gpurun call, re-submitting ONLY while gpurun answers 3 ("no box or
# slot free right now": nothing ran, nothing charged), at most ATTEMPTS times,
# SLEEP seconds apart.  Any other exit code -- success, a refusal, or a failed
# or killed GPU command -- ends the loop at once: a GPU step is never re-run.
#   scripts/gpurun_wait.sh LOG TIMEOUT 'command'
log=$1 t=$2 cmd=$3
for i in $(seq 1 "${ATTEMPTS:-12}"); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$cmd" > "$log" 2>&1
  rc=$?
  echo "attempt $i rc=$rc" >> "$log.attempts"
  [ "$rc" -ne 3 ] && break
  sleep "${SLEEP:-150}"
done
echo "rc=$rc" >> "$log"
