#!/bin/bash
# gpurun wrapper: retries ONLY when no GPU slot / box was free (gpurun exit code 3: nothing ran,
# nothing charged), up to 20 times a minute apart.  Any other outcome (including a failed or
# killed GPU command) is returned as is -- never retried.
# usage: scripts/gpu_call.sh TIMEOUT_S 'command'
t=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@"
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q '"status": "transient"' gpurun_out/.last_call.json 2>/dev/null; then exit $rc; fi
  echo "[gpu_call] no slot free (rc $rc), retry $i in 60 s" >&2
  sleep 60
done
exit 3
