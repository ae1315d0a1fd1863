#!/bin/bash
# Submit one gpurun call, re-submitting only while the pool reports no free slot / box (exit status 3: nothing ran,
# nothing was charged); any other status (including a failed command) ends it.  usage: gpurun_wait.sh TIMEOUT CMD
T=$1; shift
for i in $(seq 1 ${GPURUN_ATTEMPTS:-15}); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[gpurun_wait] no slot (attempt $i), retrying in 90 s"
  sleep 90
done
exit 3
