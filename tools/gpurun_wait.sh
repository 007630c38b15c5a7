#!/bin/bash
# Submit one gpurun call, waiting while the pool has no box (exit 3: nothing ran, nothing charged) -- at most
# $TRIES attempts, $WAIT s apart.  Any other outcome (success or a failure of the command) ends the loop: a failed GPU
# step is never re-run.   tools/gpurun_wait.sh <timeout-s> '<command>'
T=$1; shift
for i in $(seq 1 ${TRIES:-12}); do
  /usr/local/graft/bin/gpurun --timeout $T -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[gpurun_wait] no box (attempt $i), waiting ${WAIT:-150}s" >&2
  sleep ${WAIT:-150}
done
exit 3
