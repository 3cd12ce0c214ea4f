#!/bin/bash
# gpurun wrapper: retries ONLY when no box could be provided (exit 3, nothing
# ran, nothing charged).  Any other outcome -- including a failing command --
# is returned as is.
T=${GPU_TIMEOUT:-900}
for attempt in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 45
done
exit 3
