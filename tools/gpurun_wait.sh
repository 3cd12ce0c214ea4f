#!/bin/bash
# Local helper (never runs on the GPU box): submit one gpurun call, and when
# the pool has no free box (exit 3 or a "transient" status: nothing ran,
# nothing charged) wait and submit the same call again, at most 8 times.
#   tools/gpurun_wait.sh TIMEOUT 'command' > log
T=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > /tmp/gpurun_wait.$$ 2>&1
  rc=$?
  cat /tmp/gpurun_wait.$$
  if [ $rc -eq 3 ] || grep -q "status=transient" /tmp/gpurun_wait.$$; then
    sleep 90
    continue
  fi
  rm -f /tmp/gpurun_wait.$$
  exit $rc
done
rm -f /tmp/gpurun_wait.$$
exit 3
