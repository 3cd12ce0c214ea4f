#!/bin/bash
# Arbitrary PMC passes on the parse kernel, one rocprofv3 run per pass
# (kernel trace only; never combined with runtime/sys traces).
#   tools/pmc_passes.sh TAG LINES "CNT CNT ..." ["CNT ..."]...
set -euo pipefail
TAG=$1; LINES=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$O/p$i" -o run -- \
      python3 "$R/bench.py" --lines "$LINES" --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-} > "$O/p$i.log" 2>&1
done
python3 "$R/tools/sq_summary.py" "$O"
