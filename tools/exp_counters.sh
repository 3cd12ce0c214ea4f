#!/bin/bash
# SQ counters of experiment builds (logparser_amd/_dbg/exp<N>.so, 0 = product), one PMC pass each
set -uo pipefail
LINES=${LINES:-4000000}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/exp_counters
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
for e in "$@"; do
  if [ "$e" = "0" ]; then unset LOGPARSER_AMD_LIB; else export LOGPARSER_AMD_LIB=$R/logparser_amd/_dbg/exp$e.so; fi
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY \
      --kernel-trace --output-format csv -d "$O/e$e" -o run -- \
      python3 "$R/bench.py" --lines "$LINES" --steps 1 --warmup 1 --no-cpu-baseline > "$O/e$e.log" 2>&1 || exit 1
done
echo done
