#!/bin/bash
# SQ counter passes on the parse kernel (separate runs, kernel trace only).
set -euo pipefail
TAG=${1:-sq}
LINES=${2:-4000000}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$O/counters_list.txt" 2>&1 || true
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_FLAT SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$O/p$i" -o run -- \
      python3 "$R/bench.py" --lines "$LINES" --steps 1 --warmup 0 --no-cpu-baseline > "$O/p$i.log" 2>&1
done
echo done
