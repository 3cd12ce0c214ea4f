#!/bin/bash
# SQ/SQC counter passes over k_parse_lines (4M-line bench), one rocprofv3 --pmc run per pass
set -uo pipefail
LINES=${LINES:-4000000}
TAG=${TAG:-sq_probe}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_BRANCH"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P3="SQ_WAVES SQ_INST_CYCLES_SMEM SQ_LEVEL_WAVES SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_INSTS_VMEM_WR"
P4="SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQC_TC_STALL"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$O/p$i" -o run -- \
      python3 "$R/bench.py" --lines "$LINES" --steps 1 --warmup 1 --no-cpu-baseline > "$O/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
  echo "pass $i ok"
done
echo done
