#!/bin/bash
# Instruction mix and LDS pressure of the parse kernel: two PMC passes of <= 8
# SQ counters each (kernel trace only), 4M config-2 lines.
set -uo pipefail
TAG=${1:-sqmix}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM \
    --kernel-trace --output-format csv -d "$O/p1" -o run -- \
    python3 "$R/bench.py" --lines 4000000 --steps 1 --warmup 0 --no-cpu-baseline --no-delivery > "$O/p1.log" 2>&1 || { echo "p1 failed"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS \
    --kernel-trace --output-format csv -d "$O/p2" -o run -- \
    python3 "$R/bench.py" --lines 4000000 --steps 1 --warmup 0 --no-cpu-baseline --no-delivery > "$O/p2.log" 2>&1 || { echo "p2 failed"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    --kernel-trace --output-format csv -d "$O/p3" -o run -- \
    python3 "$R/bench.py" --lines 4000000 --steps 1 --warmup 0 --no-cpu-baseline --no-delivery > "$O/p3.log" 2>&1 || { echo "p3 failed"; exit 1; }
python3 "$R/tools/sq_summary.py" "$O" > "$O/summary.txt"
echo done
