#!/bin/bash
# SQ instruction mix / wave cycles of experiment builds (k_parse_chunks), 4M config-2 lines
set -uo pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp; export TMPDIR=/tmp
for n in "$@"; do
  mkdir -p $O/$n
  LOGPARSER_AMD_LIB=$R/logparser_amd/_exp/$n/liblogparser_amd.so timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM \
    --kernel-trace --output-format csv -d $O/$n/p1 -o run -- python3 $R/bench.py --lines 4000000 --steps 1 --warmup 0 --no-cpu-baseline --no-delivery > $O/$n/p1.log 2>&1 || { echo "p1 failed"; exit 1; }
  LOGPARSER_AMD_LIB=$R/logparser_amd/_exp/$n/liblogparser_amd.so timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS \
    --kernel-trace --output-format csv -d $O/$n/p3 -o run -- python3 $R/bench.py --lines 4000000 --steps 1 --warmup 0 --no-cpu-baseline --no-delivery > $O/$n/p3.log 2>&1 || { echo "p3 failed"; exit 1; }
  echo "== $n"; python3 $R/tools/sq_summary.py $O/$n | grep -A20 "^k_parse_chunks" | grep "per wave"
done
