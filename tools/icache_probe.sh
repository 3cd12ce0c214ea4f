#!/bin/bash
# Instruction-cache pressure of the parse kernel: list the counters, then one
# PMC pass (kernel trace only) with the SQ / SQC instruction-fetch counters.
set -uo pipefail
TAG=${1:-icache}
LINES=${2:-4000000}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$O/counters_list.txt" 2>&1
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQC_TC_INST[A-Z_]*\|SQ_INST_LEVEL[A-Z_]*" "$O/counters_list.txt" | sort -u > "$O/icache_names.txt"
want=""
for c in SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAIT_ANY; do
  grep -qw "$c" "$O/counters_list.txt" && want="$want $c"
done
echo "pmc:$want" > "$O/pmc_used.txt"
timeout -s KILL 200 rocprofv3 --pmc $want --kernel-trace --output-format csv -d "$O/p1" -o run -- \
    python3 "$R/bench.py" --lines "$LINES" --steps 1 --warmup 0 --no-cpu-baseline > "$O/p1.log" 2>&1
echo "rc=$?"
echo done
