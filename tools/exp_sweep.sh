#!/bin/bash
# Parse-kernel time of experiment builds (tools/build_exp.sh) x field sets.
#   tools/exp_sweep.sh LINES "lib1 lib2 ..." "fields1" "fields2" ...
set -euo pipefail
LINES=$1; LIBS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/exp
mkdir -p "$O"
for lib in $LIBS; do
  for f in "$@"; do
    path=$R/logparser_amd/_lib/liblogparser_amd.so
    [ "$lib" != base ] && path=$R/logparser_amd/_dbg/$lib.so
    LOGPARSER_AMD_LIB=$path timeout -k 10 120 python3 "$R/bench.py" --lines "$LINES" --steps 3 --warmup 1 \
        --no-cpu-baseline --fields "$f" ${BENCH_ARGS:-} > "$O/run.json" 2> "$O/run.err"
    echo "$lib | $f | $(python3 -c "import json; d=json.load(open('$O/run.json')); print(d['kernel_ms']['parse_avg'], d['status_counts'])")"
  done
done
