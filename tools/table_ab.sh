#!/bin/bash
# Device-table kernel variants (logparser_amd/_exp/<name>, make exp EXPU=table)
# against each other: tools/table_bench.py per build, twice interleaved.
#   tools/table_ab.sh TAG LINES name1 name2 ...
set -uo pipefail
TAG=$1; LINES=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for rep in 1 2; do
  for n in "$@"; do
    LOGPARSER_AMD_LIB=$R/logparser_amd/_exp/$n/liblogparser_amd.so timeout -k 10 120 python3 tools/table_bench.py "$LINES" \
        > "$O/$n.$rep.txt" 2> "$O/$n.$rep.err" || { echo "$n failed"; tail -5 "$O/$n.$rep.err"; exit 1; }
    echo "$n $rep $(tail -1 "$O/$n.$rep.txt")"
  done
done
