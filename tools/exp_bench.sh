#!/bin/bash
# Experiment builds (logparser_amd/_exp/<name>, make exp) against each other:
# a 20M-line config-2 bench per build, parse / index kernel times.
#   tools/exp_bench.sh TAG name1 name2 ...
set -uo pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for n in "$@"; do
  LOGPARSER_AMD_LIB=$R/logparser_amd/_exp/$n/liblogparser_amd.so timeout -k 10 240 python3 bench.py --lines ${LINES:-20000000} \
      --steps 5 --warmup 2 --no-cpu-baseline --no-delivery ${BENCH_ARGS:-} > "$O/$n.json" 2> "$O/$n.err" || { echo "$n failed"; tail -5 "$O/$n.err"; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);print('%-12s value %8.1f parse %7.3f index %6.3f ok %d' % ('$n', d['value'], d['kernel_ms']['parse_avg'], d['kernel_ms']['index_avg'], d['status_counts']['ok']))"
done
