#!/bin/bash
# BASELINE.json configs 3, 4 and 5 on one GPU (default sizes), one bench line each
set -uo pipefail
TAG=${1:-configs}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for w in 3 4 5; do
  timeout -k 10 400 python3 bench.py --workload $w > "$O/bench_config$w.json" 2> "$O/bench_config$w.err" || { echo "config $w failed"; tail -5 "$O/bench_config$w.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_config$w.json'));print($w, d['value'], d['kernel_ms'], d['roofline']['frac'], d['status_counts'])"
done
echo done
