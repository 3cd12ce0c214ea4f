#!/bin/bash
# BASELINE.json configs 3-5 on one GPU box (100 M lines each, the bench's
# defaults; no CPU baseline / delivery), then the LP_PROFILE stage points of
# the parse and URI kernels for configs 2-5 (tools/prof_points.py).
set -uo pipefail
TAG=${1:-configs}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
for w in 3 4 5; do
  timeout -k 10 500 python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-delivery \
      > "$O/bench_config$w.json" 2> "$O/bench_config$w.err" || { echo "config $w failed"; tail "$O/bench_config$w.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench_config$w.json').read().strip().splitlines()[-1]);print($w, d['value'], d['lines_per_s'], d['kernel_ms'], d['roofline']['frac'])"
done
for w in 2 3 4 5; do
  LP_WORKLOAD=$w timeout -k 10 300 python3 tools/prof_points.py 4000000 > "$O/stage_points_config$w.txt" 2>&1 \
      || { echo "points $w failed"; tail "$O/stage_points_config$w.txt"; exit 1; }
done
echo done
