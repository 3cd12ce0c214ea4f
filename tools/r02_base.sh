#!/bin/bash
# round-2 baseline: stage cycles of the current engine (LP_PROFILE build) + a short bench
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r02_base
mkdir -p "$O"
timeout -k 10 300 python3 "$R/tools/prof_points.py" 4000000 > "$O/points.txt" 2> "$O/points.err"
timeout -k 10 400 python3 "$R/bench.py" --lines 20000000 --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench20m.json" 2> "$O/bench20m.err"
echo done
