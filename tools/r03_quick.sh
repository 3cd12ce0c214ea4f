#!/bin/bash
# 20M-line config-2 bench with a kernel trace, then the stage profile
# (LP_PROFILE build) of both parse kernels on 4M lines.
set -uo pipefail
TAG=${1:-r03_quick}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- \
    python3 "$R/bench.py" --lines 20000000 --steps 3 --warmup 2 --no-cpu-baseline --no-delivery > "$O/bench20m.json" 2> "$O/bench20m.err" || exit 1
cd "$R"
timeout -k 10 300 python3 tools/prof_points.py 4000000 > "$O/points.txt" 2>&1 || exit 1
echo done
