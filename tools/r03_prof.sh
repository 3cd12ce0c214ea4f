#!/bin/bash
# Stage profile of both parse kernels (LP_PROFILE build, wave timestamps) and
# their SQ instruction mix / wait counters, 4M config-2 lines.
set -uo pipefail
TAG=${1:-r03_prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 tools/prof_points.py 4000000 > "$O/points.txt" 2>&1 || { echo "points failed"; exit 1; }
bash tools/sq_mix.sh "$TAG/sq" || exit 1
echo done
