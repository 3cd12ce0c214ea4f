#!/bin/bash
# Stage profile (LP_PROFILE build) of the parse and URI kernels on 4M
# config-2 lines, then the SQ instruction mix (tools/sq_mix.sh).
set -uo pipefail
TAG=${1:-r04_prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 tools/prof_points.py 4000000 > "$O/points.txt" 2>&1 || { echo "prof failed"; tail -20 "$O/points.txt"; exit 1; }
head -20 "$O/points.txt"
bash tools/sq_mix.sh "$TAG/sq" || exit 1
cat "$O/sq/summary.txt"
