#!/bin/bash
# round-2 GPU check: parity tests, stage cycles (LP_PROFILE build), 20M-line bench
set -uo pipefail
TAG=${1:-r02_check}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?
echo "tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 "$R/tools/prof_points.py" 4000000 > "$O/points.txt" 2> "$O/points.err" || exit 1
timeout -k 10 400 python3 "$R/bench.py" --lines 20000000 --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench20m.json" 2> "$O/bench20m.err"
echo done
