#!/bin/bash
# round-2 baseline: GPU parity tests, stage cycles of the current engine
# (LP_PROFILE build), a 20M-line bench under a rocprofv3 kernel trace
set -uo pipefail
TAG=${1:-r02_base}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
if [ "${SKIP_TESTS:-0}" = "0" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { echo "tests failed"; exit 1; }
fi
timeout -k 10 300 python3 "$R/tools/prof_points.py" 4000000 > "$O/points.txt" 2> "$O/points.err" || { echo "points failed"; exit 1; }
cd /tmp
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- \
    python3 "$R/bench.py" --lines 20000000 --steps 3 --warmup 2 --no-cpu-baseline > "$O/bench20m.json" 2> "$O/bench20m.err" || { echo "bench failed"; exit 1; }
echo done
