#!/bin/bash
# one optimisation iteration on a GPU box: GPU parity tests, then a 20M-line
# config-2 bench under a rocprofv3 kernel trace
set -uo pipefail
TAG=${1:-r02_iter}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
if [ "${SKIP_TESTS:-0}" = "0" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -30 "$O/gpu_tests.log"; exit 1; }
  tail -1 "$O/gpu_tests.log"
fi
cd /tmp
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- \
    python3 "$R/bench.py" --lines 20000000 --steps 3 --warmup 2 --no-cpu-baseline > "$O/bench20m.json" 2> "$O/bench20m.err" || { echo "bench failed"; tail "$O/bench20m.err"; exit 1; }
python3 -c "import json,sys;d=json.load(open('$O/bench20m.json'));print('value',d['value'],d['kernel_ms'],d['status_counts'])"
grep -h k_parse_lines "$O"/trace/*kernel_stats.csv | cut -d, -f1-4
