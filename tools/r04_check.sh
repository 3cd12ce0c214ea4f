#!/bin/bash
# Round-4 check on the GPU box: the -m gpu parity tests, then a 20M-line
# config-2 bench with a kernel trace (per-kernel times).  Every GPU step has
# its own time limit; the first failure ends the script.
set -uo pipefail
TAG=${1:-r04_check}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 \
    || { echo "gpu tests failed"; tail -40 "$O/gpu_tests.log"; exit 1; }
tail -3 "$O/gpu_tests.log"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- \
    python3 "$R/bench.py" --lines 20000000 --steps 3 --warmup 2 --no-cpu-baseline --no-delivery > "$O/bench20m.json" 2> "$O/bench20m.err" \
    || { echo "bench failed"; tail -20 "$O/bench20m.err"; exit 1; }
python3 - "$O/trace/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print("%-60s %8d calls %10.3f ms avg" % (r["Name"][:60], int(r["Calls"]), float(r["AverageNs"]) / 1e6))
PY
tail -c 600 "$O/bench20m.json"
echo done
