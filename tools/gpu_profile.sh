#!/bin/bash
# Round profile on a GPU box (run through gpurun from the repo root):
#   separate PMC passes for FETCH_SIZE and WRITE_SIZE (never combined with
#   runtime/sys traces) -> per-launch HBM bytes -> default bench run (reads
#   that summary for roofline.traffic) -> rocprofv3 kernel trace + stats.
#   Everything lands under gpurun_out/<tag>/.
set -euo pipefail
TAG=${1:-r01}
LINES=${2:-100000000}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$O/pmc_fetch" -o run -- \
    python3 "$R/bench.py" --lines "$LINES" --steps 1 --warmup 0 --no-cpu-baseline --no-delivery > "$O/pmc_fetch_bench.json" 2> "$O/pmc_fetch.err"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$O/pmc_write" -o run -- \
    python3 "$R/bench.py" --lines "$LINES" --steps 1 --warmup 0 --no-cpu-baseline --no-delivery > "$O/pmc_write_bench.json" 2> "$O/pmc_write.err"
python3 "$R/tools/pmc_traffic.py" "$O/pmc_fetch/run_counter_collection.csv" "$O/pmc_write/run_counter_collection.csv" \
    --lines "$LINES" --lib "$R/logparser_amd/_lib/liblogparser_amd.so" --out "$O/pmc_traffic.json" > /dev/null
timeout -k 10 600 python3 "$R/bench.py" --lines "$LINES" --pmc-json "$O/pmc_traffic.json" > "$O/bench.json" 2> "$O/bench.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- \
    python3 "$R/bench.py" --lines "$LINES" --steps 3 --warmup 1 --no-cpu-baseline --pmc-json "$O/pmc_traffic.json" \
    > "$O/trace_bench.json" 2> "$O/trace.err"
echo done
