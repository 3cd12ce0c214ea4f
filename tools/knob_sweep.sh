#!/bin/bash
set -euo pipefail
LINES=${1:-20000000}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/knobs
mkdir -p "$O"
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python3 "$R/bench.py" --lines "$LINES" --steps 3 --warmup 1 --no-cpu-baseline > "$O/$tag.json" 2> "$O/$tag.err"; }
run win100 LP_WIN_PCT=100
run win105 LP_WIN_PCT=105
run win110 LP_WIN_PCT=110
echo done
