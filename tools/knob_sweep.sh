#!/bin/bash
# Parse-kernel tuning knobs (env, read by launch_parse) on the config-2 bench.
set -euo pipefail
LINES=${1:-20000000}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/knobs
mkdir -p "$O"
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python3 "$R/bench.py" --lines "$LINES" --steps 3 --warmup 1 --no-cpu-baseline > "$O/$tag.json" 2> "$O/$tag.err"; }
run default LP_X=0
run nomask LP_MASKS=0
run nomask_w100 LP_MASKS=0 LP_WIN_PCT=100
run pad2k LP_LDS_PAD=2048
echo done
