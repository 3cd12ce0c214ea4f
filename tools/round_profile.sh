#!/bin/bash
# End-of-milestone GPU run: profile (tools/gpu_profile.sh) + configs 3 / 4 bench lines.
set -euo pipefail
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash "$R/tools/gpu_profile.sh" "$TAG"
O=$R/gpurun_out/$TAG
for w in 3 4 5; do
  timeout -k 10 600 python3 "$R/bench.py" --workload $w > "$O/bench_config$w.json" 2> "$O/bench_config$w.err"
done
echo done
