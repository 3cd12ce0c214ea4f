#!/bin/bash
# Round-3 record: GPU tests, smoke, PMC passes + default bench + kernel
# trace (tools/final_check.sh), then the bench lines of configs 3, 4, 5.
set -uo pipefail
TAG=${1:-r03_final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
cd "$R"
bash tools/final_check.sh "$TAG" || exit 1
for w in 3 4 5; do
  timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline > "$O/bench_config$w.json" 2> "$O/bench_config$w.err" || { echo "config $w failed"; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench_config$w.json').read().strip().splitlines()[-1]);print('config $w', d['value'], d['kernel_ms'], d['roofline']['frac'], d['status_counts'])"
done
echo all done
