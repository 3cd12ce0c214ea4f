#!/bin/bash
# Device-table check on the GPU box: the -m gpu table tests, then a 20M-line
# config-2 bench with the delivery measurement (device table phases).
set -uo pipefail
TAG=${1:-r04_table}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -k "table or golden" -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 \
    || { echo "gpu tests failed"; tail -40 "$O/gpu_tests.log"; exit 1; }
tail -2 "$O/gpu_tests.log"
timeout -k 10 400 python3 bench.py --lines ${LINES:-20000000} --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err" \
    || { echo "bench failed"; tail -20 "$O/bench.err"; exit 1; }
python3 -c "
import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], d['kernel_ms'])
print({k: v for k, v in d.get('delivery', d).items() if k.startswith('table')})"
echo done
