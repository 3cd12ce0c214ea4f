#!/bin/bash
# Round-end verification on one GPU box: GPU parity tests, smoke(), then the
# round profile (PMC passes, default bench with roofline.traffic, kernel trace)
set -uo pipefail
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { echo "tests failed"; tail -30 "$O/gpu_tests.log"; exit 1; }
tail -1 "$O/gpu_tests.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke failed"; tail "$O/smoke.log"; exit 1; }
cat "$O/smoke.log"
bash tools/gpu_profile.sh "$TAG" 100000000 || { echo "profile failed"; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('value',d['value'],d['kernel_ms'],d['roofline'])"
echo done
