#!/bin/bash
# GPU parity tests on the box, one pytest process per step, each step under
# its own time limit; stops at the first failing step.
#   tools/gpu_tests.sh TAG [pytest -k expression]
set -uo pipefail
TAG=${1:-tests}
K=${2:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
if [ -n "$K" ]; then
  timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v -s -k "$K" --timeout 300 --timeout-method thread > "$O/gpu_tests_k.log" 2>&1
  rc=$?; tail -5 "$O/gpu_tests_k.log"; grep -a "internal check" "$O/gpu_tests_k.log" | head -5
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; tail -3 "$O/gpu_tests.log"; grep -a "internal check" "$O/gpu_tests.log" | head -5
exit $rc
