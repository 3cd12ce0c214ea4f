#!/bin/bash
# One GPU call: every -m gpu test, smoke(), the default bench line (config 2,
# 100 M lines), then configs 3, 4 and 5 (bench lines only).  Each step under its
# own time limit; stops at the first failure.
#   tools/round_check.sh TAG [skip-tests]
set -uo pipefail
TAG=${1:-check}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 \
    || { echo "tests failed"; grep -a "internal check" -A3 "$O/gpu_tests.log" | head -8; tail -30 "$O/gpu_tests.log"; exit 1; }
  tail -1 "$O/gpu_tests.log"
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke failed"; tail "$O/smoke.log"; exit 1; }
  cat "$O/smoke.log"
fi
timeout -k 10 600 python3 bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo "bench failed"; tail "$O/bench.err"; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print('value',d['value'],d['kernel_ms'],d['roofline']['frac'],d.get('delivery',{}).get('table_chars_roofline_frac'))"
for w in 3 4 5; do
  timeout -k 10 500 python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-delivery \
      > "$O/bench_config$w.json" 2> "$O/bench_config$w.err" || { echo "config $w failed"; tail "$O/bench_config$w.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench_config$w.json').read().strip().splitlines()[-1]);print($w, d['value'], d['kernel_ms'], d['roofline']['frac'])"
done
echo done
