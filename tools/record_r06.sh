#!/bin/bash
# Round-6 record of the built library on one GPU box: smoke(), the round
# profile (PMC passes, default bench with roofline.traffic, kernel trace +
# stats), configs 3-5 bench lines, then the config-5 chunk-lines sweep.
#   tools/record_r06.sh TAG
set -uo pipefail
TAG=${1:-r06y}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke failed"; tail "$O/smoke.log"; exit 1; }
cat "$O/smoke.log"
bash tools/gpu_profile.sh "$TAG" 100000000 || { echo "profile failed"; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print('value',d['value'],d['kernel_ms'],d['roofline']['frac'],d['roofline']['traffic'],d.get('delivery',{}).get('table_chars_roofline_frac'))"
for w in 3 4 5; do
  timeout -k 10 500 python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-delivery \
      > "$O/bench_config$w.json" 2> "$O/bench_config$w.err" || { echo "config $w failed"; tail "$O/bench_config$w.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench_config$w.json').read().strip().splitlines()[-1]);print($w, d['value'], d['kernel_ms'], d['roofline']['frac'])"
done
LP_WORKLOAD=5 timeout -k 10 300 python3 tools/chunk_sweep.py 20000000 0,34,40,46,52,58 > "$O/sweep_c5.txt" 2>&1 && cat "$O/sweep_c5.txt"
echo done
