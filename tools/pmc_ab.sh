#!/bin/bash
# PMC traffic (separate FETCH_SIZE / WRITE_SIZE passes) of experiment builds, 20M config-2 lines
set -uo pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd /tmp; export TMPDIR=/tmp
for n in "$@"; do
  for c in FETCH_SIZE WRITE_SIZE; do
    LOGPARSER_AMD_LIB=$R/logparser_amd/_exp/$n/liblogparser_amd.so timeout -s KILL 200 rocprofv3 --pmc $c --kernel-trace --output-format csv \
      -d $O/$n.$c -o run -- python3 $R/bench.py --lines ${LINES:-20000000} --steps 1 --warmup 0 --no-cpu-baseline --no-delivery \
      > $O/$n.$c.log 2>&1 || { echo "$n $c failed"; tail -5 $O/$n.$c.log; exit 1; }
  done
  python3 $R/tools/pmc_traffic.py $O/$n.FETCH_SIZE/run_counter_collection.csv $O/$n.WRITE_SIZE/run_counter_collection.csv \
      --lines ${LINES:-20000000} --out $O/$n.pmc.json > /dev/null
  python3 -c "
import json;d=json.load(open('$O/$n.pmc.json'))['kernels']
print('$n', ' '.join('%s f%.2f w%.2f' % (k, v['fetch_bytes']/1e9, v['write_bytes']/1e9) for k, v in d.items() if k in ('k_parse_chunks','k_uri_lines')))"
done
