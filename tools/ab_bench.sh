#!/bin/bash
# usage: tools/ab_bench.sh TAG build1 build2 ...  (builds: logparser_amd/_exp/<name>, make exp)
# A/B of experiment builds: 20M-line config-2 bench each, twice, interleaved
set -uo pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for r in 1 2; do
for n in "$@"; do
  LOGPARSER_AMD_LIB=$PWD/logparser_amd/_exp/$n/liblogparser_amd.so timeout -k 10 240 python3 bench.py --lines ${LINES:-20000000} \
      --steps 5 --warmup 2 --no-cpu-baseline --no-delivery ${BENCH_ARGS:-} > $O/$n.$r.json 2> $O/$n.$r.err || { echo "$n failed"; tail -5 $O/$n.$r.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/$n.$r.json').read().strip().splitlines()[-1]);print('%-10s value %8.1f parse %7.3f pk %7.3f uk %7.3f ok %d' % ('$n', d['value'], d['kernel_ms']['parse_avg'], d['kernel_ms']['parse_kernels_avg'], d['kernel_ms']['uri_kernels_avg'], d['status_counts']['ok']))"
done; done
