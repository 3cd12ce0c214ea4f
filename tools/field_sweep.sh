#!/bin/bash
# Parse-kernel time vs cumulative requested field subsets (profiling experiment):
# which stages the config-2 kernel time goes to.
set -uo pipefail
LINES=${1:-20000000}
TAG=${2:-sweep}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
T="IP:connection.client.host,STRING:connection.client.user,STRING:request.status.last,BYTES:response.body.bytes,HTTP.USERAGENT:request.user-agent,HTTP.URI:request.referer,HTTP.FIRSTLINE:request.firstline"
TM="$T,TIME.EPOCH:request.receive.time.epoch"
FL="$TM,HTTP.METHOD:request.firstline.method,HTTP.URI:request.firstline.uri"
P0="$FL,HTTP.PATH:request.firstline.uri.path,HTTP.QUERYSTRING:request.firstline.uri.query"
Q0="$P0,STRING:request.firstline.uri.query.*"
P1="$Q0,HTTP.PATH:request.referer.path,HTTP.HOST:request.referer.host"
Q1="$P1,STRING:request.referer.query.*"
i=0
for f in "$T" "$TM" "$FL" "$P0" "$Q0" "$P1" "$Q1" all; do
  i=$((i+1))
  timeout -k 10 300 python3 "$R/bench.py" --lines "$LINES" --steps 3 --warmup 1 --no-cpu-baseline --no-delivery --fields "$f" \
      > "$O/f$i.json" 2> "$O/f$i.err" || { echo "f$i failed"; tail -5 "$O/f$i.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/f$i.json'));print('f$i', d['kernel_ms'], d['status_counts'])"
done
echo done
