#!/bin/bash
# Parse-kernel time vs requested field subsets (profiling experiment).
set -euo pipefail
LINES=${1:-20000000}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sweep
mkdir -p "$O"
i=0
for f in all \
         "IP:connection.client.host" \
         "TIME.EPOCH:request.receive.time.epoch" \
         "HTTP.URI:request.firstline.uri" \
         "HTTP.PATH:request.firstline.uri.path" \
         "STRING:request.firstline.uri.query.*" \
         "HTTP.PATH:request.referer.path" \
         "STRING:request.referer.query.*"; do
  i=$((i+1))
  timeout -k 10 300 python3 "$R/bench.py" --lines "$LINES" --steps 3 --warmup 1 --no-cpu-baseline --fields "$f" \
      > "$O/f$i.json" 2> "$O/f$i.err"
  echo "$f" > "$O/f$i.name"
done
echo done
