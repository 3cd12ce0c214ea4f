#!/bin/bash
# Kernel trace (rocprofv3 --kernel-trace --stats) of the 20M-line config-2
# bench for each experiment build: per-kernel average durations.
#   tools/exp_trace.sh TAG name1 name2 ...
set -uo pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
for n in "$@"; do
  LOGPARSER_AMD_LIB=$R/logparser_amd/_exp/$n/liblogparser_amd.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      --output-format csv -d "$O/$n" -o run -- python3 "$R/bench.py" --lines ${LINES:-20000000} --steps 3 --warmup 1 \
      --no-cpu-baseline --no-delivery > "$O/$n.json" 2> "$O/$n.err" || { echo "$n failed"; exit 1; }
  python3 - "$O/$n/run_kernel_stats.csv" "$n" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[2], " ".join("%s=%.3f" % (r["Name"].replace("lp::(anonymous namespace)::", "").replace("void ", "")[:16], float(r["AverageNs"]) / 1e6)
                            for r in rows if "lp::" in r["Name"]))
PY
done
