#!/bin/bash
# Copy the judged summaries of a gpu_profile.sh run into profiles/<tag>/.
set -euo pipefail
TAG=${1:?tag}
S=gpurun_out/$TAG
D=profiles/$TAG
mkdir -p "$D"
cp "$S/bench.json" "$D/bench_default.json"
cp "$S/trace_bench.json" "$D/trace_bench.json"
cp "$S/trace/run_kernel_stats.csv" "$D/kernel_stats.csv"
cp "$S/trace/run_kernel_trace.csv" "$D/kernel_trace.csv"
cp "$S/pmc_fetch/run_counter_collection.csv" "$D/pmc_fetch_size.csv"
cp "$S/pmc_write/run_counter_collection.csv" "$D/pmc_write_size.csv"
cp "$S/pmc_traffic.json" "$D/pmc_traffic.json"
cp "$S/pmc_traffic.json" profiles/pmc_traffic_latest.json
ls -la "$D"
