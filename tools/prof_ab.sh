#!/bin/bash
# stage points (LP_PROFILE builds under logparser_amd/_exp/prof_<name>) of config 2, 4M lines
set -uo pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for n in "$@"; do
  LP_PROF_LIB=$PWD/logparser_amd/_exp/prof_$n/liblogparser_amd.so LP_WORKLOAD=${WL:-2} timeout -k 10 300 python3 tools/prof_points.py 4000000 > $O/points_$n.txt 2>&1 || { echo "$n failed"; tail $O/points_$n.txt; exit 1; }
  grep -E "guard |first-leaf|kernel total|staged   " $O/points_$n.txt | head -6
done
