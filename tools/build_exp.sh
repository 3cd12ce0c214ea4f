#!/bin/bash
# Profiling-experiment builds: kernels.hip with -DLP_EXP=N linked into
# logparser_amd/_dbg/exp<N>.so (select with LOGPARSER_AMD_LIB=...).
set -euo pipefail
cd "$(dirname "$0")/../logparser_amd"
make -s all
for n in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DLP_EXP=$n -c csrc/kernels.hip -o _dbg/obj/kernels_exp$n.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o _dbg/exp$n.so _lib/obj/capi.o _lib/obj/plan.o _lib/obj/synth.o _dbg/obj/kernels_exp$n.o
done
