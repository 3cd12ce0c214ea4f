#!/bin/bash
# CPU parity tests with the oracle (oracle/) and the test-only emulation of the
# device code (tests/emu: lp_device.h + plan.cpp) built with AddressSanitizer
# and UndefinedBehaviorSanitizer.  Python itself is not instrumented, so the
# ASan runtime is preloaded; leak checking is off (the interpreter's own
# allocations would be reported).  Host code only: GPU sanitizers are not
# available on this pool.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
make -s -C "$R/oracle" asan
SEL=${1:-"golden or synthetic_config2 or mutated or nginx_config4 or utf8 or upstream or strftime or authority or ip_token or setup or oracle_vs or resilient or cookies"}
export LD_PRELOAD=$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1${ASAN_LOG:+:log_path=$ASAN_LOG}
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1${ASAN_LOG:+:log_path=$ASAN_LOG}
export LP_ORACLE_LIB="$R/oracle/_build/liboracle_asan.so" LP_EMU_ASAN=1
cd "$R"
python3 -m pytest tests/test_emu_parity.py tests/test_oracle.py -x -q -p no:cacheprovider -k "$SEL" ${PYTEST_ARGS:-}
