#!/bin/bash
# CPU suite against the ASan + UBSan builds of the oracle (SURVEY 5 "race detection / sanitizers").
# Usage: scripts/oracle_sanitize.sh [pytest args]   (log: profiles/r04/oracle_sanitize.log)
set -euo pipefail
cd "$(dirname "$0")/.."
make -s -C oracle sanitize
export FUTBOL_ORACLE_SANITIZE=1
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)" \
    python -m pytest tests -m "not gpu" -q -p no:cacheprovider "$@"
