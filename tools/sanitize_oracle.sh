#!/bin/bash
# The CPU test suite (-m "not gpu") against the oracle built with
# AddressSanitizer + UndefinedBehaviorSanitizer (oracle/Makefile `sanitize`,
# -fno-sanitize-recover: any report aborts the run).  In this container
# (no GPU); the log goes to profiles/<tag>_oracle_sanitize.log.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-r03}
make -s -C "$R/oracle" sanitize || exit 1
LOG="$R/profiles/${TAG}_oracle_sanitize.log"
{
  echo "# oracle/build/librav1e_oracle_san.so: gcc $(gcc -dumpversion) -fsanitize=address,undefined -fno-sanitize-recover=all"
  echo "# git $(git -C "$R" rev-parse --short HEAD)$(git -C "$R" diff --quiet || echo +dirty), $(date -u +%FT%TZ)"
  LD_PRELOAD="$(gcc -print-file-name=libasan.so)${LD_PRELOAD:+:$LD_PRELOAD}" \
  ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 \
  UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  RAV1E_ORACLE_LIB="$R/oracle/build/librav1e_oracle_san.so" \
    python -m pytest "$R/tests" -q -m "not gpu" -p no:cacheprovider 2>&1
  echo "# exit status $?"
} | tee "$LOG"
