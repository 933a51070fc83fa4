#!/bin/bash
# Run GPU steps in order on the gpurun box; each step has its own time
# limit.  A step that fails normally (exit 1: a test failure) lets the next
# step run; a crash, abort, timeout or kill (any other non-zero status)
# stops the script there.  Usage: gpu_step.sh "<secs> <log> <cmd...>" ...
mkdir -p gpurun_out
for step in "$@"; do
  secs=${step%% *}; rest=${step#* }; log=${rest%% *}; cmd=${rest#* }
  echo "== [$secs s] $cmd" | tee -a gpurun_out/steps.log
  mkdir -p "$(dirname "gpurun_out/$log")"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$log" 2>&1
  rc=$?
  echo "   rc=$rc" | tee -a gpurun_out/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after rc=$rc" | tee -a gpurun_out/steps.log
    exit $rc
  fi
done
exit 0
