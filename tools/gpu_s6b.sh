#!/bin/bash
# speed 6 at full size: the config-D GOP parity test, then the config-D bench
# line (speed 6) and a kernel trace of it.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-s6b}
export TMPDIR=/tmp
bash "$R/tools/gpu_step.sh" \
  "300 $TAG/pytest_full.log python -u -m pytest $R/tests/test_replay.py -v -m gpu --timeout 280 --timeout-method thread -k full_size_gop --durations=0" \
  "400 $TAG/bench_2160p10.log python $R/bench.py --config 2160p10" \
  "300 $TAG/trace.log rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run -- python3 $R/bench.py --config 2160p10 --no-cpu-baseline --steps 16"
