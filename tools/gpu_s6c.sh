#!/bin/bash
# the lane-group diamond kernel: diamond parity, the replay (speed 6 and 10),
# then the config-D bench line and its kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-s6c}
export TMPDIR=/tmp
bash "$R/tools/gpu_step.sh" \
  "300 $TAG/pytest_ds.log python -u -m pytest $R/tests/test_hip_parity.py -x -v -m gpu --timeout 120 --timeout-method thread -k diamond" \
  "500 $TAG/pytest_replay.log python -u -m pytest $R/tests/test_replay.py -x -v -m gpu --timeout 280 --timeout-method thread" \
  "400 $TAG/bench_2160p10.log python $R/bench.py --config 2160p10" \
  "300 $TAG/trace.log rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run -- python3 $R/bench.py --config 2160p10 --no-cpu-baseline --steps 16"
