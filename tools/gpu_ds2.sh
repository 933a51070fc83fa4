#!/bin/bash
# lane-group diamond with vector loads: diamond parity, replay parity, the
# two benches.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-ds2}
export TMPDIR=/tmp
bash "$R/tools/gpu_step.sh" \
  "300 $TAG/pytest_ds.log python -u -m pytest $R/tests/test_hip_parity.py -x -v -m gpu --timeout 120 --timeout-method thread -k diamond" \
  "500 $TAG/pytest_replay.log python -u -m pytest $R/tests/test_replay.py -x -v -m gpu --timeout 280 --timeout-method thread" \
  "300 $TAG/bench_2160p.log python $R/bench.py --config 2160p" \
  "300 $TAG/bench_2160p10.log python $R/bench.py --config 2160p10"
