#!/bin/bash
# quadrant half-res search + lookahead ME: replay parity (every schedule,
# full-size GOPs), the speed-10 and speed-6 bench lines, a kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-la}
export TMPDIR=/tmp
bash "$R/tools/gpu_step.sh" \
  "500 $TAG/pytest_replay.log python -u -m pytest $R/tests/test_replay.py -x -v -m gpu --timeout 280 --timeout-method thread" \
  "300 $TAG/bench_2160p.log python $R/bench.py --config 2160p" \
  "300 $TAG/bench_2160p10.log python $R/bench.py --config 2160p10" \
  "300 $TAG/trace.log rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run -- python3 $R/bench.py --config 2160p --no-cpu-baseline --steps 16"
