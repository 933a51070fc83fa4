#!/bin/bash
# r02b: the stream replay on the GPU -- replay parity first, then the rest
# of the GPU suite, then the default bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02b}
export TMPDIR=/tmp
bash "$R/tools/gpu_step.sh" \
  "500 $TAG/pytest_replay.log python -u -m pytest $R/tests/test_replay.py -x -v -m gpu --timeout 240 --timeout-method thread" \
  "400 $TAG/pytest_gpu.log python -u -m pytest $R/tests -x -q -m gpu --timeout 180 --timeout-method thread --deselect tests/test_replay.py" \
  "300 $TAG/bench_2160p.log python $R/bench.py --config 2160p"
