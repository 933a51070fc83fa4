#!/bin/bash
# deblocking: the plane kernel vs the oracle, then the replay with and without it.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-db}
export TMPDIR=/tmp
bash "$R/tools/gpu_step.sh" \
  "300 $TAG/pytest_deblock.log python -u -m pytest $R/tests/test_deblock.py -x -v -m gpu --timeout 120 --timeout-method thread" \
  "500 $TAG/pytest_replay.log python -u -m pytest $R/tests/test_replay.py -v -m gpu --timeout 280 --timeout-method thread"
