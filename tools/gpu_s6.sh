#!/bin/bash
# speed 6 (config D): replay parity of every schedule incl. the partition-RDO
# one (the RDO kernels were generalised under the speed-10 cases).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-s6}
export TMPDIR=/tmp
bash "$R/tools/gpu_step.sh" \
  "600 $TAG/pytest_replay.log python -u -m pytest $R/tests/test_replay.py -v -m gpu --timeout 300 --timeout-method thread"
