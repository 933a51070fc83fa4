#!/bin/bash
# The round-end checks: the whole -m gpu suite in one process, then smoke().
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-suite}
export TMPDIR=/tmp
bash "$R/tools/gpu_step.sh" \
  "900 $TAG/pytest_gpu.log python -u -m pytest $R/tests -x -q -m gpu --timeout 280 --timeout-method thread" \
  "300 $TAG/smoke.log python -c 'import __graft_entry__ as g; g.smoke()'"
