#!/bin/bash
# Round-end rehearsal: the -m gpu suite in one process, smoke(), then the
# default bench line (what the driver runs with no flags).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-final}
export TMPDIR=/tmp
bash "$R/tools/gpu_step.sh" \
  "900 $TAG/pytest_gpu.log python -u -m pytest $R/tests -x -q -m gpu --timeout 280 --timeout-method thread" \
  "300 $TAG/smoke.log python -c 'import __graft_entry__ as g; g.smoke()'" \
  "400 $TAG/bench_default.log python $R/bench.py"
