#!/bin/bash
# r02i: intra prediction parity, the VALU issue-rate microbenchmark, and
# the GPU suite.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02i}
export TMPDIR=/tmp
bash "$R/tools/gpu_step.sh" \
  "300 $TAG/pytest_intra.log python -u -m pytest $R/tests/test_hip_parity.py -x -v -m gpu -k intra --timeout 120 --timeout-method thread" \
  "120 $TAG/valu_rates.log $R/tools/ubench/valu_rates" \
  "600 $TAG/pytest_gpu.log python -u -m pytest $R/tests -x -q -m gpu --timeout 240 --timeout-method thread"
