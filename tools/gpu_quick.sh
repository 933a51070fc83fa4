#!/bin/bash
# Iteration call: GPU parity tests, the bench line, a kernel-trace profile.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-dev}
export TMPDIR=/tmp
P="$R/gpurun_out/prof_$TAG"
mkdir -p "$P"
bash "$R/tools/gpu_step.sh" \
  "420 pytest_gpu.log python -m pytest $R/tests -x -q -m gpu" \
  "420 bench.log python $R/bench.py" \
  "300 prof_trace.log cd /tmp && rocprofv3 --kernel-trace --stats -d $P/trace -o run -- python3 $R/bench.py --no-cpu-baseline --steps 16 --warmup 4"
