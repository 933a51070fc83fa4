#!/bin/bash
# Development call: GPU parity tests, then bench lines without the CPU
# baseline (extra bench.py flags from $BENCH_ARGS), all under
# gpurun_out/<tag>/.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-dev}
export TMPDIR=/tmp
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
bash "$R/tools/gpu_step.sh" \
  "300 $TAG/pytest_gpu.log python -u -m pytest $R/tests -x -v -m gpu --timeout 120 --timeout-method thread" \
  "200 $TAG/bench_2160p.log python $R/bench.py --config 2160p --steps 32 --no-cpu-baseline $BENCH_ARGS" \
  "200 $TAG/bench_1080p.log python $R/bench.py --config 1080p --steps 32 --no-cpu-baseline $BENCH_ARGS" \
  "200 $TAG/bench_2160p10.log python $R/bench.py --config 2160p10 --steps 16 --no-cpu-baseline $BENCH_ARGS"
