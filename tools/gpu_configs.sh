#!/bin/bash
# Bench every BASELINE config shape on one GPU (1 tile per GPU), each with
# its CPU baseline, under gpurun_out/<tag>/.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-cfg}
export TMPDIR=/tmp
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
bash "$R/tools/gpu_step.sh" \
  "300 $TAG/pytest_gpu.log python -u -m pytest $R/tests -x -v -m gpu --timeout 120 --timeout-method thread" \
  "300 $TAG/bench_2160p.log python $R/bench.py --config 2160p --cpu-seconds 15" \
  "300 $TAG/bench_1080p.log python $R/bench.py --config 1080p" \
  "300 $TAG/bench_2160p10.log python $R/bench.py --config 2160p10 --steps 16 --cpu-seconds 15" \
  "300 $TAG/bench_2160p444.log python $R/bench.py --config 2160p444 --steps 16 --cpu-seconds 15" \
  "300 $TAG/bench_360p.log python $R/bench.py --config 360p --steps 64"
