#!/bin/bash
# r02a: GPU parity tests (incl. full-size GOP replay parity), the default
# bench line (with the CPU baseline + bench parity) and the host CPU probe.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02a}
export TMPDIR=/tmp
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
(lscpu; echo; nproc; python3 -c 'import os; print("affinity", len(os.sched_getaffinity(0)))') > "$O/host.txt" 2>&1
bash "$R/tools/gpu_step.sh" \
  "600 $TAG/pytest_gpu.log python -u -m pytest $R/tests -x -v -m gpu --timeout 180 --timeout-method thread" \
  "400 $TAG/bench_2160p.log python $R/bench.py --config 2160p" \
  "300 $TAG/bench_1080p.log python $R/bench.py --config 1080p"
