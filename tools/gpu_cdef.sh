#!/bin/bash
# CDEF: the frame filter vs the oracle, the replay with CDEF vs the CPU
# replay, bench lines with --cdef (and the default for comparison), and a
# kernel trace of the --cdef bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-cdef}
export TMPDIR=/tmp
P="$R/gpurun_out/$TAG"
mkdir -p "$P"
bash "$R/tools/gpu_step.sh" \
  "300 $TAG/pytest_cdef.log python -u -m pytest $R/tests/test_cdef.py $R/tests/test_replay.py -x -v -m gpu --timeout 280 --timeout-method thread" \
  "300 $TAG/bench_2160p_cdef.log python $R/bench.py --config 2160p --cdef" \
  "300 $TAG/bench_1080p_cdef.log python $R/bench.py --config 1080p --cdef" \
  "200 $TAG/prof_trace.log cd /tmp && rocprofv3 --kernel-trace --stats -d $P/trace -o run -- python3 $R/bench.py --config 2160p --cdef --no-cpu-baseline --steps 16 --warmup 5"
