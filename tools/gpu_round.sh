#!/bin/bash
# One GPU box call: parity tests, the default bench line, a kernel-trace
# profile of the same bench and HBM-byte PMC passes (separate passes, as the
# MI355X guide prescribes: FETCH_SIZE and WRITE_SIZE do not fit one pass).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
export TMPDIR=/tmp
P="$R/gpurun_out/prof_$TAG"
mkdir -p "$P"
bash "$R/tools/gpu_step.sh" \
  "420 pytest_gpu.log python -u -m pytest $R/tests -x -v -m gpu --timeout 120 --timeout-method thread" \
  "420 bench.log python $R/bench.py" \
  "300 prof_trace.log cd /tmp && rocprofv3 --kernel-trace --stats -d $P/trace -o run -- python3 $R/bench.py --no-cpu-baseline --steps 16 --warmup 4" \
  "300 prof_fetch.log cd /tmp && rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o run -- python3 $R/bench.py --no-cpu-baseline --steps 8 --warmup 2" \
  "300 prof_write.log cd /tmp && rocprofv3 --pmc WRITE_SIZE -d $P/write -o run -- python3 $R/bench.py --no-cpu-baseline --steps 8 --warmup 2"
