#!/bin/bash
# One GPU box call: parity tests, the default bench line (2160p), the 1080p
# line, a kernel-trace profile of the default bench, HBM-byte PMC passes
# (separate passes, as the MI355X guide prescribes: FETCH_SIZE and WRITE_SIZE
# do not fit one pass) and one SQ counter pass (VALU / LDS instruction counts).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
export TMPDIR=/tmp
P="$R/gpurun_out/prof_$TAG"
mkdir -p "$P"
B="python3 $R/bench.py --no-cpu-baseline --steps 16 --warmup 4"
bash "$R/tools/gpu_step.sh" \
  "300 prof_$TAG/pytest_gpu.log python -u -m pytest $R/tests -x -v -m gpu --timeout 120 --timeout-method thread" \
  "300 prof_$TAG/bench.log python $R/bench.py" \
  "300 prof_$TAG/bench_1080p.log python $R/bench.py --config 1080p" \
  "200 prof_$TAG/prof_trace.log cd /tmp && rocprofv3 --kernel-trace --stats -d $P/trace -o run -- $B" \
  "200 prof_$TAG/prof_fetch.log cd /tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o run -- $B" \
  "200 prof_$TAG/prof_write.log cd /tmp && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $P/write -o run -- $B" \
  "200 prof_$TAG/prof_sq.log cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $P/sq -o run -- $B"
