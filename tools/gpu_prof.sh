#!/bin/bash
# One GPU box call: the default bench line, the other configs' lines, a
# kernel-trace profile of the default bench, HBM-byte PMC passes (separate
# passes: FETCH_SIZE and WRITE_SIZE do not fit one pass) and one SQ pass.
# Usage: gpu_prof.sh <tag> [config]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-prof}
CFG=${2:-2160p}
export TMPDIR=/tmp
P="$R/gpurun_out/prof_$TAG"
mkdir -p "$P"
B="python3 $R/bench.py --config $CFG --no-cpu-baseline --steps 16 --warmup 5"
bash "$R/tools/gpu_step.sh" \
  "200 prof_$TAG/prof_trace.log cd /tmp && rocprofv3 --kernel-trace --stats -d $P/trace -o run -- $B" \
  "200 prof_$TAG/prof_fetch.log cd /tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o run -- $B" \
  "200 prof_$TAG/prof_write.log cd /tmp && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $P/write -o run -- $B" \
  "200 prof_$TAG/prof_sq.log cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $P/sq -o run -- $B" \
  "300 prof_$TAG/bench_1080p.log python $R/bench.py --config 1080p" \
  "300 prof_$TAG/bench_2160p444.log python $R/bench.py --config 2160p444" \
  "300 prof_$TAG/bench_2160p10.log python $R/bench.py --config 2160p10" \
  "300 prof_$TAG/bench_2160p.log python $R/bench.py --config 2160p" \
  "200 prof_$TAG/bench_360p.log python $R/bench.py --config 360p" \
  "400 prof_$TAG/pytest_replay.log python -u -m pytest $R/tests/test_replay.py -x -q -m gpu --timeout 240 --timeout-method thread"
