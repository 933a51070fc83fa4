#!/bin/bash
# Bench every BASELINE config shape on one GPU (1 tile per GPU), plus PMC
# HBM-byte passes of the default bench for the profile summary.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-cfg}
export TMPDIR=/tmp
P="$R/gpurun_out/prof_$TAG"
mkdir -p "$P"
bash "$R/tools/gpu_step.sh" \
  "300 bench_1080p.log python $R/bench.py" \
  "300 bench_2160p.log python $R/bench.py --config 2160p --steps 16 --cpu-seconds 15" \
  "300 bench_2160p10.log python $R/bench.py --config 2160p10 --steps 16 --cpu-seconds 15" \
  "300 bench_2160p444.log python $R/bench.py --config 2160p444 --steps 16 --cpu-seconds 15" \
  "300 bench_360p.log python $R/bench.py --config 360p --steps 64" \
  "300 prof_trace.log cd /tmp && rocprofv3 --kernel-trace --stats -d $P/trace -o run -- python3 $R/bench.py --no-cpu-baseline --steps 16 --warmup 4" \
  "300 prof_fetch.log cd /tmp && rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o run -- python3 $R/bench.py --no-cpu-baseline --steps 8 --warmup 2" \
  "300 prof_write.log cd /tmp && rocprofv3 --pmc WRITE_SIZE -d $P/write -o run -- python3 $R/bench.py --no-cpu-baseline --steps 8 --warmup 2"
