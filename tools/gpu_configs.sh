#!/bin/bash
# Bench every BASELINE config shape on one GPU (1 tile per GPU), a kernel
# trace of the default bench and PMC HBM-byte passes (separate passes, as the
# MI355X guide prescribes), all under gpurun_out/<tag>/.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-cfg}
export TMPDIR=/tmp
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R/gpurun_out" && ln -sfn "$TAG" last && cd "$R"
bash "$R/tools/gpu_step.sh" \
  "420 $TAG/pytest_gpu.log python -u -m pytest $R/tests -x -v -m gpu --timeout 120 --timeout-method thread" \
  "300 $TAG/bench_1080p.log python $R/bench.py" \
  "300 $TAG/bench_2160p.log python $R/bench.py --config 2160p --steps 16 --cpu-seconds 15" \
  "300 $TAG/bench_2160p10.log python $R/bench.py --config 2160p10 --steps 16 --cpu-seconds 15" \
  "300 $TAG/bench_2160p444.log python $R/bench.py --config 2160p444 --steps 16 --cpu-seconds 15" \
  "300 $TAG/bench_360p.log python $R/bench.py --config 360p --steps 64" \
  "300 $TAG/prof_trace.log cd /tmp && rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 $R/bench.py --no-cpu-baseline --steps 16 --warmup 4" \
  "300 $TAG/prof_fetch.log cd /tmp && rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run -- python3 $R/bench.py --no-cpu-baseline --steps 8 --warmup 2" \
  "300 $TAG/prof_write.log cd /tmp && rocprofv3 --pmc WRITE_SIZE -d $O/write -o run -- python3 $R/bench.py --no-cpu-baseline --steps 8 --warmup 2"
