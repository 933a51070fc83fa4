#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/ab
cd $R
for i in 1 2; do
timeout -k 10 120 python bench.py --no-cpu-baseline --steps 32 > gpurun_out/ab/quad_$i.log 2>&1 || exit 1
RAV1E_HIP_RDO_SINGLE=1 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 32 > gpurun_out/ab/single_$i.log 2>&1 || exit 1
done
