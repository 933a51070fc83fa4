#!/bin/bash
# A/B of an environment switch on the 2160p bench: tools/ab_env.sh TAG VAR=VALUE
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; SW=$2
mkdir -p $R/gpurun_out/$TAG
cd $R
for i in 1 2; do
timeout -k 10 120 python bench.py --no-cpu-baseline --steps 32 > gpurun_out/$TAG/a_$i.log 2>&1 || exit 1
env $SW timeout -k 10 120 python bench.py --no-cpu-baseline --steps 32 > gpurun_out/$TAG/b_$i.log 2>&1 || exit 1
done
