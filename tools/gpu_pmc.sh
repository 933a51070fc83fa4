#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run each, <= 8 SQ counters) over a
# short bench run, under gpurun_out/<tag>/pmc<i>/.  Usage: gpu_pmc.sh <tag>
# <config>
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmc}
CFG=${2:-2160p}
export TMPDIR=/tmp
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
B="python3 $R/bench.py --config $CFG --no-cpu-baseline --steps 8 --warmup 2"
bash "$R/tools/gpu_step.sh" \
  "120 $TAG/pmc1.log cd /tmp && timeout -s KILL 110 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $O/pmc1 -o run -- $B" \
  "120 $TAG/pmc2.log cd /tmp && timeout -s KILL 110 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $O/pmc2 -o run -- $B"
