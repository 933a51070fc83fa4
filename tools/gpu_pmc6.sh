#!/bin/bash
# SQ counters of the config-D (speed 6) frame's kernels: issue, waiting, LDS.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmc6}
P=$R/gpurun_out/$TAG
B="python3 $R/bench.py --config 2160p10 --no-cpu-baseline --steps 8 --warmup 3"
export TMPDIR=/tmp
bash "$R/tools/gpu_step.sh" \
  "200 $TAG/prof_sq.log cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $P/sq -o run -- $B" \
  "200 $TAG/prof_sq2.log cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d $P/sq2 -o run -- $B"
