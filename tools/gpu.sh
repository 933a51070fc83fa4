#!/bin/bash
# The one GPU-box driver (run it through gpurun from the repo root):
#
#   tools/gpu.sh suite TAG            -m gpu suite in one process, smoke(), default bench
#   tools/gpu.sh tests TAG 'EXPR'     pytest -m gpu -k EXPR
#   tools/gpu.sh testbench TAG 'EXPR' CFG...  those tests, then a bench line per config
#   tools/gpu.sh bench TAG CFG... [-- ARGS]   one bench line per config (ARGS to each)
#   tools/gpu.sh prof TAG CFG [ARGS]  kernel trace + FETCH / WRITE / SQ PMC passes of the
#                                     bench run of CFG (default steps; one rocprofv3 pass each, the
#                                     MI355X guide's rule: FETCH_SIZE and WRITE_SIZE do not
#                                     share a pass)
#   tools/gpu.sh trace TAG CFG [ARGS] the kernel trace pass alone
#   tools/gpu.sh tracesum TAG CFG [ARGS]  the kernel trace pass, summarised on the box
#   tools/gpu.sh envbench TAG CFG "ENV=.." ... [-- ARGS]  one bench line per environment (A/B)
#   tools/gpu.sh argbench TAG CFG "ARGS" ...  one bench line per argument set (A/B)
#   tools/gpu.sh ubench TAG           tools/ubench binaries (VALU issue rates, PMC calibration)
#
# Every step has its own time limit (tools/gpu_step.sh); a crash, abort or
# timeout stops the call.  Logs and profiles land in gpurun_out/TAG/.
R=${GRAFT_REPO_ROOT:-$(pwd)}
MODE=$1; TAG=${2:-dev}; shift 2
export TMPDIR=/tmp
P="$R/gpurun_out/$TAG"
mkdir -p "$P"
PYT="python -u -m pytest $R/tests -x -q -m gpu --timeout 280 --timeout-method thread"
case "$MODE" in
  suite)
    exec bash "$R/tools/gpu_step.sh" \
      "900 $TAG/pytest_gpu.log $PYT" \
      "300 $TAG/smoke.log python -c 'import __graft_entry__ as g; g.smoke()'" \
      "400 $TAG/bench_default.log python $R/bench.py" ;;
  tests)
    exec bash "$R/tools/gpu_step.sh" "900 $TAG/pytest_k.log $PYT -v -k '$1'" ;;
  testbench)
    # testbench TAG 'EXPR' CFG...: the selected tests, then one bench line per
    # config, in one step chain (a crash stops it; a test failure does not)
    expr=$1; shift
    steps=("900 $TAG/pytest_k.log $PYT -v -k '$expr'")
    for c in "$@"; do steps+=("400 $TAG/bench_$c.log python $R/bench.py --config $c"); done
    exec bash "$R/tools/gpu_step.sh" "${steps[@]}" ;;
  bench)
    cfgs=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do cfgs+=("$1"); shift; done
    [ "$1" = "--" ] && shift
    steps=()
    for c in "${cfgs[@]}"; do steps+=("400 $TAG/bench_$c.log python $R/bench.py --config $c $*"); done
    exec bash "$R/tools/gpu_step.sh" "${steps[@]}" ;;
  prof)
    CFG=${1:-2160p}; shift
    B="python3 $R/bench.py --config $CFG --no-cpu-baseline --emulate-ranks 0 $*"
    SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
    exec bash "$R/tools/gpu_step.sh" \
      "200 $TAG/trace.log cd /tmp && rocprofv3 --kernel-trace --stats -d $P/trace -o run -- $B" \
      "200 $TAG/fetch.log cd /tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o run -- $B" \
      "200 $TAG/write.log cd /tmp && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $P/write -o run -- $B" \
      "200 $TAG/sq.log cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $SQ -d $P/sq -o run -- $B" \
      "120 $TAG/summary.log python3 $R/tools/prof_json.py $P $P/prof_$CFG.json --frames ${FRAMES:-101} --bench $P/trace.log --md $P/prof_$CFG.md" \
      "60 $TAG/slim.log $R/tools/slim_prof.sh $P" ;;
  tracesum)
    # kernel trace + its summary on the box (occupancy, gaps; no PMC passes):
    # tracesum TAG CFG [ARGS]
    CFG=${1:-2160p}; shift
    B="python3 $R/bench.py --config $CFG --no-cpu-baseline --emulate-ranks 0 $*"
    exec bash "$R/tools/gpu_step.sh" \
      "200 $TAG/trace.log cd /tmp && rocprofv3 --kernel-trace --stats -d $P/trace -o run -- $B" \
      "120 $TAG/summary.log python3 $R/tools/prof_json.py $P $P/trace_$CFG.json --frames ${FRAMES:-101} --bench $P/trace.log --md $P/trace_$CFG.md" \
      "60 $TAG/slim.log $R/tools/slim_prof.sh $P" ;;
  trace)
    # kernel trace only: trace TAG CFG [ARGS]
    CFG=${1:-2160p}; shift
    B="python3 $R/bench.py --config $CFG --no-cpu-baseline --emulate-ranks 0 $*"
    exec bash "$R/tools/gpu_step.sh" \
      "200 $TAG/trace.log cd /tmp && rocprofv3 --kernel-trace --stats -d $P/trace -o run -- $B" \
      "120 $TAG/gzip.log find $P -type f -size +256k ! -name '*.gz' -exec gzip -9 {} +" ;;
  envbench)
    # one bench line per environment setting: envbench TAG CFG "A=1" "A=2 B=1" ... [-- ARGS]
    CFG=$1; shift
    envs=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
    [ "$1" = "--" ] && shift
    steps=(); i=0
    for e in "${envs[@]}"; do
      steps+=("400 $TAG/envbench_$i.log env $e python $R/bench.py --config $CFG --no-cpu-baseline --emulate-ranks 0 $*")
      i=$((i + 1))
    done
    exec bash "$R/tools/gpu_step.sh" "${steps[@]}" ;;
  argbench)
    # one bench line per argument set: argbench TAG CFG "ARGS1" "ARGS2" ...
    CFG=$1; shift
    steps=(); i=0
    for a in "$@"; do
      steps+=("400 $TAG/argbench_$i.log python $R/bench.py --config $CFG --no-cpu-baseline --emulate-ranks 0 $a")
      i=$((i + 1))
    done
    exec bash "$R/tools/gpu_step.sh" "${steps[@]}" ;;
  ubench)
    exec bash "$R/tools/gpu_step.sh" \
      "120 $TAG/valu_rates.txt $R/tools/ubench/valu_rates" ;;
  *)
    echo "usage: tools/gpu.sh suite|tests|bench|prof|ubench TAG ..." >&2; exit 2 ;;
esac
