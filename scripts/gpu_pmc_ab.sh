#!/bin/bash
# Issue-side PMC passes of maze_step_kernel for each library in $LIBS (GPU box),
# bench setting (N = 65,536, 200 steps).  Pass 1: wave/issue counters; pass 2:
# instruction-cache counters.  Summaries: scripts/pmc_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmcab
export TMPDIR=/tmp
ARGS="--workload pointmaze --steps 200 --warmup 100 --no-cpu-baseline --no-extras ${BENCH_ARGS:-}"
if [ "${LIST:-0}" = 1 ]; then timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmcab/counters.txt 2>&1; fi
P1="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY"
P2=${P2:-"SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_CYCLES"}
for lib in $LIBS; do
  tag=$(basename $lib .so)
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    KT=""; [ $i = 2 ] && KT="--kernel-trace"
    OGBX_LIB=$PWD/$lib timeout -s KILL 90 rocprofv3 $KT --pmc $P -d gpurun_out/pmcab/${tag}_p$i -o run --output-format csv \
      -- python3 bench.py $ARGS > gpurun_out/pmcab/${tag}_p$i.log 2>&1 || { echo "pmc $tag p$i failed rc=$?"; tail -5 gpurun_out/pmcab/${tag}_p$i.log; }
  done
done
python3 scripts/pmc_summary.py gpurun_out/pmcab maze_step_kernel
