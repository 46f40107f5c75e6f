#!/bin/bash
# Issue-side counters of maze_step_kernel in the bench setting (GPU box):
# VALU/SALU instructions per wave, wave cycles, busy/wait cycles.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--workload pointmaze --steps 200 --warmup 100 --no-cpu-baseline --no-extras"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES \
  -d gpurun_out/pmc_maze_sq -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_maze_sq.log 2>&1 || exit $?
timeout -k 10 120 python3 scripts/probe_locomaze_compact.py > gpurun_out/maze_compact.log 2>&1; cat gpurun_out/maze_compact.log | grep -v amdgpu.ids
