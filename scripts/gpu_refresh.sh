#!/bin/bash
# Refresh: pointmaze profile set + default bench, full bench lines of the
# other workloads listed in $BENCH_WLS, issue counters of maze_step_kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
WLS=${WLS:-pointmaze} bash scripts/gpu_round_prof.sh || exit $?
for wl in ${BENCH_WLS:-powder-medium powder-hard}; do
  timeout -k 10 400 python bench.py --workload $wl > gpurun_out/bench_$wl.log 2>&1 || { tail -20 gpurun_out/bench_$wl.log; exit 1; }
  grep '^{' gpurun_out/bench_$wl.log | cut -c1-200
done
bash scripts/gpu_pmc_maze.sh
