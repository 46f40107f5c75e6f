#!/bin/bash
# Round 6 closing profiles (GPU box): kernel trace + FETCH_SIZE + WRITE_SIZE
# passes of every bench workload, kernel traces of the pointmaze strong-scaling
# shares, the pointmaze issue counters.  Locally afterwards:
# scripts/prof_summary.py --round r06 per workload.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
WLS=${WLS:-"pointmaze powder powder-medium powder-hard gcsample hgcsample antmaze"} DEFAULT_BENCH=0 ROUND=r06 bash scripts/gpu_round_prof.sh || exit $?
for N in 32768 16384 8192; do
  PMC=0 WL=pointmaze TAG=pointmaze-n$N STEPS=2000 BENCH_ARGS="--num-envs $N" bash scripts/gpu_prof.sh || exit $?
done
bash scripts/gpu_pmc_maze.sh || exit $?
LIBS="ogbench_amd/libogbx.so _abx/libogbx_head.so" ROUNDS=3 bash scripts/gpu_maze_ab.sh > gpurun_out/r06_final_maze_ab.txt 2>&1 || exit 5
cat gpurun_out/r06_final_maze_ab.txt
