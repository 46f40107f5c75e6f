#!/bin/bash
# Round-2 pointmaze profile set (GPU box): kernel trace + FETCH_SIZE + WRITE_SIZE
# passes of the default workload (N = 65,536) and of the 8-GPU strong share
# (N = 8,192), the issue counters, the per-N launch probe and the default bench.
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ROUND=${ROUND:-r02} WL=pointmaze KERNEL=maze_step_kernel STEPS=2000 bash scripts/gpu_prof.sh || exit $?
for N in ${EXTRA_N:-8192}; do
  ARGS="--workload pointmaze --num-envs $N --steps 2000 --warmup 100 --no-cpu-baseline --no-extras"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pointmaze_n$N -o run --output-format csv -- \
    python3 bench.py $ARGS > gpurun_out/prof_pointmaze_n$N.log 2>&1 || exit $?
  grep '^{' gpurun_out/prof_pointmaze_n$N.log
done
bash scripts/gpu_pmc_maze.sh || exit $?
timeout -k 10 240 python3 scripts/probe_maze_launch.py > gpurun_out/probe_launch.log 2>&1 || exit $?
grep N= gpurun_out/probe_launch.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
grep '^{' gpurun_out/bench_default.log
