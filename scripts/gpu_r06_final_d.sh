#!/bin/bash
# Round 6 closing profiles after the late kernel changes (GPU box): kernel
# trace + FETCH_SIZE + WRITE_SIZE passes of the workloads whose kernels or
# launch sequence changed (pointmaze, antmaze, powder medium / hard), the
# pointmaze strong-scaling shares, the pointmaze issue counters.  Locally
# afterwards: scripts/prof_summary.py --round r06 per workload.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
WLS=${WLS:-"pointmaze antmaze powder-medium powder-hard"} DEFAULT_BENCH=0 ROUND=r06 bash scripts/gpu_round_prof.sh || exit $?
for N in 32768 16384 8192; do
  PMC=0 WL=pointmaze TAG=pointmaze-n$N STEPS=2000 BENCH_ARGS="--num-envs $N" bash scripts/gpu_prof.sh || exit $?
done
bash scripts/gpu_pmc_maze.sh || exit $?
