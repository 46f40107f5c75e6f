#!/bin/bash
# rocprofv3 evidence for one bench workload (run on the GPU box):
#   1. --kernel-trace --stats   (per-kernel durations)
#   2. --pmc FETCH_SIZE         (own pass: TCC slots cannot hold both)
#   3. --pmc WRITE_SIZE
# then (locally, after gpurun merged gpurun_out/) scripts/prof_summary.py -> profiles/<round>_<wl>_kernel_stats.csv and
# profiles/traffic.json.  Usage: WL=powder KERNEL=pw_step_kernel ROUND=r01 scripts/gpu_prof.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
WL=${WL:-pointmaze}
KERNEL=${KERNEL:-maze_step_kernel}
ROUND=${ROUND:-r01}
STEPS=${STEPS:-300}
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--workload $WL --steps $STEPS --warmup ${WARMUP:-100} --no-cpu-baseline --no-extras ${BENCH_ARGS:-}"
TAG=${TAG:-$WL}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
  python3 bench.py $ARGS > gpurun_out/prof_${TAG}.log 2>&1 || exit $?
[ "${PMC:-1}" = 1 ] || { tail -1 gpurun_out/prof_${TAG}.log; exit 0; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$TAG -o run --output-format csv -- \
  python3 bench.py $ARGS > gpurun_out/pmc_fetch_${TAG}.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$TAG -o run --output-format csv -- \
  python3 bench.py $ARGS > gpurun_out/pmc_write_${TAG}.log 2>&1 || exit $?
tail -1 gpurun_out/prof_${TAG}.log
# profiles/ is written back here (gpurun returns only gpurun_out/):
#   python3 scripts/prof_summary.py --round $ROUND --workload $WL --kernel $KERNEL
