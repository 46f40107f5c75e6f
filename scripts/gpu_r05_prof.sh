#!/bin/bash
# Round 5 profiles: kernel trace + FETCH_SIZE + WRITE_SIZE passes of the
# pointmaze, GC, HGC and antmaze benches; kernel traces of the pointmaze
# strong-scaling shares; the pointmaze issue counters.  Summaries are made
# here afterwards (scripts/prof_summary.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
WLS=${WLS:-"pointmaze gcsample hgcsample antmaze"} DEFAULT_BENCH=0 bash scripts/gpu_round_prof.sh || exit $?
for N in 32768 16384 8192; do
  PMC=0 WL=pointmaze TAG=pointmaze-n$N STEPS=2000 BENCH_ARGS="--num-envs $N" bash scripts/gpu_prof.sh || exit $?
done
if [ "${ISSUE:-1}" = 1 ]; then bash scripts/gpu_pmc_maze.sh || exit $?; fi
