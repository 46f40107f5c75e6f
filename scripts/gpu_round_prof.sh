#!/bin/bash
# Round profile set: kernel trace + FETCH_SIZE + WRITE_SIZE passes for every
# bench workload (scripts/gpu_prof.sh), then the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
WL=pointmaze KERNEL=maze_step_kernel STEPS=2000 bash scripts/gpu_prof.sh || exit $?
WL=powder KERNEL=pw_step_kernel STEPS=600 bash scripts/gpu_prof.sh || exit $?
WL=powder-medium KERNEL=pwf_step_kernel STEPS=600 bash scripts/gpu_prof.sh || exit $?
WL=powder-hard KERNEL=pwf_step_kernel STEPS=600 bash scripts/gpu_prof.sh || exit $?
WL=gcsample KERNEL=gc_sample_kernel STEPS=300 bash scripts/gpu_prof.sh || exit $?
WL=hgcsample KERNEL=hgc_sample_kernel STEPS=300 bash scripts/gpu_prof.sh || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
grep '^{' gpurun_out/bench_default.log
