#!/bin/bash
# Round-4 profile set, other workloads (GPU box): kernel trace + FETCH_SIZE +
# WRITE_SIZE passes for each workload in $WLS, then the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for wl in ${WLS:-gcsample hgcsample antmaze powder powder-medium powder-hard}; do
  case $wl in
    antmaze) K=ant_step_kernel; S=2000 ;;
    gcsample) K=gc_sample_kernel; S=300 ;;
    hgcsample) K=hgc_ahead_kernel; S=300 ;;
    powder) K=pw_step_kernel; S=600 ;;
    powder-medium|powder-hard) K=pwf_light_step_kernel+pwf_step_kernel; S=600 ;;
  esac
  WL=$wl KERNEL=$K STEPS=$S bash scripts/gpu_prof.sh || exit 7
  timeout -k 10 300 python3 bench.py --workload $wl --no-cpu-baseline > gpurun_out/bench_$wl.log 2>&1 || exit 8
  grep '^{' gpurun_out/bench_$wl.log | cut -c1-200
done
[ "${1:-}" = --no-default ] && exit 0
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 9; }
grep '^{' gpurun_out/bench_default.log
