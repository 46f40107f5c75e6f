#!/bin/bash
# Round profile set: kernel trace + FETCH_SIZE + WRITE_SIZE passes for each
# bench workload in $WLS (default: all), then the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
WLS=${WLS:-"pointmaze powder powder-medium powder-hard gcsample hgcsample antmaze"}
for wl in $WLS; do
  case $wl in
    pointmaze) K=maze_step_kernel; S=2000 ;;
    powder) K=pw_step_kernel; S=600 ;;
    powder-medium|powder-hard) K=pwf_light_step_kernel+pwf_step_kernel; S=600 ;;
    gcsample) K="gc_ahead_kernel<true>"; S=300 ;;
    hgcsample) K="hgc_ahead_kernel<true>"; S=300 ;;
    antmaze) K=ant_step_kernel; S=2000 ;;
    *) echo "unknown workload $wl"; exit 2 ;;
  esac
  WL=$wl KERNEL=$K STEPS=$S bash scripts/gpu_prof.sh || exit $?
done
if [ "${DEFAULT_BENCH:-1}" = 1 ]; then
  timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
  grep '^{' gpurun_out/bench_default.log
fi
