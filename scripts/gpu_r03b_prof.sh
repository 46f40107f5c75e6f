#!/bin/bash
# Round-3 profile refresh (GPU box) for the workloads whose kernels changed in
# the second half of round 3: powder medium/hard (two worlds per CU) and the
# GC/HGC samplers (full-wave chains).  Kernel traces + FETCH/WRITE PMC passes
# via scripts/gpu_prof.sh, plus each workload's plain bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for wl in ${WLS:-powder-medium powder-hard gcsample hgcsample}; do
  case $wl in
    gcsample) K=gc_sample_kernel; S=300 ;;
    hgcsample) K=hgc_sample_kernel; S=300 ;;
    powder) K=pw_step_kernel; S=600 ;;
    powder-medium|powder-hard) K=pwf_light_step_kernel+pwf_step_kernel; S=600 ;;
  esac
  timeout -k 10 300 python3 bench.py --workload $wl --no-cpu-baseline > gpurun_out/bench_$wl.log 2>&1 || exit 4
  grep '^{' gpurun_out/bench_$wl.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$wl', r['value'], r['roofline']['kernel_ms'], r['roofline']['frac'])"
  WL=$wl KERNEL=$K STEPS=$S bash scripts/gpu_prof.sh || exit 5
done
