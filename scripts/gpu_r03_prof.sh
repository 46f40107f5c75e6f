#!/bin/bash
# Round-3 profile set (GPU box): pointmaze kernel traces at the single-GPU
# shares of the 1/2/4/8-GPU strong-scaling job (N = 65,536 / 32,768 / 16,384 /
# 8,192) with the bench line of each, PMC traffic at N = 65,536, the issue
# counters, then the other workloads' traces ($WLS).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for N in 65536 32768 16384 8192; do
  TAG=pointmaze-n$N
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python3 bench.py --workload pointmaze --num-envs $N --steps 2000 --warmup 100 --no-cpu-baseline --no-extras \
    > gpurun_out/prof_$TAG.log 2>&1 || { tail -5 gpurun_out/prof_$TAG.log; exit 3; }
  timeout -k 10 200 python3 bench.py --workload pointmaze --num-envs $N --steps 2000 --warmup 100 --no-cpu-baseline \
    --no-extras > gpurun_out/bench_$TAG.log 2>&1 || exit 4
  grep '^{' gpurun_out/bench_$TAG.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$TAG', r['value'], r['roofline']['kernel_ms'])"
done
WL=pointmaze KERNEL=maze_step_kernel STEPS=2000 bash scripts/gpu_prof.sh || exit 5
bash scripts/gpu_pmc_maze.sh || exit 6
for wl in ${WLS:-antmaze hgcsample}; do
  case $wl in
    antmaze) K=ant_step_kernel; S=2000 ;;
    gcsample) K=gc_sample_kernel; S=300 ;;
    hgcsample) K=hgc_sample_kernel; S=300 ;;
    powder) K=pw_step_kernel; S=600 ;;
    powder-medium|powder-hard) K=pwf_light_step_kernel+pwf_step_kernel; S=600 ;;
  esac
  WL=$wl KERNEL=$K STEPS=$S bash scripts/gpu_prof.sh || exit 7
done
