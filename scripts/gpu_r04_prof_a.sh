#!/bin/bash
# Round-4 check + pointmaze profile set (GPU box): the whole GPU suite and
# smoke, pointmaze kernel traces at the single-GPU shares of the strong-scaling
# job with their bench lines, PMC traffic and issue counters at N = 65,536.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_all.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
for N in 65536 32768 16384 8192; do
  TAG=pointmaze-n$N
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python3 bench.py --workload pointmaze --num-envs $N --steps 2000 --warmup 100 --no-cpu-baseline --no-extras \
    > gpurun_out/prof_$TAG.log 2>&1 || { tail -5 gpurun_out/prof_$TAG.log; exit 4; }
  timeout -k 10 200 python3 bench.py --workload pointmaze --num-envs $N --steps 2000 --warmup 100 --no-cpu-baseline \
    --no-extras > gpurun_out/bench_$TAG.log 2>&1 || exit 5
  grep '^{' gpurun_out/bench_$TAG.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$TAG', r['value'], r['roofline']['kernel_ms'])"
done
WL=pointmaze KERNEL=maze_step_kernel STEPS=2000 bash scripts/gpu_prof.sh || exit 6
bash scripts/gpu_pmc_maze.sh || exit 7
