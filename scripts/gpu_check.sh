#!/bin/bash
# Round GPU check: gpu tests, smoke, default bench, pointmaze-medium N=1 bench,
# 2-rank gloo rehearsal of the strong-scaling pointmaze bench.  Every GPU step
# has its own time limit; the script stops at the first crash / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${PYTEST_ARGS:-} \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
echo "== bench"
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 4; }
grep '^{' gpurun_out/bench.log
timeout -k 10 200 python bench.py --workload pointmaze-medium-n1 --steps 3000 > gpurun_out/bench_n1.log 2>&1 || { tail -20 gpurun_out/bench_n1.log; exit 5; }
grep '^{' gpurun_out/bench_n1.log
if [ "${DIST:-1}" = 1 ]; then
  echo "== 2-rank gloo rehearsal"
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 500 --warmup 20 --dist-backend gloo --workload pointmaze \
    --no-cpu-baseline > gpurun_out/dist_pointmaze.log 2>&1 || { tail -30 gpurun_out/dist_pointmaze.log; exit 6; }
  grep '^{' gpurun_out/dist_pointmaze.log
fi
exit $rc
