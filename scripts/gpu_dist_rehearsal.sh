#!/bin/bash
# Rehearse bench.py's multi-rank path on a one-GPU box: 2 ranks share cuda:0
# over gloo (the driver's 8-GPU run uses RCCL; this checks the code path).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for wl in pointmaze powder gcsample; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 120 --warmup 10 --dist-backend gloo --workload $wl \
    --num-envs 16384 > gpurun_out/dist_$wl.log 2>&1 || { tail -30 gpurun_out/dist_$wl.log; exit 1; }
  grep '^{' gpurun_out/dist_$wl.log | cut -c1-400
done
