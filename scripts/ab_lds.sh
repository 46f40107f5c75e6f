#!/bin/bash
# Placement A/B: dynamic LDS padding per maze step workgroup (OGBX_MAZE_LDS).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for pad in 0 40000 70000 100000; do
  OGBX_MAZE_LDS=$pad timeout -k 10 180 python bench.py --steps 2000 --warmup 100 --no-cpu-baseline --no-extras > gpurun_out/ab_lds_$pad.log 2>&1 || { tail -5 gpurun_out/ab_lds_$pad.log; exit 1; }
  python -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/ab_lds_$pad.log') if l.startswith('{')][-1])
print('lds $pad', round(d['value']/1e6,1), 'M/s kernel', round(d['roofline']['kernel_ms']*1e3,2), 'us')"
  OGBX_MAZE_LDS=$pad timeout -k 10 120 python3 scripts/probe_locomaze_compact.py 2>&1 | grep physics
done
