#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python scripts/probe_window_host.py > gpurun_out/r06_window_host2.log 2>&1 || { tail -20 gpurun_out/r06_window_host2.log; exit 2; }
tail -1 gpurun_out/r06_window_host2.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06_drv_h$r.log 2>&1 || exit 3
  grep '^{' gpurun_out/r06_drv_h$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value', d['value'], 'ms', d['ms_per_step'], 'timed', r['kernel_ms_timed_region'], 'b2b', r['kernel_ms_back_to_back'], 'host', d['extra']['host_us_per_step'])"
done
