#!/bin/bash
# Round 6, verdict r05 item 3: the driver's own command, then the window probe
# under a kernel trace (device start/end of every launch beside the host stamps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_driver_cmd_$r.log 2>&1 || { tail -20 gpurun_out/r06_driver_cmd_$r.log; exit 2; }
  grep '^{' gpurun_out/r06_driver_cmd_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value', d['value'], 'ms', d['ms_per_step'], 'timed', r['kernel_ms_timed_region'], 'b2b', r['kernel_ms_back_to_back'], 'host', d['extra']['host_us_per_step'])"
done
rm -rf gpurun_out/r06_win
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06_win -o win -- \
  python scripts/probe_window.py --out gpurun_out/r06_window_host.json > gpurun_out/r06_window.log 2>&1 || { tail -20 gpurun_out/r06_window.log; exit 3; }
tail -2 gpurun_out/r06_window.log
