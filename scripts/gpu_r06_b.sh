#!/bin/bash
# Round 6: host launch-cost micro, which envs differ across env layouts, the
# driver's command with the bound-step host path, and the locomaze tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out _mb
export TMPDIR=/tmp
hipcc -O3 --offload-arch=gfx950 scripts/micro/launch_host.hip -o _mb/launch_host 2> /dev/null || exit 2
timeout -k 10 60 ./_mb/launch_host | tee gpurun_out/r06_launch_host.txt || exit 3
timeout -k 10 200 python scripts/probe_epw_diff.py 2>&1 | tee gpurun_out/r06_epw_diff.log || exit 4
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_driver_cmd_b$r.log 2>&1 || { tail -20 gpurun_out/r06_driver_cmd_b$r.log; exit 5; }
  grep '^{' gpurun_out/r06_driver_cmd_b$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('value', d['value'], 'ms', d['ms_per_step'], 'timed', r['kernel_ms_timed_region'], 'b2b', r['kernel_ms_back_to_back'], 'host', d['extra']['host_us_per_step'])"
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_locomaze_gpu.py tests/test_c_host_gpu.py tests/test_shard_boundary_gpu.py > gpurun_out/r06_pytest_b.log 2>&1
rc=$?; tail -5 gpurun_out/r06_pytest_b.log; exit $rc
