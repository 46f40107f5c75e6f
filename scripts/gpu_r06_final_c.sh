#!/bin/bash
# Round 6 closing records after the late kernel changes (GPU box): the GPU
# suite and smoke, one bench line per workload with its CPU baseline
# (gpurun_out/records/<wl>.json), the driver's command three times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/records
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r06_pytest_final.log 2>&1
rc=$?; tail -2 gpurun_out/r06_pytest_final.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1 || { tail -20 gpurun_out/r06_smoke.log; exit 3; }
tail -1 gpurun_out/r06_smoke.log
bash scripts/gpu_r05_records.sh || exit 4
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/records/driver_cmd_$r.log 2>&1 || { tail -20 gpurun_out/records/driver_cmd_$r.log; exit 5; }
  grep '^{' gpurun_out/records/driver_cmd_$r.log | tail -1 > gpurun_out/records/driver_cmd_$r.json
done
