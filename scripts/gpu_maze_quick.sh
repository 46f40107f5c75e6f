#!/bin/bash
# Quick pointmaze check (GPU box): locomaze + shard GPU parity tests, the bench
# at N = 65,536 and N = 8,192 (timed step only), the per-N launch probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_locomaze_gpu.py tests/test_contact_pin_gpu.py tests/test_shard_gpu.py -m gpu -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/quick_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/quick_pytest.log; [ $rc -eq 0 ] || exit $rc
for N in 65536 8192; do
  timeout -k 10 200 python bench.py --num-envs $N --no-extras --no-cpu-baseline > gpurun_out/quick_bench_$N.log 2>&1 \
    || { tail -20 gpurun_out/quick_bench_$N.log; exit 4; }
  python - gpurun_out/quick_bench_$N.log <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(f"N={r['config']['total_envs']}: {r['value']/1e9:.3f} G env-steps/s, {r['ms_per_step']*1e3:.2f} us/step, "
      f"kernel {r['roofline']['kernel_ms']*1e3:.2f} us (pair median {r['roofline']['kernel_ms_event_pair_median']*1e3:.2f})")
PY
done
if [ "${PROBE:-1}" = 1 ]; then
  timeout -k 10 240 python3 scripts/probe_maze_launch.py > gpurun_out/probe_launch.log 2>&1 || exit $?
  grep N= gpurun_out/probe_launch.log
fi
