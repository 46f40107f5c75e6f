#!/bin/bash
# Round 6: powder prepared resets (parity + per-step A/B of OGBX_PWF_PREP_OPS),
# the lean stage A/B (fusion-matched explicit fma vs HEAD), and the GC/HGC
# device column tables vs by-value (dfc9b96).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -q -x --timeout 300 --timeout-method thread tests/test_powder_full_gpu.py tests/test_powder_gpu.py tests/test_gc_gpu.py tests/test_hgc_gpu.py > gpurun_out/r06_pytest_e.log 2>&1
rc=$?; tail -5 gpurun_out/r06_pytest_e.log; [ $rc -eq 0 ] || exit 2
for ops in 0 2 1 4; do
  OGBX_PWF_PREP_OPS=$ops timeout -k 10 300 python bench.py --workload powder-medium --no-cpu-baseline > gpurun_out/r06_pwm_ops$ops.log 2>&1 || { tail -20 gpurun_out/r06_pwm_ops$ops.log; exit 3; }
  grep '^{' gpurun_out/r06_pwm_ops$ops.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); x=d['extra']; print('prep_ops $ops', 'ms/step', round(d['ms_per_step'],4), 'steady', round(x.get('steady_state_ms_per_step',0),4), 'sync_reset', round(x.get('sync_reset_step_ms',0),3))"
done
LIBS="ogbench_amd/libogbx.so _abx/libogbx_head.so" ROUNDS=3 bash scripts/gpu_maze_ab.sh || exit 4
LIBS="ogbench_amd/libogbx.so _abx/libogbx_gcbyval.so" ROUNDS=3 WLS="gcsample hgcsample" bash scripts/gpu_lib_ab.sh || exit 5
