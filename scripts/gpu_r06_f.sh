#!/bin/bash
# Round 6: the whole GPU suite, the lean-stage A/B (keep-settled selects vs
# HEAD's stage), powder prepared resets per-step A/B (fork before the light
# step), and the GC/HGC host cost with by-value column tables.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_pytest_f.log 2>&1
rc=$?; tail -5 gpurun_out/r06_pytest_f.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 200 python scripts/probe_epw_diff.py 2>&1 | grep epw | tee gpurun_out/r06_epw_diff3.log || exit 3
LIBS="ogbench_amd/libogbx.so _abx/libogbx_head.so" ROUNDS=3 bash scripts/gpu_maze_ab.sh || exit 4
for ops in 0 8 4; do
  OGBX_PWF_PREP_OPS=$ops timeout -k 10 300 python bench.py --workload powder-medium --no-cpu-baseline > gpurun_out/r06_pwm2_ops$ops.log 2>&1 || { tail -20 gpurun_out/r06_pwm2_ops$ops.log; exit 5; }
  grep '^{' gpurun_out/r06_pwm2_ops$ops.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); x=d['extra']; print('prep_ops $ops', 'ms/step', round(d['ms_per_step'],4), 'steady', round(x.get('steady_state_ms_per_step',0),4), 'sync_reset', round(x.get('sync_reset_step_ms',0),3))"
done
timeout -k 10 200 python scripts/probe_gc_host.py > gpurun_out/r06_gc_host3.log 2>&1 || { tail -20 gpurun_out/r06_gc_host3.log; exit 6; }
tail -1 gpurun_out/r06_gc_host3.log
