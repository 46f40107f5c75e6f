#!/bin/bash
# A/B of the pointmaze step kernel: locomaze GPU parity tests on the in-tree
# build, then the default bench once per _variants/libogbx_*.so, then the
# path counters of the _diag/libogbx_stats.so build (if present).  Every GPU
# step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_locomaze_gpu.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/ab_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/ab_pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_run.sh || exit $?
if [ -f _diag/libogbx_stats.so ]; then
  OGBX_LIB=_diag/libogbx_stats.so timeout -k 10 120 python scripts/probe_stats.py > gpurun_out/ab_stats.log 2>&1 || exit $?
  grep step gpurun_out/ab_stats.log
fi
if [ -n "${PROBE_LIB:-}" ]; then
  OGBX_LIB=$PROBE_LIB timeout -k 10 240 python scripts/probe_maze_launch.py > gpurun_out/ab_launch.log 2>&1 || exit $?
  grep N= gpurun_out/ab_launch.log
fi
