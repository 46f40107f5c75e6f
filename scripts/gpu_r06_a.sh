#!/bin/bash
# Round 6, first GPU call: the driver's command (x2), the window probe under a
# kernel trace, the GC host probe, the replicated-lane layouts, and the tests
# the round's changes touch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_r06_window.sh || exit $?
timeout -k 10 200 python scripts/probe_gc_host.py > gpurun_out/r06_gc_host.log 2>&1 || { tail -20 gpurun_out/r06_gc_host.log; exit 5; }
tail -1 gpurun_out/r06_gc_host.log
timeout -k 10 400 python scripts/probe_epw_rep.py > gpurun_out/r06_epw_rep.log 2>&1 || { tail -20 gpurun_out/r06_epw_rep.log; exit 6; }
tail -1 gpurun_out/r06_epw_rep.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_locomaze_gpu.py tests/test_hgc_gpu.py tests/test_bench_gpu.py > gpurun_out/r06_pytest_a.log 2>&1
rc=$?; tail -5 gpurun_out/r06_pytest_a.log; exit $rc
