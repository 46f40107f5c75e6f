#!/bin/bash
# Round 6: parity after the explicit-fma lean solve (layout independence at 8
# envs per wave) and the plan's device column tables, then an A/B of the lean
# stage against HEAD's, and the GC/HGC host cost.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests/test_locomaze_gpu.py tests/test_contact_pin_gpu.py tests/test_shard_boundary_gpu.py tests/test_shard_gpu.py tests/test_gc_gpu.py tests/test_hgc_gpu.py tests/test_periodic_gpu.py > gpurun_out/r06_pytest_d.log 2>&1
rc=$?; tail -5 gpurun_out/r06_pytest_d.log; [ $rc -eq 0 ] || exit 2
timeout -k 10 200 python scripts/probe_epw_diff.py 2>&1 | grep epw | tee gpurun_out/r06_epw_diff2.log || exit 3
timeout -k 10 200 python scripts/probe_gc_host.py > gpurun_out/r06_gc_host2.log 2>&1 || { tail -20 gpurun_out/r06_gc_host2.log; exit 5; }
tail -1 gpurun_out/r06_gc_host2.log
LIBS="ogbench_amd/libogbx.so _abx/libogbx_head.so" ROUNDS=3 bash scripts/gpu_maze_ab.sh || exit 4
