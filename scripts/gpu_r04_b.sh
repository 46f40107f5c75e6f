#!/bin/bash
# Round 4: maze parity tests on the in-tree library, then the maze A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_locomaze_gpu.py tests/test_contact_pin_gpu.py tests/test_shard_boundary_gpu.py tests/test_shard_gpu.py tests/test_stream_pin_gpu.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_maze.log 2>&1
rc=$?; grep -E "FAILED|passed|failed" gpurun_out/pytest_maze.log | tail -8; echo pytest rc=$rc
[ $rc -le 1 ] || exit $rc
LIBS=${LIBS:-"ogbench_amd/libogbx.so _abx/libogbx_v1.so _abx/libogbx_salu.so"} ROUNDS=${ROUNDS:-2} bash scripts/gpu_maze_ab.sh
[ -f _abx/libogbx_stats.so ] && OGBX_LIB=$PWD/_abx/libogbx_stats.so timeout -k 10 200 python scripts/probe_bail.py 2>&1 | grep -v amdgpu.ids
