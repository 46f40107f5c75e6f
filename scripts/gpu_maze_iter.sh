#!/bin/bash
# Pointmaze kernel iteration (GPU box): the locomaze parity tests on the
# in-tree build, then the A/B bench of $LIBS (scripts/gpu_maze_ab.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_locomaze_gpu.py tests/test_contact_pin_gpu.py ${EXTRA_TESTS:-} -m gpu -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/maze_iter_tests.log 2>&1
rc=$?
tail -3 gpurun_out/maze_iter_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/maze_iter_tests.log | head -20; exit $rc; }
bash scripts/gpu_maze_ab.sh
