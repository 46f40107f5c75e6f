#!/bin/bash
# GPU-box check: gpu tests, smoke, short bench.  Stops at the first crash/timeout
# (exit codes other than 0 = pass and 1 = pytest test failures).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-1000}
echo "== pytest -m gpu"
timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc2=$?
tail -3 gpurun_out/smoke.log
if [ $rc2 -ne 0 ] && [ $rc2 -ne 1 ]; then exit $rc2; fi
echo "== bench"
timeout -k 10 400 python bench.py --steps $STEPS --warmup 100 > gpurun_out/bench.log 2>&1
rc3=$?
tail -3 gpurun_out/bench.log
exit $(( rc | rc2 | rc3 ))
