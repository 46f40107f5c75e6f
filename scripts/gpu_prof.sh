#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run (no PMC counters here).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$OLDPWD}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- \
  python3 bench.py --steps ${STEPS:-300} --warmup 20 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof_bench.log 2>&1
rc=$?
tail -2 gpurun_out/prof_bench.log
find gpurun_out/prof -name "*stats*" | head
exit $rc
