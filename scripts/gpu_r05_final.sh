#!/bin/bash
# Round-5 closing run (GPU box): the whole GPU suite, smoke, the default bench
# line, then the powder-medium / powder-hard profile sets (kernel trace +
# FETCH_SIZE + WRITE_SIZE passes) and their bench records with CPU baselines
# (scripts/gpu_r05_records.sh).  Locally afterwards: scripts/prof_summary.py
# per workload, then copy gpurun_out/records/<wl>.json to profiles/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_all.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 4; }
grep '^{' gpurun_out/bench_default.log | tail -1
WLS=${WLS:-"powder-medium powder-hard"}
WLS="$WLS" DEFAULT_BENCH=0 ROUND=r05 bash scripts/gpu_round_prof.sh || exit 5
WLS="$WLS" bash scripts/gpu_r05_records.sh || exit 6
