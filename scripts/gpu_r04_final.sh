#!/bin/bash
# Round-4 closing run (GPU box), part $PART:
#   a: the whole GPU suite, smoke, then the powder-medium / powder-hard
#      profile sets (kernel trace + FETCH_SIZE + WRITE_SIZE passes, bench line);
#   b: antmaze / gcsample / hgcsample profile sets and the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${PART:-a}" = a ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu_all.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit 2
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 3; }
  tail -1 gpurun_out/smoke.log
  WLS="powder-medium powder-hard" bash scripts/gpu_r04_prof_b.sh --no-default || exit 4
else
  for wl in powder-medium powder-hard; do  # bench lines priced with part a's traffic.json
    timeout -k 10 300 python3 bench.py --workload $wl --no-cpu-baseline > gpurun_out/bench_$wl.log 2>&1 || exit 6
  done
  WLS="antmaze gcsample hgcsample" bash scripts/gpu_r04_prof_b.sh || exit 5
fi
