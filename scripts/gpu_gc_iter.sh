#!/bin/bash
# GC/HGC iteration (GPU box): the sampler tests, then the gcsample / hgcsample
# bench lines and their rocprof traces + PMC traffic (scripts/gpu_prof.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gc_gpu.py tests/test_hgc_gpu.py tests/test_loader_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/pytest_gc.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gc.log; [ $rc -eq 0 ] || exit $rc
for wl in ${WLS:-gcsample hgcsample}; do
  timeout -k 10 200 python3 bench.py --workload $wl --no-cpu-baseline > gpurun_out/bench_$wl.log 2>&1 || exit 4
  grep '^{' gpurun_out/bench_$wl.log | python3 -c "import json,sys; r=json.loads(sys.stdin.read()); print('$wl', r['value'], r['roofline']['kernel_ms'], r['extra'])"
  [ "${PROF:-1}" = 1 ] || continue
  case $wl in gcsample) K=gc_sample_kernel ;; hgcsample) K=hgc_sample_kernel ;; esac
  WL=$wl KERNEL=$K STEPS=300 bash scripts/gpu_prof.sh || exit 5
done
