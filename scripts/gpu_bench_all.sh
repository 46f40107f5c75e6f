#!/bin/bash
# One full bench line (extras + cpu_baseline) per workload -> gpurun_out/bench_<wl>.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for wl in ${WLS:-powder powder-medium powder-hard gcsample hgcsample}; do
  timeout -k 10 400 python bench.py --workload $wl > gpurun_out/bench_$wl.log 2>&1 || { tail -20 gpurun_out/bench_$wl.log; exit 1; }
  grep '^{' gpurun_out/bench_$wl.log | tail -n 1 > gpurun_out/bench_$wl.json
  cut -c1-200 gpurun_out/bench_$wl.json
done
