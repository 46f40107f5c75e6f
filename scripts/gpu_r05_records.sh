#!/bin/bash
# Round 5 bench records: one bench.py line per workload WITH its CPU baseline
# (the oracle port on this box's host, bounded sample), saved under
# gpurun_out/records/<wl>.json (copied to profiles/r05_<wl>_bench.json here).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/records
export TMPDIR=/tmp
for wl in ${WLS:-pointmaze powder powder-medium powder-hard gcsample hgcsample antmaze pointmaze-medium-n1}; do
  extra=""
  [ "$wl" = pointmaze-medium-n1 ] && extra="--steps 3000"
  timeout -k 10 400 python bench.py --workload $wl $extra > gpurun_out/records/$wl.log 2>&1 \
    || { tail -20 gpurun_out/records/$wl.log; exit 4; }
  grep '^{' gpurun_out/records/$wl.log | tail -1 > gpurun_out/records/$wl.json
  python -c "import json,sys; r=json.load(open(sys.argv[1])); print(sys.argv[2], r['value'], r['ms_per_step'], (r.get('cpu_baseline') or {}).get('value'))" gpurun_out/records/$wl.json $wl
done
