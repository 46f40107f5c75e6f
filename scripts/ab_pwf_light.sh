#!/bin/bash
# A/B of the render-only split for powderworld medium/hard (OGBX_PWF_LIGHT).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for wl in powder-medium powder-hard; do
for L in 0 1; do
  OGBX_PWF_LIGHT=$L timeout -k 10 300 python bench.py --workload $wl --steps 900 --warmup 60 --no-cpu-baseline --no-extras > gpurun_out/ab_pwf_${wl}_$L.log 2>&1 || { tail -5 gpurun_out/ab_pwf_${wl}_$L.log; exit 1; }
  python -c "
import json
d=json.loads([l for l in open('gpurun_out/ab_pwf_${wl}_$L.log') if l.startswith('{')][-1])
print('$wl light=$L', round(d['value']/1e6,3), 'M/s  ms/step', round(d['ms_per_step'],4))"
done
done
