#!/bin/bash
# Runs the default bench workload once per _variants/libogbx_*.so (GPU box).
# WL / STEPS select the workload; prints one summary line per variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
WL=${WL:-pointmaze}
for f in _variants/libogbx_*.so; do
  name=$(basename $f .so)
  OGBX_LIB=$f timeout -k 10 180 python bench.py --workload $WL --steps ${STEPS:-2000} --warmup 100 \
    --no-cpu-baseline --no-extras > gpurun_out/ab_${WL}_$name.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab_${WL}_$name.log; exit $rc; fi
  python - "$name" gpurun_out/ab_${WL}_$name.log <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith('{')][-1]
d = json.loads(line)
print(f"{sys.argv[1]:32s} value {d['value']/1e6:10.2f} M/s  kernel {d['roofline']['kernel_ms']*1e3:8.2f} us", flush=True)
PY
done
