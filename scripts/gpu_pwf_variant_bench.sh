#!/bin/bash
# bench.py powder-medium under each _ab/libogbx_pwf_*.so (tuning only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for f in _ab/libogbx_pwf_*.so; do
  echo "== $f"
  OGBX_LIB=$f timeout -k 10 200 python bench.py --workload powder-medium --steps 600 --warmup 60 --no-extras --no-cpu-baseline > gpurun_out/vb.log 2>&1 || exit $?
  tail -n 1 gpurun_out/vb.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4g env-steps/s kern %.3f ms' % (d['value'], d['roofline']['kernel_ms']))"
done
