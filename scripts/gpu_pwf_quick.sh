#!/bin/bash
# Powderworld medium/hard check (GPU box): full-rule parity tests, then the
# powder-medium and powder-hard bench (timed single steps only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_powder_full_gpu.py tests/test_powder_gpu.py -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/pwf_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/pwf_pytest.log; [ $rc -eq 0 ] || exit $rc
for wl in powder-medium powder-hard; do
  timeout -k 10 300 python bench.py --workload $wl --steps 600 --warmup 60 --no-extras --no-cpu-baseline \
    > gpurun_out/pwf_bench_$wl.log 2>&1 || { tail -20 gpurun_out/pwf_bench_$wl.log; exit 4; }
  tail -n 1 gpurun_out/pwf_bench_$wl.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl %.4g env-steps/s kern %.3f ms frac %.3f' % (d['value'], d['roofline']['kernel_ms'], d['roofline']['frac']))"
done
