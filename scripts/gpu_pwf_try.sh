#!/bin/bash
# Powder medium/hard A/B (GPU box): parity tests + bench for the in-tree build,
# then for each _abx/libogbx_pwf_*.so variant (parity + bench).  Tuning only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
one() {  # $1 = tag, OGBX_LIB from the env
  timeout -k 10 300 python -u -m pytest tests/test_powder_full_gpu.py -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/pwf_try_$1.log 2>&1
  rc=$?; echo "$1 tests: $(tail -1 gpurun_out/pwf_try_$1.log)"; [ $rc -eq 0 ] || return $rc
  for wl in ${WLS:-powder-medium}; do
    timeout -k 10 200 python bench.py --workload $wl --steps 600 --warmup 60 --no-extras --no-cpu-baseline \
      > gpurun_out/pwf_try_b_$1.log 2>&1 || return 4
    tail -n 1 gpurun_out/pwf_try_b_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 $wl %.4g env-steps/s kern %.3f ms frac %.3f' % (d['value'], d['roofline']['kernel_ms'], d['roofline']['frac']))"
  done
}
one intree || exit $?
for f in _abx/libogbx_pwf_*.so; do
  [ -f "$f" ] || continue
  t=$(basename $f .so); OGBX_LIB=$f one ${t#libogbx_pwf_} || exit $?
done
