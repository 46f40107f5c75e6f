#!/bin/bash
# A/B of sampler builds (GPU box): GC/HGC parity tests on the in-tree build,
# then the gcsample / hgcsample bench (timed B = 1024 call only) under each
# library in $LIBS, alternating, $ROUNDS rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gc_gpu.py tests/test_hgc_gpu.py -m gpu -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/gc_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/gc_pytest.log; [ $rc -eq 0 ] || exit $rc
LIBS=${LIBS:-"ogbench_amd/libogbx.so $(ls _abx/libogbx_*.so 2>/dev/null | tr '\n' ' ')"}
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in $LIBS; do
    for wl in gcsample hgcsample; do
      OGBX_LIB=$PWD/$lib timeout -k 10 120 python bench.py --workload $wl --no-extras --no-cpu-baseline \
        > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 4; }
      python - gpurun_out/ab.log "$lib" "$wl" <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
rf = r['roofline']
print(f"{sys.argv[2]:34s} {sys.argv[3]:9s}: {r['value']/1e6:.1f} M samples/s, {r['ms_per_step']*1e3:.2f} us/call, "
      f"kernel {rf['kernel_ms']*1e3:.2f} us (b2b {rf.get('kernel_ms_back_to_back', 0)*1e3:.2f})", flush=True)
PY
    done
  done
done
