#!/bin/bash
# A/B of powder builds (GPU box): the powder / powder-medium bench (timed step
# only) under the in-tree library and each _abx/libogbx_pwf_*.so,
# alternating, $ROUNDS rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIBS=${LIBS:-"ogbench_amd/libogbx.so $(ls _abx/libogbx_pwf_*.so 2>/dev/null | tr '\n' ' ')"}
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in $LIBS; do
    for wl in ${WLS:-powder powder-medium}; do
      OGBX_LIB=$PWD/$lib timeout -k 10 200 python bench.py --workload $wl --steps ${STEPS:-600} --warmup 60 --no-extras \
        --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 4; }
      python - gpurun_out/ab.log "$lib" "$wl" <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
rf = r['roofline']
print(f"{sys.argv[2]:34s} {sys.argv[3]:13s}: {r['value']/1e6:.2f} M env-steps/s, kernel {rf['kernel_ms']*1e3:.1f} us, frac {rf['frac']:.3f}", flush=True)
PY
    done
  done
done
