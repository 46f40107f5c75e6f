#!/bin/bash
# A/B of library builds (GPU box): bench.py --workload $wl (timed step only)
# under the in-tree library and each _abx/libogbx_*.so ($LIBS), alternating,
# $ROUNDS rounds; one line per run with the workload's kernel time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIBS=${LIBS:-"ogbench_amd/libogbx.so $(ls _abx/libogbx_*.so 2>/dev/null | tr '\n' ' ')"}
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in $LIBS; do
    for wl in ${WLS:-gcsample hgcsample}; do
      OGBX_LIB=$PWD/$lib timeout -k 10 200 python bench.py --workload $wl --steps ${STEPS:-2000} --warmup 100 --no-extras ${EXTRA:-} \
        --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 4; }
      python - gpurun_out/ab.log "$lib" "$wl" <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
rf = r['roofline']
print(f"{sys.argv[2]:34s} {sys.argv[3]:13s}: {r['value']/1e6:.2f} M {r['unit']}, step {r['ms_per_step']*1e3:.2f} us, "
      f"kernel {rf['kernel_ms']*1e3:.2f} us (b2b {rf.get('kernel_ms_back_to_back', 0)*1e3:.2f}, timed {rf.get('kernel_ms_timed_region', 0)*1e3:.2f})", flush=True)
PY
    done
  done
done
