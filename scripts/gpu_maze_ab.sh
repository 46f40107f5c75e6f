#!/bin/bash
# A/B of locomaze builds (GPU box): the timed pointmaze bench at N = 65,536 and
# 8,192 under each library in $LIBS (default: the in-tree libogbx.so and every
# _abx/libogbx_*.so), alternating, $ROUNDS rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS=${LIBS:-"ogbench_amd/libogbx.so $(ls _abx/libogbx_*.so 2>/dev/null | tr '\n' ' ')"}
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in $LIBS; do
    for N in ${NS:-65536 8192}; do
      OGBX_LIB=$PWD/$lib timeout -k 10 120 python bench.py --num-envs $N --no-extras --no-cpu-baseline \
        > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 4; }
      python - gpurun_out/ab.log "$lib" <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(f"{sys.argv[2]:40s} N={r['config']['total_envs']:6d}: {r['value']/1e9:.3f} G env-steps/s, "
      f"{r['ms_per_step']*1e3:.2f} us/step, kernel {r['roofline']['kernel_ms']*1e3:.2f} us", flush=True)
PY
    done
  done
done
