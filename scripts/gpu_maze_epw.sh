#!/bin/bash
# Envs-per-wave sweep of the pointmaze step at the strong-scaling shares (GPU
# box): bench.py --num-envs N with OGBX_EPW in {64, 32, 16}.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for N in ${NS:-8192 16384 32768}; do
  for E in ${EPWS:-64 32 16}; do
    OGBX_EPW=$E timeout -k 10 120 python bench.py --num-envs $N --steps 2000 --no-extras --no-cpu-baseline \
      > gpurun_out/epw.log 2>&1 || { tail -20 gpurun_out/epw.log; exit 4; }
    python - gpurun_out/epw.log "$E" <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(f"epw={sys.argv[2]:>2} N={r['config']['total_envs']:6d}: {r['ms_per_step']*1e3:.2f} us/step, "
      f"kernel {r['roofline']['kernel_ms']*1e3:.2f} us", flush=True)
PY
  done
done
