#!/bin/bash
# Round 5 check B: the GPU suite, the sampler benches and the maze A/B
# against the variants in _abx/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread ${PYTEST_ARGS:-} \
  > gpurun_out/r05_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r05_gpu.log; [ $rc -eq 0 ] || exit $rc
for w in ${SAMPLERS:-gcsample hgcsample}; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > gpurun_out/r05_$w.log 2>&1 \
    || { tail -20 gpurun_out/r05_$w.log; exit 4; }
  python - gpurun_out/r05_$w.log <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
f = r['roofline']
print(f"{r['config']['workload']}: {r['value']/1e6:.1f} M/s, {r['ms_per_step']*1e3:.2f} us/step, {f['kernel']} "
      f"timed {f['kernel_ms_timed_region']*1e3:.2f} b2b {f['kernel_ms_back_to_back']*1e3:.2f} us host {r['extra'].get('host_us_per_call', 0):.2f} us")
PY
done
ROUNDS=${ROUNDS:-2} bash scripts/gpu_maze_ab.sh
