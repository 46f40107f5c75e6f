#!/bin/bash
# Round 4: maze A/B (in-tree lib vs _abx variants), GC/HGC look-ahead A/B
# with full bench lines, kernel trace of the GC look-ahead.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS=${LIBS:-"ogbench_amd/libogbx.so _abx/libogbx_v1.so _abx/libogbx_v1c.so"} ROUNDS=${ROUNDS:-2} bash scripts/gpu_maze_ab.sh || exit $?
for la in 1 0 1 0; do
  for w in gcsample hgcsample; do
    OGBX_GC_LOOKAHEAD=$la timeout -k 10 120 python bench.py --workload $w --no-extras --no-cpu-baseline > gpurun_out/gc_ab.log 2>&1 || { tail -5 gpurun_out/gc_ab.log; exit 4; }
    python - gpurun_out/gc_ab.log $w $la <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
f = r['roofline']
print(f"{sys.argv[2]:10s} lookahead={sys.argv[3]}: {r['value']/1e6:.1f} M/s, {r['ms_per_step']*1e3:.2f} us/call, "
      f"kernel {f['kernel_ms']*1e3:.2f} us (timed region {f.get('kernel_ms_timed_region', 0)*1e3:.2f}, "
      f"b2b {f.get('kernel_ms_back_to_back', 0)*1e3:.2f})", flush=True)
PY
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gcla -o run --output-format csv -- python3 bench.py --workload gcsample --steps 300 --warmup 100 --no-cpu-baseline --no-extras > gpurun_out/prof_gcla.log 2>&1 || exit 5
find gpurun_out/prof_gcla -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-150
