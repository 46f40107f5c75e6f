#!/bin/bash
# After a gpurun of scripts/gpu_refresh.sh: write the pointmaze profile set
# (kernel stats, traffic, bench lines, issue-counter PMC) into profiles/.
set -e
cd "$(dirname "$0")/.."
python scripts/prof_summary.py --round r01 --workload pointmaze --kernel maze_step_kernel
grep '^{' gpurun_out/bench_default.log > profiles/r01_pointmaze_bench.json
grep '^{' gpurun_out/prof_pointmaze.log > profiles/r01_pointmaze_bench_under_rocprof.json
python - <<'PY'
import csv, glob, json, collections
f = sorted(glob.glob('gpurun_out/pmc_maze_sq/**/*counter_collection.csv', recursive=True))[-1]
acc = collections.defaultdict(float); disp = set()
for r in csv.DictReader(open(f)):
    if 'maze_step_kernel' not in r['Kernel_Name']:
        continue
    acc[r['Counter_Name']] += float(r['Counter_Value']); disp.add(r['Dispatch_Id'])
n = len(disp); c = {k: v / n for k, v in sorted(acc.items())}
d = {'kernel': 'maze_step_kernel', 'workload': 'pointmaze', 'dispatches': n, 'counters_avg_per_dispatch': c,
     'valu_per_wave': c['SQ_INSTS_VALU'] / c['SQ_WAVES'], 'salu_per_wave': c['SQ_INSTS_SALU'] / c['SQ_WAVES'],
     'wave_cycles_per_wave_x4': c['SQ_WAVE_CYCLES'] / c['SQ_WAVES'] * 4}
json.dump(d, open('profiles/r01_pointmaze_issue_pmc.json', 'w'), indent=1)
print(json.dumps(d, indent=1))
PY
