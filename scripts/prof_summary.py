"""Summarise rocprofv3 runs of bench.py into profiles/ (run on the GPU box or
after gpurun merged gpurun_out/ back).

For one workload it reads
  gpurun_out/prof_<wl>/        --kernel-trace --stats   (kernel_stats.csv)
  gpurun_out/pmc_fetch_<wl>/   --pmc FETCH_SIZE         (counter_collection.csv)
  gpurun_out/pmc_write_<wl>/   --pmc WRITE_SIZE
and writes profiles/<round>_<wl>_kernel_stats.csv (copy of the stats table) and
the entry of the workload's dominant kernel in profiles/traffic.json:
  hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024, averaged over
  that kernel's dispatches (FETCH_SIZE/WRITE_SIZE in KiB; FETCH_SIZE doubled per
  the gfx950 note in MI355X_MICROARCH.md section HBM).

  python scripts/prof_summary.py --round r02 --workload powder --kernel pw_step_kernel --units 4096
"""

import argparse
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _one(pattern):
    files = sorted(glob.glob(pattern, recursive=True))
    if not files:
        raise SystemExit(f'no file matches {pattern}')
    return files[-1]


def counter_avg(d, counter, kernel):
    path = _one(os.path.join(d, '**', '*counter_collection.csv'))
    vals = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get('Counter_Name') != counter or kernel not in row.get('Kernel_Name', ''):
                continue
            key = row.get('Dispatch_Id') or row.get('Correlation_Id')
            vals[key] = vals.get(key, 0.0) + float(row['Counter_Value'])
    if not vals:
        raise SystemExit(f'no {counter} rows for {kernel} in {path}')
    return sum(vals.values()) / len(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--round', required=True)
    ap.add_argument('--workload', required=True)
    ap.add_argument('--kernel', required=True)
    ap.add_argument('--label', default=None, help="traffic.json key's kernel name (default: --kernel), as bench.py names it")
    ap.add_argument('--units', type=int, required=True, help='envs or samples per launch of the profiled run')
    ap.add_argument('--world', type=int, default=1)
    ap.add_argument('--out', default=os.path.join(ROOT, 'gpurun_out'))
    a = ap.parse_args()
    stats = _one(os.path.join(a.out, f'prof_{a.workload}', '**', '*kernel_stats.csv'))
    dst = os.path.join(ROOT, 'profiles', f'{a.round}_{a.workload}_kernel_stats.csv')
    shutil.copyfile(stats, dst)
    with open(stats) as f:
        rows = list(csv.DictReader(f))
    # '+'-joined kernels (a step made of several launches): per-step duration
    # and bytes are the sums over the parts, each part weighted by its share of
    # the steps (a part may skip steps: the powder light kernel is not launched
    # on steps where every env runs the full kernel); steps = the most calls
    parts = a.kernel.split('+')
    per = []
    for k in parts:
        # every row whose name contains the part (template instances of one
        # kernel, e.g. the powder step kernel's dense and sparse forms)
        tot, n = 0.0, 0
        for row in rows:
            if k in row['Name']:
                tot += float(row['TotalDurationNs'])
                n += int(row['Calls'])
        avg = tot / n if n else 0.0
        fk, nfk = counter_avg(os.path.join(a.out, f'pmc_fetch_{a.workload}'), 'FETCH_SIZE', k)
        wk, nwk = counter_avg(os.path.join(a.out, f'pmc_write_{a.workload}'), 'WRITE_SIZE', k)
        per.append((avg, n, fk, nfk, wk, nwk))
    calls = max(p[1] for p in per)
    nf = max(p[3] for p in per)
    nw = max(p[5] for p in per)
    avg_ns = sum(p[0] * p[1] for p in per) / calls
    fetch = sum(p[2] * p[3] for p in per) / nf
    write = sum(p[4] * p[5] for p in per) / nw
    rec = dict(
        workload=a.workload,
        round=a.round,
        fetch_size_kib_avg=fetch,
        write_size_kib_avg=write,
        hbm_bytes_per_launch=(2.0 * fetch + write) * 1024.0,
        pmc_dispatches=[nf, nw],
        kernel_trace_avg_ns=avg_ns,
        kernel_trace_calls=calls,
        stats_file=os.path.relpath(dst, ROOT),
        units=a.units,
        world=a.world,
    )
    tpath = os.path.join(ROOT, 'profiles', 'traffic.json')
    data = {}
    if os.path.exists(tpath):
        with open(tpath) as f:
            data = json.load(f)
    # keyed by workload; bench.py uses it only for a run of the same units and world size
    data[f'{a.label or a.kernel}@{a.workload}'] = rec
    with open(tpath, 'w') as f:
        json.dump(data, f, indent=1, sort_keys=True)
    print(json.dumps({a.kernel: rec}))


if __name__ == '__main__':
    main()
