"""Per-wave averages of rocprofv3 --pmc counter CSVs for one kernel.
usage: python scripts/pmc_summary.py <dir with <tag>_p<k>/ subdirs> <kernel substring>"""
import collections
import csv
import glob
import os
import sys

root, kern = sys.argv[1], sys.argv[2]
res = collections.defaultdict(dict)
for d in sorted(glob.glob(os.path.join(root, '*_p*'))):
    if not os.path.isdir(d):
        continue
    tag = os.path.basename(d).rsplit('_p', 1)[0]
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        sums, n = collections.defaultdict(float), collections.defaultdict(int)
        for row in csv.DictReader(open(f)):
            if kern not in row.get('Kernel_Name', ''):
                continue
            sums[row['Counter_Name']] += float(row['Counter_Value'])
            n[row['Counter_Name']] += 1
        for k in sums:
            res[tag][k] = sums[k] / max(1, n[k])  # per dispatch
    for f in glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True):
        ds = [int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in csv.DictReader(open(f))
              if kern in r.get('Kernel_Name', '')]
        if ds:
            res[tag]['_kernel_ns'] = sum(ds) / len(ds)
for tag, c in res.items():
    if '_kernel_ns' in c and 'GRBM_GUI_ACTIVE' in c:
        # GRBM_GUI_ACTIVE is summed over the 8 XCCs
        print(tag, f'kernel {c["_kernel_ns"] / 1e3:.2f} us, GUI_ACTIVE/XCC {c["GRBM_GUI_ACTIVE"] / 8:.0f} clk '
              f'-> {c["GRBM_GUI_ACTIVE"] / 8 / c["_kernel_ns"]:.3f} GHz')
    w = c.get('SQ_WAVES', 1.0) or 1.0
    print(tag, ' '.join(f'{k}={v / w:.1f}' for k, v in sorted(c.items()) if k not in ('SQ_WAVES', '_kernel_ns')), f'waves={w:.0f}')
