"""Line up scripts/probe_window.py's host stamps with the kernel trace of the
same run (rocprofv3 --kernel-trace --output-format csv): per window, when the
host issued each env.step, when each maze_step_kernel started and ended on the
device, and where the device sat idle inside the HIP event span.

  python scripts/window_summary.py gpurun_out/r06_window_host.json gpurun_out/r06_win
"""

import csv
import glob
import json
import os
import sys


def main():
    host = json.load(open(sys.argv[1]))
    trace = sorted(glob.glob(os.path.join(sys.argv[2], '**', '*kernel_trace.csv'), recursive=True))[-1]
    ks = []
    with open(trace) as f:
        for r in csv.DictReader(f):
            if 'maze_step_kernel' in r['Kernel_Name']:
                ks.append((int(r['Start_Timestamp']), int(r['End_Timestamp'])))
    ks.sort()
    K = host['steps']
    out = []
    for w in host['windows']:
        off = w['boottime_minus_monotonic_ns']
        h = [t + off for t in w['host_ns']]  # host stamps on the trace's clock
        t0, t_end = h[0], h[-1]
        mine = [k for k in ks if t0 <= k[0] <= t_end]
        if len(mine) != K:
            out.append(dict(error=f'{len(mine)} kernels in window'))
            continue
        first_start = mine[0][0] - t0  # host's event record -> first kernel start
        gaps = [mine[i + 1][0] - mine[i][1] for i in range(K - 1)]
        durs = [e - s for s, e in mine]
        lag = [mine[i][0] - h[i + 1] for i in range(K)]  # kernel start - host return of its call
        out.append(dict(host_call_us=[(h[i + 1] - h[i]) / 1e3 for i in range(K)],
                        first_kernel_after_t0_us=first_start / 1e3,
                        kernel_us=[d / 1e3 for d in durs], gap_us=[g / 1e3 for g in gaps],
                        start_minus_host_return_us=[x / 1e3 for x in lag],
                        span_per_step_us=w['span_ms'] * 1e3 / K,
                        sum_kernel_us=sum(durs) / 1e3, sum_gap_us=sum(gaps) / 1e3,
                        tail_us=(t_end - mine[-1][1]) / 1e3))
    print(json.dumps(dict(host_us=host['host_us'], b2b_ms=host['kernel_ms_back_to_back'], windows=out), indent=1))


if __name__ == '__main__':
    main()
