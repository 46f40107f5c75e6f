"""Host time of each env.step call inside bench.py's 20-step window, without a
profiler (round 6): 60 windows of the driver's shape (synchronize, 20 calls,
synchronize); per call position the median and the count of slow calls, and
the distribution of the window's device span per step against back to back.
  python scripts/probe_window_host.py"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    n, K = 65536, 20
    env, acts = bench._maze_job(n, 0, n, 128, dev)
    views = list(acts.unbind(0))
    for i in range(5):
        env.step(views[i % 128])
    calls, spans, walls = [], [], []
    for w in range(60):
        torch.cuda.synchronize(dev)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        t = [time.perf_counter_ns()]
        for i in range(K):
            env.step(views[i % 128])
            t.append(time.perf_counter_ns())
        b.record()
        torch.cuda.synchronize(dev)
        t_end = time.perf_counter_ns()
        calls.append(np.diff(t) / 1e3)
        spans.append(a.elapsed_time(b) * 1e3 / K)
        walls.append((t_end - t[0]) / 1e3 / K)
    c = np.array(calls)
    b2b = bench._per_launch_ms(lambda i: env.step(views[i % 128]), 1000, dev, 60.0) * 1e3
    res = dict(b2b_us=b2b, call_us_median_by_position=np.median(c, 0).round(2).tolist(),
               slow_calls_over_15us_by_position=(c > 15).sum(0).tolist(),
               call_us_p50=float(np.median(c)), call_us_p99=float(np.percentile(c, 99)), call_us_max=float(c.max()),
               span_per_step_us=dict(p10=float(np.percentile(spans, 10)), p50=float(np.median(spans)),
                                     p90=float(np.percentile(spans, 90))),
               wall_per_step_us=dict(p10=float(np.percentile(walls, 10)), p50=float(np.median(walls)),
                                     p90=float(np.percentile(walls, 90))))
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
