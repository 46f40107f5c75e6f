"""What makes the first launch after a synchronize slow (round 6, the driver
window)?  Wave-stamp build (OGBX_WAVE_STAMPS).  Each case: synchronize, then
the case's lead-in, then ONE bench step of the 65,536-env job, synchronize,
and that launch's duration from its waves' stamps (first wave start to last
wave end) and shader clock; 20 repetitions each, means.
  plain       nothing in between (the driver window's first step)
  spin        a 30-us spin kernel queued first (no idle gap, other code ran)
  fill        a 4-KB torch fill kernel first (other code, short)
  small_maze  a 64-env maze step of another handle first (same kernel code)
  second      a first bench step, then the stamped one (launch 2 of a window)
  idle_1ms    the host sleeps 1 ms after the synchronize
  OGBX_LIB=_abx/libogbx_stamps.so python scripts/probe_cold_start.py"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from ogbench_amd import _lib  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    n = 65536
    L = _lib.lib()
    env, acts = bench._maze_job(n, 0, n, 128, dev)
    small, sacts = bench._maze_job(64, 0, 64, 4, dev)
    views = list(acts.unbind(0))
    sviews = list(sacts.unbind(0))
    buf = (ctypes.c_ulonglong * (4096 * 4))()
    nw = n // 64
    scratch = torch.empty(1024, dtype=torch.float32, device=dev)

    def stamp():
        L.ogbx_diag_wave_stamps(buf)
        a = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 4)[:nw].astype(np.int64)
        t0, t1, cyc = a[:, 0], a[:, 1], a[:, 2]
        return float((t1.max() - t0.min()) / 100.0), float(cyc.sum() / ((t1 - t0).sum() / 100.0) / 1e3)

    i = 0
    for _ in range(50):
        env.step(views[i % 128]); i += 1
        small.step(sviews[i % 4])
    leads = {
        'plain': lambda: None,
        'spin': lambda: torch.cuda._sleep(int(30e-6 * 2.4e9)),
        'fill': lambda: scratch.fill_(1.0),
        'small_maze': lambda: small.step(sviews[0]),
        'second': lambda: env.step(views[0]),
        'idle_1ms': lambda: time.sleep(1e-3),
    }
    res = {}
    for rep in range(20):
        for name, lead in leads.items():
            torch.cuda.synchronize(dev)
            lead()
            env.step(views[i % 128]); i += 1
            torch.cuda.synchronize(dev)
            res.setdefault(name, []).append(stamp())
    torch.cuda.synchronize(dev)
    torch.cuda._sleep(int(1000 * 60e-6 * 2.4e9))
    for _ in range(500):
        env.step(views[i % 128]); i += 1
    torch.cuda.synchronize(dev)
    out = {k: dict(launch_us=float(np.mean([s[0] for s in v])), ghz=float(np.mean([s[1] for s in v])))
           for k, v in res.items()}
    us, ghz = stamp()
    out['back_to_back_last'] = dict(launch_us=us, ghz=ghz)
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
