"""Is a kernel right after a synchronize slower than one in a back-to-back run
(round 6, the driver window)?  With the wave-stamp build (OGBX_WAVE_STAMPS:
per wave s_memrealtime at entry/exit and shader cycles of the last launch),
for k = 1..20: synchronize, k bench steps, synchronize, read the stamps of
the k-th launch -- its duration (first wave start to last wave end) and the
effective shader clock (cycles / wall time of its waves); then the same after
1,000 back-to-back launches behind a spin kernel.
  OGBX_LIB=_abx/libogbx_stages.so python scripts/probe_window_clock.py"""
import ctypes
import json
import os
import sys

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
    views = list(acts.unbind(0))
    buf = (ctypes.c_ulonglong * (4096 * 4))()
    nw = n // 64

    def stamp():
        L.ogbx_diag_wave_stamps(buf)
        a = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 4)[:nw].astype(np.int64)
        t0, t1, cyc = a[:, 0], a[:, 1], a[:, 2]
        return dict(launch_us=float((t1.max() - t0.min()) / 100.0), wave_us_mean=float((t1 - t0).mean() / 100.0),
                    ghz=float(cyc.sum() / ((t1 - t0).sum() / 100.0) / 1e3))

    i = 0
    for _ in range(5):
        env.step(views[i % 128]); i += 1
    by_k = {}
    for rep in range(3):
        for k in range(1, 21):
            torch.cuda.synchronize(dev)
            for _ in range(k):
                env.step(views[i % 128]); i += 1
            torch.cuda.synchronize(dev)
            by_k.setdefault(k, []).append(stamp())
    # back to back behind a spin kernel, then the last launch's stamps
    torch.cuda.synchronize(dev)
    torch.cuda._sleep(int(1000 * 60e-6 * 2.4e9))
    for _ in range(1000):
        env.step(views[i % 128]); i += 1
    torch.cuda.synchronize(dev)
    b2b = stamp()
    res = dict(after_sync={k: dict(launch_us=float(np.mean([s['launch_us'] for s in v])),
                                   ghz=float(np.mean([s['ghz'] for s in v]))) for k, v in by_k.items()},
               back_to_back_last=b2b)
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
