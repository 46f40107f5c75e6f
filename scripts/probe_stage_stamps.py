"""Diagnostic (verdict r05 item 4): what the slowest waves of maze_step_kernel
wait on, at lean-stage granularity.  Bench setting (pointmaze-large, N envs,
task i%5+1, auto-reset, uniform actions, warmed); every 10th step of 300 is
stamped.  Per wave: its lifetime in shader cycles (OGBX_WAVE_STAMPS) and the
lean stage's parts summed over the step's 20 stages (OGBX_STAGE_STAMPS):
collision, piece solve, edge mask, slots, active-set iterations, RK update,
plus iteration trips.  Reports the median wave against the slowest 1 % (by
lifetime) among waves that ran the contact loop.

Run with OGBX_LIB=_abx/libogbx_stages.so built by
  scripts/build_maze_variant.sh stages -DOGBX_STAGE_STAMPS -DOGBX_WAVE_STAMPS
"""
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

PARTS = ['collision', 'solve', 'mask', 'slots', 'iterations', 'rk_update']


def main():
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    L = _lib.lib()
    env, acts = bench._maze_job(n, 0, n, 128, dev)
    views = list(acts.unbind(0))
    nw = (n + 63) // 64
    wbuf = (ctypes.c_ulonglong * (4096 * 4))()
    sbuf = (ctypes.c_ulonglong * (4096 * 8))()
    life, parts = [], []
    for i in range(300):
        stamp = i >= 100 and i % 10 == 0
        if stamp:
            torch.cuda.synchronize()
            L.ogbx_diag_wave_stages(sbuf)  # clear
        env.step(views[i % 128])
        if stamp:
            torch.cuda.synchronize()
            L.ogbx_diag_wave_stamps(wbuf)
            L.ogbx_diag_wave_stages(sbuf)
            w = np.frombuffer(wbuf, dtype=np.uint64).reshape(4096, 4)[:nw].astype(np.int64)
            s = np.frombuffer(sbuf, dtype=np.uint64).reshape(4096, 8)[:nw].astype(np.int64)
            life.append(w[:, 2])
            parts.append(s.copy())
    life = np.concatenate(life)
    parts = np.concatenate(parts)
    ran = parts[:, :6].sum(1) > 0  # waves that ran the lean loop
    lf, pt = life[ran], parts[ran]
    order = np.argsort(lf)
    med = order[len(order) // 2 - len(order) // 100: len(order) // 2 + len(order) // 100 + 1]
    top = order[int(0.99 * len(order)):]
    res = dict(num_envs=n, waves=int(len(life)), contact_waves=int(ran.sum()))
    for name, sel in (('median_band', med), ('slowest_1pct', top)):
        res[name] = dict(wave_cycles=float(lf[sel].mean()),
                         **{p: float(pt[sel, k].mean()) for k, p in enumerate(PARTS)},
                         iteration_trips=float(pt[sel, 6].mean()), stages_iterated=float(pt[sel, 7].mean()))
    m, t = res['median_band'], res['slowest_1pct']
    res['slowest_minus_median'] = {p: t[p] - m[p] for p in ['wave_cycles'] + PARTS + ['iteration_trips']}
    print(json.dumps(res), flush=True)
    env.close()


if __name__ == '__main__':
    main()
