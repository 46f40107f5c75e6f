"""Would spreading the contact envs evenly over the wavefronts shorten the
slowest wave (round 6)?  With the mask-trace build (OGBX_MASK_TRACE), pairs
of consecutive bench steps of pointmaze-large at N = 65,536: step t gives each
env's contact flag (some lean-stage mask non-zero), step t + 1 each env's
set of lean stages that iterated (start mask != settled mask; stage 0's
Newton step excluded).  A wave runs the iterations of the union of its envs'
sets, so for a layout (env -> wave) the wave's iterated-stage count is the
popcount of that union.  Compared: the contiguous layout the kernel uses,
the step-t contact envs dealt round-robin over the waves (the layout a
contact-balancing permutation would give, from the previous step's flags),
and random layouts.  Reported: max and slowest-1 % mean over waves.
  OGBX_LIB=_abx/libogbx_masks.so python scripts/probe_wave_balance.py"""
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


def union_counts(sets, layout, nw):
    """sets: [n] uint32 stage bitmasks; layout: [n] wave of each env."""
    u = np.zeros(nw, np.uint32)
    np.bitwise_or.at(u, layout, sets)
    return np.array([bin(int(x)).count('1') for x in u])


def main():
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    n, nw = 65536, 1024
    L = _lib.lib()
    env, acts = bench._maze_job(n, 0, n, 128, dev)
    views = list(acts.unbind(0))
    buf = (ctypes.c_uint32 * (65536 * 40))()
    rng = np.random.default_rng(0)
    rows = []

    def trace(i):
        env.step(views[i % 128])
        torch.cuda.synchronize()
        L.ogbx_diag_mask_trace(buf)
        return np.frombuffer(buf, dtype=np.uint32).reshape(n, 20, 2).copy()

    for i in range(400):
        if i >= 100 and i % 20 == 0:
            a0 = trace(i)
            a1 = trace(i + 1)
            contact0 = ((a0[:, :, 0] | a0[:, :, 1]) != 0).any(1)
            start, end = a1[:, :, 0], a1[:, :, 1] & 0x1FF
            it = start != end
            it[:, 0] = False
            sets = (it.astype(np.uint32) << np.arange(20, dtype=np.uint32)).sum(1).astype(np.uint32)
            contig = np.arange(n) // 64
            # balanced: contact envs (by step-t flags) dealt round-robin, then the free envs
            order = np.concatenate([np.flatnonzero(contact0), np.flatnonzero(~contact0)])
            bal = np.empty(n, np.int64)
            bal[order] = np.arange(n) % nw
            res = {}
            for name, lay in (('contiguous', contig), ('balanced', bal), ('random', rng.permutation(n) // 64)):
                c = np.sort(union_counts(sets, lay, nw))
                res[name] = (int(c[-1]), float(c[-max(1, nw // 100):].mean()), float(c.mean()))
            res['contact_envs'] = int(contact0.sum())
            res['contact_per_wave_max_contiguous'] = int(np.bincount(contig[contact0], minlength=nw).max())
            rows.append(res)
        else:
            env.step(views[i % 128])
    out = {k: dict(max=float(np.mean([r[k][0] for r in rows])), top1pct=float(np.mean([r[k][1] for r in rows])),
                   mean=float(np.mean([r[k][2] for r in rows])))
           for k in ('contiguous', 'balanced', 'random')}
    out['samples'] = len(rows)
    out['contact_envs'] = float(np.mean([r['contact_envs'] for r in rows]))
    out['contact_per_wave_max_contiguous'] = float(np.mean([r['contact_per_wave_max_contiguous'] for r in rows]))
    print(json.dumps(out), flush=True)
    env.close()


if __name__ == '__main__':
    main()
