"""Diagnostic (round 6): where the lean loop's active-set iterations come
from.  With the mask-trace build (OGBX_MASK_TRACE: per env and lean stage the
mask the stage started from and the one it settled on), one bench step of
pointmaze-large at N = 65,536 after `warm` steps; for every stage that had to
iterate (start != settled), is the settled mask the one the same RK phase
settled on in the previous substep (stage e - 4), the one two stages back, or
a mask not seen before in the step?  Reported over all envs and over the envs
with the most iterating stages (the slowest waves' envs).
  OGBX_LIB=_abx/libogbx_masks.so python scripts/probe_mask_trace.py"""
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
    buf = (ctypes.c_uint32 * (65536 * 40))()
    stats = []
    for i in range(300):
        env.step(views[i % 128])
        if i >= 100 and i % 20 == 0:
            torch.cuda.synchronize()
            # zero the trace, step once, read it
            L.ogbx_diag_mask_trace(buf)
            a = np.frombuffer(buf, dtype=np.uint32).reshape(65536, 20, 2).copy()
            stats.append(a)
    a = np.concatenate(stats)  # [samples*envs, 20, 2]
    start, end = a[:, :, 0], a[:, :, 1] & 0x1FF
    contact = (a[:, :, 0] | a[:, :, 1]) != 0
    envs = contact.any(1)
    it = (start != end)
    it[:, 0] = False  # stage 0 always runs its Newton step (start is the u = 0 mask)
    per_env = it.sum(1)
    res = dict(samples=int(a.shape[0]), contact_envs=int(envs.sum()), iterating_stage_fraction=float(it[envs].mean()))
    # predictors for a stage e >= 4 that iterated: settled == settled at e - 4 (same RK phase), e - 2, e - 1's start
    e_idx = np.arange(20)
    for name, lag in (('same_phase_prev_substep', 4), ('two_back', 2), ('one_back_start', None)):
        hits = tot = 0
        for e in range(4, 20):
            m = it[:, e]
            if lag is None:
                pred = start[:, e - 1]
            else:
                pred = end[:, e - lag]
            hits += int((end[m, e] == pred[m]).sum())
            tot += int(m.sum())
        res[f'pred_{name}'] = hits / max(1, tot)
    order = np.argsort(per_env)[::-1]
    top = order[: max(1, int(0.01 * envs.sum()))]
    res['top1pct_env_iterating_stages'] = float(per_env[top].mean())
    res['median_contact_env_iterating_stages'] = float(np.median(per_env[envs]))
    hits = tot = 0
    for e in range(4, 20):
        m = it[top, e]
        hits += int((end[top][m, e] == end[top][m, e - 4]).sum())
        tot += int(m.sum())
    res['top1pct_pred_same_phase'] = hits / max(1, tot)
    # iterating stages per RK phase (e % 4) over all contact envs
    res['iterating_by_phase'] = [float(it[envs][:, p::4].mean()) for p in range(4)]
    # how often would the same-phase predictor change a stage that did NOT iterate (a wrong warm start)?
    bad = tot2 = 0
    for e in range(4, 20):
        m = ~it[:, e] & envs
        bad += int((end[m, e - 4] != start[m, e]).sum())
        tot2 += int(m.sum())
    res['same_phase_pred_wrong_on_settled_stages'] = bad / max(1, tot2)
    print(json.dumps(res), flush=True)
    env.close()


if __name__ == '__main__':
    main()
