"""oracle/gcdataset_np.py -- TEST INFRASTRUCTURE ONLY.

NumPy restatement of the reference offline sampler, the checker for
libogbx's gc_sample_kernel.  Pinned against tests/golden/gc_golden.npz, which
holds outputs of the reference's own impls/utils/datasets.py with the
recorded np.random draws.

  Dataset.get_random_idxs / get_subset  impls/utils/datasets.py:65-83
  GCDataset.__post_init__               impls/utils/datasets.py:182-211
  GCDataset.sample                      impls/utils/datasets.py:213-294
  GCDataset.sample_goals                impls/utils/datasets.py:296-327
  load_dataset (compact / regular)      ogbench/utils.py:14-96
"""

import numpy as np


def load_dataset(raw, compact_dataset=False, add_info=False):
    """ogbench/utils.py:14-96 on an in-memory dict of the .npz arrays."""
    d = {'observations': raw['observations'].astype(np.float32),
         'actions': raw['actions'].astype(np.float32),
         'terminals': raw['terminals'].astype(np.float32)}
    info = [k for k in ('qpos', 'qvel', 'button_states') if add_info and k in raw]
    for k in info:
        d[k] = raw[k]
    t = d['terminals']
    shifted = np.concatenate([t[1:], np.ones(1, np.float32)])
    if compact_dataset:
        d['valids'] = 1.0 - t
        d['terminals'] = np.minimum(t + shifted, 1.0).astype(np.float32)
    else:
        keep = (1.0 - t).astype(bool)
        keep_next = np.concatenate([[False], keep[:-1]])
        d['next_observations'] = d['observations'][keep_next]
        d['observations'] = d['observations'][keep]
        d['actions'] = d['actions'][keep]
        d['terminals'] = shifted[keep].astype(np.float32)
        for k in info:
            d[k] = d[k][keep]
    return d


def traj_end(terminals):
    locs = np.nonzero(terminals > 0)[0]
    return locs[np.searchsorted(locs, np.arange(len(terminals)))]


def sample(data, cfg, draws, idxs=None):
    """One GCDataset.sample with the given draws (names as ogbx_gc_draws)."""
    size = max(len(v) for v in data.values())
    valid = np.nonzero(data['valids'] > 0)[0] if 'valids' in data else None
    if idxs is None:
        idxs = valid[draws['pick']] if valid is not None else draws['pick']
    idxs = np.asarray(idxs, np.int64)
    fin = traj_end(data['terminals'])[idxs]

    def goals(p, pre):
        rnd = valid[draws[p + 'pick']] if valid is not None else draws[p + 'pick']
        if cfg[pre + '_geom_sample']:
            traj = np.minimum(idxs + draws[p + 'geom'], fin)
        else:
            d = draws[p + 'dist']
            traj = np.round(np.minimum(idxs + 1, fin) * d + fin * (1 - d)).astype(np.int64)
        if cfg[pre + '_p_curgoal'] == 1.0:
            return idxs
        thr = cfg[pre + '_p_trajgoal'] / (1.0 - cfg[pre + '_p_curgoal'])
        g = np.where(draws[p + 'u_traj'] < thr, traj, rnd)
        return np.where(draws[p + 'u_cur'] < cfg[pre + '_p_curgoal'], idxs, g)

    vg, ag = goals('v_', 'value'), goals('a_', 'actor')
    out = {k: v[idxs] for k, v in data.items()}
    if 'next_observations' not in data:
        out['next_observations'] = data['observations'][np.minimum(idxs + 1, size - 1)]
    src = data['oracle_reps'] if 'oracle_reps' in data else data['observations']
    out['value_goals'] = src[vg]
    out['actor_goals'] = src[ag]
    s = (idxs == vg).astype(float)
    out['masks'] = 1.0 - s
    out['rewards'] = s - (1.0 if cfg['gc_negative'] else 0.0)
    return out, idxs, vg, ag
