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


def prepare(data):
    """What GCDataset.__post_init__ computes once (impls/utils/datasets.py:
    59-60, 182-190): valid_idxs and terminal_locs.  Pass it as `prep` to
    sample / hgc_sample so that a timed loop (bench.py's cpu_baseline) does
    per call only what the reference does per call."""
    return dict(valid=np.nonzero(data['valids'] > 0)[0] if 'valids' in data else None,
                term_locs=np.nonzero(data['terminals'] > 0)[0])


def _final(prep, idxs):
    # final_state_idxs = terminal_locs[searchsorted(terminal_locs, idxs)] (datasets.py:309)
    return prep['term_locs'][np.searchsorted(prep['term_locs'], idxs)]


def sample(data, cfg, draws, idxs=None, prep=None):
    """One GCDataset.sample with the given draws (names as ogbx_gc_draws)."""
    size = max(len(v) for v in data.values())
    prep = prepare(data) if prep is None else prep
    valid = prep['valid']
    if idxs is None:
        idxs = valid[draws['pick']] if valid is not None else draws['pick']
    idxs = np.asarray(idxs, np.int64)
    fin = _final(prep, idxs)

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


def compute_high_next_idxs(idxs, fin, goal, steps):
    """HGCDataset.compute_high_next_idxs (impls/utils/datasets.py:478-491)."""
    s = np.minimum(np.full(len(idxs), steps, np.int64), fin - idxs)
    diff = goal - idxs
    s = np.where((0 <= diff) & (diff < s), diff, s)
    return idxs + s, s


def hgc_sample(data, cfg, draws, prep=None):
    """One HGCDataset.sample (impls/utils/datasets.py:496-643) with the given
    draws (pick, v_*, [l_*], a_*).  Returns the batch dict (reference keys and
    order) and the goal indices."""
    size = max(len(v) for v in data.values())
    prep = prepare(data) if prep is None else prep
    valid = prep['valid']
    idxs = (valid[draws['pick']] if valid is not None else draws['pick']).astype(np.int64)
    fin = _final(prep, idxs)

    def goals(p, p_cur, p_traj, geom):
        rnd = valid[draws[p + 'pick']] if valid is not None else draws[p + 'pick']
        if geom:
            traj = np.minimum(idxs + draws[p + 'geom'], fin)
        else:
            d = draws[p + 'dist']
            traj = np.round(np.minimum(idxs + 1, fin) * d + fin * (1 - d)).astype(np.int64)
        if p_cur == 1.0:
            return idxs
        g = np.where(draws[p + 'u_traj'] < p_traj / (1.0 - p_cur), traj, rnd)
        return np.where(draws[p + 'u_cur'] < p_cur, idxs, g)

    obs = data['observations']
    src = data['oracle_reps'] if 'oracle_reps' in data else obs
    disc = cfg['discount']
    out = {k: v[idxs] for k, v in data.items()}
    if 'next_observations' not in data:
        out['next_observations'] = obs[np.minimum(idxs + 1, size - 1)]
    hvg = goals('v_', cfg['value_p_curgoal'], cfg['value_p_trajgoal'], cfg['value_geom_sample'])
    high = cfg.get('high_subgoal_steps', cfg['subgoal_steps'])
    vsteps = high if cfg.get('value_subgoal_steps') is None else cfg['value_subgoal_steps']
    hv_next, hv_s = compute_high_next_idxs(idxs, fin, hvg, vsteps)
    out['high_value_reps'] = out['observations']
    out['high_value_goals'] = src[hvg]
    out['high_value_actions'] = src[hv_next]
    out['high_value_next_observations'] = obs[hv_next]
    out['high_value_offsets'] = hvg - idxs
    succ = (hv_s < vsteps).astype(float)
    out['high_value_subgoal_steps'] = hv_s
    out['high_value_masks'] = 1.0 - succ
    out['high_value_rewards'] = (-(1 - disc ** hv_s) / (1 - disc) if cfg['gc_negative'] else (disc ** hv_s) * succ)
    lsteps = cfg.get('low_subgoal_steps', cfg['subgoal_steps'])
    lv_next, lv_s = compute_high_next_idxs(idxs, fin, hvg, lsteps)
    out['low_value_next_observations'] = obs[lv_next]
    succ = (lv_s < lsteps).astype(float)
    out['low_value_subgoal_steps'] = lv_s
    out['low_value_masks'] = 1.0 - succ
    out['low_value_rewards'] = (-(1 - disc ** lv_s) / (1 - disc) if cfg['gc_negative'] else (disc ** lv_s) * succ)
    lvg = None
    if cfg.get('low_discount') is not None:
        lvg = goals('l_', cfg['value_p_curgoal'], cfg['value_p_trajgoal'], True)
        out['low_value_goals'] = src[lvg]
        s = (idxs == lvg).astype(float)
        out['low_value_masks'] = 1.0 - s
        out['low_value_rewards'] = s - (1.0 if cfg['gc_negative'] else 0.0)
    s = (idxs == hvg).astype(float)
    out['value_goals'] = out['high_value_goals']
    out['masks'] = 1.0 - s
    out['rewards'] = s - (1.0 if cfg['gc_negative'] else 0.0)
    hag = goals('a_', cfg['actor_p_curgoal'], cfg['actor_p_trajgoal'], cfg['actor_geom_sample'])
    asteps = high if cfg.get('actor_subgoal_steps') is None else cfg['actor_subgoal_steps']
    ha_next, _ = compute_high_next_idxs(idxs, fin, hag, asteps)
    out['high_actor_goals'] = src[hag]
    out['high_actor_actions'] = src[ha_next]
    out['high_actor_next_observations'] = obs[ha_next]
    out['high_actor_targets'] = out['high_actor_actions']
    la_goal = np.minimum(idxs + asteps, fin)
    out['low_actor_goals'] = src[la_goal]
    out['low_actor_goal_observations'] = obs[la_goal]
    la_next, _ = compute_high_next_idxs(idxs, fin, hag, lsteps)
    out['low_actor_next_observations'] = obs[la_next]
    return out, dict(idxs=idxs, hvg=hvg, hag=hag, lvg=lvg)
