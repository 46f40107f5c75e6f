"""Golden fixtures for the offline sampler, from the reference's own code.

Imports ogbench/utils.py (load_dataset) and impls/utils/datasets.py
(Dataset, GCDataset, HGCDataset) with in-process stand-ins for the absent
third-party modules (gymnasium; jax.tree_util / jax.jit; flax FrozenDict),
builds small synthetic ragged trajectory buffers through the reference
load_dataset (compact and regular), runs the reference samplers under a fixed
np.random seed and records every np.random draw in call order.  Saves inputs,
draws and outputs only (tests/golden/gc_golden.npz).
"""

import importlib.util
import os
import sys
import types

import numpy as np

REF = os.environ.get('OGBENCH_REF', '/root/reference')
OUT = os.path.dirname(os.path.abspath(__file__))


def _stub_modules():
    gym = types.ModuleType('gymnasium')
    sys.modules.setdefault('gymnasium', gym)
    jax = types.ModuleType('jax')
    tu = types.ModuleType('jax.tree_util')

    def tree_map(f, tree, *rest):
        if isinstance(tree, dict) or hasattr(tree, '_dict'):
            d = tree._dict if hasattr(tree, '_dict') else tree
            return {k: tree_map(f, d[k], *[r[k] for r in rest]) for k in d}
        return f(tree, *rest)

    def tree_leaves(tree):
        if isinstance(tree, dict) or hasattr(tree, '_dict'):
            d = tree._dict if hasattr(tree, '_dict') else tree
            out = []
            for k in d:
                out += tree_leaves(d[k])
            return out
        return [tree]

    tu.tree_map = tree_map
    tu.tree_leaves = tree_leaves
    jax.tree_util = tu
    jax.jit = lambda f=None, **kw: (f if f is not None else (lambda g: g))
    jax.vmap = lambda f, *a, **k: f
    jax.lax = types.SimpleNamespace(dynamic_slice=None)
    jnp = types.ModuleType('jax.numpy')
    jax.numpy = jnp
    sys.modules['jax'] = jax
    sys.modules['jax.tree_util'] = tu
    sys.modules['jax.numpy'] = jnp
    flax = types.ModuleType('flax')
    core = types.ModuleType('flax.core')
    fd = types.ModuleType('flax.core.frozen_dict')

    class FrozenDict(dict):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            self._dict = dict(self)

        def copy(self, add_or_replace=None):
            d = dict(self._dict)
            d.update(add_or_replace or {})
            return type(self)(d)

    fd.FrozenDict = FrozenDict
    sys.modules['flax'] = flax
    sys.modules['flax.core'] = core
    sys.modules['flax.core.frozen_dict'] = fd


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def reference_modules():
    _stub_modules()
    pkg = types.ModuleType('ogbench')
    pkg.__path__ = [os.path.join(REF, 'ogbench')]
    sys.modules['ogbench'] = pkg
    relabel = _load('ogbench.relabel_utils', os.path.join(REF, 'ogbench/relabel_utils.py'))
    utils = _load('ogbench.utils', os.path.join(REF, 'ogbench/utils.py'))
    ds = _load('ref_datasets', os.path.join(REF, 'impls/utils/datasets.py'))
    return utils, ds, relabel


class Recorder:
    """Wrap np.random.{randint,geometric,rand} and log (name, value) in order."""

    def __init__(self):
        self.log = []
        self._saved = {}

    def __enter__(self):
        for name in ('randint', 'geometric', 'rand'):
            fn = getattr(np.random, name)
            self._saved[name] = fn

            def wrap(*a, _fn=fn, _name=name, **k):
                v = _fn(*a, **k)
                self.log.append((_name, np.array(v)))
                return v

            setattr(np.random, name, wrap)
        return self

    def __exit__(self, *exc):
        for name, fn in self._saved.items():
            setattr(np.random, name, fn)


def synthetic_npz(path, rng, n_traj, ob_dim, act_dim, min_len=3, max_len=40):
    """A raw OGBench-format .npz: trajectories of ragged length, terminals=1 at
    each trajectory's last row (as data_gen_scripts write them), qpos too."""
    obs, act, term, qpos = [], [], [], []
    for _ in range(n_traj):
        L = rng.randint(min_len, max_len + 1)
        obs.append(rng.normal(size=(L, ob_dim)).astype(np.float32))
        act.append(rng.uniform(-1, 1, (L, act_dim)).astype(np.float32))
        t = np.zeros(L, np.float32)
        t[-1] = 1
        term.append(t)
        qpos.append(rng.uniform(-4, 40, (L, 2)).astype(np.float32))
    np.savez(path, observations=np.concatenate(obs), actions=np.concatenate(act),
             terminals=np.concatenate(term), qpos=np.concatenate(qpos))


CONFIGS = {
    'gciql': dict(discount=0.99, value_p_curgoal=0.2, value_p_trajgoal=0.5, value_p_randomgoal=0.3,
                  value_geom_sample=True, actor_p_curgoal=0.0, actor_p_trajgoal=1.0, actor_p_randomgoal=0.0,
                  actor_geom_sample=False, gc_negative=True, p_aug=0.0, frame_stack=None),
    'crl': dict(discount=0.995, value_p_curgoal=0.0, value_p_trajgoal=1.0, value_p_randomgoal=0.0,
                value_geom_sample=True, actor_p_curgoal=0.0, actor_p_trajgoal=0.5, actor_p_randomgoal=0.5,
                actor_geom_sample=False, gc_negative=False, p_aug=None, frame_stack=None),
    'curone': dict(discount=0.9, value_p_curgoal=1.0, value_p_trajgoal=0.0, value_p_randomgoal=0.0,
                   value_geom_sample=False, actor_p_curgoal=0.3, actor_p_trajgoal=0.3, actor_p_randomgoal=0.4,
                   actor_geom_sample=True, gc_negative=True, p_aug=None, frame_stack=None),
}


def _draws_from_log(log, B, cfg):
    """Map the reference's np.random call log of one GCDataset.sample to the
    named draw vectors of ogbx_gc_draws (datasets.py:65-70, 296-327)."""
    it = iter(log)
    d = {}
    name, v = next(it)
    assert name == 'randint'
    d['pick'] = v.astype(np.int64)
    for pre in ('value', 'actor'):
        p = pre[0] + '_'
        name, v = next(it)
        assert name == 'randint'
        d[p + 'pick'] = v.astype(np.int64)
        name, v = next(it)
        if cfg[pre + '_geom_sample']:
            assert name == 'geometric'
            d[p + 'geom'] = v.astype(np.int64)
            d[p + 'dist'] = np.zeros(B)
        else:
            assert name == 'rand'
            d[p + 'dist'] = v.astype(np.float64)
            d[p + 'geom'] = np.zeros(B, np.int64)
        if cfg[pre + '_p_curgoal'] == 1.0:
            d[p + 'u_traj'] = np.ones(B)
            d[p + 'u_cur'] = np.zeros(B)
        else:
            name, v = next(it)
            assert name == 'rand'
            d[p + 'u_traj'] = v.astype(np.float64)
            name, v = next(it)
            assert name == 'rand'
            d[p + 'u_cur'] = v.astype(np.float64)
    return d


def main():
    utils, dsm, _ = reference_modules()
    rng = np.random.RandomState(777)
    out = {}
    import tempfile

    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, 'synth.npz')
        synthetic_npz(path, rng, n_traj=37, ob_dim=5, act_dim=3)
        raw = dict(np.load(path))
        for k, v in raw.items():
            out[f'raw_{k}'] = v
        for compact in (True, False):
            tag = 'compact' if compact else 'regular'
            d = utils.load_dataset(path, compact_dataset=compact, add_info=True)
            for k, v in d.items():
                out[f'load_{tag}_{k}'] = v
        d = utils.load_dataset(path, compact_dataset=True, add_info=False)
        for cname, cfg in CONFIGS.items():
            for oracle in (False, True):
                data = dict(d)
                if oracle:
                    data['oracle_reps'] = raw['qpos'][: len(data['observations'])].astype(np.float32)
                dataset = dsm.Dataset.create(**data)
                gc = dsm.GCDataset(dataset, dict(cfg))
                tag = f'{cname}_{"oracle" if oracle else "obs"}'
                B = 257
                np.random.seed(sum(map(ord, tag)))
                with Recorder() as rec:
                    batch = gc.sample(B)
                draws = _draws_from_log(rec.log, B, cfg)
                for k, v in draws.items():
                    out[f'gc_{tag}_draw_{k}'] = v
                for k, v in batch.items():
                    out[f'gc_{tag}_out_{k}'] = np.asarray(v)
        # explicit idxs + regular dataset (next_observations stored)
        dreg = utils.load_dataset(path, compact_dataset=False, add_info=False)
        dataset = dsm.Dataset.create(**dreg)
        gc = dsm.GCDataset(dataset, dict(CONFIGS['crl']))
        idxs = rng.randint(0, len(dreg['observations']), 64)
        np.random.seed(5)
        with Recorder() as rec:
            batch = gc.sample(64, idxs=idxs)
        log = [('randint', idxs)] + rec.log
        draws = _draws_from_log(log, 64, CONFIGS['crl'])
        out['gc_regidx_idxs'] = idxs.astype(np.int64)
        for k, v in draws.items():
            out[f'gc_regidx_draw_{k}'] = v
        for k, v in batch.items():
            out[f'gc_regidx_out_{k}'] = np.asarray(v)
        # geometric formula pin: legacy RandomState inversion
        us, gs = [], []
        for seed in range(3000):
            r = np.random.RandomState(seed)
            us.append(r.random_sample())
            r = np.random.RandomState(seed)
            gs.append(r.geometric(1 - 0.99))
        out['geom_u'] = np.array(us)
        out['geom_g'] = np.array(gs, np.int64)
    np.savez_compressed(os.path.join(OUT, 'gc_golden.npz'), **out)
    print('gc golden:', len(out), 'arrays')


HGC_CONFIGS = {
    # HIQL-style (impls/agents/hiql.py defaults; subgoal_steps shortened for short trajectories)
    'hiql': dict(discount=0.99, value_p_curgoal=0.2, value_p_trajgoal=0.5, value_p_randomgoal=0.3,
                 value_geom_sample=True, actor_p_curgoal=0.0, actor_p_trajgoal=1.0, actor_p_randomgoal=0.0,
                 actor_geom_sample=False, gc_negative=True, p_aug=0.0, frame_stack=None, subgoal_steps=10),
    # separate value/actor/low subgoal steps, low-level value goals, positive rewards
    'hlow': dict(discount=0.97, value_p_curgoal=0.3, value_p_trajgoal=0.4, value_p_randomgoal=0.3,
                 value_geom_sample=False, actor_p_curgoal=0.2, actor_p_trajgoal=0.5, actor_p_randomgoal=0.3,
                 actor_geom_sample=True, gc_negative=False, p_aug=None, frame_stack=None, subgoal_steps=6,
                 value_subgoal_steps=7, actor_subgoal_steps=4, low_subgoal_steps=3, low_discount=0.95),
    # current-state value goals (no u draws), high_subgoal_steps override
    'hcur': dict(discount=0.9, value_p_curgoal=1.0, value_p_trajgoal=0.0, value_p_randomgoal=0.0,
                 value_geom_sample=True, actor_p_curgoal=0.0, actor_p_trajgoal=0.5, actor_p_randomgoal=0.5,
                 actor_geom_sample=False, gc_negative=True, p_aug=None, frame_stack=None, subgoal_steps=5,
                 high_subgoal_steps=12, low_discount=0.9),
}


def hgc_draws_from_log(log, B, cfg):
    """Map the np.random call log of one HGCDataset.sample (datasets.py:496-643)
    to named draws: pick, v_*, [l_*], a_* (same layout as ogbx_hgc_draws)."""
    it = iter(log)
    d = {}
    name, v = next(it)
    assert name == 'randint'
    d['pick'] = v.astype(np.int64)

    def goal(p, p_cur, geom):
        name, v = next(it)
        assert name == 'randint'
        d[p + 'pick'] = v.astype(np.int64)
        name, v = next(it)
        if geom:
            assert name == 'geometric'
            d[p + 'geom'] = v.astype(np.int64)
            d[p + 'dist'] = np.zeros(B)
        else:
            assert name == 'rand'
            d[p + 'dist'] = v.astype(np.float64)
            d[p + 'geom'] = np.zeros(B, np.int64)
        if p_cur == 1.0:
            d[p + 'u_traj'] = np.ones(B)
            d[p + 'u_cur'] = np.zeros(B)
        else:
            for k in ('u_traj', 'u_cur'):
                name, v = next(it)
                assert name == 'rand'
                d[p + k] = v.astype(np.float64)

    goal('v_', cfg['value_p_curgoal'], cfg['value_geom_sample'])
    if cfg.get('low_discount') is not None:
        goal('l_', cfg['value_p_curgoal'], True)
    goal('a_', cfg['actor_p_curgoal'], cfg['actor_geom_sample'])
    return d


def main_hgc():
    utils, dsm, _ = reference_modules()
    rng = np.random.RandomState(4321)
    out = {}
    import tempfile

    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, 'synth.npz')
        synthetic_npz(path, rng, n_traj=41, ob_dim=4, act_dim=2, min_len=2, max_len=30)
        raw = dict(np.load(path))
        for k, v in raw.items():
            out[f'raw_{k}'] = v
        d = utils.load_dataset(path, compact_dataset=True, add_info=False)
        for cname, cfg in HGC_CONFIGS.items():
            for oracle in (False, True):
                data = dict(d)
                if oracle:
                    data['oracle_reps'] = raw['qpos'][: len(data['observations'])].astype(np.float32)
                hgc = dsm.HGCDataset(dsm.Dataset.create(**data), dict(cfg))
                tag = f'{cname}_{"oracle" if oracle else "obs"}'
                B = 301
                np.random.seed(sum(map(ord, tag)) + 11)
                with Recorder() as rec:
                    batch = hgc.sample(B)
                for k, v in hgc_draws_from_log(rec.log, B, cfg).items():
                    out[f'hgc_{tag}_draw_{k}'] = v
                for k, v in batch.items():
                    out[f'hgc_{tag}_out_{k}'] = np.asarray(v)
                out[f'hgc_{tag}_keys'] = np.array(list(batch.keys()))
    np.savez_compressed(os.path.join(OUT, 'hgc_golden.npz'), **out)
    print('hgc golden:', len(out), 'arrays')


class PickRecorder(Recorder):
    """Recorder whose randint calls (the sample and goal picks of
    get_random_idxs, datasets.py:65-70) return the reference's own draws with
    the first entries replaced by ``forced`` picks, logging what it returned."""

    def __init__(self, forced):
        super().__init__()
        self.forced = np.asarray(forced, np.int64)

    def __enter__(self):
        super().__enter__()
        inner = np.random.randint

        def randint(*a, **k):
            v = np.array(inner(*a, **k))
            n = min(len(self.forced), v.size)
            v[:n] = self.forced[:n]
            self.log[-1] = ('randint', v.copy())
            return v

        np.random.randint = randint
        return self


def periodic_npz(path, rng, n_traj, L, ob_dim, act_dim):
    """A raw .npz of n_traj equal trajectories of L rows (the OGBench layout:
    every episode the same length, terminals = 1 at its last row)."""
    R = n_traj * L
    term = np.zeros(R, np.float32)
    term[L - 1::L] = 1
    np.savez(path, observations=rng.normal(size=(R, ob_dim)).astype(np.float32),
             actions=rng.uniform(-1, 1, (R, act_dim)).astype(np.float32), terminals=term,
             qpos=rng.uniform(-4, 40, (R, 2)).astype(np.float32))


def main_periodic():
    """Equal-length trajectories (30 x 50 rows; after the compact load the last
    row of each is invalid: 49 picks per 50-row period, trajectory end at
    offset 48).  libogbx samples such a buffer through its closed form
    (ogbx_gc_buffer.period); these are the reference GCDataset / HGCDataset
    outputs on it, with every pick, value-goal pick and actor-goal pick forced
    to the period boundaries q*49 - 1, q*49 (and 0, npick - 1) in its first
    entries and the reference's own draws elsewhere."""
    utils, dsm, _ = reference_modules()
    rng = np.random.RandomState(2024)
    n_traj, L = 30, 50
    out = {}
    import tempfile

    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, 'periodic.npz')
        periodic_npz(path, rng, n_traj, L, ob_dim=5, act_dim=3)
        raw = dict(np.load(path))
        for k, v in raw.items():
            out[f'raw_{k}'] = v
        d = utils.load_dataset(path, compact_dataset=True, add_info=False)
        npick = int((d['valids'] > 0).sum())
        assert npick == n_traj * (L - 1)
        q = np.arange(1, n_traj)
        forced = np.concatenate([[0, npick - 1], q * (L - 1) - 1, q * (L - 1), q * (L - 1) + 1])
        out['forced_picks'] = forced
        B = 256
        for cname, cfg in CONFIGS.items():
            gc = dsm.GCDataset(dsm.Dataset.create(**d), dict(cfg))
            tag = f'gc_{cname}'
            np.random.seed(sum(map(ord, tag)) + 3)
            with PickRecorder(forced) as rec:
                batch = gc.sample(B)
            for k, v in _draws_from_log(rec.log, B, cfg).items():
                out[f'{tag}_draw_{k}'] = v
            for k, v in batch.items():
                out[f'{tag}_out_{k}'] = np.asarray(v)
        for cname, cfg in HGC_CONFIGS.items():
            hgc = dsm.HGCDataset(dsm.Dataset.create(**d), dict(cfg))
            tag = f'hgc_{cname}'
            np.random.seed(sum(map(ord, tag)) + 5)
            with PickRecorder(forced) as rec:
                batch = hgc.sample(B)
            for k, v in hgc_draws_from_log(rec.log, B, cfg).items():
                out[f'{tag}_draw_{k}'] = v
            for k, v in batch.items():
                out[f'{tag}_out_{k}'] = np.asarray(v)
            out[f'{tag}_keys'] = np.array(list(batch.keys()))
    np.savez_compressed(os.path.join(OUT, 'gc_periodic_golden.npz'), **out)
    print('gc periodic golden:', len(out), 'arrays')


def main_relabel():
    """relabel_dataset / add_oracle_reps (maze branch) of the reference
    ogbench/relabel_utils.py with a stand-in env (the attributes they read)."""
    _, _, relabel = reference_modules()
    rng = np.random.RandomState(99)
    out = {}

    class _Unwrapped:
        _reward_task_id = 2
        _goal_tol = 1.0

    class _Env:
        unwrapped = _Unwrapped()

        def reset(self):
            return None

    for qdt in ('f32', 'f64'):
        n = 5000
        goal = np.array([28.0, 16.0])
        q = np.concatenate([rng.uniform(-4, 40, (n, 2)), rng.normal(size=(n, 13))], 1)
        # exact-boundary rows: distance exactly 1.0 and one ulp around it
        q[:4, 0] = goal[0] + np.array([1.0, np.nextafter(1.0, 2), np.nextafter(1.0, 0), 0.6])
        q[:4, 1] = goal[1] + np.array([0.0, 0.0, 0.0, 0.8])
        q[4:200, :2] = goal + rng.uniform(-1.2, 1.2, (196, 2))
        q = q.astype(np.float32 if qdt == 'f32' else np.float64)
        env = _Env()
        env.unwrapped.cur_goal_xy = goal
        ds = dict(qpos=q.copy())
        relabel.relabel_dataset('pointmaze-large-singletask-task2-v0', env, ds)
        relabel.add_oracle_reps('pointmaze-large-oraclerep-v0', env, ds)
        out[f'{qdt}_qpos'] = q
        out[f'{qdt}_goal'] = goal
        for k in ('rewards', 'masks', 'oracle_reps'):
            out[f'{qdt}_{k}'] = ds[k]
    np.savez_compressed(os.path.join(OUT, 'relabel_golden.npz'), **out)
    print('relabel golden:', len(out), 'arrays')


NAME_CASES = [
    'pointmaze-large-navigate-v0', 'pointmaze-medium-stitch-v0', 'antmaze-giant-explore-v0',
    'humanoidmaze-large-navigate-v0', 'pointmaze-large-navigate-singletask-v0',
    'pointmaze-large-navigate-singletask-task2-v0', 'antmaze-teleport-stitch-singletask-task5-v0',
    'pointmaze-large-navigate-oraclerep-v0', 'antmaze-medium-navigate-oraclerep-v0', 'powderworld-easy-play-v0',
    'visual-antmaze-large-navigate-v0',
]


def main_names():
    """make_env_and_datasets' name grammar (utils.py:160-182), recorded from the
    reference with gymnasium.make and download_datasets replaced by recorders."""
    import json

    utils, _, _ = reference_modules()
    rec = {}

    def fake_make(name, **kw):
        rec['env_name'], rec['env_kwargs'] = name, kw
        return object()

    class _Stop(Exception):
        pass

    def fake_download(names, dataset_dir=None):
        rec['file_name'] = names[0]
        raise _Stop()

    utils.gymnasium.make = fake_make
    utils.download_datasets = fake_download
    out = []
    for name in NAME_CASES:
        rec.clear()
        try:
            utils.make_env_and_datasets(name, dataset_dir='/nonexistent')
        except _Stop:
            pass
        out.append(dict(dataset_name=name, env_name=rec['env_name'], env_kwargs=rec['env_kwargs'],
                        file_name=rec['file_name']))
    with open(os.path.join(OUT, 'names_golden.json'), 'w') as f:
        json.dump(out, f, indent=1)
    print('names golden:', len(out))


if __name__ == '__main__':
    main()
    main_hgc()
    main_periodic()
    main_relabel()
    main_names()
