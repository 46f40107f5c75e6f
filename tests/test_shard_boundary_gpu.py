"""GPU: shard boundaries that are NOT multiples of 64 reproduce the single run
through maze_step_kernel (include/ogbx.h env_base contract).

Three handles at env_base 0 / 1,000 / 2,731 split a 4,096-env pointmaze-large
job so that wavefronts straddle every boundary differently from the single
run.  Near-wall states (many contact steps, lean-loop bails), staggered episode
clocks (TimeLimit ends at every step) and auto-reset (Philox reset noise keyed
by the global env index) run through env.step, env.rollout (K fused steps) and
env.rollout_until_done; every per-env output must be bit-identical to the one
4,096-env handle.  A permuted multi-step run pins per-env independence of the
wavefront composition over many steps (not just one physics call).
"""

import numpy as np
import pytest
import torch

import ogbench_amd
from oracle import locomaze as orc

pytestmark = pytest.mark.gpu
TOTAL = 4096
BOUNDS = (0, 1000, 2731, TOTAL)
SEED = 0x5EED


def _env(gpu, base, n, **kw):
    return ogbench_amd.MazeEnv('point', 'large', num_envs=n, device=gpu, env_base=base, **kw)


def _near_wall_state(env, rng, stagger):
    """Reset env state replaced by near-wall positions (offsets up to 1.9 from
    the cell centre) and staggered elapsed counters."""
    mp, _ = orc.tables('large')
    cells = np.argwhere(mp == 0)
    c = cells[rng.randint(len(cells), size=TOTAL)]
    q = np.stack([c[:, 1] * 4.0 - 4 + rng.uniform(-1.9, 1.9, TOTAL),
                  c[:, 0] * 4.0 - 4 + rng.uniform(-1.9, 1.9, TOTAL)], 1)
    sd = env.state_dict()
    sd['qpos'] = torch.tensor(q, device=env.device)
    sd['elapsed'] = torch.tensor(np.arange(TOTAL) % stagger, dtype=torch.int32, device=env.device)
    return sd


def _split(sd, b, e):
    return {k: (v[b:e].clone() if isinstance(v, torch.Tensor) else v) for k, v in sd.items()}


def _setup(gpu, **kw):
    single = _env(gpu, 0, TOTAL, **kw)
    shards = [_env(gpu, b, e - b, **kw) for b, e in zip(BOUNDS[:-1], BOUNDS[1:])]
    task = torch.arange(TOTAL, dtype=torch.int32) % 5 + 1
    single.reset(seed=SEED, options=dict(task_id=task))
    for s, b, e in zip(shards, BOUNDS[:-1], BOUNDS[1:]):
        s.reset(seed=SEED, options=dict(task_id=task[b:e]))
    return single, shards


def _contact_fraction(env, sd, a):
    _, contact = env.physics(sd['qpos'], a)
    return float(contact.float().mean())


def test_step_with_auto_reset_any_boundary(gpu):
    single, shards = _setup(gpu, auto_reset=True, max_episode_steps=40)
    rng = np.random.RandomState(7)
    sd = _near_wall_state(single, rng, 40)
    single.load_state_dict(sd)
    for s, b, e in zip(shards, BOUNDS[:-1], BOUNDS[1:]):
        s.load_state_dict(_split(sd, b, e))
    acts = torch.tensor(rng.uniform(-1, 1, (60, TOTAL, 2)).astype(np.float32))
    assert _contact_fraction(single, sd, acts[0]) > 0.2
    ends = 0
    for t in range(60):
        o, r, te, tr, info = single.step(acts[t])
        ref = [x.cpu().numpy().copy() for x in (o, r, te, tr, info['success'])]
        done = ref[2] | ref[3]
        ref_final = info['final_observation'].cpu().numpy()[done]
        ends += int(done.sum())
        for s, b, e in zip(shards, BOUNDS[:-1], BOUNDS[1:]):
            o, r, te, tr, info = s.step(acts[t, b:e])
            got = [x.cpu().numpy() for x in (o, r, te, tr, info['success'])]
            for name, g, x in zip(('obs', 'reward', 'terminated', 'truncated', 'success'), got, ref):
                assert np.array_equal(g, x[b:e]), (t, b, name)
            d = done[b:e]
            assert np.array_equal(info['final_observation'].cpu().numpy()[d], ref_final[done[:b].sum():][:d.sum()])
    assert ends > TOTAL  # every env ended (TimeLimit) at least once: auto-reset ran everywhere
    for s, b, e in zip(shards, BOUNDS[:-1], BOUNDS[1:]):
        assert torch.equal(s.get_xy(), single.get_xy()[b:e])


def test_rollout_and_rollout_until_done_any_boundary(gpu):
    rng = np.random.RandomState(8)
    # K fused steps with auto-reset
    single, shards = _setup(gpu, auto_reset=True, max_episode_steps=25)
    sd = _near_wall_state(single, rng, 25)
    single.load_state_dict(sd)
    for s, b, e in zip(shards, BOUNDS[:-1], BOUNDS[1:]):
        s.load_state_dict(_split(sd, b, e))
    acts = torch.tensor(rng.uniform(-1, 1, (48, TOTAL, 2)).astype(np.float32))
    ref = {k: v.cpu().numpy() for k, v in single.rollout(acts).items()}
    assert ref['truncated'].sum() > TOTAL
    for s, b, e in zip(shards, BOUNDS[:-1], BOUNDS[1:]):
        got = s.rollout(acts[:, b:e])
        for k, v in got.items():
            assert np.array_equal(v.cpu().numpy(), ref[k][:, b:e]), (b, k)
    # evaluation episodes (no auto-reset, per-env stop, wave-ballot exit)
    single, shards = _setup(gpu, auto_reset=False, max_episode_steps=30)
    sd = _near_wall_state(single, rng, 30)
    single.load_state_dict(sd)
    for s, b, e in zip(shards, BOUNDS[:-1], BOUNDS[1:]):
        s.load_state_dict(_split(sd, b, e))
    acts = torch.tensor(rng.uniform(-1, 1, (40, TOTAL, 2)).astype(np.float32))
    ref = {k: v.cpu().numpy() for k, v in single.rollout_until_done(acts).items()}
    assert len(np.unique(ref['steps'])) > 20
    for s, b, e in zip(shards, BOUNDS[:-1], BOUNDS[1:]):
        got = s.rollout_until_done(acts[:, b:e])
        for k, v in got.items():
            x = ref[k][b:e] if k == 'steps' else ref[k][:, b:e]
            assert np.array_equal(v.cpu().numpy(), x), (b, k)
        assert torch.equal(s.get_xy(), single.get_xy()[b:e])


def test_permuted_multistep_rollout(gpu):
    """60 steps of near-wall envs (no auto-reset: no Philox draw depends on
    the env index) in order and permuted: every row identical."""
    rng = np.random.RandomState(9)
    a_env, p_env = _env(gpu, 0, TOTAL, max_episode_steps=1000), _env(gpu, 0, TOTAL, max_episode_steps=1000)
    a_env.reset(seed=SEED, options=dict(task_id=3))
    p_env.reset(seed=SEED, options=dict(task_id=3))
    sd = _near_wall_state(a_env, rng, 1)
    perm = torch.tensor(rng.permutation(TOTAL))
    a_env.load_state_dict(sd)
    p_env.load_state_dict({k: (v[perm.to(v.device)] if isinstance(v, torch.Tensor) else v) for k, v in sd.items()})
    acts = torch.tensor(rng.uniform(-1, 1, (60, TOTAL, 2)).astype(np.float32))
    ref = a_env.rollout(acts)
    got = p_env.rollout(acts[:, perm])
    pd = perm.to(gpu)
    for k in ref:
        assert torch.equal(got[k], ref[k][:, pd]), k
    assert torch.equal(p_env.get_xy(), a_env.get_xy()[pd])
