"""GPU parity: the medium/hard powderworld kernels (every PWSim rule, through
the C-ABI) vs the reference's own outputs (tests/golden/powder_full_golden.npz,
rand fields recorded and injected) and the NumPy oracle
(oracle/powder_full_np.py) on seeded inputs.  Float32 velocities included, the
bar is bit-exact: the kernels follow the reference op by op."""

import os

import numpy as np
import pytest
import torch

import ogbench_amd
from ogbench_amd import _lib
from oracle import powder_full_np as orc

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), 'golden', 'powder_full_golden.npz')


@pytest.fixture(scope='module')
def gold():
    return dict(np.load(GOLD))


def _env(gpu, n, ne=5, size=32, **kw):
    name = {5: 'powderworld-medium-v0', 8: 'powderworld-hard-v0'}[ne]
    return ogbench_amd.make(name, num_envs=n, device=gpu, world_size=size, **kw)


def _diff(a, b):
    a, b = np.asarray(a), np.asarray(b)
    bad = np.argwhere(a != b)
    return f'{len(bad)} mismatches, first {bad[:5].tolist()}'


@pytest.mark.parametrize('size', [32, 64])
def test_forward_matches_reference(gpu, gold, size):
    env = _env(gpu, 1, size=size)
    w0, outs, rands = gold[f'full{size}_in'], gold[f'full{size}_out'], gold[f'full{size}_rand']
    # one forward at a time from the reference's own inputs
    w = w0
    for t in range(outs.shape[0]):
        got = env.forward_full(w, 1, rand=rands[t][None]).cpu().numpy()
        assert np.array_equal(got, outs[t]), (t, _diff(got, outs[t]))
        w = outs[t]
    # all six chained in one launch
    got = env.forward_full(w0, outs.shape[0], rand=rands).cpu().numpy()
    assert np.array_equal(got, outs[-1]), _diff(got, outs[-1])


def test_render_with_velocity(gpu, gold):
    env = _env(gpu, 1)
    out, img = env.forward_full(gold['render_vel_world'], 0, render=True)
    assert np.array_equal(out.cpu().numpy(), gold['render_vel_world'])
    got = img.cpu().numpy()[0]
    assert np.array_equal(got, gold['render_vel_img']), _diff(got, gold['render_vel_img'])


def _seeded_world(rng, n, size, ne):
    """Random full worlds: elements of the set, walls on the border, random
    velocities and momenta (the states a trajectory reaches)."""
    elems = orc.ELEM_IDS[ne] + [0, 0, 0]
    ids = rng.choice(elems, size=(n, size, size))
    ids[:, 0, :] = ids[:, -1, :] = ids[:, :, 0] = ids[:, :, -1] = orc.WALL
    w = orc.from_ids(ids)
    w[:, 3:5] = (rng.randn(n, 2, size, size) * 2.5).astype(np.float32) * (rng.rand(n, 1, size, size) < 0.3)
    w[:, 6] = rng.choice([-2, 0, 2], size=(n, size, size)) * np.isin(ids, orc.FLUIDS)
    w[:, 8] = rng.rand(n, size, size) < 0.2
    stone = ids == orc.STONE
    w[:, 2] = np.where(stone, rng.rand(n, size, size) < 0.5, w[:, 2])
    return w.astype(np.float32)


@pytest.mark.parametrize('ne,size', [(5, 32), (8, 32), (8, 64)])
def test_forward_matches_oracle_seeded(gpu, ne, size):
    rng = np.random.RandomState(100 + ne + size)
    n, steps = 3, 8
    w = _seeded_world(rng, n, size, ne)
    rand = rng.rand(steps, n, 3, size, size).astype(np.float32)
    env = _env(gpu, 1, ne=ne, size=size)
    got = env.forward_full(w, steps, rand=rand).cpu().numpy()
    ref = w
    for t in range(steps):
        ref = orc.forward(ref, [rand[t][:, k] for k in range(3)])
    assert np.array_equal(got, ref), _diff(got, ref)


@pytest.mark.parametrize('walls', [True, False])
def test_forward_sparse_rows_matches_oracle(gpu, walls):
    """64x64 worlds where fire / lava sit in a few rows only, so the fire
    rule's per-row skipping (rows with no hot cell within one row, and rows
    with no burn flag within one row, periodic) is exercised next to the rows
    it runs on; without border walls, hot cells at rows 0 / 63 reach across
    the periodic boundary (impulses use np.roll).  Bit-exact vs the oracle."""
    rng = np.random.RandomState(7 if walls else 8)
    n, size, steps = 3, 64, 8
    ids = np.zeros((n, size, size), np.int64)
    burn = [orc.WOOD, orc.PLANT, orc.GAS, orc.DUST, orc.SAND, orc.WATER, orc.ICE, orc.STONE]
    for e in range(n):
        rows = rng.choice(np.arange(size), size=10, replace=False)
        for r in rows:  # sparse rows of burnables and others
            cols = rng.rand(size) < 0.5
            ids[e, r, cols] = rng.choice(burn, size=int(cols.sum()))
        hot = [1, 2, 62] if walls else [1, 31]
        for r in hot + [int(rows[0])]:
            cols = rng.rand(size) < 0.3
            ids[e, r, cols] = rng.choice([orc.FIRE, orc.LAVA, orc.DUST, orc.WOOD], size=int(cols.sum()))
        if not walls:  # dust at row 0 burns next to row 1's fire and pushes row 63 (periodic)
            ids[e, 0, :] = orc.DUST
            ids[e, 1, ::2] = orc.FIRE
    if walls:
        ids[:, 0, :] = ids[:, -1, :] = ids[:, :, 0] = ids[:, :, -1] = orc.WALL
    w = orc.from_ids(ids)
    w[:, 3:5] = (rng.randn(n, 2, size, size) * 2.5).astype(np.float32) * (rng.rand(n, 1, size, size) < 0.05)
    w = w.astype(np.float32)
    rand = rng.rand(steps, n, 3, size, size).astype(np.float32)
    env = _env(gpu, 1, ne=8, size=size)
    got = env.forward_full(w, steps, rand=rand).cpu().numpy()
    ref = w
    for t in range(steps):
        ref = orc.forward(ref, [rand[t][:, k] for k in range(3)])
    assert np.array_equal(got, ref), _diff(got, ref)
    one = env.forward_full(w, 1, rand=rand[:1]).cpu().numpy()
    assert np.array_equal(one, orc.forward(w, [rand[0][:, k] for k in range(3)]))


def _padded_reset_rand(env, r, task):
    """[1, R, 3, H, W]: goal rows then the reset forward at row len(task)."""
    H = env._world_size
    rows = env._max_seq + 1
    out = np.zeros((1, rows, 3, H, H), np.float32)
    out[0, :r.shape[0]] = r
    assert r.shape[0] == len(env.task_infos[task - 1]['action_seq']) + 1
    return out


@pytest.mark.parametrize('ne', [5, 8])
def test_env_trace_matches_reference(gpu, gold, ne):
    tag = f'env{ne}_tr0'
    task = int(gold[f'{tag}_task'])
    env = _env(gpu, 1, ne=ne)
    ob, info = env.reset(seed=0, options=dict(task_id=task, reset_action=gold[f'{tag}_reset_action'][None],
                                              rand=_padded_reset_rand(env, gold[f'{tag}_reset_rand'], task)))
    assert np.array_equal(env.goal_ids()[0].cpu().numpy(), gold[f'{tag}_goal_world'])
    assert np.array_equal(info['goal'][0].cpu().numpy(), gold[f'{tag}_goal_ob'])
    assert np.array_equal(ob[0].cpu().numpy(), gold[f'{tag}_reset_ob'])
    acts, rands = gold[f'{tag}_actions'], gold[f'{tag}_step_rand']
    for t in range(len(acts)):
        ob, rew, term, trunc, info = env.step([int(acts[t])], rand=rands[t][None])
        assert np.array_equal(ob[0].cpu().numpy(), gold[f'{tag}_obs'][t]), (t, _diff(ob[0].cpu(), gold[f'{tag}_obs'][t]))
        assert float(rew[0]) == gold[f'{tag}_reward'][t]
    fw = env.world_full()[0].cpu().numpy()
    assert np.array_equal(fw, gold[f'{tag}_final_world']), _diff(fw, gold[f'{tag}_final_world'])


def test_env_fused_rollout_matches_steps(gpu, gold):
    """K steps in one launch == K single-step launches (injected rands)."""
    tag = 'env5_tr0'
    task = int(gold[f'{tag}_task'])
    acts, rands = gold[f'{tag}_actions'], gold[f'{tag}_step_rand']
    opts = dict(task_id=task, reset_action=gold[f'{tag}_reset_action'][None])
    a = _env(gpu, 1)
    a.reset(seed=0, options=dict(opts, rand=_padded_reset_rand(a, gold[f'{tag}_reset_rand'], task)))
    out = a.rollout(acts[:, None], rand=rands[:, None])
    assert np.array_equal(out['obs'][:, 0].cpu().numpy(), gold[f'{tag}_obs'])
    assert np.array_equal(a.world_full()[0].cpu().numpy(), gold[f'{tag}_final_world'])


def _host_errors(world, goal):
    match = np.zeros(goal.shape, bool)
    for dx, dy in [(0, 0), (1, 0), (-1, 0), (0, 1), (0, -1)]:
        match |= goal == np.roll(world, (dy, dx), axis=(0, 1))
    return int((~match).sum())


@pytest.mark.parametrize('ne,size', [(5, 32), (8, 64)])
def test_philox_batch_consistency(gpu, ne, size):
    """Philox-driven batch: every env's step is the oracle forward of its
    previous state under SOME rand field -> check what is rand-independent:
    determinism per seed, state restore, success == goal-match < tol, obs ==
    oracle render of the state, goals differ across envs (stochastic replay)."""
    n, K = 16, 24
    env = _env(gpu, n, ne=ne, size=size)
    tasks = torch.arange(n, device=gpu) % env.num_tasks + 1
    env.reset(seed=7, options=dict(task_id=tasks))
    goals = env.goal_ids().cpu().numpy()
    assert len({g.tobytes() for g in goals}) > env.num_tasks  # per-env stochastic goals
    sd = env.state_dict()
    rng = np.random.RandomState(3)
    acts = rng.randint(0, max(ne, env._xy_action_size) + 2, size=(K, n))  # some invalid -> Philox draws
    outs = []
    for t in range(K):
        ob, rew, term, trunc, info = env.step(acts[t])
        w = env.world_full().cpu().numpy()
        tids = env.cur_task_ids.cpu().numpy()
        for e in range(n):
            ref = orc.render(w[e])
            assert np.array_equal(ob[e, ..., :3].cpu().numpy(), ref)
            err = _host_errors(w[e, 0].astype(np.uint8), goals[e])
            assert bool(info['success'][e]) == (err < env.task_infos[tids[e] - 1]['tol'])
        outs.append(ob.clone())
    # same seed + restored state -> identical trajectory
    env.load_state_dict(sd)
    for t in range(K):
        ob, *_ = env.step(acts[t])
        assert torch.equal(ob, outs[t])


def test_auto_reset_replays_goal(gpu):
    """max_episode_steps truncation with auto_reset: the next episode has a
    fresh goal replay (new Philox stream) and a fresh world."""
    env = _env(gpu, 8, max_episode_steps=6, auto_reset=True)
    env.reset(seed=11, options=dict(task_id=2))
    g0 = env.goal_ids().clone()
    for t in range(6):
        ob, rew, term, trunc, info = env.step(np.full(8, t % 3, np.int64))
    assert bool(trunc.all())
    g1 = env.goal_ids()
    assert not torch.equal(g0, g1)  # replayed with new randomness
    assert int(env._state_views()[2].max()) == 0  # elapsed reset
    # goal of task 2 (water fill + plant square) still looks like it
    assert ((g1 == orc.PLANT).sum(dim=(1, 2)) > 20).all()


def test_full_errors(gpu):
    env = _env(gpu, 2)
    with pytest.raises(ValueError):
        env.goal_worlds()
    with pytest.raises(ValueError):
        env.forward(np.zeros((1, 32, 32), np.uint8))
    easy = ogbench_amd.make('powderworld-easy-v0', num_envs=1, device=gpu)
    with pytest.raises(ValueError):
        easy.step([0], rand=np.zeros((1, 3, 32, 32), np.float32))


@pytest.mark.parametrize('ne,size', [(8, 32), (5, 64)])
def test_fused_rollout_with_auto_reset_matches_single_steps(gpu, ne, size):
    """Philox mode, auto-reset inside the launch: K steps fused in one launch ==
    K single-step launches from the same state (outputs and final state)."""
    n, K = 6, 40
    a = _env(gpu, n, ne=ne, size=size, max_episode_steps=9, auto_reset=True)
    b = _env(gpu, n, ne=ne, size=size, max_episode_steps=9, auto_reset=True)
    opts = dict(task_id=torch.arange(n, device=gpu) % 5 + 1)
    a.reset(seed=5, options=opts)
    b.reset(seed=5, options=opts)
    rng = np.random.RandomState(4)
    acts = rng.randint(0, max(ne, a._xy_action_size) + 1, size=(K, n))
    out = a.rollout(acts)
    for t in range(K):
        ob, rew, term, trunc, info = b.step(acts[t])
        assert torch.equal(out['obs'][t], ob), t
        assert torch.equal(out['reward'][t], rew), t
        assert torch.equal(out['truncated'][t].bool(), trunc), t
    sa, sb = a.state_dict(), b.state_dict()
    for k in ('world', 'ctrl', 'elapsed', 'episode', 'momentum', 'velocity', 'goal'):
        assert torch.equal(sa[k], sb[k]), k
    assert int(out['truncated'].sum()) >= n * 4  # several auto-resets happened in the launch


def test_masked_reset_leaves_other_envs(gpu):
    env = _env(gpu, 4)
    env.reset(seed=3, options=dict(task_id=2))
    for t in range(6):
        env.step(np.full(4, t % 3))
    before = env.state_dict()
    mask = torch.tensor([1, 0, 1, 0], dtype=torch.uint8, device=gpu)
    env.reset(options=dict(task_id=4), mask=mask)
    after = env.state_dict()
    for k in ('world', 'momentum', 'velocity', 'goal'):
        assert torch.equal(after[k][1], before[k][1]) and torch.equal(after[k][3], before[k][3]), k
        assert not torch.equal(after[k][0], before[k][0]) or k in ('momentum', 'velocity'), k
    assert env.cur_task_ids.tolist() == [4, 2, 4, 2]
    assert (env._state_views()[2][[0, 2]] == 0).all()


def test_forward_rand_threshold_edges(gpu):
    """Rand values at and one ulp around every threshold the rules compare
    against (sand 0.5; fluid (rm + ch6) + mom > 0.5 with its float32 rounding;
    ice/plant/fire/water thresholds): the kernel's exact reduction of the three
    fields to decision bits must agree with the reference's float32 arithmetic."""
    rng = np.random.RandomState(77)
    f32 = np.float32
    edges = []
    for t in (0.5, 0.02, 0.05, 0.2, 0.3, 0.4):
        t = f32(t)
        edges += [np.nextafter(t, f32(0)), t, np.nextafter(t, f32(1))]
    edges += [f32(0.5) + f32(2 ** -24), f32(0.5) - f32(2 ** -25), f32(0.0), np.nextafter(f32(1), f32(0))]
    edges = np.array(edges, np.float32)
    n, size, steps = 4, 32, 6
    w = _seeded_world(rng, n, size, 8)
    rand = edges[rng.randint(0, len(edges), size=(steps, n, 3, size, size))]
    env = _env(gpu, 1, ne=8, size=size)
    got = env.forward_full(w, steps, rand=rand).cpu().numpy()
    ref = w
    for t in range(steps):
        ref = orc.forward(ref, [rand[t][:, k] for k in range(3)])
    assert np.array_equal(got, ref), _diff(got, ref)


@pytest.mark.parametrize('ne,size', [(5, 64), (8, 32)])
def test_mixed_stages_single_steps_match_fused(gpu, ne, size):
    """Envs at different stages of the action machine in one launch: a single
    step splits them between the render-only kernel (stage 0/1, no reset) and
    the full-rule kernel; the fused rollout keeps all in one kernel.  Both from
    the same state must agree bit for bit (outputs and final state)."""
    n, K = 9, 15
    a = _env(gpu, n, ne=ne, size=size, max_episode_steps=7, auto_reset=True)
    a.reset(seed=21, options=dict(task_id=torch.arange(n, device=gpu) % 5 + 1))
    rng = np.random.RandomState(9)
    hi = max(ne, a._xy_action_size) + 1
    for t in range(2):
        a.step(rng.randint(0, hi, size=n))
    # re-reset a third of the envs: stages 0 / 1 / 2 now coexist
    a.reset(options=dict(task_id=3), mask=torch.tensor([i % 3 == 0 for i in range(n)], dtype=torch.uint8,
                                                         device=gpu))
    stages = (a.state_dict()['ctrl'] & 3).tolist()
    assert len(set(stages)) >= 2, stages
    b = _env(gpu, n, ne=ne, size=size, max_episode_steps=7, auto_reset=True)
    b.reset(seed=21, options=dict(task_id=1))
    b.load_state_dict(a.state_dict())
    acts = rng.randint(0, hi, size=(K, n))
    out = b.rollout(acts)
    for t in range(K):
        ob, rew, term, trunc, info = a.step(acts[t])
        assert torch.equal(out['obs'][t], ob), t
        assert torch.equal(out['reward'][t], rew), t
        assert torch.equal(out['truncated'][t].bool(), trunc), t
        assert torch.equal(out['success'][t].bool(), info['success']), t
    sa, sb = a.state_dict(), b.state_dict()
    for k in ('world', 'ctrl', 'elapsed', 'episode', 'momentum', 'velocity', 'goal'):
        assert torch.equal(sa[k], sb[k]), k


@pytest.mark.parametrize('ne,size', [(5, 64), (8, 32)])
def test_render_cache_paths_agree(gpu, ne, size):
    """Render-only steps take their colours from the env's render cache; a step
    after the world / velocity pointers were handed out (world_full,
    state_dict, load_state_dict) renders from the state and rewrites the cache.
    Both paths, and a cache made stale by load_state_dict, give the same
    observations bit for bit."""
    n, K, T = 8, 30, 13
    a, b, c = (_env(gpu, n, ne=ne, size=size, max_episode_steps=11, auto_reset=True) for _ in range(3))
    opts = dict(task_id=torch.arange(n, device=gpu) % 5 + 1)
    a.reset(seed=2, options=opts)
    b.reset(seed=2, options=opts)
    c.reset(seed=99, options=dict(task_id=1))
    rng = np.random.RandomState(5)
    acts = rng.randint(0, max(ne, a._xy_action_size) + 1, size=(K, n))
    for t in range(K):
        oa, ra, *_ = a.step(acts[t])  # cache path on render-only steps
        b._state_views()  # a writable hand-out: b renders every step from the state
        ob, rb, *_ = b.step(acts[t])
        assert torch.equal(oa, ob) and torch.equal(ra, rb), t
        if t > T:
            oc, *_ = c.step(acts[t])
            assert torch.equal(oa, oc), t
        if t == T:
            assert bool(((a._scalar_view("ctrl") & 3) != 2).any())  # the next step has render-only envs
            c.load_state_dict(a.state_dict())  # c's cache still holds its own worlds' colours
    for k in ('world', 'momentum', 'velocity'):
        assert torch.equal(a.state_dict()[k], c.state_dict()[k]), k


def test_kept_pointer_write_and_read_only_views(gpu):
    """a host that keeps the writable world pointer and writes
    through it after later steps announces the write with
    ogbx_powder_state_written; readers use the const view
    (ogbx_powder_state_view), which keeps the render cache.  The env written
    through its kept pointer steps bit-identically to one restored with
    load_state_dict, and world_ids / world_full read every step leave the
    observations unchanged."""
    n, K, T = 8, 24, 11
    a, c, d = (_env(gpu, n, ne=5, size=64, max_episode_steps=50, auto_reset=True) for _ in range(3))
    opts = dict(task_id=torch.arange(n, device=gpu) % 5 + 1)
    a.reset(seed=3, options=opts)
    c.reset(seed=3, options=opts)
    d.reset(seed=77, options=dict(task_id=2))
    w_keep = a._state_views()[0]  # writable, kept across steps
    m_keep, v_keep, _ = a._full_views()
    rng = np.random.RandomState(8)
    acts = rng.randint(0, max(5, a._xy_action_size) + 1, size=(K, n))
    for t in range(K):
        ids_before = a.world_ids().clone()
        full_before = a.world_full()
        oa, ra, *_ = a.step(acts[t])
        oc, rc, *_ = c.step(acts[t])
        assert torch.equal(oa, oc) and torch.equal(ra, rc), t
        assert torch.equal(ids_before, (full_before[:, 0]).to(torch.uint8)), t
        if t == T:
            assert bool(((a._scalar_view("ctrl") & 3) != 2).any())  # the next step has render-only envs
            other = d.state_dict()
            sd = a.state_dict()
            sd.update(world=other['world'], momentum=other['momentum'], velocity=other['velocity'])
            c.load_state_dict(sd)
            w_keep.copy_(other['world'])  # through the pointers a handed out before the steps
            m_keep.copy_(other['momentum'])
            v_keep.copy_(other['velocity'])
            _lib.check(_lib.lib().ogbx_powder_state_written(a._h))
    for k in ('world', 'momentum', 'velocity'):
        assert torch.equal(a.state_dict()[k], c.state_dict()[k]), k


@pytest.mark.parametrize('ne,size', [(5, 64), (8, 32)])
def test_out_of_phase_envs_after_full_reset_match_fused(gpu, ne, size):
    """A mixed-stage state loaded after an all-env reset: load_state_dict drops
    the host's phase guess (ogbx_powder_env::phase), so every step launches the
    light kernel and the one-env full kernel; the steps must match the fused
    rollout from the same state bit for bit (a wrong guess:
    test_wrong_phase_hint_matches_fused)."""
    n, K = 9, 16
    src = _env(gpu, n, ne=ne, size=size, max_episode_steps=7, auto_reset=True)
    src.reset(seed=4, options=dict(task_id=torch.arange(n, device=gpu) % 5 + 1))
    rng = np.random.RandomState(12)
    hi = max(ne, src._xy_action_size) + 1
    src.step(rng.randint(0, hi, size=n))
    src.reset(options=dict(task_id=2), mask=torch.tensor([i % 3 == 1 for i in range(n)], dtype=torch.uint8,
                                                           device=gpu))
    src.step(rng.randint(0, hi, size=n))
    sd = src.state_dict()
    assert len(set((sd['ctrl'] & 3).tolist())) >= 2
    a = _env(gpu, n, ne=ne, size=size, max_episode_steps=7, auto_reset=True)
    b = _env(gpu, n, ne=ne, size=size, max_episode_steps=7, auto_reset=True)
    a.reset(seed=4, options=dict(task_id=1))  # all-env reset: phase 0 on the host
    a.load_state_dict(sd)                       # ... but the envs are not in that phase
    b.reset(seed=4, options=dict(task_id=1))
    b.load_state_dict(sd)
    acts = rng.randint(0, hi, size=(K, n))
    out = b.rollout(acts)
    for t in range(K):
        ob, rew, term, trunc, info = a.step(acts[t])
        assert torch.equal(out['obs'][t], ob), t
        assert torch.equal(out['reward'][t], rew), t
        assert torch.equal(out['truncated'][t].bool(), trunc), t
    sa, sb = a.state_dict(), b.state_dict()
    for k in ('world', 'ctrl', 'elapsed', 'episode', 'momentum', 'velocity', 'goal'):
        assert torch.equal(sa[k], sb[k]), k


@pytest.mark.parametrize('ne,size,phase', [(5, 64, 0), (5, 64, 1), (8, 32, 2), (8, 64, 5)])
def test_wrong_phase_hint_matches_fused(gpu, ne, size, phase):
    """A wrong phase hint (set_step_phase on a mixed-stage state) makes the host
    pick the wrong launch plan on most steps: no light kernel on a step where
    some envs are render-only (the dense full kernel steps them), and the
    sparse full kernel (8 envs per workgroup, pwf_step_kernel<WS, true>) on
    render-only steps where some envs need a forward or an auto-reset.  Both
    must step bit-for-bit as the fused rollout from the same state."""
    n, K = 19, 18
    src = _env(gpu, n, ne=ne, size=size, max_episode_steps=7, auto_reset=True)
    src.reset(seed=6, options=dict(task_id=torch.arange(n, device=gpu) % 5 + 1))
    rng = np.random.RandomState(30 + phase)
    hi = max(ne, src._xy_action_size) + 1
    src.step(rng.randint(0, hi, size=n))
    src.reset(options=dict(task_id=3), mask=torch.tensor([i % 3 != 0 for i in range(n)], dtype=torch.uint8,
                                                           device=gpu))
    src.step(rng.randint(0, hi, size=n))
    src.reset(options=dict(task_id=4), mask=torch.tensor([i % 4 == 1 for i in range(n)], dtype=torch.uint8,
                                                           device=gpu))
    sd = src.state_dict()
    assert len(set((sd['ctrl'] & 3).tolist())) == 3
    a = _env(gpu, n, ne=ne, size=size, max_episode_steps=7, auto_reset=True)
    b = _env(gpu, n, ne=ne, size=size, max_episode_steps=7, auto_reset=True)
    for x in (a, b):
        x.reset(seed=6, options=dict(task_id=1))
        x.load_state_dict(sd)
    a.set_step_phase(phase)
    acts = rng.randint(0, hi, size=(K, n))
    out = b.rollout(acts)
    for t in range(K):
        ob, rew, term, trunc, info = a.step(acts[t])
        assert torch.equal(out['obs'][t], ob), t
        assert torch.equal(out['reward'][t], rew), t
        assert torch.equal(out['truncated'][t].bool(), trunc), t
    sa, sb = a.state_dict(), b.state_dict()
    for k in ('world', 'ctrl', 'elapsed', 'episode', 'momentum', 'velocity', 'goal'):
        assert torch.equal(sa[k], sb[k]), k


@pytest.mark.parametrize('ne', [5, 8])
def test_prepared_resets_match_inline_replays(gpu, ne, monkeypatch):
    """OGBX_PWF_PREP_OPS (off by default): next-episode reset
    states prepared on the low-priority side stream and loaded by the
    synchronized auto-reset step give exactly the in-line goal replays'
    outputs and state, and the reset step loads instead of replaying."""
    n, T, K = 8, 45, 100
    monkeypatch.setenv('OGBX_PWF_PREP_OPS', '8')
    a = _env(gpu, n, ne=ne, size=32, max_episode_steps=T, auto_reset=True)
    monkeypatch.delenv('OGBX_PWF_PREP_OPS')
    b = _env(gpu, n, ne=ne, size=32, max_episode_steps=T, auto_reset=True)
    opts = dict(task_id=torch.arange(n, device=gpu) % 5 + 1)
    a.reset(seed=11, options=opts)
    b.reset(seed=11, options=opts)
    rng = np.random.RandomState(2)
    acts = torch.tensor(rng.randint(0, max(ne, a._xy_action_size), size=(K, n)), dtype=torch.int32, device=gpu)
    ms = {}
    for t in range(K):
        outs = {}
        for name, env in (('a', a), ('b', b)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ob, rew, term, trunc, info = env.step(acts[t])
            e1.record()
            outs[name] = [x.clone() for x in (ob, rew, term, trunc, info['success'])]
            if t == T - 1:
                torch.cuda.synchronize()
                ms[name] = e0.elapsed_time(e1)
        for k, (x, y) in enumerate(zip(outs['a'], outs['b'])):
            assert torch.equal(x, y), (t, k)
    sa, sb = a.state_dict(), b.state_dict()
    for k in ('world', 'ctrl', 'elapsed', 'episode', 'momentum', 'velocity', 'goal'):
        assert torch.equal(sa[k], sb[k]), k
    # the synchronized reset at step T-1 loaded prepared states (no replay)
    assert ms['a'] < ms['b'] / 3, ms
