"""GPU parity: libogbx locomaze kernels (through the C-ABI) vs the oracle and the
reference golden vectors.  Tolerances: bit-exact for indices, masks, reset
arithmetic and free-space steps; 1e-9 abs for contact dynamics (north_star
allows 1e-5; the oracle solves the same model with a different solver)."""

import numpy as np
import pytest
import torch

import ogbench_amd
from oracle import locomaze as orc

pytestmark = pytest.mark.gpu
TOL = 1e-9


def _env(gpu, n, maze='large', **kw):
    return ogbench_amd.MazeEnv('point', maze, num_envs=n, device=gpu, **kw)


def test_free_space_bit_exact(gpu, golden_locomaze):
    q = torch.tensor(golden_locomaze['free_qpos'])
    env = _env(gpu, 1)
    for kind in ('32', '64'):
        a = torch.tensor(golden_locomaze[f'free_act{kind}'])
        out, contact = env.physics(q, a)
        ref, rc = orc.physics('large', q.numpy(), a.numpy())
        assert np.array_equal(contact.cpu().numpy(), rc)
        free = rc == 0
        assert free.sum() > 1000
        assert np.array_equal(out.cpu().numpy()[free], golden_locomaze[f'free_out{kind}'][free])


@pytest.mark.parametrize('maze', ['medium', 'large', 'giant', 'arena'])
@pytest.mark.parametrize('f64', [False, True])
def test_physics_matches_oracle_with_contacts(gpu, maze, f64):
    rng = np.random.RandomState(sum(map(ord, maze)) + 7 * int(f64))
    mp, _ = orc.tables(maze)
    cells = np.argwhere(mp == 0)
    n = 20000
    c = cells[rng.randint(len(cells), size=n)]
    # positions concentrated near walls: offsets up to 1.9 from the cell centre
    q = np.stack([c[:, 1] * 4.0 - 4 + rng.uniform(-1.9, 1.9, n), c[:, 0] * 4.0 - 4 + rng.uniform(-1.9, 1.9, n)], 1)
    a = rng.uniform(-1, 1, (n, 2)).astype(np.float64 if f64 else np.float32)
    env = _env(gpu, 1, maze)
    out, contact = env.physics(torch.tensor(q), torch.tensor(a))
    ref, rc = orc.physics(maze, q, a, nthreads=8)
    got = out.cpu().numpy()
    assert np.array_equal(contact.cpu().numpy(), rc)
    assert rc.mean() > (0.05 if maze == "arena" else 0.2)  # the test really exercises contacts
    assert np.abs(got - ref).max() <= TOL
    assert np.array_equal(got[rc == 0], ref[rc == 0])


@pytest.mark.parametrize('k', [1, 8, 63])
def test_physics_waves_mixing_contact_and_free_lanes(gpu, k):
    """Waves of 64 envs with exactly k contact lanes: the free lanes run the
    contact loop alongside (point_step) and must still return the exact free
    step and contact flag 0; the contact lanes match the oracle."""
    rng = np.random.RandomState(100 + k)
    mp, _ = orc.tables('large')
    cells = np.argwhere(mp == 0)
    n = 40000
    c = cells[rng.randint(len(cells), size=n)]
    q = np.stack([c[:, 1] * 4.0 - 4 + rng.uniform(-1.9, 1.9, n), c[:, 0] * 4.0 - 4 + rng.uniform(-1.9, 1.9, n)], 1)
    a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
    _, rc = orc.physics('large', q, a, nthreads=8)
    ci, fi = np.flatnonzero(rc == 1), np.flatnonzero(rc == 0)
    waves = min(len(ci) // k, len(fi) // (64 - k), 128)
    order = np.concatenate([np.concatenate([ci[w * k:(w + 1) * k], fi[w * (64 - k):(w + 1) * (64 - k)]])
                            for w in range(waves)])
    qm, am = q[order], a[order]
    env = _env(gpu, 1)
    out, contact = env.physics(torch.tensor(qm), torch.tensor(am))
    ref, rcm = orc.physics('large', qm, am, nthreads=8)
    got = out.cpu().numpy()
    assert np.array_equal(contact.cpu().numpy(), rcm)
    assert rcm.reshape(waves, 64).sum(1).tolist() == [k] * waves
    assert np.array_equal(got[rcm == 0], ref[rcm == 0])
    assert np.abs(got - ref).max() <= TOL


def test_xy_to_ij_bit_exact(gpu, golden_locomaze):
    env = _env(gpu, 1)
    ij = env.xy_to_ij(torch.tensor(golden_locomaze['xy2ij_in']))
    assert np.array_equal(ij.cpu().numpy(), golden_locomaze['xy2ij_out'])


def test_success_mask_bit_exact(gpu, golden_locomaze):
    pos, goal = golden_locomaze['succ_pos'], golden_locomaze['succ_goal']
    n = len(pos)
    env = _env(gpu, n, success_timing='pre')
    env.reset(options=dict(task_id=1, noise=torch.zeros(n, 4, dtype=torch.float64)))
    sd = env.state_dict()
    sd['qpos'] = torch.tensor(pos)
    sd['goal'] = torch.tensor(goal)
    env.load_state_dict(sd)
    _, _, _, _, info = env.step(torch.zeros(n, 2))
    assert np.array_equal(info['success'].cpu().numpy(), golden_locomaze['succ_out'].astype(bool))


@pytest.mark.parametrize('maze', ['medium', 'large'])
def test_reset_with_injected_noise(gpu, golden_locomaze, maze):
    tid = golden_locomaze[f'reset_{maze}_task']
    noise = golden_locomaze[f'reset_{maze}_noise']
    env = _env(gpu, len(tid), maze)
    obs, info = env.reset(options=dict(task_id=torch.tensor(tid), noise=torch.tensor(noise)))
    exp = golden_locomaze[f'reset_{maze}_out']
    assert np.array_equal(obs.cpu().numpy(), exp[:, :2])
    assert np.array_equal(info['goal'].cpu().numpy(), exp[:, 2:])


@pytest.mark.parametrize('maze', ['medium', 'large', 'giant'])
def test_oracle_subgoal_bit_exact(gpu, golden_locomaze, maze):
    env = _env(gpu, 1, maze)
    s = torch.tensor(golden_locomaze[f'subgoal_{maze}_start'])
    g = torch.tensor(golden_locomaze[f'subgoal_{maze}_goal'])
    out = env.get_oracle_subgoal(s, g)
    assert np.array_equal(out.cpu().numpy(), golden_locomaze[f'subgoal_{maze}_out'])


@pytest.mark.parametrize('fused', [False, True])
def test_env_rollout_matches_oracle(gpu, fused):
    """300 steps of N envs with auto-reset (Philox reset draws), vs the oracle."""
    n, k = 4096, 300
    env = _env(gpu, n, 'large', auto_reset=True, max_episode_steps=120)
    rng = np.random.RandomState(7)
    tid = (np.arange(n) % 5 + 1).astype(np.int32)
    noise = rng.uniform(-1, 1, (n, 4))
    seed = 0x1234_5678_9ABC
    env.reset(seed=seed, options=dict(task_id=torch.tensor(tid), noise=torch.tensor(noise)))
    st = orc.reset('large', tid, noise, max_steps=120)
    # drive envs toward their goals part of the time so that successes happen
    acts = rng.uniform(-1, 1, (k, n, 2)).astype(np.float32)
    key = orc.philox_key(seed, orc.TAG_MAZE_RESET)
    ref = orc.step('large', st, acts, auto_reset=1, key=key, nthreads=8)
    if fused:
        out = env.rollout(torch.tensor(acts))
        got = {k2: v.cpu().numpy() for k2, v in out.items()}
    else:
        got = dict(obs=[], reward=[], terminated=[], truncated=[], success=[])
        for t in range(k):
            o, r, te, tr, info = env.step(torch.tensor(acts[t]))
            got['obs'].append(o.cpu().numpy().copy())
            got['reward'].append(r.cpu().numpy().copy())
            got['terminated'].append(te.cpu().numpy().copy())
            got['truncated'].append(tr.cpu().numpy().copy())
            got['success'].append(info['success'].cpu().numpy().copy())
        got = {k2: np.stack(v) for k2, v in got.items()}
    assert np.abs(got['obs'] - ref['obs']).max() <= TOL
    for key2 in ('terminated', 'truncated', 'success'):
        assert np.array_equal(got[key2].astype(bool), ref[key2].astype(bool)), key2
    assert np.array_equal(got['reward'], ref['reward'])
    assert ref['truncated'].sum() > 0


@pytest.mark.parametrize('f64', [False, True])
def test_rollout_until_done_matches_single_steps(gpu, f64):
    """Evaluation rollout (no auto-reset, SURVEY 7.3 wave-ballot exit): every
    row an env writes equals K single env.step calls; rows after its episode
    ended are untouched; the env's state is the state at its last step."""
    n, k = 4096, 200
    kw = dict(max_episode_steps=150)
    rng = np.random.RandomState(11)
    tid = torch.tensor((np.arange(n) % 5 + 1).astype(np.int32))
    noise = torch.tensor(rng.uniform(-1, 1, (n, 4)))
    envs = [_env(gpu, n, 'large', **kw) for _ in range(2)]
    obs0 = [e.reset(seed=5, options=dict(task_id=tid, noise=noise))[0] for e in envs]
    # goals within a few units of the start (half of the envs), the task goal
    # otherwise; heading straight for them ends some episodes at the goal and
    # the rest at the TimeLimit
    sd = envs[0].state_dict()
    near = torch.tensor(rng.uniform(-3, 3, (n, 2)), device=gpu) + obs0[0]
    sd['goal'] = torch.where(torch.arange(n, device=gpu)[:, None] % 2 == 0, near, sd['goal'])
    for e in envs:
        e.load_state_dict(sd)
    goal = sd['goal'].cpu().numpy()
    d = goal - obs0[0].cpu().numpy()
    acts = np.clip(d / np.maximum(np.abs(d).max(1, keepdims=True), 1e-9), -1, 1)
    acts = np.repeat(acts[None], k, 0) + rng.normal(0, 0.3, (k, n, 2))
    acts = torch.tensor(np.clip(acts, -1, 1).astype(np.float64 if f64 else np.float32))
    sentinel = -7.0
    out = dict(obs=torch.full((k, n, 2), sentinel, dtype=torch.float64, device=gpu),
               reward=torch.full((k, n), sentinel, dtype=torch.float32, device=gpu),
               terminated=torch.full((k, n), 9, dtype=torch.uint8, device=gpu),
               truncated=torch.full((k, n), 9, dtype=torch.uint8, device=gpu),
               success=torch.full((k, n), 9, dtype=torch.uint8, device=gpu),
               steps=torch.zeros(n, dtype=torch.int32, device=gpu))
    got = {key: v.cpu().numpy() for key, v in envs[0].rollout_until_done(acts, out).items()}
    steps = got['steps']
    ref = dict(obs=[], reward=[], terminated=[], truncated=[], success=[])
    for t in range(k):
        o, r, te, tr, info = envs[1].step(acts[t])
        for key, v in (('obs', o), ('reward', r), ('terminated', te), ('truncated', tr), ('success', info['success'])):
            ref[key].append(v.cpu().numpy().copy())
    ref = {key: np.stack(v) for key, v in ref.items()}
    done = ref['terminated'].astype(bool) | ref['truncated'].astype(bool)
    first = np.where(done.any(0), done.argmax(0) + 1, k)
    assert np.array_equal(steps, first)
    assert (first < 150).sum() > 100 and (first == 150).sum() > 100  # goal ends and TimeLimit ends
    rows = np.arange(k)[:, None] < steps[None, :]
    for key in ('obs', 'reward', 'terminated', 'truncated', 'success'):
        g, r = got[key], ref[key].astype(got[key].dtype)
        assert np.array_equal(g[rows], r[rows]), key
        assert (g[~rows] == (sentinel if key in ('obs', 'reward') else 9)).all(), key
    final = got['obs'][steps - 1, np.arange(n)]
    assert np.array_equal(envs[0].get_xy().cpu().numpy(), final)


def test_truncation_singletask_reward(gpu):
    n = 64
    env = ogbench_amd.make('pointmaze-medium-singletask-task2-v0', num_envs=n, device=gpu, max_episode_steps=4)
    obs, info = env.reset(seed=3)
    # singletask: fixed task 2, no goal noise
    goal = info['goal'].cpu().numpy()
    assert np.array_equal(goal, np.tile([[20.0, 0.0]], (n, 1)))  # task2 goal (1,6)
    for t in range(4):
        obs, rew, term, trunc, info = env.step(torch.zeros(n, 2))
        assert (rew.cpu().numpy() == -1.0).all()
        assert trunc.cpu().numpy().all() == (t == 3)


def test_step_before_reset_and_bad_task(gpu):
    env = _env(gpu, 4)
    with pytest.raises(Exception, match='reset'):
        env.step(torch.zeros(4, 2))
    with pytest.raises(AssertionError, match='Task ID must be in'):
        env.reset(options=dict(task_id=9))


def test_teleport_moves_state_but_not_obs(gpu):
    env = _env(gpu, 2, 'teleport')
    env.reset(seed=1, options=dict(task_id=1, noise=torch.zeros(2, 4, dtype=torch.float64)))
    sd = env.state_dict()
    sd['qpos'] = torch.tensor([[20.0, 12.0], [5.0, 0.0]])  # first env on the in-portal (4,6)
    env.load_state_dict(sd)
    obs, *_ = env.step(torch.zeros(2, 2))
    q = env.get_xy().cpu().numpy()
    assert np.array_equal(obs.cpu().numpy()[0], [20.0, 12.0])
    assert tuple(q[0]) in {(24.0, 0.0), (0.0, 20.0), (36.0, 20.0)}
    assert np.array_equal(q[1], [5.0, 0.0])


def test_teleport_maze_matches_oracle(gpu):
    """Teleport maze: agents around the in-portals, 3 fused steps; the GPU and
    the oracle (same Philox key for the out-portal draw) agree on every
    teleport destination bit-exactly and on the dynamics to TOL."""
    rng = np.random.RandomState(21)
    n = 20000
    ins = np.array([[20.0, 12.0], [0.0, 16.0]])
    centre = ins[np.arange(n) % 2]
    ang = rng.uniform(0, 2 * np.pi, n)
    q = centre + np.stack([np.cos(ang), np.sin(ang)], 1) * rng.uniform(0, 2.2, n)[:, None]
    env = _env(gpu, n, 'teleport')
    env.reset(seed=77, options=dict(task_id=1))
    sd = env.state_dict()
    sd['qpos'] = torch.tensor(q, device=gpu)
    env.load_state_dict(sd)
    st = dict(qpos=q.copy(), goal=sd['goal'].cpu().numpy().copy(), elapsed=sd['elapsed'].cpu().numpy().copy(),
              task=sd['task'].cpu().numpy().copy(), episode=sd['episode'].cpu().numpy().view(np.uint32).copy(),
              opts=orc._opts())
    a = rng.uniform(-1, 1, (3, n, 2)).astype(np.float32)
    out = env.rollout(torch.tensor(a, device=gpu))
    ref = orc.step('teleport', st, a, key=orc.philox_key(77, orc.TAG_MAZE_RESET))
    got_q = env.get_xy().cpu().numpy()
    assert np.abs(out['obs'].cpu().numpy() - ref['obs']).max() <= TOL
    assert np.abs(got_q - st['qpos']).max() <= TOL
    outs = np.array([[24.0, 0.0], [0.0, 20.0], [36.0, 20.0]])
    tele = (np.abs(st['qpos'][:, None, :] - outs[None]).max(-1) == 0).any(1)
    assert tele.sum() > 200  # teleported at the last step (earlier ones moved on; all are checked above)
    assert np.array_equal(got_q[tele], st['qpos'][tele])


def test_headline_n65536_matches_oracle(gpu):
    """The BASELINE configuration itself: pointmaze-large, N = 65,536, task
    i%5+1, Philox reset noise (seed 0), TimeLimit 1000, same-step auto-reset,
    150 single-step launches vs the OpenMP oracle.  Episode clocks start
    staggered (elapsed = i % 1000) so that ~15 % of the envs hit the TimeLimit
    and auto-reset with Philox draws inside the window."""
    n, k, seed = 65536, 150, 0
    env = ogbench_amd.make('pointmaze-large-v0', num_envs=n, device=gpu, auto_reset=True)
    tid = (np.arange(n) % 5 + 1).astype(np.int32)
    obs, info = env.reset(seed=seed, options=dict(task_id=torch.tensor(tid, device=gpu)))
    st = orc.reset('large', tid, orc.reset_draws(n, seed))
    assert np.array_equal(obs.cpu().numpy(), st['qpos']) and np.array_equal(info['goal'].cpu().numpy(), st['goal'])
    sd = env.state_dict()
    sd['elapsed'] = torch.tensor(np.arange(n) % 1000, dtype=torch.int32)
    env.load_state_dict(sd)
    st['elapsed'][:] = np.arange(n) % 1000
    acts = (torch.rand(k, n, 2, generator=torch.Generator().manual_seed(1)) * 2 - 1).float()
    key = orc.philox_key(seed, orc.TAG_MAZE_RESET)
    resets = 0
    for t in range(k):
        o, r, te, tr, inf = env.step(acts[t].to(gpu))
        ref = orc.step('large', st, acts[t].numpy()[None], auto_reset=1, key=key, nthreads=16)
        assert np.abs(o.cpu().numpy() - ref['obs'][0]).max() <= TOL, t
        assert np.array_equal(inf['success'].cpu().numpy(), ref['success'][0].astype(bool)), t
        assert np.array_equal(te.cpu().numpy(), ref['terminated'][0].astype(bool)), t
        assert np.array_equal(tr.cpu().numpy(), ref['truncated'][0].astype(bool)), t
        assert np.array_equal(r.cpu().numpy(), ref['reward'][0]), t
        resets += int(ref['truncated'][0].sum() + ref['terminated'][0].sum())
    assert resets >= 0.14 * n
    assert np.abs(env.get_xy().cpu().numpy() - st['qpos']).max() <= TOL
    assert np.array_equal(env.cur_goal_xy.cpu().numpy(), st['goal'])


@pytest.mark.parametrize('task', [1, 4])
def test_medium_single_env_timelimit_episode(gpu, task):
    """pointmaze-medium-v0 with ONE env (BASELINE configs[0], the Gymnasium
    surface): make -> reset(seed, task_id) -> 1000 steps of U[-1,1]^2 float32
    actions (torch.Generator seed 0) -> truncated exactly at step 1000, every
    step against the oracle."""
    seed = 5 + task
    env = ogbench_amd.make('pointmaze-medium-v0', num_envs=1, device=gpu)
    assert env.max_episode_steps == 1000 and env.observation_space.shape == (1, 2)
    obs, info = env.reset(seed=seed, options=dict(task_id=task))
    st = orc.reset('medium', np.array([task], np.int32), orc.reset_draws(1, seed))
    assert np.array_equal(obs.cpu().numpy(), st['qpos']) and np.array_equal(info['goal'].cpu().numpy(), st['goal'])
    acts = (torch.rand(1000, 1, 2, generator=torch.Generator().manual_seed(0)) * 2 - 1).float()
    contacts = 0
    for t in range(1000):
        prev = env.get_xy().cpu().numpy()
        o, r, te, tr, inf = env.step(acts[t].to(gpu))
        ref = orc.step('medium', st, acts[t].numpy()[None])
        got = o.cpu().numpy()
        assert np.abs(got - ref['obs'][0]).max() <= TOL, t
        free = prev + (0.2 * acts[t].numpy()).astype(np.float64)
        contacts += int(not np.array_equal(got, free))
        assert bool(te[0]) == bool(ref['terminated'][0, 0]) and bool(inf['success'][0]) == bool(ref['success'][0, 0])
        assert bool(tr[0]) == (t == 999) == bool(ref['truncated'][0, 0]), t
        assert float(r[0]) == float(ref['reward'][0, 0])
    assert contacts > 20  # the episode really exercises wall contacts


def test_rollout_until_done_teleport_matches_single_steps(gpu):
    """pointmaze-teleport evaluation rollout: envs placed around the in-portals
    so that many teleport inside the window; every written row (and the
    out-portal each teleport picks, which follows the reset seed) equals K
    single env.step calls (the rollout used a different key)."""
    n, k = 4096, 12
    rng = np.random.RandomState(23)
    ins = np.array([[20.0, 12.0], [0.0, 16.0]])
    centre = ins[np.arange(n) % 2]
    ang = rng.uniform(0, 2 * np.pi, n)
    q = centre + np.stack([np.cos(ang), np.sin(ang)], 1) * rng.uniform(0, 2.2, n)[:, None]
    envs = [_env(gpu, n, 'teleport', max_episode_steps=150) for _ in range(2)]
    for e in envs:
        e.reset(seed=91, options=dict(task_id=1))
        sd = e.state_dict()
        sd['qpos'] = torch.tensor(q, device=gpu)
        e.load_state_dict(sd)
    acts = torch.tensor(rng.uniform(-1, 1, (k, n, 2)).astype(np.float32))
    out = dict(obs=torch.zeros((k, n, 2), dtype=torch.float64, device=gpu),
               reward=torch.zeros((k, n), dtype=torch.float32, device=gpu),
               terminated=torch.zeros((k, n), dtype=torch.uint8, device=gpu),
               truncated=torch.zeros((k, n), dtype=torch.uint8, device=gpu),
               success=torch.zeros((k, n), dtype=torch.uint8, device=gpu),
               steps=torch.zeros(n, dtype=torch.int32, device=gpu))
    got = {key: v.cpu().numpy() for key, v in envs[0].rollout_until_done(acts, out).items()}
    ref = dict(obs=[], reward=[], terminated=[], truncated=[], success=[])
    for t in range(k):
        o, r, te, tr, info = envs[1].step(acts[t])
        for key, v in (('obs', o), ('reward', r), ('terminated', te), ('truncated', tr), ('success', info['success'])):
            ref[key].append(v.cpu().numpy().copy())
    ref = {key: np.stack(v) for key, v in ref.items()}
    rows = np.arange(k)[:, None] < got['steps'][None, :]
    for key in ('obs', 'reward', 'terminated', 'truncated', 'success'):
        assert np.array_equal(got[key][rows], ref[key].astype(got[key].dtype)[rows]), key
    qa, qb = envs[0].get_xy().cpu().numpy(), envs[1].get_xy().cpu().numpy()
    alive = got['steps'] == k
    assert np.array_equal(qa[alive], qb[alive])
    outs = np.array([[24.0, 0.0], [0.0, 20.0], [36.0, 20.0]])
    moved = (np.abs(qb[:, None, :] - outs[None]).max(-1) < 2.5).any(1)
    assert moved.sum() > 200  # many envs went through a portal inside the window


def test_results_do_not_depend_on_wavefront_composition(gpu):
    """Every contact-path choice is per lane (lean loop, full-loop redo,
    generic collider), so an env's step is the same whichever envs share its
    64-lane wavefront: near-wall states (many lean-loop bails) plus states
    inside wall cells (generic collider), stepped in order and permuted, agree
    bit for bit.  This is what lets any sharding of the envs reproduce the
    single-GPU run."""
    rng = np.random.RandomState(31)
    mp, _ = orc.tables('large')
    free_cells, wall_cells = np.argwhere(mp == 0), np.argwhere(mp == 1)
    n = 24000
    c = free_cells[rng.randint(len(free_cells), size=n)]
    q = np.stack([c[:, 1] * 4.0 - 4 + rng.uniform(-1.95, 1.95, n), c[:, 0] * 4.0 - 4 + rng.uniform(-1.95, 1.95, n)], 1)
    k = n // 50
    wc = wall_cells[rng.randint(len(wall_cells), size=k)]
    q[:k] = np.stack([wc[:, 1] * 4.0 - 4 + rng.uniform(-2, 2, k), wc[:, 0] * 4.0 - 4 + rng.uniform(-2, 2, k)], 1)
    a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
    perm = rng.permutation(n)
    env = _env(gpu, 1)
    out, contact = env.physics(torch.tensor(q), torch.tensor(a))
    outp, contactp = env.physics(torch.tensor(q[perm]), torch.tensor(a[perm]))
    assert np.array_equal(outp.cpu().numpy(), out.cpu().numpy()[perm])
    assert np.array_equal(contactp.cpu().numpy(), contact.cpu().numpy()[perm])
    assert contact.cpu().numpy().mean() > 0.2


def test_state_restore_into_other_handle_carries_seed(gpu):
    """load_state_dict into a handle reset with another seed: the restored
    handle keys its auto-reset draws with the saved seed (ogbx_maze_set_seed),
    so both continue identically through several auto-resets."""
    n, K = 256, 40
    a = _env(gpu, n, max_episode_steps=7, auto_reset=True)
    b = _env(gpu, n, max_episode_steps=7, auto_reset=True)
    a.reset(seed=3)
    b.reset(seed=77)
    g = torch.Generator().manual_seed(2)
    acts = (torch.rand(K, n, 2, generator=g) * 2 - 1).to(gpu)
    for t in range(3):
        a.step(acts[t])
    b.load_state_dict(a.state_dict())
    for t in range(3, K):
        oa, ra, _, tra, _ = a.step(acts[t])
        ob, rb, _, trb, _ = b.step(acts[t])
        assert torch.equal(oa, ob) and torch.equal(tra, trb), t
    assert torch.equal(a.cur_goal_xy, b.cur_goal_xy)


def test_results_do_not_depend_on_envs_per_wave(gpu):
    """ogbx_maze_set_envs_per_wave (16 / 32 / 64 envs per 64-lane wave, the
    layout knob for small per-GPU shares) changes which envs share a
    wavefront, never an env's result: near-wall states stepped with auto-reset
    through env.step and through K fused steps agree bit for bit across the
    three layouts (the contact path decides everything per lane)."""
    from ogbench_amd import _lib

    rng = np.random.RandomState(17)
    mp, _ = orc.tables('large')
    free_cells = np.argwhere(mp == 0)
    n, K = 3000, 12
    c = free_cells[rng.randint(len(free_cells), size=n)]
    q = np.stack([c[:, 1] * 4.0 - 4 + rng.uniform(-1.9, 1.9, n), c[:, 0] * 4.0 - 4 + rng.uniform(-1.9, 1.9, n)], 1)
    acts = torch.tensor(rng.uniform(-1, 1, (K, n, 2)).astype(np.float32)).to(gpu)
    res = {}
    for epw in (64, 32, 16, 8, 32 | 0x100, 16 | 0x100, 8 | 0x100):  # 0x100: OGBX_EPW_REPLICATE
        env = _env(gpu, n, max_episode_steps=9, auto_reset=True)
        _lib.check(env._L.ogbx_maze_set_envs_per_wave(env._h, epw))
        env.reset(seed=5)
        sd = env.state_dict()
        sd['qpos'] = torch.tensor(q, dtype=torch.float64)
        env.load_state_dict(sd)
        rows = []
        for t in range(K):
            ob, rew, term, trunc, info = env.step(acts[t])
            rows.append(torch.cat([ob.flatten(), rew.double(), term.double(), info['success'].double()]).cpu())
        roll = env.rollout(acts)
        rows.append(torch.cat([roll[k].double().flatten().cpu() for k in ('obs', 'reward', 'terminated', 'success')]))
        res[epw] = torch.cat(rows)
    for epw, r in res.items():
        assert torch.equal(res[64], r), epw
