"""GPU parity: libogbx powderworld-easy kernels (through the C-ABI) vs the
reference golden vectors (tests/golden/powder_golden.npz) and the NumPy oracle
(oracle/powder_np.py).  Everything here is integer/byte work: bit-exact."""

import os

import numpy as np
import pytest
import torch

import ogbench_amd
from ogbench_amd.powder_tasks import easy_task_sequences
from oracle import powder_np as orc

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), 'golden', 'powder_golden.npz')


@pytest.fixture(scope='module')
def gold():
    return dict(np.load(GOLD))


def _env(gpu, n, size=32, **kw):
    return ogbench_amd.make('powderworld-easy-v0', num_envs=n, device=gpu, world_size=size, **kw)


def pack(ids, grav, didg):
    return (np.asarray(ids) | (np.asarray(grav) << 5) | (np.asarray(didg) << 6)).astype(np.uint8)


def unpack(w):
    w = np.asarray(w).astype(np.int32)
    return w & 31, (w >> 5) & 1, (w >> 6) & 1


@pytest.mark.parametrize('size', [32, 64])
def test_goal_worlds(gpu, gold, size):
    env = _env(gpu, 1, size)
    assert np.array_equal(env.goal_worlds(), gold[f'env{size}_goal_world'])
    for t in range(1, 6):
        _, info = env.reset(seed=t, options=dict(task_id=t))
        assert np.array_equal(info['goal'][0].cpu().numpy(), gold[f'env{size}_goal_ob'][t - 1])


@pytest.mark.parametrize('size', [32, 64])
def test_forward_random_worlds(gpu, gold, size):
    w_in, w_out = gold[f'fwd{size}_in'], gold[f'fwd{size}_out']
    packed = np.stack([pack(w[0].astype(np.int32), w[2].astype(np.int32), w[8].astype(np.int32)) for w in w_in])
    env = _env(gpu, 1, size)
    cur = torch.tensor(packed)
    for t in range(w_out.shape[0]):
        cur = env.forward(cur)
        exp = np.stack([pack(w[0].astype(np.int32), w[2].astype(np.int32), w[8].astype(np.int32))
                        for w in w_out[t]])
        assert np.array_equal(cur.cpu().numpy(), exp), t
    # fused multi-step forward == repeated single steps
    fused = env.forward(torch.tensor(packed), steps=w_out.shape[0])
    assert np.array_equal(fused.cpu().numpy(), cur.cpu().numpy())


def _trace_inputs(gold, size):
    n_tr = 6
    resets = np.stack([gold[f'env{size}_tr{tr}_reset'] for tr in range(n_tr)])
    acts = np.stack([gold[f'env{size}_tr{tr}_actions'] for tr in range(n_tr)], 1)
    draws = np.stack([gold[f'env{size}_tr{tr}_draws'] for tr in range(n_tr)], 1)
    return n_tr, resets, acts, draws


@pytest.mark.parametrize('size', [32, 64])
def test_reference_traces_step(gpu, gold, size):
    """The reference's recorded episodes (valid + invalid actions with their
    np.random draws) replayed as one batch, one step() per time step."""
    n_tr, resets, acts, draws = _trace_inputs(gold, size)
    env = _env(gpu, n_tr, size)
    ob, info = env.reset(seed=0, options=dict(task_id=torch.tensor(resets[:, 0]), reset_action=resets[:, 1:]))
    for tr in range(n_tr):
        assert np.array_equal(ob[tr].cpu().numpy(), gold[f'env{size}_tr{tr}_reset_ob'])
        assert np.array_equal(info['goal'][tr].cpu().numpy(), gold[f'env{size}_goal_ob'][resets[tr, 0] - 1])
    for t in range(acts.shape[0]):
        ob, rew, term, trunc, info = env.step(acts[t], draws=draws[t])
        ob, rew, term = ob.cpu().numpy(), rew.cpu().numpy(), term.cpu().numpy()
        for tr in range(n_tr):
            assert np.array_equal(ob[tr], gold[f'env{size}_tr{tr}_obs'][t]), (tr, t)
            assert rew[tr] == gold[f'env{size}_tr{tr}_reward'][t]
            assert term[tr] == gold[f'env{size}_tr{tr}_terminated'][t]
        assert not trunc.any()
        assert np.array_equal(info['success'].cpu().numpy(), term)
    ids = env.world_ids().cpu().numpy()
    for tr in range(n_tr):
        assert np.array_equal(ids[tr], gold[f'env{size}_tr{tr}_final_world'])


@pytest.mark.parametrize('size', [32, 64])
def test_reference_traces_fused_rollout(gpu, gold, size):
    n_tr, resets, acts, draws = _trace_inputs(gold, size)
    env = _env(gpu, n_tr, size)
    env.reset(seed=0, options=dict(task_id=torch.tensor(resets[:, 0]), reset_action=resets[:, 1:]))
    out = env.rollout(acts, draws=draws)
    obs = out['obs'].cpu().numpy()
    for tr in range(n_tr):
        assert np.array_equal(obs[:, tr], gold[f'env{size}_tr{tr}_obs'])
        assert np.array_equal(out['reward'][:, tr].cpu().numpy(), gold[f'env{size}_tr{tr}_reward'])
        assert np.array_equal(out['terminated'][:, tr].cpu().numpy().astype(bool),
                              gold[f'env{size}_tr{tr}_terminated'])


def _oracle_batch(size, tasks, reset_actions, goals):
    envs = []
    for t, (e, x, y) in zip(tasks, reset_actions):
        env = orc.Env(size)
        env.reset(goals[t - 1].astype(np.int32), int(e), int(x), int(y))
        envs.append(env)
    return envs


@pytest.mark.parametrize('size', [32, 64])
def test_random_batch_vs_oracle(gpu, size):
    """256 envs x 150 steps of random (mostly valid) actions, bit-exact against the oracle."""
    rng = np.random.RandomState(7 + size)
    n, T = 256, 150
    env = _env(gpu, n, size)
    goals = env.goal_worlds()
    xy = env._xy_action_size
    tasks = rng.randint(1, 6, n)
    ra = np.stack([rng.randint(0, 2, n), rng.randint(0, xy, n), rng.randint(0, xy, n)], 1)
    env.reset(seed=1, options=dict(task_id=torch.tensor(tasks), reset_action=ra))
    oracles = _oracle_batch(size, tasks, ra, goals)
    for t in range(T):
        hi = 2 if t % 3 == 0 else xy
        a = rng.randint(0, hi + 2, n)  # some invalid
        d = rng.randint(0, hi, n)
        ob, rew, term, _, _ = env.step(a, draws=d)
        if t % 10 == 9 or t == T - 1:
            ob, rew, term = ob.cpu().numpy(), rew.cpu().numpy(), term.cpu().numpy()
        for i, o in enumerate(oracles):
            eo, er, es = o.step(int(a[i]), int(d[i]))
            if t % 10 == 9 or t == T - 1:
                assert np.array_equal(ob[i], eo), (i, t)
                assert rew[i] == er and term[i] == es
    w = env._state_views()[0].cpu().numpy()
    for i, o in enumerate(oracles):
        assert np.array_equal(w[i], pack(*o.state)), i


def test_task_replay_reaches_success(gpu):
    """Replaying each task's own action sequence from a random start reaches
    success exactly when the oracle does (success must actually occur)."""
    size = 32
    seqs = easy_task_sequences()
    n = 5
    env = _env(gpu, n, size)
    goals = env.goal_worlds()
    tasks = np.arange(1, 6)
    ra = np.array([[1, 3, 2], [0, 0, 0], [1, 7, 7], [0, 4, 5], [1, 2, 6]])
    env.reset(seed=3, options=dict(task_id=torch.tensor(tasks), reset_action=ra))
    oracles = _oracle_batch(size, tasks, ra, goals)
    L = max(len(s) for s in seqs)
    ever = np.zeros(n, bool)
    for k in range(L):
        for stage in range(3):
            a = np.zeros(n, np.int64)
            for i in range(n):
                e, x, y = seqs[i][k % len(seqs[i])]
                a[i] = (e, x, y)[stage]
            _, rew, term, _, info = env.step(a)
            term = term.cpu().numpy()
            for i, o in enumerate(oracles):
                _, _, es = o.step(int(a[i]))
                assert term[i] == es, (i, k, stage)
            ever |= term
    assert ever.all()


def test_auto_reset_truncation_and_success(gpu):
    size = 32
    n = 64
    env = _env(gpu, n, size, max_episode_steps=7, auto_reset=True)
    env.reset(seed=11, options=dict(task_id=1))
    for t in range(1, 22):
        ob, rew, term, trunc, info = env.step(np.full(n, 0))
        expect_trunc = t % 7 == 0
        assert bool(trunc.all()) == expect_trunc and bool(trunc.any()) == expect_trunc
        el = env._state_views()[2].cpu().numpy()
        assert (el == (t % 7)).all()
    # after a reset the world is blank + one random brush (a valid reset world)
    blanks = {}
    o = orc.Env(size)
    for e in range(2):
        for x in range(8):
            for y in range(8):
                ids, grav, didg = o.blank()
                ids, grav, didg = orc.forward(ids, grav, didg)
                blanks[pack(*orc.paint(ids, grav, didg, orc.EASY_ELEMS[e], x, y)).tobytes()] = 1
    env2 = _env(gpu, n, size, max_episode_steps=500, auto_reset=True)
    env2.reset(seed=5, options=dict(task_id=1))
    w = env2._state_views()[0].cpu().numpy()
    assert all(w[i].tobytes() in blanks for i in range(n))
    # resets with different seeds differ; the same seed reproduces
    env2.reset(seed=5, options=dict(task_id=1))
    assert np.array_equal(env2._state_views()[0].cpu().numpy(), w)
    env2.reset(seed=6, options=dict(task_id=1))
    assert not np.array_equal(env2._state_views()[0].cpu().numpy(), w)


def test_auto_reset_on_success(gpu):
    """Task 1 (plant everywhere): painting plant over the whole grid succeeds;
    with auto_reset the same step returns the next episode's first obs."""
    size = 32
    env = _env(gpu, 1, size, auto_reset=True)
    env.reset(seed=2, options=dict(task_id=1, reset_action=[[0, 0, 0]]))
    seq = easy_task_sequences()[0]
    done_at = None
    for k, (e, x, y) in enumerate(seq):
        for stage, a in enumerate((e, x, y)):
            ob, rew, term, trunc, info = env.step([a])
            if bool(term[0]):
                done_at = (k, stage)
                assert rew[0].item() == 1.0 and bool(info['success'][0])
                assert int(env._state_views()[2][0]) == 0  # elapsed reset
                w = env.world_ids()[0].cpu().numpy()
                assert (w[1:-1, 1:-1] == 8).sum() <= 16  # fresh world: one brush at most
                break
        if done_at:
            break
    assert done_at is not None


def test_errors(gpu):
    with pytest.raises(ValueError):
        _env(gpu, 1, 48)
    env = _env(gpu, 2)
    with pytest.raises(Exception):
        env.step([0, 0])  # step before reset
    with pytest.raises(AssertionError):
        env.reset(options=dict(task_id=6))
