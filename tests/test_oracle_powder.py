"""CPU: pin the powderworld-easy oracle (oracle/powder_np.py) against the
reference's own sim.py / powderworld_env.py outputs (tests/golden/powder_golden.npz)."""

import os

import numpy as np
import pytest

from oracle import powder_np as orc

GOLD = os.path.join(os.path.dirname(__file__), 'golden', 'powder_golden.npz')


@pytest.fixture(scope='module')
def gold():
    return dict(np.load(GOLD))


def test_render_lut(gold):
    assert np.array_equal(orc.render_lut(), gold['render_lut'])


@pytest.mark.parametrize('size', [32, 64])
def test_forward_periodic_random_worlds(gold, size):
    w_in = gold[f'fwd{size}_in']
    w_out = gold[f'fwd{size}_out']
    for e in range(w_in.shape[0]):
        ids, grav, didg = orc.from_channels(w_in[e])
        for t in range(w_out.shape[0]):
            ids, grav, didg = orc.forward(ids, grav, didg)
            ref = w_out[t, e]
            assert np.array_equal(ids, ref[0]) and np.array_equal(grav, ref[2]) and np.array_equal(didg, ref[8])
            # every other channel is a function of the id or zero (easy worlds)
            assert np.array_equal(ref[1], orc.DENSITY[ids]) and not ref[3:8].any()


@pytest.mark.parametrize('size', [32, 64])
def test_env_traces(gold, size):
    env = orc.Env(size)
    goals = gold[f'env{size}_goal_world']
    for tr in range(6):
        task, elem, x, y = gold[f'env{size}_tr{tr}_reset']
        ob = env.reset(goals[task - 1].astype(np.int32), elem, x, y)
        assert np.array_equal(ob, gold[f'env{size}_tr{tr}_reset_ob'])
        acts, draws = gold[f'env{size}_tr{tr}_actions'], gold[f'env{size}_tr{tr}_draws']
        for t, (a, d) in enumerate(zip(acts, draws)):
            ob, rew, succ = env.step(int(a), int(d))
            assert np.array_equal(ob, gold[f'env{size}_tr{tr}_obs'][t]), (tr, t)
            assert rew == gold[f'env{size}_tr{tr}_reward'][t]
            assert succ == gold[f'env{size}_tr{tr}_terminated'][t]
        assert np.array_equal(env.state[0], gold[f'env{size}_tr{tr}_final_world'])


@pytest.mark.parametrize('size', [32, 64])
def test_goal_worlds_replay(gold, size):
    """The easy goal worlds are the replay of each task's action sequence."""
    from ogbench_amd.powder_tasks import easy_task_sequences

    env = orc.Env(size)
    for t, seq in enumerate(easy_task_sequences()):
        ids, grav, didg = env.blank()
        for elem, x, y in seq:
            ids, grav, didg = orc.forward(ids, grav, didg)
            ids, grav, didg = orc.paint(ids, grav, didg, orc.EASY_ELEMS[elem], x, y)
        assert np.array_equal(ids, gold[f'env{size}_goal_world'][t])
        ob = orc.observe(ids, 0, 0, 0)
        assert np.array_equal(ob, gold[f'env{size}_goal_ob'][t])
        assert orc.error_count(ids, ids) == 0
