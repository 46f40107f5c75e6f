"""CPU: pin the medium/hard powderworld restatement (oracle/powder_full_np.py)
against the reference's own sim.py / powderworld_env.py outputs with the rand
fields recorded (tests/golden/powder_full_golden.npz)."""

import os

import numpy as np
import pytest

from oracle import powder_full_np as orc

GOLD = os.path.join(os.path.dirname(__file__), 'golden', 'powder_full_golden.npz')


@pytest.fixture(scope='module')
def gold():
    return dict(np.load(GOLD))


@pytest.mark.parametrize('size', [32, 64])
def test_full_forward_matches_reference(gold, size):
    w = gold[f'full{size}_in']
    outs, rands = gold[f'full{size}_out'], gold[f'full{size}_rand']
    for t in range(outs.shape[0]):
        w = orc.forward(w, [rands[t][:, k] for k in range(3)])
        assert np.array_equal(w, outs[t]), t  # every channel, bit for bit (velocities included)
    assert np.abs(outs[-1][:, 3:5]).max() > 1.0  # the velocity rule really ran


def test_render_with_velocity(gold):
    w = gold['render_vel_world'][0]
    assert np.array_equal(orc.render(w), gold['render_vel_img'])


@pytest.mark.parametrize('ne', [5, 8])
def test_env_trace(gold, ne):
    tag = f'env{ne}_tr0'
    env = orc.Env(ne, 32)
    task = int(gold[f'{tag}_task'])
    from ogbench_amd.powder_tasks import task_sequences

    seq = task_sequences(ne)[task - 1]
    rr = gold[f'{tag}_reset_rand']
    goal = env.replay(seq, rr[:-1])
    assert np.array_equal(goal[0, 0].astype(np.uint8), gold[f'{tag}_goal_world'])
    gob = np.zeros((32, 32, 6), np.uint8)
    gob[..., :3] = orc.render(goal[0])
    assert np.array_equal(gob, gold[f'{tag}_goal_ob'])
    e, x, y = gold[f'{tag}_reset_action']
    ob = env.reset(goal[0, 0], int(e), int(x), int(y), rr[-1])
    assert np.array_equal(ob, gold[f'{tag}_reset_ob'])
    for t, a in enumerate(gold[f'{tag}_actions']):
        ob = env.step(int(a), gold[f'{tag}_step_rand'][t])
        assert np.array_equal(ob, gold[f'{tag}_obs'][t]), t
    assert np.array_equal(env.w[0], gold[f'{tag}_final_world'])


def test_blur_order_matches_reference_conv2d():
    """The velocity blur's einsum summation order, against the reference conv2d
    run here (tests/golden/make_golden_powder.py imports it)."""
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(__file__), 'golden'))
    try:
        import make_golden_powder as m

        sim, _ = m.reference_modules()
    except Exception:  # reference absent (GPU box): the golden traces above still pin it
        pytest.skip('reference sources not available here')
    rng = np.random.RandomState(3)
    x = (rng.normal(0, 3, (2, 1, 32, 32)) * (rng.rand(2, 1, 32, 32) < 0.6)).astype(np.float32)
    ref = sim.conv2d(x, np.ones((1, 1, 3, 3), np.float32) / 18, padding=1)[:, 0]
    assert np.array_equal(orc.blur(x[:, 0]), ref)


@pytest.mark.parametrize('ne', [2, 5, 8])
def test_task_tables_match_reference(gold, ne):
    from ogbench_amd.powder_tasks import task_names, task_sequences, task_tols

    for t, (seq, tol, name) in enumerate(zip(task_sequences(ne), task_tols(ne), task_names(ne))):
        assert np.array_equal(np.array(seq, np.int64), gold[f'tasks{ne}_{t + 1}_seq']), (ne, t)
        assert tol == int(gold[f'tasks{ne}_{t + 1}_tol']) and name == str(gold[f'tasks{ne}_{t + 1}_name'])
