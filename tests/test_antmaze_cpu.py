"""CPU: the antmaze wrapper oracle (oracle/antmaze_np.py) pinned against the
fixture tests/golden/antmaze_golden.npz, generated from the reference's own
MazeEnv/AntEnv methods by make_golden_ant.py: reset ob and goal from the
recorded draws, then 40 wrapper steps on given post-physics states (ob,
success with the fma-rounded 2-norm, terminated, reward, TimeLimit) for
success_timing 'post' and 'pre'.  The GPU kernel is held to the same fixture
in tests/test_antmaze_gpu.py."""

import os

import numpy as np
import pytest

from oracle import antmaze_np as am

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'antmaze_golden.npz')


@pytest.mark.parametrize('timing', ['post', 'pre'])
def test_oracle_matches_reference_fixture(timing):
    d = np.load(GOLDEN)
    g = {k[len(timing) + 1:]: d[k] for k in d.files if k.startswith(timing + '_')}
    ob0, goal = am.reset_obs(g['task'], g['noise'], g['body_draws'])
    assert np.array_equal(ob0, g['reset_obs'])
    assert np.array_equal(goal, g['reset_goal'])
    assert np.array_equal(am.goal_obs(goal, g['goal_states']), g['reset_goal_ob'])
    b = am.Batch(g['task'], g['noise'], g['body_draws'], max_steps=int(d['max_episode_steps']), timing=timing)
    for k in range(g['obs'].shape[0]):
        obs, rew, term, trunc, succ = b.step(g['qpos_post'][k], g['qvel_post'][k])
        assert np.array_equal(obs, g['obs'][k])
        assert np.array_equal(succ, g['success'][k].astype(bool))
        assert np.array_equal(term, g['terminated'][k].astype(bool))
        assert np.array_equal(trunc, g['truncated'][k].astype(bool))
        assert np.array_equal(rew, g['reward'][k])
    assert g['success'].sum() > 50


def test_within_decides_boundary_exactly():
    # pairs whose plain sum and fma-rounded sum fall on opposite sides of 0.5
    rng = np.random.RandomState(0)
    ang = rng.uniform(0, 2 * np.pi, 20000)
    r = 0.5 + rng.normal(0, 1, 20000) * 1e-16
    dx, dy = r * np.cos(ang), r * np.sin(ang)
    from fractions import Fraction

    exact = np.array([np.sqrt(float(Fraction(float(y)) ** 2 + Fraction(float(x * x)))) <= 0.5
                      for x, y in zip(dx, dy)])
    assert np.array_equal(am.within(dx, dy), exact)
