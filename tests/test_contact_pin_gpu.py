"""GPU: maze_step/point_physics contact dynamics (through the C-ABI) against the
independent MuJoCo-formulation model of tests/mjmodel_np.py (see
tests/test_contact_pin.py): the straight one-face push-out and the symmetric
inside corner in closed form to 1e-12, and the enumeration model on contact
states spread over pointmaze-large to 1e-10 (north_star allows 1e-5)."""

import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import mjmodel_np as mj  # noqa: E402
import test_contact_pin as cp  # noqa: E402

import ogbench_amd  # noqa: E402

pytestmark = pytest.mark.gpu


def _physics(gpu, q, f64=True):
    env = ogbench_amd.MazeEnv('point', 'large', num_envs=1, device=gpu)
    q = torch.tensor(np.asarray(q, np.float64))
    a = torch.zeros(q.shape[0], 2, dtype=torch.float64 if f64 else torch.float32)
    out, contact = env.physics(q, a)
    return out.cpu().numpy(), contact.cpu().numpy()


def test_kernel_matches_closed_forms(gpu):
    cases = cp.pushout_cases() + cp.corner_cases()
    q0 = np.array([c[0] for c in cases])
    exp = np.array([c[1] for c in cases])
    # the same states inside a wave of 64 lanes with free lanes mixed in
    # (every lane of a wave with a contact lane runs the contact loop)
    for got, contact in (_physics(gpu, q0), _physics(gpu, np.concatenate([q0, np.tile([[0.0, 0.0]], (64, 1))]))):
        assert contact[:len(q0)].all()
        err = np.abs(got[:len(q0)] - exp).max()
        assert err <= cp.TOL_CLOSED, err
    # pushed straight out: no tangential motion at all
    npush = len(cp.DEPTHS)
    got, _ = _physics(gpu, q0[:npush])
    assert np.array_equal(got[:, 1], q0[:npush, 1])


def test_kernel_matches_mujoco_model_on_contact_states(gpu):
    boxes = mj.wall_boxes(cp.maze_map())
    q = cp.random_contact_states(400, seed=3)
    got, contact = _physics(gpu, q)
    assert contact.all()
    exp = np.array([mj.point_step(x, boxes)[0] for x in q])
    err = np.abs(got - exp).max()
    assert err <= cp.TOL_MODEL, err


def test_step_kernel_matches_mujoco_model(gpu):
    """The env step (maze_step_kernel) from restored contact states: the
    post-step observation is the model's qpos after qpos + 0.2 a (f64 actions
    of 0, so the action product is exact)."""
    boxes = mj.wall_boxes(cp.maze_map())
    q = cp.random_contact_states(128, seed=5)
    n = len(q)
    env = ogbench_amd.make('pointmaze-large-v0', num_envs=n, device=gpu)
    env.reset(seed=0)
    sd = env.state_dict()
    sd['qpos'] = torch.tensor(q, device=gpu)
    sd['goal'] = torch.full_like(sd['qpos'], 1e3)  # no success, no termination
    sd['elapsed'].zero_()
    env.load_state_dict(sd)
    obs, _, term, trunc, _ = env.step(torch.zeros(n, 2, dtype=torch.float64, device=gpu))
    exp = np.array([mj.point_step(x, boxes)[0] for x in q])
    assert not term.any() and not trunc.any()
    err = np.abs(obs.cpu().numpy() - exp).max()
    assert err <= cp.TOL_MODEL, err
