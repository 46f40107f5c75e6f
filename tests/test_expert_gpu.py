"""GPU: the point-maze expert (expert_action_kernel), set_goal and the
on-device collector, against the oracle restatement (bit-exact with injected
draws) and distributional checks for the Philox draws."""

import numpy as np
import pytest
import torch

import ogbench_amd
from ogbench_amd.datagen import collect_locomaze, maze_cells
from oracle import locomaze as orc

pytestmark = pytest.mark.gpu


def _states(maze, n, rng):
    mp, _ = orc.tables(maze)
    cells = np.argwhere(mp == 0)
    c = cells[rng.randint(len(cells), size=n)]
    xy = np.stack([c[:, 1] * 4.0 - 4 + rng.uniform(-2, 2, n), c[:, 0] * 4.0 - 4 + rng.uniform(-2, 2, n)], 1)
    g = cells[rng.randint(len(cells), size=n)]
    goal = np.stack([g[:, 1] * 4.0 - 4 + rng.uniform(-1, 1, n), g[:, 0] * 4.0 - 4 + rng.uniform(-1, 1, n)], 1)
    return xy, goal


@pytest.mark.parametrize('maze', ['medium', 'large', 'giant'])
def test_expert_action_injected_matches_oracle(gpu, maze):
    rng = np.random.RandomState(5)
    xy, goal = _states(maze, 20000, rng)
    normal = rng.normal(0, 0.2, xy.shape)
    env = ogbench_amd.MazeEnv('point', maze, num_envs=1, device=gpu)
    got = env.expert_action(noise=0.2, normal=torch.tensor(normal), start_xy=torch.tensor(xy),
                            goal_xy=torch.tensor(goal)).cpu().numpy()
    assert np.array_equal(got, orc.expert_action(maze, xy, goal, normal))


def test_expert_action_philox_noise_statistics(gpu):
    rng = np.random.RandomState(6)
    xy, goal = _states('large', 200000, rng)
    env = ogbench_amd.MazeEnv('point', 'large', num_envs=1, device=gpu)
    a = env.expert_action(noise=0.2, start_xy=torch.tensor(xy), goal_xy=torch.tensor(goal), seed=3).cpu().numpy()
    clean = orc.expert_action('large', xy, goal, np.zeros_like(xy))
    # components whose clean value is far from the clip bounds carry the raw noise
    # (clipping beyond 0.7 = 3.5 sigma is negligible)
    d = (a - clean)[np.abs(clean) < 0.3]
    assert d.size > 50000
    assert abs(d.mean()) < 2e-3 and abs(d.std() - 0.2) < 3e-3
    b = env.expert_action(noise=0.2, start_xy=torch.tensor(xy), goal_xy=torch.tensor(goal), seed=3).cpu().numpy()
    assert not np.array_equal(a, b)  # successive calls draw fresh noise


def test_expert_reads_env_state(gpu):
    env = ogbench_amd.make('pointmaze-large-v0', num_envs=512, device=gpu)
    env.reset(seed=1)
    z = torch.zeros(512, 2, dtype=torch.float64, device=gpu)
    a = env.expert_action(normal=z).cpu().numpy()
    exp = orc.expert_action('large', env.get_xy().cpu().numpy(), env.cur_goal_xy.cpu().numpy(), np.zeros((512, 2)))
    assert np.array_equal(a, exp)


def test_set_goal_injected_noise(gpu):
    n = 256
    env = ogbench_amd.make('pointmaze-large-v0', num_envs=n, device=gpu)
    env.reset(seed=2)
    before = env.cur_goal_xy.cpu().numpy()
    rng = np.random.RandomState(3)
    _, vert = maze_cells(env.maze_map)
    ij = vert[rng.randint(len(vert), size=n)]
    r = rng.uniform(-1, 1, (n, 2))
    mask = rng.rand(n) < 0.5
    env.set_goal(torch.tensor(ij), mask=torch.tensor(mask), noise=torch.tensor(r))
    got = env.cur_goal_xy.cpu().numpy()
    exp_x = (ij[:, 1] * 4.0 - 4) + r[:, 0] * 4.0 / 4
    exp_y = (ij[:, 0] * 4.0 - 4) + r[:, 1] * 4.0 / 4
    assert np.array_equal(got[mask], np.stack([exp_x, exp_y], 1)[mask])
    assert np.array_equal(got[~mask], before[~mask])


def test_collect_navigate(gpu):
    N, T = 64, 120
    d = collect_locomaze('pointmaze-medium-v0', 'navigate', num_envs=N, max_episode_steps=T, noise=0.2, seed=1,
                         device=gpu)
    obs, act, term = d['observations'].cpu().numpy(), d['actions'].cpu().numpy(), d['terminals'].cpu().numpy()
    assert obs.shape == (N * T, 2) and obs.dtype == np.float32 and term.dtype == np.bool_
    assert np.array_equal(np.nonzero(term)[0], np.arange(T - 1, N * T, T))
    assert np.abs(act).max() <= 1.0
    # within a trajectory consecutive positions differ by at most the step size (0.2 per axis + contact)
    o = obs.reshape(N, T, 2)
    assert np.abs(np.diff(o, axis=1)).max() < 0.5
