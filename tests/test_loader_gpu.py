"""GPU: HBM dataset loader (compact / regular), relabel and oracle reps against
the reference's own load_dataset / relabel_dataset / add_oracle_reps outputs
(tests/golden/gc_golden.npz load_*, relabel_golden.npz).  Bit-exact."""

import os

import numpy as np
import pytest
import torch

import ogbench_amd
from ogbench_amd.utils import add_oracle_reps, load_dataset, make_env_and_datasets, relabel_dataset

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), 'golden')


@pytest.fixture(scope='module')
def raw_npz(tmp_path_factory):
    g = np.load(os.path.join(G, 'gc_golden.npz'))
    raw = {k[4:]: g[k] for k in g.files if k.startswith('raw_')}
    d = tmp_path_factory.mktemp('ds')
    path = str(d / 'pointmaze-large-navigate-v0.npz')
    np.savez(path, **raw)
    np.savez(path.replace('.npz', '-val.npz'), **{k: v[:200] for k, v in raw.items()})
    return path, g


@pytest.mark.parametrize('compact', [True, False])
def test_load_dataset_matches_reference(gpu, raw_npz, compact):
    path, g = raw_npz
    tag = 'compact' if compact else 'regular'
    exp = {k[len(f'load_{tag}_'):]: g[k] for k in g.files if k.startswith(f'load_{tag}_')}
    d = load_dataset(path, compact_dataset=compact, add_info=True, device=gpu)
    assert list(d) == list(exp)
    for k, v in exp.items():
        got = d[k].cpu().numpy()
        assert got.dtype == v.dtype and np.array_equal(got, v), k


class _StubEnv:
    """The attributes relabel_dataset / add_oracle_reps read (maze branch)."""

    def __init__(self, goal):
        self.unwrapped = self
        self._reward_task_id = 2
        self._goal_tol = 1.0
        self.cur_goal_xy = np.asarray(goal)

    def reset(self):
        return None


@pytest.mark.parametrize('qdt', ['f32', 'f64'])
def test_relabel_and_oracle_reps_match_reference(gpu, qdt):
    g = np.load(os.path.join(G, 'relabel_golden.npz'))
    ds = {'qpos': torch.tensor(g[f'{qdt}_qpos'], device=gpu)}
    env = _StubEnv(g[f'{qdt}_goal'])
    relabel_dataset('pointmaze-large-singletask-task2-v0', env, ds)
    add_oracle_reps('pointmaze-large-oraclerep-v0', env, ds)
    for k in ('rewards', 'masks', 'oracle_reps'):
        got = ds[k].cpu().numpy()
        assert got.dtype == g[f'{qdt}_{k}'].dtype and np.array_equal(got, g[f'{qdt}_{k}']), k
    assert (g[f'{qdt}_masks'] == 0).sum() > 50  # the fixture really has successes


def test_make_env_and_datasets_singletask_and_oraclerep(gpu, raw_npz):
    path, _ = raw_npz
    env, train, val = make_env_and_datasets('pointmaze-large-navigate-singletask-task2-v0', dataset_path=path,
                                            compact_dataset=True, num_envs=4, device=gpu)
    assert isinstance(env, ogbench_amd.MazeEnv) and env._reward_task_id == 2
    assert set(train) == {'observations', 'actions', 'terminals', 'valids', 'rewards', 'masks'}
    assert train['rewards'].dtype == torch.float32 and len(val['rewards']) == 200
    # rewards follow the task-2 goal (exact cell centre: no goal noise in single-task mode)
    raw = np.load(path)
    goal = np.array(env.task_infos[1]['goal_xy'])
    q = raw['qpos'].astype(np.float64)
    succ = (np.sqrt((q[:, 0] - goal[0]) ** 2 + (q[:, 1] - goal[1]) ** 2) <= 1.0).astype(np.float32)
    assert np.array_equal(train['rewards'].cpu().numpy(), succ - 1.0)
    env2, tr2, _ = make_env_and_datasets('pointmaze-large-navigate-oraclerep-v0', dataset_path=path,
                                         num_envs=2, device=gpu)
    assert env2._use_oracle_rep and 'next_observations' in tr2
    assert tr2['oracle_reps'].shape == (tr2['observations'].shape[0], 2)
    e3 = make_env_and_datasets('powderworld-easy-play-v0', env_only=True, num_envs=2, device=gpu)
    assert isinstance(e3, ogbench_amd.PowderworldEnv)
