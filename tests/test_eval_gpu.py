"""GPU: eval counters kernel (ogbx_eval_accumulate) and batched evaluate()."""

import numpy as np
import pytest
import torch

import ogbench_amd
from ogbench_amd.evaluation import accumulate, evaluate

pytestmark = pytest.mark.gpu


def test_accumulate_matches_host_recount(gpu):
    rng = np.random.RandomState(0)
    n, T, steps = 100_000, 5, 12
    task = rng.randint(1, T + 1, n).astype(np.int32)
    rem = rng.randint(0, 3, n).astype(np.int32)
    counters = torch.zeros(T, 2, dtype=torch.int64, device=gpu)
    remaining = torch.tensor(rem, device=gpu)
    exp = np.zeros((T, 2), np.int64)
    for _ in range(steps):
        s = rng.rand(n) < 0.3
        te = rng.rand(n) < 0.2
        tr = rng.rand(n) < 0.1
        accumulate(counters, torch.tensor(s, device=gpu).view(torch.uint8), torch.tensor(te, device=gpu).view(torch.uint8),
                   torch.tensor(tr, device=gpu).view(torch.uint8), torch.tensor(task, device=gpu), remaining)
        done = (te | tr) & (rem > 0)
        np.add.at(exp[:, 0], task[done] - 1, s[done].astype(np.int64))
        np.add.at(exp[:, 1], task[done] - 1, 1)
        rem = rem - done
    assert np.array_equal(counters.cpu().numpy(), exp)
    assert np.array_equal(remaining.cpu().numpy(), rem)


def test_evaluate_greedy_pointmaze_arena(gpu):
    env = ogbench_amd.make('pointmaze-arena-v0', num_envs=2048, device=gpu, auto_reset=True, max_episode_steps=200)

    def greedy(obs, goal):
        return torch.clamp((goal - obs) / 0.2, -1, 1).to(torch.float32)

    metrics, total, local = evaluate(greedy, env, episodes_per_env=2, seed=3)
    assert total[:, 1].sum().item() == 2048 * 2
    assert metrics['evaluation/overall_success'] == 1.0


def test_evaluate_counts_every_episode_powder(gpu):
    env = ogbench_amd.make('powderworld-easy-v0', num_envs=500, device=gpu, auto_reset=True, max_episode_steps=6)
    gen = torch.Generator(device=gpu)
    gen.manual_seed(0)

    def rand_policy(obs, goal):
        return torch.randint(0, 8, (obs.shape[0],), device=gpu, generator=gen, dtype=torch.int32)

    metrics, total, _ = evaluate(rand_policy, env, episodes_per_env=3, seed=1)
    t = total.cpu().numpy()
    assert t[:, 1].sum() == 1500
    assert np.array_equal(t[:, 1], np.bincount(np.arange(500) % 5, minlength=5) * 3)
    assert set(metrics) == {f'evaluation/{ti["task_name"]}_success' for ti in env.task_infos} | {
        'evaluation/overall_success'}


def test_rccl_cabi_allgather_single_rank(gpu):
    """The C-ABI RCCL communicator (ogbx_comm_create / ogbx_eval_allgather) on
    one rank: the gather is the identity, and gather_counters(comm=...) sums it."""
    import torch

    from ogbench_amd.evaluation import RcclComm, comm_unique_id, gather_counters

    uid = comm_unique_id()
    assert len(uid) == 128
    comm = RcclComm(1, 0, gpu, uid)
    c = torch.arange(10, dtype=torch.int64, device=gpu).view(5, 2) * 7 + 3
    out = comm.allgather(c)
    assert out.shape == (1, 5, 2) and torch.equal(out[0], c)
    total, per_rank = gather_counters(c, comm=comm)
    assert torch.equal(total, c) and per_rank.shape == (1, 5, 2)
    comm.close()
