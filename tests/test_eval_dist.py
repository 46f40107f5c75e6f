"""CPU: the eval reduction's collective and metric summary (gloo, world_size 2).

Reference metric: impls/main.py:251-258 (per-task mean of the final-step
success; overall = mean over tasks)."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ogbench_amd.evaluation import gather_counters, summarize


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_counters(rank, T=5):
    rng = np.random.RandomState(100 + rank)
    cnt = rng.randint(1, 40, T)
    succ = np.minimum(rng.randint(0, 40, T), cnt)
    return np.stack([succ, cnt], 1).astype(np.int64)


def _worker(rank, world, port, out):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        local = torch.tensor(_rank_counters(rank))
        total, stacked = gather_counters(local)
        out[rank] = (total.numpy().tolist(), stacked.numpy().tolist(), summarize(total))
    finally:
        dist.destroy_process_group()


def test_gather_counters_gloo_world2():
    world = 2
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    exp_total = sum(_rank_counters(r) for r in range(world))
    for r in range(world):
        total, stacked, metrics = res[r]
        assert np.array_equal(np.array(total), exp_total)
        assert np.array_equal(np.array(stacked), np.stack([_rank_counters(q) for q in range(world)]))
        assert metrics == res[0][2]  # every rank derives the same metrics
    per_task = exp_total[:, 0] / exp_total[:, 1]
    m0 = res[0][2]
    assert m0['evaluation/overall_success'] == pytest.approx(float(np.mean(per_task)), abs=0)
    for t in range(5):
        assert m0[f'evaluation/task{t + 1}_success'] == per_task[t]


def test_gather_without_group_is_identity():
    c = torch.tensor([[3, 4], [0, 2]], dtype=torch.int64)
    total, stacked = gather_counters(c)
    assert torch.equal(total, c) and stacked.shape == (1, 2, 2)


def test_summarize_names_and_empty_tasks():
    c = np.array([[1, 2], [0, 0], [3, 3]])
    infos = [dict(task_name='a'), dict(task_name='b'), dict(task_name='c')]
    m = summarize(c, infos)
    assert m == {'evaluation/a_success': 0.5, 'evaluation/c_success': 1.0, 'evaluation/overall_success': 0.75}
