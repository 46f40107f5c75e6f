"""CPU: env sharding -- the block layout, global-index Philox keying
(checked on the oracle restatement, which keys its auto-reset draws exactly as
libogbx does) and the world-size-2 gloo path: two ranks each step half of the
envs with their global ``env_base`` and all-gather eval counters that equal the
single-process run's."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ogbench_amd.evaluation import gather_counters
from ogbench_amd.sharding import rank_of_env, shard
from oracle import locomaze as orc

SEED = 0xC0FFEE
N, K = 512, 160


def test_shard_blocks_cover_envs_contiguously():
    assert [shard(65536, 8, r) for r in range(8)] == [(r * 8192, 8192) for r in range(8)]
    assert [shard(65536, 1, 0)] == [(0, 65536)]
    # uneven totals: 64-aligned blocks, the last one takes the rest
    blocks = [shard(1000, 3, r) for r in range(3)]
    assert blocks == [(0, 384), (384, 384), (768, 232)]
    for i in (0, 383, 384, 767, 768, 999):
        r = rank_of_env(i, 1000, 3)
        b, n = blocks[r]
        assert b <= i < b + n
    with pytest.raises(ValueError):
        shard(100, 4, 2)  # 64-aligned blocks leave rank 2 empty
    with pytest.raises(ValueError):
        shard(10, 2, 2)


def _run(base, n, acts):
    tid = (np.arange(base, base + n) % 5 + 1).astype(np.int32)
    st = orc.reset('large', tid, orc.reset_draws(n, SEED, env_base=base), max_steps=40)
    key = orc.philox_key(SEED, orc.TAG_MAZE_RESET)
    out = orc.step('large', st, np.ascontiguousarray(acts[:, base:base + n]), auto_reset=1, key=key,
                   env_base=base)
    cnt = np.zeros((5, 2), np.int64)
    done = (out['terminated'] | out['truncated']).astype(bool)
    for t in range(5):
        m = done & (tid[None, :] == t + 1)
        cnt[t] = (out['success'][m].sum(), m.sum())
    return out, st, cnt


def _actions():
    return np.random.RandomState(3).uniform(-1, 1, (K, N, 2)).astype(np.float32)


def test_oracle_shards_reproduce_single_run():
    acts = _actions()
    ref, ref_st, ref_cnt = _run(0, N, acts)
    assert ref['truncated'].sum() > 0  # auto-resets (Philox draws) happen
    tot = np.zeros_like(ref_cnt)
    for r in range(4):
        b, n = shard(N, 4, r)
        out, st, cnt = _run(b, n, acts)
        for k in ('obs', 'reward', 'terminated', 'truncated', 'success'):
            assert np.array_equal(out[k], ref[k][:, b:b + n]), k
        assert np.array_equal(st['qpos'], ref_st['qpos'][b:b + n])
        tot += cnt
    assert np.array_equal(tot, ref_cnt)
    # keying by the LOCAL index (the round-1 behaviour) would break it
    out, _, _ = _run(0, N // 2, acts[:, N // 2:].copy())
    assert not np.array_equal(out['obs'], ref['obs'][:, N // 2:])


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        b, n = shard(N, world, rank)
        res, _, cnt = _run(b, n, _actions())
        total, per_rank = gather_counters(torch.tensor(cnt))
        out[rank] = (b, n, res['obs'].tobytes(), total.numpy().tolist(), per_rank.numpy().tolist())
    finally:
        dist.destroy_process_group()


def test_gloo_world2_sharded_eval_equals_single_run():
    world = 2
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    ref, _, ref_cnt = _run(0, N, _actions())
    for r in range(world):
        b, n, obs, total, per_rank = res[r]
        got = np.frombuffer(obs, np.float64).reshape(K, n, 2)
        assert np.array_equal(got, ref['obs'][:, b:b + n])
        assert np.array_equal(np.array(total), ref_cnt)
        assert np.array_equal(np.array(per_rank).sum(0), ref_cnt)

