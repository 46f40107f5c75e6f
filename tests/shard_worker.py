"""Sharded-rollout workload shared by the sharding test (tests/test_shard_gpu.py).

Run as a script it is ONE rank of a gloo job (RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT from the environment; every rank uses cuda:0, the ranks share the
one GPU of the test box).  Each rank steps its contiguous block of the job's
envs (``ogbench_amd.sharding.shard``) with a handle created at that block's
``env_base``, all-gathers the eval counters over the process group and saves
its per-env outputs to ``<out>/rank<r>.npz``.  Imported, ``run_maze`` /
``run_powder`` give the single-process (G = 1) run the test compares against.

Workloads:
  pointmaze-large, auto-reset, max_episode_steps 250 (short tasks reach the goal), task_id = i%5+1 (global
  i), Philox reset noise under one shared seed, expert actions (on-device
  oracle-subgoal policy + Philox noise keyed by the global env index);
  powderworld-easy 32x32, auto-reset, random actions with invalid values (the
  random replacement draws are Philox keyed by the global env index).
"""

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

MAZE_TOTAL, MAZE_STEPS, SEED = 4096, 300, 0xC0FFEE
POWDER_TOTAL, POWDER_STEPS = 128, 30


def run_maze(base, n, dev, total=MAZE_TOTAL, steps=MAZE_STEPS, seed=SEED):
    import torch

    import ogbench_amd
    from ogbench_amd.evaluation import accumulate, env_task_ids

    env = ogbench_amd.make('pointmaze-large-v0', num_envs=n, device=dev, auto_reset=True, max_episode_steps=250,
                           env_base=base)
    task = (torch.arange(base, base + n, dtype=torch.int32) % 5 + 1).to(dev)
    obs0, info = env.reset(seed=seed, options=dict(task_id=task))
    out = dict(obs0=obs0.cpu().numpy().copy(), goal0=info['goal'].cpu().numpy().copy())
    rec = {k: [] for k in ('obs', 'reward', 'terminated', 'truncated', 'success')}
    counters = torch.zeros(env.num_tasks, 2, dtype=torch.int64, device=dev)
    remaining = torch.full((n,), 1 << 30, dtype=torch.int32, device=dev)
    tid = env_task_ids(env)
    for t in range(steps):
        a = env.expert_action(noise=0.2, seed=seed)
        o, r, te, tr, inf = env.step(a)
        accumulate(counters, inf['success'].view(torch.uint8), te.view(torch.uint8), tr.view(torch.uint8), tid,
                   remaining)
        for k, v in (('obs', o), ('reward', r), ('terminated', te), ('truncated', tr), ('success', inf['success'])):
            rec[k].append(v.cpu().numpy().copy())
    out.update({k: np.stack(v) for k, v in rec.items()})
    out['qpos'] = env.get_xy().cpu().numpy()
    out['counters'] = counters.cpu().numpy()
    env.close()
    return out, counters


def run_powder(base, n, dev, total=POWDER_TOTAL, steps=POWDER_STEPS, seed=SEED):
    import torch

    import ogbench_amd

    env = ogbench_amd.make('powderworld-easy-v0', num_envs=n, device=dev, world_size=32, auto_reset=True,
                           max_episode_steps=12, env_base=base)
    task = torch.arange(base, base + n, dtype=torch.int32) % 5 + 1
    obs0, _ = env.reset(seed=seed, options=dict(task_id=task))
    out = dict(obs0=obs0.cpu().numpy().copy())
    g = torch.Generator().manual_seed(11)
    acts = torch.randint(-2, 10, (steps, total), generator=g, dtype=torch.int32)  # invalid values included
    rec = {k: [] for k in ('obs', 'reward', 'terminated', 'truncated', 'success')}
    for t in range(steps):
        o, r, te, tr, inf = env.step(acts[t, base:base + n].to(dev))
        for k, v in (('obs', o), ('reward', r), ('terminated', te), ('truncated', tr), ('success', inf['success'])):
            rec[k].append(v.cpu().numpy().copy())
    out.update({k: np.stack(v) for k, v in rec.items()})
    env.close()
    return out


def main():
    import torch
    import torch.distributed as dist

    from ogbench_amd.evaluation import gather_counters
    from ogbench_amd.sharding import shard

    out_dir = sys.argv[1]
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    dist.init_process_group('gloo', rank=rank, world_size=world)
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    base, n = shard(MAZE_TOTAL, world, rank)
    maze, counters = run_maze(base, n, dev)
    total, per_rank = gather_counters(counters)
    maze['gathered_total'] = total.cpu().numpy()
    maze['gathered_per_rank'] = per_rank.cpu().numpy()
    pbase, pn = shard(POWDER_TOTAL, world, rank)
    powder = run_powder(pbase, pn, dev)
    np.savez(os.path.join(out_dir, f'rank{rank}.npz'), base=base, n=n, pbase=pbase, pn=pn,
             **{f'maze_{k}': v for k, v in maze.items()}, **{f'powder_{k}': v for k, v in powder.items()})
    dist.barrier()
    dist.destroy_process_group()
    print(f'rank {rank}: envs [{base}, {base + n}) done', flush=True)


if __name__ == '__main__':
    main()
