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
  random replacement draws are Philox keyed by the global env index);
  antmaze-large wrapper (BASELINE configs[4]), auto-reset with caller reset
  states and Philox bodies, goal observations from caller goal states.
"""

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

MAZE_TOTAL, MAZE_STEPS, SEED = 4096, 300, 0xC0FFEE
POWDER_TOTAL, POWDER_STEPS = 128, 30
ANT_TOTAL, ANT_STEPS = 1024, 60


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


def run_ant(base, n, dev, total=ANT_TOTAL, steps=ANT_STEPS, seed=SEED):
    """antmaze-large wrapper: post-physics states from a job-global generator
    (sliced to this block), even global envs walking toward their goal (goal
    ends + auto-reset), the rest wandering (TimeLimit ends); auto-reset bodies
    from the caller's reset states on even steps and Philox on odd steps."""
    import torch

    import ogbench_amd
    from ogbench_amd.evaluation import accumulate, env_task_ids

    env = ogbench_amd.MazeEnv('ant', 'large', num_envs=n, device=dev, auto_reset=True, max_episode_steps=25,
                              env_base=base)
    task = (torch.arange(base, base + n, dtype=torch.int32) % 5 + 1).to(dev)
    g = torch.Generator().manual_seed(5)
    gstates = torch.randn(total, 29, generator=g, dtype=torch.float64)
    obs0, info = env.reset(seed=seed, options=dict(task_id=task, goal_states=gstates[base:base + n].to(dev)))
    out = dict(obs0=obs0.cpu().numpy().copy(), goal0=info['goal'].cpu().numpy().copy())
    qn = torch.randn(steps, total, 15, generator=g, dtype=torch.float64)
    vn = torch.randn(steps, total, 14, generator=g, dtype=torch.float64)
    rs = torch.randn(steps, total, 29, generator=g, dtype=torch.float64)
    walk = (torch.arange(base, base + n) % 2 == 0).to(dev)[:, None]
    rec = {k: [] for k in ('obs', 'final_obs', 'reward', 'terminated', 'truncated', 'success')}
    counters = torch.zeros(env.num_tasks, 2, dtype=torch.int64, device=dev)
    remaining = torch.full((n,), 1 << 30, dtype=torch.int32, device=dev)
    tid = env_task_ids(env)
    for t in range(steps):
        xy, goal = env.get_xy(), env.cur_goal_xy
        q = qn[t, base:base + n].to(dev)
        step_xy = torch.where(walk, (goal - xy).clamp(-1.5, 1.5), 0.05 * q[:, :2])
        q[:, :2] = xy + step_xy
        reset_states = rs[t, base:base + n].to(dev) if t % 2 == 0 else None
        o, r, te, tr, inf = env.wrap_step(q, vn[t, base:base + n].to(dev), reset_states=reset_states)
        accumulate(counters, inf['success'].view(torch.uint8), te.view(torch.uint8), tr.view(torch.uint8), tid,
                   remaining)
        done = (te | tr).cpu().numpy()
        fo = np.where(done[:, None], inf['final_observation'].cpu().numpy(), 0.0)
        for k, v in (('obs', o), ('reward', r), ('terminated', te), ('truncated', tr), ('success', inf['success'])):
            rec[k].append(v.cpu().numpy().copy())
        rec['final_obs'].append(fo)
    out.update({k: np.stack(v) for k, v in rec.items()})
    bq, bv = env.body_state()
    out['body'] = np.concatenate([bq.cpu().numpy(), bv.cpu().numpy()], 1)
    out['goal_xy'] = env.cur_goal_xy.cpu().numpy()
    out['counters'] = counters.cpu().numpy()
    env.close()
    return out, counters


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
    abase, an = shard(ANT_TOTAL, world, rank)
    ant, acounters = run_ant(abase, an, dev)
    atotal, aper_rank = gather_counters(acounters)
    ant['gathered_total'] = atotal.cpu().numpy()
    ant['gathered_per_rank'] = aper_rank.cpu().numpy()
    np.savez(os.path.join(out_dir, f'rank{rank}.npz'), base=base, n=n, pbase=pbase, pn=pn, abase=abase, an=an,
             **{f'maze_{k}': v for k, v in maze.items()}, **{f'powder_{k}': v for k, v in powder.items()},
             **{f'ant_{k}': v for k, v in ant.items()})
    dist.barrier()
    dist.destroy_process_group()
    print(f'rank {rank}: envs [{base}, {base + n}) done', flush=True)


if __name__ == '__main__':
    main()
