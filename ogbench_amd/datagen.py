"""On-device data collection for point mazes (no host round trips per step).

Batched counterpart of data_gen_scripts/generate_locomaze.py (hliuson/ogbench)
for the point agent, whose actor is the oracle subgoal direction (:44-46):
every step is one ``expert_action`` launch (BFS-table subgoal, normalised
direction, Gaussian action noise, clip) and one ``step`` launch; 'navigate'
resamples the goal of the envs that reached theirs (``set_goal``).  N envs run
their episodes in lock step (terminate_at_goal=False, so every episode lasts
max_episode_steps), and the result is laid out trajectory-major exactly like
the reference's saved arrays (observations / actions / qpos float32,
terminals bool).  qvel (info only) is not recorded.
"""

from __future__ import annotations

import numpy as np


def _torch():
    import torch

    return torch


def maze_cells(maze_map):
    """(all empty cells, vertex cells) as in generate_locomaze.py:62-90."""
    all_cells, vertex_cells = [], []
    m = maze_map
    for i in range(m.shape[0]):
        for j in range(m.shape[1]):
            if m[i, j] != 0:
                continue
            all_cells.append((i, j))
            if m[i - 1, j] == 0 and m[i + 1, j] == 0 and m[i, j - 1] == 1 and m[i, j + 1] == 1:
                continue
            if m[i, j - 1] == 0 and m[i, j + 1] == 0 and m[i - 1, j] == 1 and m[i + 1, j] == 1:
                continue
            vertex_cells.append((i, j))
    return np.array(all_cells, np.int32), np.array(vertex_cells, np.int32)


def collect_locomaze(env_name='pointmaze-large-v0', dataset_type='navigate', num_envs=1024, num_rounds=1,
                     max_episode_steps=1001, noise=0.2, seed=0, device=None):
    """Collect num_envs x num_rounds episodes of max_episode_steps transitions.

    Returns a dict of device tensors (trajectory-major): observations f32
    [E*T, 2], actions f32 [E*T, 2], terminals bool [E*T], qpos f32 [E*T, 2]."""
    torch = _torch()
    from .registry import make

    assert dataset_type in ('path', 'navigate'), 'point-maze collection supports path and navigate'
    env = make(env_name, num_envs=num_envs, device=device, terminate_at_goal=False,
               max_episode_steps=max_episode_steps, seed=seed)
    if env._loco_env_type != 'point':
        raise NotImplementedError('only the point agent has an oracle actor (ant/humanoid experts are SAC nets)')
    dev = env.device
    all_cells, vertex_cells = maze_cells(env.maze_map)
    all_t = torch.as_tensor(all_cells, device=dev)
    vert_t = torch.as_tensor(vertex_cells, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(int(seed))
    T, N = int(max_episode_steps), int(num_envs)
    obs = torch.empty(num_rounds, T, N, 2, dtype=torch.float32, device=dev)
    act = torch.empty_like(obs)
    qpos = torch.empty_like(obs)
    term = torch.empty(num_rounds, T, N, dtype=torch.bool, device=dev)
    unit, off = env._maze_unit, env._offset_x
    for r in range(num_rounds):
        init_ij = all_t[torch.randint(len(all_t), (N,), device=dev, generator=gen)]
        goal_ij = vert_t[torch.randint(len(vert_t), (N,), device=dev, generator=gen)]
        task_xy = torch.stack([init_ij[:, 1] * unit - off, init_ij[:, 0] * unit - off,
                               goal_ij[:, 1] * unit - off, goal_ij[:, 0] * unit - off], 1).to(torch.float64)
        ob, _ = env.reset(seed=seed * 1000003 + r, options=dict(task_info=task_xy))
        for t in range(T):
            a = env.expert_action(noise=noise)
            obs[r, t] = ob
            qpos[r, t] = ob  # prev_qpos of a point agent is its observation
            act[r, t] = a
            ob, _, terminated, truncated, info = env.step(a)
            term[r, t] = terminated | truncated
            if dataset_type == 'navigate':
                new_ij = vert_t[torch.randint(len(vert_t), (N,), device=dev, generator=gen)]
                env.set_goal(new_ij, mask=info['success'])
    # [R, T, N, ...] -> trajectory-major [R, N, T, ...] -> rows
    def rows(x):
        x = x.permute(0, 2, 1, *range(3, x.dim())).contiguous()
        return x.reshape(num_rounds * N * T, *x.shape[3:])

    env.close()
    return dict(observations=rows(obs), actions=rows(act), terminals=rows(term), qpos=rows(qpos))
