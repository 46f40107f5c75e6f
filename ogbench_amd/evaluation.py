"""Batched evaluation with an all-gathered success reduction.

Reference: ``evaluate`` (impls/utils/evaluation.py:36-123) runs
``num_eval_episodes`` episodes of one task and averages the final-step
``info['success']``; impls/main.py:226-258 loops over tasks and reports
``evaluation/{task_name}_success`` plus ``evaluation/overall_success`` (the
mean over tasks).

Batched restatement: every env of a batch runs one task (default env i runs
task ``i % num_tasks + 1``) with same-step auto-reset, so one launch per step
advances all episodes of all tasks.  The step outputs feed
``ogbx_eval_accumulate``, which adds each finished episode's success into an
int64[num_tasks, 2] block {success_sum, episode_count}.  Across ranks the
blocks are all-gathered (RCCL over xGMI on GPU, gloo on CPU) and summed; every
rank then derives the same metrics.  This is the path's one collective
(SURVEY.md section 8e).
"""

from __future__ import annotations

import numpy as np

from . import _lib


def _torch():
    import torch

    return torch


def accumulate(counters, success, terminated, truncated, task_id, remaining):
    """counters[task-1] += {success, 1} for the envs whose episode ended this
    step and still owe episodes (``remaining`` is decremented).  Device tensors."""
    torch = _torch()
    n = success.shape[0]
    for t, dt in ((success, torch.uint8), (terminated, torch.uint8), (truncated, torch.uint8)):
        assert t.dtype in (dt, torch.bool) and t.is_contiguous() and t.shape[0] == n
    assert task_id.dtype == torch.int32 and remaining.dtype == torch.int32
    assert counters.dtype == torch.int64 and counters.is_contiguous() and counters.dim() == 2
    _lib.check(
        _lib.lib().ogbx_eval_accumulate(
            _lib.ptr(success), _lib.ptr(terminated), _lib.ptr(truncated), _lib.ptr(task_id.contiguous()),
            _lib.ptr(remaining), n, counters.shape[0], _lib.ptr(counters), _lib.stream_of(success.device)
        ),
        'eval_accumulate',
    )


def comm_unique_id():
    """RCCL unique id (bytes) for RcclComm; rank 0 creates it and ships it to
    the other ranks out of band."""
    buf = (_lib.ctypes.c_uint8 * 128)()
    _lib.check(_lib.lib().ogbx_comm_unique_id(_lib.ctypes.cast(buf, _lib.c_void_p)), 'comm_unique_id')
    return bytes(buf)


class RcclComm:
    """An RCCL communicator owned by libogbx (``ogbx_comm_create``): the C-ABI
    all-gather for hosts that do not run torch.distributed.  Python callers
    normally use ``gather_counters(counters)`` over the default process group;
    this path is the same collective bound directly."""

    def __init__(self, world_size, rank, device, unique_id):
        assert len(unique_id) == 128
        self.world_size, self.rank = int(world_size), int(rank)
        self.device = _lib_device(device)
        buf = (_lib.ctypes.c_uint8 * 128).from_buffer_copy(unique_id)
        self._h = _lib.c_void_p()
        _lib.check(_lib.lib().ogbx_comm_create(_lib.ctypes.cast(buf, _lib.c_void_p), self.world_size, self.rank,
                                               self.device.index, self._h), 'comm_create')

    def allgather(self, counters):
        """int64 device tensor [...] -> [world_size, ...] (every rank's block)."""
        torch = _torch()
        local = counters.contiguous()
        assert local.dtype == torch.int64 and local.is_cuda
        out = torch.empty((self.world_size,) + tuple(local.shape), dtype=torch.int64, device=local.device)
        _lib.check(_lib.lib().ogbx_eval_allgather(self._h, _lib.ptr(local), local.numel(), _lib.ptr(out),
                                                  _lib.stream_of(local.device)), 'eval_allgather')
        return out

    def close(self):
        if getattr(self, '_h', None) is not None and self._h.value:
            _lib.lib().ogbx_comm_destroy(self._h)
            self._h = _lib.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _lib_device(device):
    torch = _torch()
    d = torch.device(device)
    return torch.device('cuda', torch.cuda.current_device() if d.index is None else d.index)


def gather_counters(counters, group=None, comm=None):
    """All-gather every rank's int64[num_tasks, 2] counters and sum them.

    Uses ``torch.distributed.all_gather_into_tensor`` on the default (or given)
    process group, or ``comm`` (an RcclComm) when given; a no-op without either.
    Returns the summed counters (same device as the input) and the per-rank
    stack.
    """
    torch = _torch()
    import torch.distributed as dist

    if comm is not None:
        out = comm.allgather(counters)
        return out.sum(0), out
    if not (dist.is_available() and dist.is_initialized()):
        return counters.clone(), counters.unsqueeze(0).clone()
    world = dist.get_world_size(group)
    out = torch.empty((world,) + tuple(counters.shape), dtype=counters.dtype, device=counters.device)
    if dist.get_backend(group) == 'gloo':  # host tensors (gloo's CUDA coverage is partial)
        parts = [torch.empty(tuple(counters.shape), dtype=counters.dtype) for _ in range(world)]
        dist.all_gather(parts, counters.detach().cpu().contiguous(), group=group)
        out = torch.stack(parts).to(counters.device)
    else:
        dist.all_gather_into_tensor(out, counters.contiguous(), group=group)
    return out.sum(0), out


def summarize(counters, task_infos=None):
    """Reference metric dict (main.py:251-258) from summed counters [T, 2]."""
    c = np.asarray(counters.cpu() if hasattr(counters, 'cpu') else counters, dtype=np.int64)
    metrics = {}
    per_task = []
    for t in range(c.shape[0]):
        if c[t, 1] == 0:
            continue
        name = task_infos[t]['task_name'] if task_infos is not None else f'task{t + 1}'
        v = float(c[t, 0]) / float(c[t, 1])
        metrics[f'evaluation/{name}_success'] = v
        per_task.append(v)
    if per_task:
        metrics['evaluation/overall_success'] = float(np.mean(per_task))
    return metrics


def env_task_ids(env):
    """int32 [N] task id of every env's running episode (device)."""
    torch = _torch()
    if hasattr(env, 'cur_task_ids'):
        return env.cur_task_ids.to(torch.int32).contiguous()
    return env._state_views()[3]


def evaluate(policy, env, task_ids=None, episodes_per_env=1, max_steps=None, check_every=16, seed=0,
             group=None):
    """Batched ``evaluate`` over all tasks at once.

    policy(obs, goal) -> action tensor for every env (device).  ``env`` must
    have ``auto_reset=True``.  Env i runs ``task_ids[i]`` (default
    ``i % num_tasks + 1``) for ``episodes_per_env`` episodes.  Returns
    (metrics, summed counters int64[T,2], this rank's counters).
    """
    torch = _torch()
    assert env.auto_reset, 'evaluate() needs an env created with auto_reset=True'
    n, T = env.num_envs, env.num_tasks
    dev = env.device
    if task_ids is None:
        task_ids = torch.arange(n, device=dev, dtype=torch.int32) % T + 1
    task_ids = torch.as_tensor(task_ids).to(dev, torch.int32)
    obs, info = env.reset(seed=seed, options=dict(task_id=task_ids))
    goal = info['goal']
    counters = torch.zeros(T, 2, dtype=torch.int64, device=dev)
    remaining = torch.full((n,), int(episodes_per_env), dtype=torch.int32, device=dev)
    limit = max_steps if max_steps is not None else env.max_episode_steps * episodes_per_env
    tid = env_task_ids(env)
    for step in range(int(limit)):
        g = env.cur_goal_xy if hasattr(env, 'cur_goal_xy') else goal
        action = policy(obs, g)
        obs, rew, term, trunc, inf = env.step(action)
        accumulate(counters, inf['success'].view(torch.uint8), term.view(torch.uint8), trunc.view(torch.uint8),
                   tid, remaining)
        if (step + 1) % check_every == 0 and int(remaining.max()) == 0:
            break
    total, _ = gather_counters(counters, group)
    task_infos = getattr(env, 'task_infos', None)
    return summarize(total, task_infos), total, counters
