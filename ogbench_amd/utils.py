"""Dataset loading and the env/dataset factory, with the datasets in HBM.

Batched, device-side counterparts of ogbench/utils.py and
ogbench/relabel_utils.py (hliuson/ogbench):

  load_dataset            ~ utils.py:14-96 (compact and regular conversions run
                            on the device: ogbx_compact_terminals, hipCUB
                            selection + ogbx_gather_rows)
  relabel_dataset         ~ relabel_utils.py:4-113 (maze branch, ogbx_relabel_maze)
  add_oracle_reps         ~ relabel_utils.py:116-166 (maze branch, same pass)
  make_env_and_datasets   ~ utils.py:134-236 (same name grammar: singletask,
                            oraclerep; returns a batched env and dicts of
                            device tensors)

There is no download here (no network): ``dataset_path`` or
``dataset_dir/<name>.npz`` must exist.  Manipulation (cube/scene/puzzle)
relabels are out of scope and raise NotImplementedError.
"""

from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib

DEFAULT_DATASET_DIR = '~/.ogbench/data'
INFO_KEYS = ('qpos', 'qvel', 'button_states')


def _torch():
    import torch

    return torch


def _bind():
    L = _lib.lib()
    if not getattr(L, '_loader_bound', False):
        vp, i64, i32, f64 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_double
        L.ogbx_compact_terminals.restype = i32
        L.ogbx_compact_terminals.argtypes = [vp, i64, vp, vp, vp, vp]
        L.ogbx_gather_rows.restype = i32
        L.ogbx_gather_rows.argtypes = [vp, i64, vp, i64, vp, vp]
        L.ogbx_relabel_maze.restype = i32
        L.ogbx_relabel_maze.argtypes = [vp, i32, i64, i64, f64, f64, f64, vp, vp, vp, vp]
        L._loader_bound = True
    return L


def _device(device):
    torch = _torch()
    device = torch.device('cuda' if device is None else device)
    if device.type != 'cuda':
        raise RuntimeError('ogbench_amd datasets live in HBM (no CPU fallback); got device %s' % device)
    if device.index is None:
        device = torch.device('cuda', torch.cuda.current_device())
    return device


def gather_rows(src, idx):
    """src[idx] along dim 0 for a dense device tensor (one libogbx launch)."""
    torch = _torch()
    src = src.contiguous()
    idx = idx.to(torch.int64).contiguous()
    out = torch.empty((idx.numel(),) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    row_bytes = (src[0].numel() if src.dim() > 1 else 1) * src.element_size()
    _lib.check(_bind().ogbx_gather_rows(_lib.ptr(src), row_bytes, _lib.ptr(idx), idx.numel(), _lib.ptr(out),
                                        _lib.stream_of(src.device)), 'gather_rows')
    return out


def load_dataset(dataset_path, ob_dtype=np.float32, action_dtype=np.float32, compact_dataset=False, add_info=False,
                 device=None):
    """utils.py:14-96: load an OGBench .npz into HBM (dict of device tensors).

    Keys and dtypes as the reference: observations, actions, terminals,
    [qpos, qvel, button_states if add_info], and valids (compact) or
    next_observations (regular)."""
    torch = _torch()
    dev = _device(device)
    from .datasets import nonzero_positive

    L = _bind()
    stream = _lib.stream_of(dev)
    with np.load(dataset_path) as f:
        host = {}
        for k in ('observations', 'actions', 'terminals'):
            dtype = ob_dtype if k == 'observations' else (action_dtype if k == 'actions' else np.float32)
            host[k] = f[k][...].astype(dtype, copy=False)
        info_keys = [k for k in INFO_KEYS if add_info and k in f.files]
        for k in info_keys:
            host[k] = f[k][...]
    d = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in host.items()}
    del host
    t = d['terminals']
    n = t.numel()
    if compact_dataset:
        valids = torch.empty_like(t)
        terms = torch.empty_like(t)
        _lib.check(L.ogbx_compact_terminals(_lib.ptr(t), n, _lib.ptr(terms), _lib.ptr(valids), None, stream))
        d['terminals'] = terms
        d['valids'] = valids
    else:
        shifted = torch.empty_like(t)
        valids = torch.empty_like(t)
        _lib.check(L.ogbx_compact_terminals(_lib.ptr(t), n, None, _lib.ptr(valids), _lib.ptr(shifted), stream))
        sel = nonzero_positive(valids)                    # ob_mask = (1 - terminals) != 0
        nxt = sel + 1
        nxt = nxt[nxt < n]                                # next_ob_mask = [False] + ob_mask[:-1]
        obs = d['observations']
        d['next_observations'] = gather_rows(obs, nxt)
        d['observations'] = gather_rows(obs, sel)
        d['actions'] = gather_rows(d['actions'], sel)
        d['terminals'] = gather_rows(shifted, sel)
        for k in info_keys:
            d[k] = gather_rows(d[k], sel)
        # reference key order: observations, actions, terminals, info..., next_observations
        d = {k: d[k] for k in ['observations', 'actions', 'terminals', *info_keys, 'next_observations']}
    return d


def _maze_relabel(env, dataset, rewards_masks, oracle_reps):
    torch = _torch()
    q = dataset['qpos']
    assert q.dim() == 2 and q.shape[1] >= 2, 'qpos must be [rows, nq]'
    q = q.contiguous()
    n = q.shape[0]
    dev = q.device
    goal = env.unwrapped.cur_goal_xy
    goal = goal[0] if hasattr(goal, 'dim') and goal.dim() == 2 else goal
    gx, gy = (float(v) for v in (goal.cpu().numpy() if hasattr(goal, 'cpu') else np.asarray(goal)))
    rew = msk = reps = None
    if rewards_masks:
        rew = torch.empty(n, dtype=torch.float32, device=dev)
        msk = torch.empty(n, dtype=torch.float32, device=dev)
    if oracle_reps:
        reps = torch.empty(n, 2, dtype=torch.float32, device=dev)
    _lib.check(_bind().ogbx_relabel_maze(
        _lib.ptr(q), int(q.dtype == torch.float64), n, q.shape[1], gx, gy, float(env.unwrapped._goal_tol),
        _lib.ptr(rew), _lib.ptr(msk), _lib.ptr(reps), _lib.stream_of(dev)), 'relabel_maze')
    return rew, msk, reps


def relabel_dataset(env_name, env, dataset):
    """relabel_utils.py:4-113: rewards/masks of the env's fixed task (maze branch)."""
    assert env.unwrapped._reward_task_id is not None, 'The environment is not in the single-task mode.'
    env.reset()  # Set the task.
    if 'maze' in env_name:
        rew, msk, _ = _maze_relabel(env, dataset, True, False)
    elif 'soccer' in env_name or 'cube' in env_name or 'scene' in env_name or 'puzzle' in env_name:
        raise NotImplementedError(f'relabel for {env_name} needs the manipulation/soccer envs (out of scope)')
    else:
        raise ValueError(f'Unsupported environment: {env_name}')
    dataset['rewards'] = rew
    dataset['masks'] = msk


def add_oracle_reps(env_name, env, dataset):
    """relabel_utils.py:116-166: oracle goal representations (maze branch: qpos[:, :2])."""
    if 'maze' in env_name:
        _, _, reps = _maze_relabel(env, dataset, False, True)
    elif 'soccer' in env_name or 'cube' in env_name or 'scene' in env_name or 'puzzle' in env_name:
        raise NotImplementedError(f'oracle reps for {env_name} need the manipulation/soccer envs (out of scope)')
    else:
        raise ValueError(f'Unsupported environment: {env_name}')
    dataset['oracle_reps'] = reps


def parse_dataset_name(dataset_name):
    """The name grammar of utils.py:160-182 -> (env_name, file dataset_name, mode)."""
    splits = dataset_name.split('-')
    if 'singletask' in splits:
        pos = splits.index('singletask')
        env_name = '-'.join(splits[: pos - 1] + splits[pos:])
        return env_name, '-'.join(splits[:pos] + splits[-1:]), 'singletask'
    if 'oraclerep' in splits:
        return '-'.join(splits[:-3] + splits[-1:]), '-'.join(splits[:-2] + splits[-1:]), 'oraclerep'
    return '-'.join(splits[:-2] + splits[-1:]), dataset_name, 'goal'


def make_env_and_datasets(dataset_name, dataset_dir=DEFAULT_DATASET_DIR, dataset_path=None, compact_dataset=False,
                          env_only=False, dataset_only=False, cur_env=None, add_info=False, num_envs=1, device=None,
                          **env_kwargs):
    """utils.py:134-236 with a batched env of ``num_envs`` and HBM datasets."""
    from .registry import make

    env_name, file_name, mode = parse_dataset_name(dataset_name)
    env = cur_env
    dataset_add_info = add_info or mode in ('singletask', 'oraclerep')
    if not dataset_only:
        kw = dict(env_kwargs)
        if mode == 'oraclerep':
            kw['use_oracle_rep'] = True
        env = make(env_name, num_envs=num_envs, device=device, **kw)
    if env_only:
        return env
    if dataset_path is None:
        dataset_dir = os.path.expanduser(dataset_dir)
        train_path = os.path.join(dataset_dir, f'{file_name}.npz')
        val_path = os.path.join(dataset_dir, f'{file_name}-val.npz')
        if not os.path.exists(train_path):
            raise FileNotFoundError(f'{train_path} not found (datasets are not downloaded here; pass dataset_path)')
    else:
        train_path = dataset_path
        val_path = dataset_path.replace('.npz', '-val.npz')
    ob_dtype = np.uint8 if ('visual' in env_name or 'powderworld' in env_name) else np.float32
    action_dtype = np.int32 if 'powderworld' in env_name else np.float32
    dev = env.device if env is not None and hasattr(env, 'device') else device
    kw = dict(ob_dtype=ob_dtype, action_dtype=action_dtype, compact_dataset=compact_dataset,
              add_info=dataset_add_info, device=dev)
    train = load_dataset(train_path, **kw)
    val = load_dataset(val_path, **kw)
    if mode == 'singletask':
        relabel_dataset(env_name, env, train)
        relabel_dataset(env_name, env, val)
    if mode == 'oraclerep':
        add_oracle_reps(env_name, env, train)
        add_oracle_reps(env_name, env, val)
    if not add_info:
        for k in INFO_KEYS:
            train.pop(k, None)
            val.pop(k, None)
    if dataset_only:
        return train, val
    return env, train, val
