"""Env-id registry: the batched analogue of ``gymnasium.make`` for the ids that
ogbench registers (ogbench/locomaze/__init__.py, ogbench/powderworld/__init__.py)."""

from __future__ import annotations

import re


def registered_env_ids():
    ids = []
    for loco, mazes in (('point', ('medium', 'large', 'giant', 'teleport')),
                        ('ant', ('medium', 'large', 'giant', 'teleport')),
                        ('humanoid', ('medium', 'large', 'giant', 'teleport'))):
        for m in mazes:
            ids.append(f'{loco}maze-{m}-v0')
            for t in ('', '-task1', '-task2', '-task3', '-task4', '-task5'):
                ids.append(f'{loco}maze-{m}-singletask{t}-v0')
    ids += ['powderworld-easy-v0', 'powderworld-medium-v0', 'powderworld-hard-v0']
    return ids


def make(env_id, num_envs=1, device=None, **kwargs):
    """Create a batch of ``num_envs`` envs of the registered ``env_id``.

    Keyword arguments override the registry kwargs, exactly like
    ``gymnasium.make(env_id, **env_kwargs)`` (ogbench/utils.py:143).
    """
    from .locomaze import MazeEnv, parse_env_id

    spec = parse_env_id(env_id)
    if spec is not None:
        spec.update(kwargs)
        return MazeEnv(num_envs=num_envs, device=device, **spec)
    m = re.fullmatch(r'powderworld-(easy|medium|hard)-v0', env_id)
    if m is not None:
        from .powderworld import PowderworldEnv

        num_elems = {'easy': 2, 'medium': 5, 'hard': 8}[m.group(1)]
        spec = dict(num_elems=num_elems, max_episode_steps=500)
        spec.update(kwargs)
        return PowderworldEnv(num_envs=num_envs, device=device, **spec)
    raise ValueError(f'Environment {env_id} doesn\'t exist.')
