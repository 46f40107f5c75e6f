"""ctypes wrapper of oracle/_build/liboracle.so (oracle/locomaze_ref.c).

TEST INFRASTRUCTURE ONLY -- the checker for libogbx's locomaze kernels.
Wall-contact dynamics are pinned to MuJoCo's published formulation by the
independent model tests/mjmodel_np.py, not to MuJoCo's output (MuJoCo absent);
see locomaze_ref.c and DESIGN.md section 6.
"""

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, '_build', 'liboracle.so')
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            subprocess.run(['make', '-C', _HERE], check=True, capture_output=True)
        _lib = ctypes.CDLL(_SO)
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def tables(maze):
    L = lib()
    H, W, T = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    assert L.orc_maze_tables(maze.encode(), ctypes.byref(H), ctypes.byref(W), ctypes.byref(T), None, None) == 0
    mp = np.zeros((H.value, W.value), np.int32)
    tk = np.zeros((T.value, 4), np.int32)
    L.orc_maze_tables(maze.encode(), ctypes.byref(H), ctypes.byref(W), ctypes.byref(T), _p(mp), _p(tk))
    return mp, tk


def physics(maze, qpos, action, nthreads=1):
    """qpos [n,2] f64, action [n,2] f32|f64 -> (qpos_out, contact)."""
    q = np.ascontiguousarray(qpos, np.float64)
    a = np.ascontiguousarray(action)
    assert a.dtype in (np.float32, np.float64)
    out = np.zeros_like(q)
    c = np.zeros(len(q), np.uint8)
    lib().orc_point_physics(maze.encode(), _p(q), _p(a), int(a.dtype == np.float64), ctypes.c_int64(len(q)),
                            _p(out), _p(c), int(nthreads))
    return out, c


def xy_to_ij(xy):
    xy = np.ascontiguousarray(xy, np.float64)
    ij = np.zeros((len(xy), 2), np.int32)
    lib().orc_xy_to_ij(_p(xy), ctypes.c_int64(len(xy)), _p(ij))
    return ij


def oracle_subgoal(maze, start_xy, goal_xy):
    s = np.ascontiguousarray(start_xy, np.float64)
    g = np.ascontiguousarray(goal_xy, np.float64)
    out = np.zeros_like(s)
    lib().orc_oracle_subgoal(maze.encode(), _p(s), _p(g), ctypes.c_int64(len(s)), _p(out))
    return out


def expert_action(maze, xy, goal_xy, normal):
    """generate_locomaze.py point expert with injected normal draws [n,2]."""
    xy = np.ascontiguousarray(xy, np.float64)
    g = np.ascontiguousarray(goal_xy, np.float64)
    z = np.ascontiguousarray(normal, np.float64)
    out = np.zeros_like(xy)
    lib().orc_expert_action(maze.encode(), _p(xy), _p(g), _p(z), ctypes.c_int64(len(xy)), _p(out))
    return out


def _opts(success_pre=0, terminate_at_goal=1, add_noise_to_goal=1, reward_task_id=-1, max_steps=1000,
          not_point=0):
    return np.array([success_pre, terminate_at_goal, add_noise_to_goal, reward_task_id, max_steps, not_point],
                    np.int32)


def reset(maze, task_id, noise, **opts):
    """Reset n envs with injected uniform(-1,1) draws noise [n,4]; returns a state dict."""
    o = _opts(**opts)
    task_id = np.ascontiguousarray(task_id, np.int32)
    noise = np.ascontiguousarray(noise, np.float64)
    n = len(task_id)
    st = dict(qpos=np.zeros((n, 2)), goal=np.zeros((n, 2)), elapsed=np.zeros(n, np.int32),
              task=np.zeros(n, np.int32), episode=np.ones(n, np.uint32), opts=o)
    lib().orc_maze_reset(maze.encode(), _p(o), _p(task_id), _p(noise), ctypes.c_int64(n), _p(st['qpos']),
                         _p(st['goal']), _p(st['elapsed']), _p(st['task']))
    return st


def step(maze, st, actions, auto_reset=0, key=(0, 0), nthreads=1, env_base=0):
    """k steps (actions [k,n,2]) of the env-level oracle; st is updated in place.
    env_base: global index of env 0 (Philox counter of the auto-reset draws)."""
    a = np.ascontiguousarray(actions)
    k, n = a.shape[0], a.shape[1]
    out = dict(obs=np.zeros((k, n, 2)), reward=np.zeros((k, n), np.float32),
               terminated=np.zeros((k, n), np.uint8), truncated=np.zeros((k, n), np.uint8),
               success=np.zeros((k, n), np.uint8))
    lib().orc_maze_step(maze.encode(), _p(st['opts']), _p(st['qpos']), _p(st['goal']), _p(st['elapsed']),
                        _p(st['task']), _p(st['episode']), ctypes.c_int64(n), _p(a), int(a.dtype == np.float64),
                        int(k), _p(out['obs']), _p(out['reward']), _p(out['terminated']), _p(out['truncated']),
                        _p(out['success']), int(auto_reset), ctypes.c_uint32(key[0]), ctypes.c_uint32(key[1]),
                        int(nthreads), ctypes.c_int64(env_base))
    return out


def reset_draws(n, seed, env_base=0, episode=1):
    """The Philox uniform(-1,1) reset draws [n,4] libogbx uses for a reset with
    `seed` of envs env_base..env_base+n-1 (episode counter after the reset)."""
    k0, k1 = philox_key(seed, TAG_MAZE_RESET)
    out = np.zeros((n, 4))
    lib().orc_reset_draws(ctypes.c_int64(n), ctypes.c_int64(env_base), ctypes.c_uint32(episode), ctypes.c_uint32(k0),
                          ctypes.c_uint32(k1), _p(out))
    return out


def philox4x32(ctr, k0, k1):
    c = np.ascontiguousarray(ctr, np.uint32)
    o = np.zeros(4, np.uint32)
    lib().orc_philox4x32(_p(c), ctypes.c_uint32(k0), ctypes.c_uint32(k1), _p(o))
    return o


def philox_key(seed, tag):
    """Key derivation of libogbx (common.h seed_key)."""
    return seed & 0xFFFFFFFF, ((seed >> 32) ^ tag) & 0xFFFFFFFF


TAG_MAZE_RESET = 0x4D5A0001
