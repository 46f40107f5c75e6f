"""Batched locomaze (pointmaze) environments on MI355X.

``MazeEnv`` is the batched counterpart of the reference ``make_maze_env(...)``
class (ogbench/locomaze/maze.py:13-567): the same constructor options, task
tables, ``reset(options=...)``/``step(action)`` semantics and helper methods,
but every env of the batch lives in HBM and one ``step`` is one HIP launch
(``ogbx_maze_step`` in libogbx).  Tensors are PyTorch-ROCm tensors with a
leading batch dimension N.

Differences that follow from batching (documented in DESIGN.md):
  * returned tensors are views of env-owned buffers that the next ``step``
    overwrites (clone them to keep them);
  * ``info['success']``, ``terminated`` and ``truncated`` are bool tensors;
  * with ``auto_reset=True`` finished envs are reset inside the same step
    (gymnasium same-step autoreset); ``info['final_observation']`` then holds
    the terminal observation;
  * reset noise comes from a counter-based Philox stream keyed by ``seed``
    (the reference draws np.random.uniform), and can be injected exactly with
    ``options['noise']`` for parity tests.
"""

from __future__ import annotations

import re
import warnings

import numpy as np

from . import _lib
from .spaces import Box

LOCO_TYPES = {'point': 0, 'ant': 1, 'humanoid': 2}
MAZE_TYPES = ('arena', 'medium', 'large', 'giant', 'teleport')


def _torch():
    import torch

    return torch


def _resolve_device(device):
    torch = _torch()
    if device is None:
        device = 'cuda'
    device = torch.device(device)
    if device.type != 'cuda':
        raise RuntimeError('ogbench_amd envs run on the GPU only (no CPU fallback); got device %s' % device)
    if device.index is None:
        device = torch.device('cuda', torch.cuda.current_device())
    return device


def static_tables(maze_type):
    """(maze_map int32[H,W], tasks int32[T,4]) without touching the GPU."""
    L = _lib.lib()
    H, W, T = _lib.c_int32(), _lib.c_int32(), _lib.c_int32()
    _lib.check(L.ogbx_maze_static_tables(maze_type.encode(), H, W, T, None, None))
    mp = np.zeros((H.value, W.value), np.int32)
    tk = np.zeros((T.value, 4), np.int32)
    _lib.check(
        L.ogbx_maze_static_tables(
            maze_type.encode(), H, W, T, mp.ctypes.data_as(_lib.c_void_p), tk.ctypes.data_as(_lib.c_void_p)
        )
    )
    return mp, tk


class MazeEnv:
    """Batch of ``num_envs`` maze environments (reference: maze.py:31-567)."""

    def __init__(
        self,
        loco_env_type='point',
        maze_type='large',
        num_envs=1,
        device=None,
        maze_unit=4.0,
        maze_height=0.5,
        terminate_at_goal=True,
        success_timing='post',
        ob_type='states',
        add_noise_to_goal=True,
        reward_task_id=None,
        use_oracle_rep=False,
        max_episode_steps=1000,
        auto_reset=False,
        seed=None,
        env_base=0,
    ):
        """env_base: global index of env 0 of this batch.  Every Philox stream
        is counted by the global env index, so G shards [r*N/G, (r+1)*N/G) with
        the same seed reproduce one batch of N envs bit for bit.
        Any boundary works (every contact-solver choice is made per env, so
        results do not depend on which envs share a wavefront);
        ogbench_amd.sharding.shard keeps blocks 64-aligned for full wavefronts."""
        if loco_env_type not in LOCO_TYPES:
            raise ValueError(f'Unknown locomotion environment type: {loco_env_type}')
        if maze_type not in MAZE_TYPES:
            raise ValueError(f'Unknown maze type: {maze_type}')
        assert ob_type in ['states', 'pixels']
        assert success_timing in ['pre', 'post']
        if ob_type == 'pixels':
            raise NotImplementedError('pixel observations (MuJoCo rendering) are out of scope')
        if maze_unit != 4.0 or maze_height != 0.5:
            raise NotImplementedError('only the registered maze_unit=4.0 / maze_height=0.5 are supported')
        torch = _torch()
        self.device = _resolve_device(device)
        self.num_envs = int(num_envs)
        self._loco_env_type = loco_env_type
        self._maze_type = maze_type
        self._maze_unit = maze_unit
        self._maze_height = maze_height
        self._terminate_at_goal = terminate_at_goal
        self._success_timing = success_timing
        self._ob_type = ob_type
        self._add_noise_to_goal = add_noise_to_goal
        self._reward_task_id = reward_task_id
        self._use_oracle_rep = use_oracle_rep
        self._offset_x = 4
        self._offset_y = 4
        self._noise = 1
        self._goal_tol = 1.0 if loco_env_type == 'point' else 0.5
        self.max_episode_steps = int(max_episode_steps)
        self._auto_i = int(bool(auto_reset))

        opts = _lib.MazeOpts(
            loco_type=LOCO_TYPES[loco_env_type],
            success_timing=0 if success_timing == 'post' else 1,
            terminate_at_goal=int(bool(terminate_at_goal)),
            add_noise_to_goal=int(bool(add_noise_to_goal)),
            reward_task_id=-1 if reward_task_id is None else int(reward_task_id),
            max_episode_steps=self.max_episode_steps,
            env_base=int(env_base),
        )
        self.env_base = int(env_base)
        L = _lib.lib()
        h = _lib.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(L.ogbx_maze_create(maze_type.encode(), self.num_envs, self.device.index, opts, h))
        self._h = h
        self._L = L
        self._wrap_fn = L.ogbx_antmaze_step
        self._wrap_bound = L.ogbx_antmaze_step_bound

        self.maze_map, tasks = static_tables(maze_type)
        self.task_infos = []
        for i, t in enumerate(tasks):
            init_ij, goal_ij = (int(t[0]), int(t[1])), (int(t[2]), int(t[3]))
            self.task_infos.append(
                dict(
                    task_name=f'task{i + 1}',
                    init_ij=init_ij,
                    init_xy=self.ij_to_xy(init_ij),
                    goal_ij=goal_ij,
                    goal_xy=self.ij_to_xy(goal_ij),
                )
            )
        self.num_tasks = len(self.task_infos)
        if self._reward_task_id == 0:
            self._reward_task_id = 1  # Default task (maze.py:361-362).

        ob_dim = 2 if loco_env_type == 'point' else (29 if loco_env_type == 'ant' else 69)
        act_dim = 2 if loco_env_type == 'point' else (8 if loco_env_type == 'ant' else 21)
        self.single_observation_space = Box(-np.inf, np.inf, (ob_dim,), np.float64)
        self.single_action_space = Box(-1.0, 1.0, (act_dim,), np.float32)
        self.observation_space = Box(-np.inf, np.inf, (self.num_envs, ob_dim), np.float64)
        self.action_space = Box(-1.0, 1.0, (self.num_envs, act_dim), np.float32)

        n = self.num_envs
        kw = dict(device=self.device)
        self._ob_dim = 2 if loco_env_type == 'point' else ob_dim
        self._obs = torch.zeros(n, self._ob_dim, dtype=torch.float64, **kw)
        self._goal = torch.zeros(n, 2, dtype=torch.float64, **kw)
        # ant: info['goal'] is the 29-d goal observation (maze.py:407-418)
        self._goal_ob = torch.zeros(n, ob_dim, dtype=torch.float64, **kw) if loco_env_type == 'ant' else None
        self._final_obs = torch.zeros(n, self._ob_dim, dtype=torch.float64, **kw)
        self._reward = torch.zeros(n, dtype=torch.float32, **kw)
        self._term = torch.zeros(n, dtype=torch.uint8, **kw)
        self._trunc = torch.zeros(n, dtype=torch.uint8, **kw)
        self._succ = torch.zeros(n, dtype=torch.uint8, **kw)
        # step() outputs are fixed buffers: their pointers and bool views once
        self._step_out = (_lib.ptr(self._obs), _lib.ptr(self._reward), _lib.ptr(self._term),
                          _lib.ptr(self._trunc), _lib.ptr(self._succ),
                          _lib.ptr(self._final_obs))  # written only by an auto-reset
        self._ant_qshape, self._ant_vshape, self._f64 = torch.Size((n, 15)), torch.Size((n, 14)), torch.float64
        # the steady step (step()'s fast path): outputs bound once in the
        # handle (ogbx_maze_bind_step, re-bound when auto_reset changes), then
        # one 4-argument call per step with the raw stream handle
        self._bound_auto = None
        self._step_bound = L.ogbx_maze_step_bound
        self._raw_stream = torch._C._cuda_getCurrentRawStream
        self._Tensor, self._f32, self._f64t = torch.Tensor, torch.float32, torch.float64
        self._act_shape = torch.Size((n, 2))
        self._is_point = loco_env_type == 'point'
        self._term_b = self._term.view(torch.bool)
        self._trunc_b = self._trunc.view(torch.bool)
        self._succ_b = self._succ.view(torch.bool)
        self._wrap_cache = {}
        self._dev_idx = self.device.index
        self._seed = None
        self._init_seed = seed
        self._has_reset = False
        self.cur_task_id = None

    @property
    def auto_reset(self):
        return bool(self._auto_i)

    @auto_reset.setter
    def auto_reset(self, value):
        self._auto_i = int(bool(value))

    # ------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, '_h', None) is not None and self._h.value:
            self._L.ogbx_maze_destroy(self._h)
            self._h = _lib.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def unwrapped(self):
        return self

    def _stream(self):
        return _lib.stream_of(self.device)

    # ------------------------------------------------------------ helpers
    def xy_to_ij(self, xy):
        """maze.py:552-556 (Python int() truncation).  Scalars or [n,2] tensors."""
        if isinstance(xy, (tuple, list)) or (isinstance(xy, np.ndarray) and xy.ndim == 1):
            maze_unit = self._maze_unit
            i = int((xy[1] + self._offset_y + 0.5 * maze_unit) / maze_unit)
            j = int((xy[0] + self._offset_x + 0.5 * maze_unit) / maze_unit)
            return i, j
        torch = _torch()
        xy = xy.to(self.device, torch.float64).contiguous()
        ij = torch.empty(xy.shape[0], 2, dtype=torch.int32, device=self.device)
        _lib.check(self._L.ogbx_maze_xy_to_ij(self._h, _lib.ptr(xy), xy.shape[0], _lib.ptr(ij), self._stream()))
        return ij

    def ij_to_xy(self, ij):
        """maze.py:558-562."""
        if isinstance(ij, (tuple, list)) or (isinstance(ij, np.ndarray) and ij.ndim == 1):
            i, j = ij
            x = j * self._maze_unit - self._offset_x
            y = i * self._maze_unit - self._offset_y
            return x, y
        torch = _torch()
        ij = ij.to(self.device, torch.int32).contiguous()
        xy = torch.empty(ij.shape[0], 2, dtype=torch.float64, device=self.device)
        _lib.check(self._L.ogbx_maze_ij_to_xy(self._h, _lib.ptr(ij), ij.shape[0], _lib.ptr(xy), self._stream()))
        return xy

    def get_oracle_subgoal(self, start_xy, goal_xy):
        """Batched maze.py:503-550: BFS next-hop subgoal for each (start, goal) pair."""
        torch = _torch()
        s = start_xy.to(self.device, torch.float64).contiguous()
        g = goal_xy.to(self.device, torch.float64).contiguous()
        out = torch.empty_like(s)
        _lib.check(
            self._L.ogbx_maze_oracle_subgoal(
                self._h, _lib.ptr(s), _lib.ptr(g), s.shape[0], _lib.ptr(out), self._stream()
            )
        )
        return out

    def expert_action(self, noise=0.2, normal=None, start_xy=None, goal_xy=None, out=None, seed=None):
        """Point-maze expert of data_gen_scripts/generate_locomaze.py:147-166:
        clip(subgoal direction + N(0, noise), -1, 1) as float64 [N,2] (one launch).

        Without start_xy/goal_xy it reads the envs' own qpos and goal (no host
        round trip).  normal: injected np.random.normal(0, noise) draws [N,2]."""
        torch = _torch()
        n = self.num_envs if start_xy is None else int(start_xy.shape[0])
        if out is None:
            out = torch.empty(n, 2, dtype=torch.float64, device=self.device)
        s = g = None
        if start_xy is not None or goal_xy is not None:
            assert start_xy is not None and goal_xy is not None, 'give both start_xy and goal_xy'
            s = start_xy.to(self.device, torch.float64).contiguous()
            g = goal_xy.to(self.device, torch.float64).contiguous()
        z = None if normal is None else torch.as_tensor(normal).to(self.device, torch.float64).contiguous()
        calls = getattr(self, '_expert_calls', 0)
        self._expert_calls = calls + 1
        sd = seed if seed is not None else (self._seed if self._seed is not None else 0)
        _lib.check(self._L.ogbx_maze_expert_action(self._h, _lib.ptr(s), _lib.ptr(g), n, float(noise), _lib.ptr(z),
                                                    int(sd) & ((1 << 64) - 1), calls, _lib.ptr(out),
                                                    self._stream()), 'expert_action')
        return out

    def set_goal(self, goal_ij, mask=None, noise=None):
        """MazeEnv.set_goal(goal_ij) (maze.py:492-501) per env: goal_ij int [N,2]
        (+ add_noise draws from Philox, or injected uniform(-1,1) `noise` [N,2])."""
        torch = _torch()
        ij = torch.as_tensor(goal_ij).to(self.device, torch.int32).reshape(self.num_envs, 2).contiguous()
        m = None if mask is None else torch.as_tensor(mask).to(self.device, torch.uint8).contiguous()
        z = None if noise is None else torch.as_tensor(noise).to(self.device, torch.float64).contiguous()
        calls = getattr(self, '_goal_calls', 0)
        self._goal_calls = calls + 1
        sd = self._seed if self._seed is not None else 0
        _lib.check(self._L.ogbx_maze_set_goal(self._h, _lib.ptr(ij), _lib.ptr(m), _lib.ptr(z), int(sd), calls,
                                              self._stream()), 'set_goal')

    def _state_ptrs(self):
        q, g, e, t, ep = (_lib.c_void_p() for _ in range(5))
        _lib.check(self._L.ogbx_maze_state(self._h, q, g, e, t, ep))
        return q.value, g.value, e.value, t.value, ep.value

    def _state_views(self):
        """torch views of the env-owned state (qpos, goal, elapsed, task, episode)."""
        torch = _torch()
        q, g, e, t, ep = self._state_ptrs()
        n = self.num_envs

        return (
            _from_ptr(q, (n, 2), torch.float64, self.device),
            _from_ptr(g, (n, 2), torch.float64, self.device),
            _from_ptr(e, (n,), torch.int32, self.device),
            _from_ptr(t, (n,), torch.int32, self.device),
            _from_ptr(ep, (n,), torch.int32, self.device),  # uint32 counter, viewed as int32
        )

    def get_xy(self):
        return self._state_views()[0].clone()

    @property
    def cur_goal_xy(self):
        return self._state_views()[1].clone()

    def state_dict(self):
        q, g, e, t, ep = self._state_views()
        sd = dict(qpos=q.clone(), goal=g.clone(), elapsed=e.clone(), task=t.clone(), episode=ep.clone(),
                  seed=self._seed)
        if self._loco_env_type == 'ant':
            bq, bv = self.body_state()
            sd.update(body_qpos=bq.clone(), body_qvel=bv.clone())
        return sd

    def load_state_dict(self, sd):
        q, g, e, t, ep = self._state_views()
        q.copy_(sd['qpos'])
        g.copy_(sd['goal'])
        e.copy_(sd['elapsed'])
        t.copy_(sd['task'])
        if 'episode' in sd:
            ep.copy_(sd['episode'])
        if self._loco_env_type == 'ant' and 'body_qpos' in sd:
            bq, bv = self.body_state()
            bq.copy_(sd['body_qpos'])
            bv.copy_(sd['body_qvel'])
        if sd.get('seed') is not None:
            self._seed = int(sd['seed'])
            _lib.check(self._L.ogbx_maze_set_seed(self._h, self._seed))
        self._has_reset = True

    # ------------------------------------------------------------ reset/step
    def _task_tensor(self, task_id):
        torch = _torch()
        if isinstance(task_id, (int, np.integer)):
            assert 1 <= task_id <= self.num_tasks, f'Task ID must be in [1, {self.num_tasks}].'
            return torch.full((self.num_envs,), int(task_id), dtype=torch.int32, device=self.device)
        t = torch.as_tensor(task_id).to(self.device, torch.int32).reshape(-1).contiguous()
        assert t.numel() == self.num_envs, 'task_id tensor must have one entry per env'
        lo, hi = int(t.min()), int(t.max())
        assert 1 <= lo and hi <= self.num_tasks, f'Task ID must be in [1, {self.num_tasks}].'
        return t

    def _task_xy_tensor(self, task_info):
        torch = _torch()
        if isinstance(task_info, dict):
            ix, iy = self.ij_to_xy(task_info['init_ij'])
            gx, gy = self.ij_to_xy(task_info['goal_ij'])
            row = torch.tensor([ix, iy, gx, gy], dtype=torch.float64, device=self.device)
            return row.expand(self.num_envs, 4).contiguous()
        t = torch.as_tensor(task_info).to(self.device, torch.float64).contiguous()
        assert t.shape == (self.num_envs, 4), 'task_info tensor must be [num_envs, 4] (init_xy, goal_xy)'
        return t

    def reset(self, *, seed=None, options=None, mask=None):
        """MazeEnv.reset (maze.py:373-431) for every env (or those in ``mask``).

        options: ``task_id`` (int or [N] tensor), ``task_info`` (dict with
        init_ij/goal_ij, or an [N,4] xy tensor), ``noise`` ([N,4] injected
        uniform(-1,1) draws; test hook), ``render_goal`` (unsupported); ant
        handles also take ``body_draws`` ([N,29] injected AntEnv.reset_model
        draws: 15 uniform(-0.1,0.1), 14 standard normal) and ``goal_states``
        ([N,29] f64, the body state (qpos, qvel) the caller's physics reached
        after the goal reset and its 5 random-action steps, maze.py:408-413).
        Returns (obs, {'goal': goal}): point obs/goal [N,2] f64; ant obs [N,29]
        and goal = the goal observation [N,29] (goal_states with qpos[:2] :=
        goal_xy, maze.py:416-418; without goal_states the goal reset's
        unstepped reset_model state stands in), or the goal xy [N,2] under
        use_oracle_rep (maze.py:418,482-484).
        """
        if self._loco_env_type == 'humanoid':
            raise NotImplementedError('humanoid dynamics and its observation layout are out of scope')
        torch = _torch()
        options = {} if options is None else options
        if options.get('render_goal'):
            raise NotImplementedError('render_goal needs MuJoCo rendering (out of scope)')
        if seed is not None:
            # gymnasium reseeding: the Philox stream of every reset env restarts
            self._seed = int(seed) & ((1 << 64) - 1)
            _zero_episodes(self._state_views()[4], mask, self.device)
        elif self._seed is None:
            self._seed = (
                int(self._init_seed) if self._init_seed is not None else int(np.random.randint(0, 2**63 - 1))
            )
        task_t = task_xy = None
        if self._reward_task_id is not None:
            self.cur_task_id = self._reward_task_id
        elif 'task_id' in options:
            task_t = self._task_tensor(options['task_id'])
            self.cur_task_id = options['task_id'] if isinstance(options['task_id'], int) else None
        elif 'task_info' in options:
            task_xy = self._task_xy_tensor(options['task_info'])
            task_t = torch.ones(self.num_envs, dtype=torch.int32, device=self.device)
            self.cur_task_id = None
        else:
            self.cur_task_id = None  # drawn per env on the device
        noise = options.get('noise')
        if noise is not None:
            noise = torch.as_tensor(noise).to(self.device, torch.float64).contiguous()
            assert noise.shape == (self.num_envs, 4)
        m = None
        if mask is not None:
            m = torch.as_tensor(mask).to(self.device, torch.uint8).contiguous()
        if self._loco_env_type == 'ant':
            bd = options.get('body_draws')
            if bd is not None:
                bd = torch.as_tensor(bd).to(self.device, torch.float64).contiguous()
                assert bd.shape == (self.num_envs, 29)
            gs = options.get('goal_states')
            if gs is not None:
                gs = torch.as_tensor(gs).to(self.device, torch.float64).contiguous()
                assert gs.shape == (self.num_envs, 29), 'goal_states must be [num_envs, 29] (qpos, qvel)'
            elif not self._use_oracle_rep and not getattr(self, '_warned_goal_states', False):
                # the reference's goal observation is the body state after 5
                # random-action physics steps (maze.py:408-418) -- the caller's
                # physics; without it the unstepped reset_model state stands in
                self._warned_goal_states = True
                warnings.warn('antmaze reset without options["goal_states"]: info["goal"] is the unstepped '
                              'reset_model pose, not the reference goal observation (pass the body state your '
                              'physics reached after the goal reset, or use_oracle_rep=True)', stacklevel=2)
            gob = None if self._use_oracle_rep else self._goal_ob
            _lib.check(
                self._L.ogbx_antmaze_reset(self._h, _lib.ptr(task_t), _lib.ptr(task_xy), _lib.ptr(m),
                                           _lib.ptr(noise), _lib.ptr(bd), _lib.ptr(gs), _lib.ptr(self._obs),
                                           _lib.ptr(self._goal), _lib.ptr(gob), self._seed, self._stream()),
                'reset',
            )
            self._has_reset = True
            return self._obs, {'goal': self._goal if self._use_oracle_rep else self._goal_ob}
        _lib.check(
            self._L.ogbx_maze_reset(
                self._h,
                _lib.ptr(task_t),
                _lib.ptr(task_xy),
                _lib.ptr(m),
                _lib.ptr(noise),
                _lib.ptr(self._obs),
                _lib.ptr(self._goal),
                self._seed,
                self._stream(),
            ),
            'reset',
        )
        self._has_reset = True
        return self._obs, {'goal': self._goal}

    def _action(self, action):
        torch = _torch()
        if not isinstance(action, torch.Tensor):
            action = torch.as_tensor(np.asarray(action))
        if action.device != self.device:
            action = action.to(self.device)
        if action.dtype not in (torch.float32, torch.float64):
            action = action.to(torch.float32)
        if not action.is_contiguous():
            action = action.contiguous()
        return action

    def step(self, action):
        """One env step of all envs (maze.py:433-466 + point.py:64-95 + TimeLimit).

        action: [N,2] float32 (NEP-50 float32 scaling) or float64.
        Returns (obs, reward, terminated, truncated, info) with info['success'].
        """
        a = action
        # fast path: a contiguous [N, 2] float32 / float64 tensor on this device
        # (the common case; a few attribute reads instead of _action's checks)
        if (type(a) is self._Tensor and self._is_point and a.is_cuda and a.shape == self._act_shape
                and a.get_device() == self._dev_idx and a.is_contiguous()):
            dt = a.dtype
            f64 = 0 if dt is self._f32 else (1 if dt is self._f64t else -1)
        else:
            f64 = -1
        if f64 < 0:
            if not self._is_point:
                raise NotImplementedError(
                    f'{self._loco_env_type} dynamics are out of scope: advance body_state() with your physics '
                    'engine and call wrap_step(qpos, qvel)')
            a = self._action(action)
            if a.shape != (self.num_envs, 2):
                raise ValueError(f'action must have shape ({self.num_envs}, 2), got {tuple(a.shape)}')
            f64 = int(a.dtype == self._f64t)
        auto = self._auto_i
        if auto != self._bound_auto:
            _lib.check(self._L.ogbx_maze_bind_step(self._h, *self._step_out, auto), 'step')
            self._bound_auto = auto
        st = self._step_bound(self._h, a.data_ptr(), f64, self._raw_stream(self._dev_idx))
        if st:
            _lib.check(st, 'step')
        info = {'success': self._succ_b}
        if auto:
            info['final_observation'] = self._final_obs
        return self._obs, self._reward, self._term_b, self._trunc_b, info

    # ------------------------------------------------------------ antmaze wrapper
    def body_state(self):
        """Ant handles: device views (qpos f64[N,15], qvel f64[N,14]) of the body
        state -- what a physics engine reads and overwrites in place."""
        torch = _torch()
        if self._loco_env_type != 'ant':
            raise ValueError('body_state() is for ant handles')
        q, v = _lib.c_void_p(), _lib.c_void_p()
        _lib.check(self._L.ogbx_antmaze_state(self._h, q, v))
        n = self.num_envs
        return (_from_ptr(q.value, (n, 15), torch.float64, self.device),
                _from_ptr(v.value, (n, 14), torch.float64, self.device))

    def wrap_step(self, qpos, qvel, reset_states=None):
        """MazeEnv.step + TimeLimit (maze.py:433-466) around caller-supplied ant
        physics: qpos [N,15] / qvel [N,14] f64 = the post-physics state (the
        tensors of body_state(), stepped in place, or any other buffers).

        Returns (obs [N,29], reward, terminated, truncated, info{'success'}) as
        ``step`` does; with auto_reset, ``reset_states`` [N,29] (optional) are
        the caller's reset states for the envs that end (xy := init_xy)."""
        # Per-call host cost matters here (a 16k-env launch is ~5 us).  Fast
        # path: a (qpos, qvel) pair seen before -- the handle's own body_state()
        # views of an in-place engine, or a fixed ring of state buffers -- skips
        # the dtype / device checks: the pair's validated raw pointers are
        # cached by tensor identity (the cache holds the tensors, so their ids
        # stay unique while cached) and a hit only re-reads the pointers, shapes
        # and contiguity.  Anything else takes the checked path once and is
        # cached (at most 8 pairs).
        rs = None
        if reset_states is not None:
            torch = _torch()
            rs = torch.as_tensor(reset_states).to(self.device, torch.float64).contiguous()
            assert rs.shape == (self.num_envs, 29)
            rs = rs.data_ptr()
        hit = self._wrap_cache.get((id(qpos), id(qvel)))
        # a hit is re-checked against the storage pointer, strides and row
        # count it was validated with (set_ / .data = / a reallocating resize_
        # move the pointer; transpose_ and a reshaping resize_ change the
        # strides; an in-place shrinking resize_ keeps both but not the rows);
        # anything else revalidates.  (~0.2 us per tensor call; the launch is
        # ~5 us)
        n = self.num_envs
        if (hit is not None and hit[0] is qpos and hit[1] is qvel and qpos.data_ptr() == hit[2]
                and qvel.data_ptr() == hit[3] and qpos.stride() == (15, 1) and qvel.stride() == (14, 1)
                and qpos.shape[0] == n and qvel.shape[0] == n):
            qp, vp = hit[2], hit[3]
        else:
            qp, vp = self._wrap_validate(qpos, qvel)
        auto = self._auto_i
        if auto != self._bound_auto:
            _lib.check(self._L.ogbx_maze_bind_step(self._h, *self._step_out, auto), 'wrap_step')
            self._bound_auto = auto
        st = self._wrap_bound(self._h, qp, vp, rs, _raw_stream(self._dev_idx))
        if st != 0:
            _lib.check(st, 'wrap_step')
        info = {'success': self._succ_b}
        if self.auto_reset:
            info['final_observation'] = self._final_obs
        return self._obs, self._reward, self._term_b, self._trunc_b, info

    def _wrap_validate(self, qpos, qvel):
        if self._loco_env_type != 'ant':
            raise ValueError('wrap_step() is for ant handles; point envs use step(action)')
        q, v = qpos, qvel
        if (q.shape != self._ant_qshape or v.shape != self._ant_vshape or q.dtype != self._f64 or v.dtype != self._f64
                or q.get_device() != self.device.index or v.get_device() != self.device.index):
            raise ValueError(f'wrap_step: qpos/qvel must be float64 {tuple(self._ant_qshape)}/{tuple(self._ant_vshape)} '
                             f'on {self.device}')
        if not (q.is_contiguous() and v.is_contiguous()):
            # a strided pair is copied each call, never cached; the copies stay
            # referenced by the handle until the next such call, past the launch
            self._wrap_tmp = (q.contiguous(), v.contiguous())
            return self._wrap_tmp[0].data_ptr(), self._wrap_tmp[1].data_ptr()
        if len(self._wrap_cache) >= 8:  # a small ring of engine buffers; bounds what the cache keeps alive
            self._wrap_cache.clear()
        qp, vp = q.data_ptr(), v.data_ptr()
        self._wrap_cache[(id(q), id(v))] = (q, v, qp, vp)
        return qp, vp

    def rollout(self, actions, out=None):
        """K fused steps in ONE launch: actions [K,N,2] -> per-step outputs [K,N,...].

        Equivalent to K calls of ``step`` with the same auto_reset setting.
        """
        torch = _torch()
        a = self._action(actions)
        K = a.shape[0]
        if a.shape != (K, self.num_envs, 2):
            raise ValueError(f'actions must have shape (K, {self.num_envs}, 2)')
        if out is None:
            kw = dict(device=self.device)
            out = dict(
                obs=torch.empty(K, self.num_envs, 2, dtype=torch.float64, **kw),
                reward=torch.empty(K, self.num_envs, dtype=torch.float32, **kw),
                terminated=torch.empty(K, self.num_envs, dtype=torch.uint8, **kw),
                truncated=torch.empty(K, self.num_envs, dtype=torch.uint8, **kw),
                success=torch.empty(K, self.num_envs, dtype=torch.uint8, **kw),
            )
        _lib.check(
            self._L.ogbx_maze_step(
                self._h,
                _lib.ptr(a),
                int(a.dtype == torch.float64),
                K,
                _lib.ptr(out['obs']),
                _lib.ptr(out['reward']),
                _lib.ptr(out['terminated']),
                _lib.ptr(out['truncated']),
                _lib.ptr(out['success']),
                None,
                int(self.auto_reset),
                self._stream(),
            ),
            'rollout',
        )
        return out

    def rollout_until_done(self, actions, out=None):
        """Evaluation episodes in ONE launch (no auto-reset): env i steps with
        actions[k, i] until its episode ends (terminated | truncated) or the K
        actions run out -- the reference's ``while not done: env.step(...)``
        loop (impls/utils/evaluation.py:83-112) for the whole batch.

        Returns the rollout dict of ``rollout`` plus ``steps`` (int32 [N], rows
        written per env); rows k >= steps[i] are left as they were.  Each wave
        of 64 envs stops once all its episodes ended."""
        torch = _torch()
        if self.auto_reset:
            raise ValueError('rollout_until_done needs auto_reset=False (an auto-reset episode never ends)')
        a = self._action(actions)
        K = a.shape[0]
        if a.shape != (K, self.num_envs, 2):
            raise ValueError(f'actions must have shape (K, {self.num_envs}, 2)')
        if out is None:
            kw = dict(device=self.device)
            out = dict(
                obs=torch.zeros(K, self.num_envs, 2, dtype=torch.float64, **kw),
                reward=torch.zeros(K, self.num_envs, dtype=torch.float32, **kw),
                terminated=torch.zeros(K, self.num_envs, dtype=torch.uint8, **kw),
                truncated=torch.zeros(K, self.num_envs, dtype=torch.uint8, **kw),
                success=torch.zeros(K, self.num_envs, dtype=torch.uint8, **kw),
                steps=torch.zeros(self.num_envs, dtype=torch.int32, **kw),
            )
        _lib.check(
            self._L.ogbx_maze_rollout_until_done(
                self._h,
                _lib.ptr(a),
                int(a.dtype == torch.float64),
                K,
                _lib.ptr(out['obs']),
                _lib.ptr(out['reward']),
                _lib.ptr(out['terminated']),
                _lib.ptr(out['truncated']),
                _lib.ptr(out['success']),
                _lib.ptr(out['steps']),
                self._stream(),
            ),
            'rollout_until_done',
        )
        return out

    def physics(self, qpos, action):
        """Free-standing PointEnv physics (point.py:68-73) for [n,2] qpos/actions."""
        torch = _torch()
        q = qpos.to(self.device, torch.float64).contiguous()
        a = self._action(action)
        out = torch.empty_like(q)
        contact = torch.empty(q.shape[0], dtype=torch.uint8, device=self.device)
        _lib.check(
            self._L.ogbx_point_physics(
                self._h,
                _lib.ptr(q),
                _lib.ptr(a),
                int(a.dtype == torch.float64),
                q.shape[0],
                _lib.ptr(out),
                _lib.ptr(contact),
                self._stream(),
            )
        )
        return out, contact


def _zero_episodes(episode, mask, device):
    """Restart the per-env Philox reset counters (all envs, or those in mask)."""
    if mask is None:
        episode.zero_()
    else:
        m = _torch().as_tensor(mask).to(device).bool().reshape(-1)
        episode.masked_fill_(m, 0)


def _raw_stream(device_index):
    """hipStream_t (as an int) of torch's current stream on device_index."""
    global _raw_stream
    _raw_stream = _torch()._C._cuda_getCurrentRawStream  # bind once
    return _raw_stream(device_index)


def _from_ptr(addr, shape, dtype, device):
    """Non-owning torch view of device memory owned by libogbx."""
    torch = _torch()
    numel = int(np.prod(shape))
    nbytes = numel * torch.empty((), dtype=dtype).element_size()
    iface = {
        'shape': tuple(shape),
        'typestr': {torch.float64: '<f8', torch.int32: '<i4', torch.uint8: '|u1', torch.int8: '|i1',
                    torch.float32: '<f4'}[dtype],
        'data': (addr, False),
        'version': 3,
        'strides': None,
    }

    class _Holder:
        __cuda_array_interface__ = iface

    t = torch.as_tensor(_Holder(), device=device)
    assert t.numel() * t.element_size() == nbytes
    return t


# ---------------------------------------------------------------- registry
_LOCO_MAX_STEPS = {'point': 1000, 'ant': 1000, 'humanoid': 2000}


def parse_env_id(env_id):
    """Registry entries of ogbench/locomaze/__init__.py:16-527 as kwargs."""
    m = re.fullmatch(r'(visual-)?(point|ant|humanoid)maze-(arena|medium|large|giant|teleport)'
                     r'(-singletask(?:-task(\d))?)?-v0', env_id)
    if m is None:
        return None
    visual, loco, maze, single, task = m.groups()
    if visual:
        raise NotImplementedError(f'{env_id}: pixel observations are out of scope')
    max_steps = _LOCO_MAX_STEPS[loco]
    if loco == 'humanoid' and maze == 'giant':
        max_steps = 4000
    kwargs = dict(loco_env_type=loco, maze_type=maze, max_episode_steps=max_steps)
    if single:
        kwargs.update(
            reward_task_id=0 if task is None else int(task), add_noise_to_goal=False, success_timing='pre'
        )
    return kwargs
