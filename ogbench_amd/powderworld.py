"""Batched powderworld environments on MI355X.

``PowderworldEnv`` is the batched counterpart of the reference
``PowderworldEnv`` (ogbench/powderworld/powderworld_env.py:21-476) in 'task'
mode under gymnasium's TimeLimit (registry: ogbench/powderworld/__init__.py):
the same constructor options, Discrete action protocol (element, x, y over
three steps), task table, goal observation and tolerance-based success.  Every
env's world lives in HBM; a step is one ``ogbx_powder_step`` launch in which
each env's 256-thread workgroup runs the cellular automaton in LDS.

Differences that follow from batching (documented in DESIGN.md):
  * returned tensors are views of env-owned buffers that the next ``step``
    overwrites (clone them to keep them);
  * ``info['success']``, ``terminated`` and ``truncated`` are bool tensors;
  * random draws (the initial random semantic action, the random task when no
    ``task_id`` is given, and the replacement of invalid actions) come from a
    counter-based Philox stream keyed by ``seed``; they can be injected
    exactly (``options['reset_action']``, ``step(..., draws=...)``) for parity
    tests.
  * medium/hard (num_elems 5/8) run every rule of PWSim (sand, fluids, ice,
    water, fire, plant, velocity); their forward draws three float32 rand
    fields per call, which come from Philox on the device and can be
    injected exactly (``options['rand']``, ``step(..., rand=...)``,
    ``forward_full(..., rand=...)``).  Their goal worlds are replayed per env
    at every reset (the forward is stochastic) and kept on the device
    (``goal_ids()``).
"""

from __future__ import annotations

import numpy as np

from . import _lib
from .locomaze import _from_ptr, _resolve_device, _torch, _zero_episodes
from .powder_tasks import task_names, task_sequences, task_tols
from .spaces import Box, Discrete

ELEM_NAMES = {2: ['plant', 'stone'],
              5: ['sand', 'water', 'fire', 'plant', 'stone'],
              8: ['sand', 'water', 'fire', 'plant', 'stone', 'gas', 'wood', 'ice']}


class PowderworldEnv:
    """Batch of ``num_envs`` powderworld envs (reference: powderworld_env.py:21-476)."""

    def __init__(
        self,
        num_envs=1,
        device=None,
        env_type='easy',
        world_size=32,
        grid_size=4,
        brush_size=4,
        num_elems=2,
        mode='task',
        max_episode_steps=500,
        auto_reset=False,
        seed=None,
        env_base=0,
    ):
        assert mode in ('task', 'data'), 'mode must be task or data'
        if mode != 'task':
            raise NotImplementedError("only mode='task' is implemented (data collection runs on the host)")
        if num_elems not in ELEM_NAMES:
            raise ValueError(f'num_elems must be one of {sorted(ELEM_NAMES)}')
        torch = _torch()
        self.device = _resolve_device(device)
        self.num_envs = int(num_envs)
        self._world_size = int(world_size)
        self._grid_size = int(grid_size)
        self._brush_size = int(brush_size)
        self._num_elems = int(num_elems)
        self._mode = mode
        self._elem_names = list(ELEM_NAMES[num_elems])
        self.max_episode_steps = int(max_episode_steps)
        self.auto_reset = bool(auto_reset)

        opts = _lib.PowderOpts(
            world_size=self._world_size,
            grid_size=self._grid_size,
            brush_size=self._brush_size,
            num_elems=self._num_elems,
            max_episode_steps=self.max_episode_steps,
            env_base=int(env_base),
        )
        self.env_base = int(env_base)
        L = _lib.lib()
        h = _lib.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(L.ogbx_powder_create(opts, self.num_envs, self.device.index, h))
        self._h, self._L = h, L
        ws, xy, ne, nt, tol = (_lib.c_int32() for _ in range(5))
        _lib.check(L.ogbx_powder_describe(h, ws, xy, ne, nt, tol))
        self._xy_action_size = xy.value
        self.num_tasks = nt.value
        self._tol = tol.value
        self._full = self._num_elems != 2
        seqs, names, tols = task_sequences(num_elems), task_names(num_elems), task_tols(num_elems)
        self.task_infos = [
            dict(task_name=names[i], action_seq=[(self._elem_names[e], x, y) for e, x, y in seqs[i]], tol=tols[i])
            for i in range(self.num_tasks)
        ]
        self._max_seq = max(len(q) for q in seqs)

        H = W = self._world_size
        self.single_observation_space = Box(0, 255, (H, W, 6), np.uint8)
        self.single_action_space = Discrete(max(self._num_elems, self._xy_action_size))
        self.observation_space = Box(0, 255, (self.num_envs, H, W, 6), np.uint8)

        n = self.num_envs
        kw = dict(device=self.device)
        self._obs = torch.zeros(n, H, W, 6, dtype=torch.uint8, **kw)
        self._goal = torch.zeros(n, H, W, 6, dtype=torch.uint8, **kw)
        self._reward = torch.zeros(n, dtype=torch.float32, **kw)
        self._term = torch.zeros(n, dtype=torch.uint8, **kw)
        self._trunc = torch.zeros(n, dtype=torch.uint8, **kw)
        self._succ = torch.zeros(n, dtype=torch.uint8, **kw)
        self._seed = None
        self._init_seed = seed
        self.cur_task_id = None

    # ------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, '_h', None) is not None and self._h.value:
            self._L.ogbx_powder_destroy(self._h)
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

    # ------------------------------------------------------------ state
    def goal_worlds(self):
        """Element ids of every task's goal world, uint8 [num_tasks, H, W] (host).

        Easy only: medium/hard goals are stochastic and per env (goal_ids())."""
        if self._full:
            raise ValueError('medium/hard goal worlds are replayed per env at reset; use goal_ids()')
        H = W = self._world_size
        out = np.zeros((self.num_tasks, H, W), np.uint8)
        _lib.check(self._L.ogbx_powder_goal_worlds(self._h, out.ctypes.data_as(_lib.c_void_p)))
        return out

    def _state_views(self):
        torch = _torch()
        w, c, e, ep = (_lib.c_void_p() for _ in range(4))
        _lib.check(self._L.ogbx_powder_state(self._h, w, c, e, ep))
        n, H = self.num_envs, self._world_size
        return (_from_ptr(w.value, (n, H, H), torch.uint8, self.device),
                _from_ptr(c.value, (n,), torch.int32, self.device),
                _from_ptr(e.value, (n,), torch.int32, self.device),
                _from_ptr(ep.value, (n,), torch.int32, self.device))

    def _scalar_view(self, which):
        """One of ctrl / elapsed / episode, int32 / uint32 [N], without asking
        for the world pointer (handing that out marks the render cache stale,
        ogbx_powder_state)."""
        torch = _torch()
        ptrs = [None, None, None, None]
        k = {'ctrl': 1, 'elapsed': 2, 'episode': 3}[which]
        ptrs[k] = _lib.c_void_p()
        _lib.check(self._L.ogbx_powder_state(self._h, *ptrs))
        return _from_ptr(ptrs[k].value, (self.num_envs,), torch.int32, self.device)

    def _read_views(self):
        """Read-only (world, momentum, velocity, goal ids) views through
        ogbx_powder_state_view: no writable pointer is handed out, so the
        render cache stays valid (momentum/velocity/goal None for easy)."""
        torch = _torch()
        ptrs = [_lib.c_void_p() for _ in range(4)]
        if not self._full:
            ptrs[1:] = [None, None, None]
        _lib.check(self._L.ogbx_powder_state_view(self._h, *ptrs))
        n, H = self.num_envs, self._world_size
        w = _from_ptr(ptrs[0].value, (n, H, H), torch.uint8, self.device)
        if not self._full:
            return w, None, None, None
        return (w, _from_ptr(ptrs[1].value, (n, H, H), torch.int8, self.device),
                _from_ptr(ptrs[2].value, (n, H, H, 2), torch.float32, self.device),
                _from_ptr(ptrs[3].value, (n, H, H), torch.uint8, self.device))

    def _full_views(self):
        torch = _torch()
        m, v, g = (_lib.c_void_p() for _ in range(3))
        _lib.check(self._L.ogbx_powder_full_state(self._h, m, v, g))
        n, H = self.num_envs, self._world_size
        return (_from_ptr(m.value, (n, H, H), torch.int8, self.device),
                _from_ptr(v.value, (n, H, H, 2), torch.float32, self.device),
                _from_ptr(g.value, (n, H, H), torch.uint8, self.device))

    def goal_ids(self):
        """Goal element ids per env, uint8 [N, H, W] (reference cur_goal_world)."""
        if self._full:
            return self._read_views()[3]
        torch = _torch()
        g = torch.as_tensor(self.goal_worlds(), device=self.device)
        return g[(self.cur_task_ids.long() - 1).clamp(min=0)]

    def world_full(self):
        """Worlds in the reference's (N, 9, H, W) float32 layout."""
        torch = _torch()
        w, m, v, _ = self._read_views()
        ids = (w & 31).long()
        dens = torch.tensor([1, 4, 3, 2, 0, 4, 4, 0, 4, 3, 3, 2, 2, 4, 2, 4, 3, 3, 3, 4, 3, 0, 0, 0, 0, 0, 0, 0, 0,
                             0, 0, 0], dtype=torch.float32, device=self.device)
        out = torch.zeros(self.num_envs, 9, *w.shape[1:], dtype=torch.float32, device=self.device)
        out[:, 0] = ids.float()
        out[:, 1] = dens[ids]
        out[:, 2] = ((w >> 5) & 1).float()
        out[:, 8] = ((w >> 6) & 1).float()
        if self._full:
            out[:, 3] = v[..., 0]
            out[:, 4] = v[..., 1]
            out[:, 6] = m.float()
        return out

    def world_ids(self):
        """Element id of every cell, uint8 [N, H, W] (reference self._world[:, 0])."""
        return self._read_views()[0] & 31

    @property
    def cur_task_ids(self):
        return (self._scalar_view('ctrl') >> 16) & 255

    def state_dict(self):
        w, m, v, g = self._read_views()
        c, e, ep = (self._scalar_view(k) for k in ('ctrl', 'elapsed', 'episode'))
        sd = dict(world=w.clone(), ctrl=c.clone(), elapsed=e.clone(), episode=ep.clone(), seed=self._seed)
        if self._full:
            sd.update(momentum=m.clone(), velocity=v.clone(), goal=g.clone())
        return sd

    def load_state_dict(self, sd):
        w, c, e, ep = self._state_views()
        w.copy_(sd['world'])
        c.copy_(sd['ctrl'])
        e.copy_(sd['elapsed'])
        if 'episode' in sd:
            ep.copy_(sd['episode'])
        if sd.get('seed') is not None:
            self._seed = int(sd['seed'])
            _lib.check(self._L.ogbx_powder_set_seed(self._h, self._seed))
        if self._full:
            m, v, g = self._full_views()
            m.copy_(sd['momentum'])
            v.copy_(sd['velocity'])
            g.copy_(sd['goal'])
        _lib.check(self._L.ogbx_powder_state_written(self._h))

    def set_step_phase(self, phase):
        """Declare that every env steps in phase, `phase` steps after a common
        all-env reset (-1: unknown, what load_state_dict leaves).  Only the
        launch plan of medium/hard steps uses it; a wrong hint costs time, not
        results (include/ogbx.h ogbx_powder_set_phase)."""
        _lib.check(self._L.ogbx_powder_set_phase(self._h, int(phase)))

    def forward(self, worlds, steps=1):
        """PWSim.forward (sim.py:363-380) on packed worlds uint8 [n, H, W]."""
        torch = _torch()
        if self._full:
            raise ValueError('medium/hard worlds carry velocity and momentum; use forward_full')
        w = torch.as_tensor(worlds).to(self.device, torch.uint8).contiguous()
        out = torch.empty_like(w)
        _lib.check(self._L.ogbx_powder_forward(self._h, _lib.ptr(w), w.shape[0], int(steps), _lib.ptr(out),
                                               self._stream()))
        return out

    def forward_full(self, worlds, steps=1, rand=None, render=False):
        """PWSim.forward with every rule on (n, 9, H, W) float32 worlds.

        rand: float32 [steps, n, 3, H, W] (rand_movement, rand_interact,
        rand_element per forward) or None (Philox).  render: also return
        PWRenderer.render of the result, uint8 [n, H, W, 3]."""
        torch = _torch()
        w = torch.as_tensor(worlds).to(self.device, torch.float32).contiguous()
        n, H = w.shape[0], self._world_size
        assert tuple(w.shape[1:]) == (9, H, H), f'worlds must be (n, 9, {H}, {H})'
        r = None
        if rand is not None:
            r = torch.as_tensor(rand).to(self.device, torch.float32).contiguous()
            assert tuple(r.shape) == (int(steps), n, 3, H, H), 'rand must be [steps, n, 3, H, W]'
        out = torch.empty_like(w)
        img = torch.empty(n, H, H, 3, dtype=torch.uint8, device=self.device) if render else None
        _lib.check(self._L.ogbx_powder_forward_full(self._h, _lib.ptr(w), n, int(steps), _lib.ptr(r), _lib.ptr(out),
                                                    _lib.ptr(img), self._stream()), 'forward_full')
        return (out, img) if render else out

    def _rand(self, rand, shape):
        if rand is None:
            return None
        if not self._full:
            raise ValueError('rand fields apply to medium/hard worlds only')
        torch = _torch()
        r = torch.as_tensor(rand).to(self.device, torch.float32).contiguous()
        if tuple(r.shape) != shape:
            raise ValueError(f'rand must have shape {shape}, got {tuple(r.shape)}')
        return r

    # ------------------------------------------------------------ reset/step
    def reset(self, *, seed=None, options=None, mask=None):
        """PowderworldEnv.reset (powderworld_env.py:284-352) for all envs (or ``mask``).

        options: ``task_id`` (int or [N] tensor), ``reset_action`` ([N,3]
        (elem index, x, y) of the random initial semantic action; test hook),
        ``rand`` (medium/hard test hook: float32 [N, R, 3, H, W] rand fields,
        row s < len(task) for goal action s, row len(task) for the reset's
        forward, R >= longest task + 1), ``render_goal`` (unsupported).  Returns (obs [N,H,W,6] u8, {'goal': ...}).
        """
        torch = _torch()
        options = {} if options is None else options
        if options.get('render_goal'):
            raise NotImplementedError('render_goal (PIL upscaling) is out of scope; use info["goal"]')
        if 'task_info' in options:
            raise NotImplementedError('custom task_info action sequences are not supported on the device')
        if seed is not None:
            # gymnasium reseeding: the Philox stream of every reset env restarts
            self._seed = int(seed) & ((1 << 64) - 1)
            _zero_episodes(self._scalar_view('episode'), mask, self.device)
        elif self._seed is None:
            self._seed = (int(self._init_seed) if self._init_seed is not None
                          else int(np.random.randint(0, 2**63 - 1)))
        task_t = None
        if 'task_id' in options:
            tid = options['task_id']
            if isinstance(tid, (int, np.integer)):
                assert 1 <= tid <= self.num_tasks, f'Task ID must be in [1, {self.num_tasks}].'
                task_t = torch.full((self.num_envs,), int(tid), dtype=torch.int32, device=self.device)
                self.cur_task_id = int(tid)
            else:
                task_t = torch.as_tensor(tid).to(self.device, torch.int32).reshape(-1).contiguous()
                assert task_t.numel() == self.num_envs, 'task_id tensor must have one entry per env'
                assert 1 <= int(task_t.min()) and int(task_t.max()) <= self.num_tasks, \
                    f'Task ID must be in [1, {self.num_tasks}].'
                self.cur_task_id = None
        else:
            self.cur_task_id = None
        ra = options.get('reset_action')
        if ra is not None:
            ra = torch.as_tensor(ra).to(self.device, torch.int32).reshape(self.num_envs, 3).contiguous()
            assert int(ra[:, 0].max()) < self._num_elems and int(ra[:, 1:].max()) < self._xy_action_size
        m = None
        if mask is not None:
            m = torch.as_tensor(mask).to(self.device, torch.uint8).contiguous()
        rand, rows = options.get('rand'), 0
        if rand is not None:
            rows = int(np.shape(rand)[1])
            H = self._world_size
            rand = self._rand(rand, (self.num_envs, rows, 3, H, H))
        _lib.check(
            self._L.ogbx_powder_reset(self._h, _lib.ptr(task_t), _lib.ptr(m), _lib.ptr(ra), _lib.ptr(rand), rows,
                                      _lib.ptr(self._obs), _lib.ptr(self._goal), self._seed, self._stream()),
            'reset',
        )
        return self._obs, {'goal': self._goal}

    def _actions(self, action, shape):
        torch = _torch()
        if not isinstance(action, torch.Tensor):
            action = torch.as_tensor(np.asarray(action))
        action = action.to(self.device, torch.int32).contiguous()
        if tuple(action.shape) != shape:
            raise ValueError(f'action must have shape {shape}, got {tuple(action.shape)}')
        return action

    def step(self, action, draws=None, rand=None):
        """One PowderworldEnv.step (powderworld_env.py:354-427) + TimeLimit for all envs.

        action: int [N].  draws: optional int [N] replacement values for
        invalid actions (the reference's np.random.randint; test hook).
        rand: medium/hard test hook, float32 [N, 3, H, W] rand fields of this
        step's forward (used by envs at their third action step).
        """
        a = self._actions(action, (self.num_envs,))
        d = None if draws is None else self._actions(draws, (self.num_envs,))
        H = self._world_size
        r = self._rand(rand, (self.num_envs, 3, H, H))
        _lib.check(
            self._L.ogbx_powder_step(self._h, _lib.ptr(a), 1, _lib.ptr(d), _lib.ptr(r), _lib.ptr(self._obs),
                                     _lib.ptr(self._reward), _lib.ptr(self._term), _lib.ptr(self._trunc),
                                     _lib.ptr(self._succ), int(self.auto_reset), self._stream()),
            'step',
        )
        torch = _torch()
        info = {'success': self._succ.view(torch.bool)}
        return self._obs, self._reward, self._term.view(torch.bool), self._trunc.view(torch.bool), info

    def rollout(self, actions, draws=None, out=None, rand=None):
        """K fused steps in ONE launch: actions [K,N] -> per-step outputs [K,N,...]."""
        torch = _torch()
        K = int(np.shape(actions)[0])
        a = self._actions(actions, (K, self.num_envs))
        d = None if draws is None else self._actions(draws, (K, self.num_envs))
        H = self._world_size
        r = self._rand(rand, (K, self.num_envs, 3, H, H))
        if out is None:
            kw = dict(device=self.device)
            out = dict(
                obs=torch.empty(K, self.num_envs, H, H, 6, dtype=torch.uint8, **kw),
                reward=torch.empty(K, self.num_envs, dtype=torch.float32, **kw),
                terminated=torch.empty(K, self.num_envs, dtype=torch.uint8, **kw),
                truncated=torch.empty(K, self.num_envs, dtype=torch.uint8, **kw),
                success=torch.empty(K, self.num_envs, dtype=torch.uint8, **kw),
            )
        _lib.check(
            self._L.ogbx_powder_step(self._h, _lib.ptr(a), K, _lib.ptr(d), _lib.ptr(r), _lib.ptr(out['obs']),
                                     _lib.ptr(out['reward']), _lib.ptr(out['terminated']),
                                     _lib.ptr(out['truncated']), _lib.ptr(out['success']), int(self.auto_reset),
                                     self._stream()),
            'rollout',
        )
        return out

    def semantic_action_to_action(self, elem_name, x, y, action_step):
        """powderworld_env.py:429-437 (the action step is per env here)."""
        if action_step == 0:
            return self._elem_names.index(elem_name)
        return x if action_step == 1 else y
