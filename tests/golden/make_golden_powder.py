"""Golden fixtures for powderworld, from the reference's own NumPy code.

Imports ogbench/powderworld/sim.py (pure NumPy) and powderworld_env.py (with a
small in-process stand-in for gymnasium.Env / spaces) by file path, runs them
in-process and saves inputs/outputs only (tests/golden/powder_golden.npz):

  * PWSim.forward on random easy-element worlds (ids {0,1,8,9} with random
    gravity / did-gravity channels, no border -> exercises the periodic rolls
    and zero-padded convolutions), 32x32 and 64x64;
  * PWRenderer.render colour LUT;
  * PowderworldEnv(num_elems=2) at world_size 32 and 64: the 5 task goal worlds
    and goal observations, resets with recorded np.random draws, and step
    traces (valid and invalid actions, recorded np.random draws).
"""

import importlib.util
import os
import sys
import types

import numpy as np

REF = os.environ.get('OGBENCH_REF', '/root/reference')
OUT = os.path.dirname(os.path.abspath(__file__))


def _gym_stub():
    gym = types.ModuleType('gymnasium')

    class Env:
        pass

    spaces = types.ModuleType('gymnasium.spaces')

    class Box:
        def __init__(self, low, high, shape, dtype):
            self.shape, self.dtype = shape, dtype

    class Discrete:
        def __init__(self, n):
            self.n = n

    spaces.Box, spaces.Discrete = Box, Discrete
    gym.Env, gym.spaces = Env, spaces
    sys.modules['gymnasium'] = gym
    sys.modules['gymnasium.spaces'] = spaces


def reference_modules():
    _gym_stub()
    pkg = types.ModuleType('ogbench')
    pkg.__path__ = [os.path.join(REF, 'ogbench')]
    sys.modules.setdefault('ogbench', pkg)
    sub = types.ModuleType('ogbench.powderworld')
    sub.__path__ = [os.path.join(REF, 'ogbench/powderworld')]
    sys.modules['ogbench.powderworld'] = sub

    def load(name, path):
        spec = importlib.util.spec_from_file_location(name, path)
        mod = importlib.util.module_from_spec(spec)
        sys.modules[name] = mod
        spec.loader.exec_module(mod)
        return mod

    sim = load('ogbench.powderworld.sim', os.path.join(REF, 'ogbench/powderworld/sim.py'))
    env = load('ogbench.powderworld.powderworld_env', os.path.join(REF, 'ogbench/powderworld/powderworld_env.py'))
    return sim, env


class Recorder:
    def __init__(self, names=('randint', 'choice', 'rand')):
        self.names, self.log, self._saved = names, [], {}

    def __enter__(self):
        for name in self.names:
            fn = getattr(np.random, name)
            self._saved[name] = fn

            def wrap(*a, _fn=fn, _name=name, **k):
                v = _fn(*a, **k)
                self.log.append((_name, v))
                return v

            setattr(np.random, name, wrap)
        return self

    def __exit__(self, *exc):
        for k, fn in self._saved.items():
            setattr(np.random, k, fn)


def main():
    sim, envm = reference_modules()
    rng = np.random.RandomState(4242)
    out = {}
    pw = sim.PWSim()
    # --- forward on random easy worlds (ids + flag channels), with rand fields recorded
    for size in (32, 64):
        n = 6
        ids = rng.choice([0, 0, 0, 1, 8, 9, 9], size=(n, size, size))
        world = pw.id_to_pw(ids).astype(np.float32)
        # random stone gravity and did-gravity states
        world[:, 2] = np.where(ids == 9, rng.randint(0, 2, (n, size, size)), world[:, 2])
        world[:, 8] = rng.randint(0, 2, (n, size, size)) * (ids != 1)
        w0 = world.copy()
        outs = [w0]
        for _ in range(4):
            outs.append(pw.forward(outs[-1].copy()))
        out[f'fwd{size}_in'] = w0
        out[f'fwd{size}_out'] = np.stack(outs[1:])
    # --- renderer LUT (float32 colour * 255 -> uint8) for every element id
    r = sim.PWRenderer()
    allids = np.arange(21).reshape(1, 21, 1)
    wid = pw.id_to_pw(np.repeat(allids, 2, axis=2)).astype(np.float32)
    out['render_lut'] = r.render(wid)[:, 0, :]
    # --- env: tasks, resets and step traces
    for size in (32, 64):
        env = envm.PowderworldEnv(world_size=size, num_elems=2)
        goals, gobs = [], []
        for t in range(1, 6):
            np.random.seed(t)
            ob, info = env.reset(options=dict(task_id=t))
            goals.append(env.cur_goal_world.astype(np.uint8))
            gobs.append(info['goal'])
        out[f'env{size}_goal_world'] = np.stack(goals)
        out[f'env{size}_goal_ob'] = np.stack(gobs)
        # traces: reset (recorded draws) then steps with mixed valid/invalid actions
        n_tr, T = 6, 90
        xy = env._xy_action_size
        for tr in range(n_tr):
            np.random.seed(100 + tr)
            task = 1 + tr % 5
            with Recorder(('randint', 'choice')) as rec:
                ob, info = env.reset(options=dict(task_id=task))
            # reset draws: choice(elem_names), randint(xy), randint(xy)
            names = [v for k, v in rec.log]
            elem = env._elem_names.index(names[-3])
            out[f'env{size}_tr{tr}_reset'] = np.array([task, elem, names[-2], names[-1]], np.int64)
            out[f'env{size}_tr{tr}_reset_ob'] = ob
            obs, rews, terms, succs, acts, draws = [], [], [], [], [], []
            for t in range(T):
                if rng.rand() < 0.15:
                    a = int(rng.randint(max(2, xy), max(2, xy) + 3))  # invalid for every stage
                else:
                    a = int(rng.randint(0, 2 if env._action_step == 0 else xy))
                with Recorder(('randint',)) as rec:
                    ob, rew, term, trunc, info = env.step(a)
                draws.append(int(rec.log[0][1]) if rec.log else -1)
                acts.append(a)
                obs.append(ob)
                rews.append(rew)
                terms.append(term)
                succs.append(info['success'])
            out[f'env{size}_tr{tr}_actions'] = np.array(acts, np.int64)
            out[f'env{size}_tr{tr}_draws'] = np.array(draws, np.int64)
            out[f'env{size}_tr{tr}_obs'] = np.stack(obs)
            out[f'env{size}_tr{tr}_reward'] = np.array(rews, np.float64)
            out[f'env{size}_tr{tr}_terminated'] = np.array(terms, bool)
            out[f'env{size}_tr{tr}_success'] = np.array(succs, np.float64)
            out[f'env{size}_tr{tr}_final_world'] = env._world[0, 0].astype(np.uint8)
    np.savez_compressed(os.path.join(OUT, 'powder_golden.npz'), **out)
    print('powder golden:', len(out), 'arrays')


class RandRecorder:
    """Record the float32 rand fields PWSim.forward draws (np.random.rand)."""

    def __init__(self):
        self.log = []

    def __enter__(self):
        self._fn = np.random.rand

        def wrap(*a, **k):
            v = self._fn(*a, **k)
            self.log.append(np.asarray(v).astype(np.float32))  # as PWSim.forward casts them
            return v

        np.random.rand = wrap
        return self

    def __exit__(self, *exc):
        np.random.rand = self._fn


def full_worlds(pw, rng, n, size):
    """Random medium/hard worlds: every element the 5/8-element envs place, walls,
    dust/lava/acid, stone supports, fluid momentum and velocity fields (some above
    the velocity rule's 1.0 and 2.0 thresholds)."""
    # elements the 5- and 8-element envs can produce (no dust/lava/acid/agents)
    ids = rng.choice([0, 0, 0, 0, 1, 2, 3, 3, 4, 5, 6, 7, 8, 9, 9], size=(n, size, size))
    world = pw.id_to_pw(ids).astype(np.float32)
    world[:, 2] = np.where(ids == 9, rng.randint(0, 2, (n, size, size)), world[:, 2])
    world[:, 8] = rng.randint(0, 2, (n, size, size)) * (ids != 1)
    fluid = np.isin(ids, [0, 3, 4])
    world[:, 6] = np.where(fluid, rng.choice([-2.0, 0.0, 2.0], size=(n, size, size)), 0.0)
    vel = rng.normal(0, 1.5, (n, 2, size, size)).astype(np.float32)
    vel *= (rng.rand(n, 1, size, size) < 0.3)
    world[:, 3:5] = vel
    return world


def main_full():
    """PWSim.forward with every rule active on medium/hard-style worlds, the
    rand fields recorded per forward; and PowderworldEnv(num_elems=5/8) traces
    with every draw recorded (goal replay, reset action, steps)."""
    sim, envm = reference_modules()
    rng = np.random.RandomState(9090)
    out = {}
    pw = sim.PWSim()
    for size in (32, 64):
        n = 4 if size == 32 else 2
        w0 = full_worlds(pw, rng, n, size)
        outs, rands = [w0], []
        np.random.seed(size)
        for _ in range(6):
            with RandRecorder() as rec:
                outs.append(pw.forward(outs[-1].copy()))
            rands.append(np.stack(rec.log, 1))  # [n, 3, 1, H, W]
        out[f'full{size}_in'] = w0
        out[f'full{size}_out'] = np.stack(outs[1:])
        out[f'full{size}_rand'] = np.stack(rands)[:, :, :, 0]  # [T, n, 3, H, W]
    # renderer with velocity blending
    r = sim.PWRenderer()
    w = full_worlds(pw, rng, 1, 32)
    w[:, 3:5] *= 4.0
    out['render_vel_world'] = w
    out['render_vel_img'] = r.render(w)
    # env traces, num_elems 5 and 8 (world 32): every np.random draw recorded
    for ne, tasks in ((5, (1,)), (8, (3,))):  # the shorter goal sequences (64 and 70 actions)
        env = envm.PowderworldEnv(world_size=32, num_elems=ne)
        for tr, task in enumerate(tasks):
            np.random.seed(1000 * ne + tr)
            with RandRecorder() as rrec:
                saved = {}
                picks = []
                for name in ('randint', 'choice'):
                    fn = getattr(np.random, name)
                    saved[name] = fn

                    def wrap(*a, _fn=fn, _name=name, **k):
                        v = _fn(*a, **k)
                        picks.append((_name, v))
                        return v

                    setattr(np.random, name, wrap)
                try:
                    ob, info = env.reset(options=dict(task_id=task))
                finally:
                    for name, fn in saved.items():
                        setattr(np.random, name, fn)
            n_goal_fwd = len(env.task_infos[task - 1]['action_seq'])
            rands = np.stack(rrec.log, 0)[:, 0, 0]  # [F, H, W] in call order
            assert len(rrec.log) == 3 * (n_goal_fwd + 1)
            elem = env._elem_names.index(picks[-3][1])
            tag = f'env{ne}_tr{tr}'
            out[f'{tag}_task'] = np.array(task)
            out[f'{tag}_reset_rand'] = rands.reshape(n_goal_fwd + 1, 3, 32, 32)
            out[f'{tag}_reset_action'] = np.array([elem, picks[-2][1], picks[-1][1]], np.int64)
            out[f'{tag}_goal_world'] = env.cur_goal_world.astype(np.uint8)
            out[f'{tag}_goal_ob'] = info['goal']
            out[f'{tag}_reset_ob'] = ob
            acts, step_rands, obs, rews = [], [], [], []
            for t in range(30):
                a = int(rng.randint(0, ne if env._action_step == 0 else env._xy_action_size))
                with RandRecorder() as srec:
                    ob, rew, term, trunc, info = env.step(a)
                acts.append(a)
                step_rands.append(np.stack(srec.log, 0)[:, 0, 0] if srec.log else np.zeros((3, 32, 32), np.float32))
                obs.append(ob)
                rews.append(rew)
            out[f'{tag}_actions'] = np.array(acts, np.int64)
            out[f'{tag}_step_rand'] = np.stack(step_rands)
            out[f'{tag}_obs'] = np.stack(obs)
            out[f'{tag}_reward'] = np.array(rews, np.float64)
            out[f'{tag}_final_world'] = env._world[0].astype(np.float32)
    # every task table (semantic actions as element indices, tolerances, names)
    for ne in (2, 5, 8):
        env = envm.PowderworldEnv(world_size=32, num_elems=ne)
        for t, info in enumerate(env.task_infos):
            seq = [(env._elem_names.index(e), x, y) for e, x, y in info['action_seq']]
            out[f'tasks{ne}_{t + 1}_seq'] = np.array(seq, np.int64)
            out[f'tasks{ne}_{t + 1}_tol'] = np.array(info['tol'])
            out[f'tasks{ne}_{t + 1}_name'] = np.array(info['task_name'])
    np.savez_compressed(os.path.join(OUT, 'powder_full_golden.npz'), **out)
    print('powder full golden:', len(out), 'arrays')


if __name__ == '__main__':
    main()
    main_full()
