"""Generate tests/golden/antmaze_golden.npz from the reference's antmaze wrapper.

Run in the build container (where /root/reference exists):
    python tests/golden/make_golden_ant.py

ogbench/locomaze/maze.py and ant.py import mujoco / gymnasium at module top,
so neither module is imported.  Instead the reference's own methods are
extracted with `ast` and compiled into two classes with the reference's
inheritance: the AntEnv methods (get_ob, get_xy, set_xy, reset_model, step;
ant.py:69-122) over a stub MujocoEnv whose do_simulation loads a given
post-physics state (the ant's articulated dynamics are out of scope), and the
MazeEnv methods (reset, step, compute_success, set_goal, xy_to_ij, ij_to_xy,
add_noise, set_tasks; maze.py:308-567) on top, so `super()` resolves as in the
reference.  gymnasium's TimeLimit is restated (elapsed += 1; truncated when
elapsed >= max_episode_steps).  Every draw is recorded: np.random.uniform of
add_noise and the env's np_random draws of reset_model.  Only inputs and
outputs are saved.

info['goal'] is the reference's goal observation (maze.py:407-418): the stub's
5 random steps load the last of five given states, so `goal_states` (that
state) is the input and `reset_goal_ob` (info['goal'] itself) the output.

Provenance: the npz records the sha256 of every method source extracted from
the reference (`src_sha256`, one line per method) and the reference's git HEAD
when readable, so a reviewer can audit what was executed.  Run it only in a
sandbox (this container): it executes reference code.
"""

import ast
import hashlib
import os
import textwrap

import numpy as np

REF = os.environ.get('OGBENCH_REF', '/root/reference')
OUT = os.path.dirname(os.path.abspath(__file__))
_PROVENANCE = {}


def _ref_head():
    try:
        head = open(os.path.join(REF, '.git', 'HEAD')).read().strip()
        if head.startswith('ref: '):
            head = open(os.path.join(REF, '.git', head[5:])).read().strip()
        return head
    except OSError:
        return 'unknown'


def _methods(path, cls_name, names, factory=None):
    src = open(os.path.join(REF, path)).read()
    tree = ast.parse(src)
    body = tree.body
    if factory is not None:
        body = next(n for n in body if isinstance(n, ast.FunctionDef) and n.name == factory).body
    cls = next(n for n in body if isinstance(n, ast.ClassDef) and n.name == cls_name)
    out = []
    for node in cls.body:
        if isinstance(node, ast.FunctionDef) and node.name in names:
            seg = textwrap.dedent(ast.get_source_segment(src, node))
            _PROVENANCE[f'{path}:{cls_name}.{node.name}'] = hashlib.sha256(seg.encode()).hexdigest()
            out.append(seg)
    assert len(out) == len(names), (cls_name, names)
    return out


class _Rec:
    """Recording stand-in for np.random / self.np_random."""

    def __init__(self, rng):
        self.rng = rng
        self.log = []

    def uniform(self, low=0.0, high=1.0, size=None):
        v = self.rng.uniform(low, high, size)
        self.log.append(('uniform', np.array(v, np.float64)))
        return v

    def standard_normal(self, size=None):
        v = self.rng.standard_normal(size)
        self.log.append(('normal', np.array(v, np.float64)))
        return v

    def randint(self, *a, **k):
        raise AssertionError('no teleport in the fixture mazes')


class _NP:
    def __init__(self, rec):
        self.random = rec

    def __getattr__(self, k):
        return getattr(np, k)


_STUB_BASE = '''
class _MujocoStub:
    def __init__(self, feed, np_random):
        self.init_qpos = np.array([0, 0, 0.75, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0], np.float64)
        self.init_qvel = np.zeros(14)
        self.data = types.SimpleNamespace(qpos=self.init_qpos.copy(), qvel=self.init_qvel.copy())
        self.model = types.SimpleNamespace(nq=15, nv=14, geom=lambda name: self._geoms.setdefault(
            name, types.SimpleNamespace(pos=np.zeros(3))))
        self._geoms = {}
        self.frame_skip = 5
        self.render_mode = None
        self.np_random = np_random
        self.action_space = types.SimpleNamespace(sample=lambda: np.zeros(8, np.float32))
        self._feed = feed

    def do_simulation(self, action, n_frames):
        q, v = next(self._feed)
        self.data.qpos[:] = q
        self.data.qvel[:] = v

    def set_state(self, qpos, qvel):
        self.data.qpos[:] = qpos
        self.data.qvel[:] = qvel

    def reset(self, *args, **kwargs):
        self.data.qpos[:] = self.init_qpos
        self.data.qvel[:] = self.init_qvel
        return self.reset_model(), {}
'''


def build_classes(np_proxy):
    import types

    ns = {'np': np_proxy, 'types': types, 'loco_env_type': 'ant'}
    exec(_STUB_BASE, ns)
    ant = _methods('ogbench/locomaze/ant.py', 'AntEnv', ['step', 'get_ob', 'reset_model', 'get_xy', 'set_xy'])
    src = 'class _Ant(_MujocoStub):\n' + ''.join(textwrap.indent(m, '    ') + '\n' for m in ant)
    exec(compile(src, '<reference ant.py methods>', 'exec'), ns)
    maze = _methods('ogbench/locomaze/maze.py', 'MazeEnv',
                    ['set_tasks', 'reset', 'step', 'get_oracle_rep', 'compute_success', 'set_goal', 'xy_to_ij',
                     'ij_to_xy', 'add_noise'], factory='make_maze_env')
    src = 'class _Maze(_Ant):\n' + ''.join(textwrap.indent(m, '    ') + '\n' for m in maze)
    exec(compile(src, '<reference maze.py methods>', 'exec'), ns)
    return ns['_Maze']


def make_env(cls, maze_type, feed, np_random, success_timing):
    env = cls.__new__(cls)
    type(env).__mro__[2].__init__(env, feed, np_random)  # _MujocoStub.__init__
    env._maze_type = maze_type
    env._maze_unit = 4.0
    env._offset_x = 4
    env._offset_y = 4
    env._noise = 1
    env._goal_tol = 0.5  # maze.py:86 (ant)
    env._reset_noise_scale = 0.1  # ant.py:28
    env._success_timing = success_timing
    env._terminate_at_goal = True
    env._add_noise_to_goal = True
    env._reward_task_id = None
    env._teleport_info = None
    env._ob_type = 'states'
    env._use_oracle_rep = False
    env.task_infos = []  # maze.py:189-194 (__init__ tail)
    env.cur_task_id = None
    env.cur_task_info = None
    env.set_tasks()
    env.num_tasks = len(env.task_infos)
    env.cur_goal_xy = np.zeros(2)
    return env


def antmaze_golden(rng, n=24, T=40, max_steps=30):
    out = {}
    for timing in ('post', 'pre'):
        rec = _Rec(np.random.RandomState(int(rng.randint(1 << 30))))
        cls = build_classes(_NP(rec))
        tasks = (np.arange(n) % 5 + 1).astype(np.int32)
        noise = np.zeros((n, 4))
        body = np.zeros((n, 29))
        robs = np.zeros((n, 29))
        rgoal = np.zeros((n, 2))
        gstates = np.zeros((n, 29))
        gob = np.zeros((n, 29))
        qpost = np.zeros((T, n, 15))
        vpost = np.zeros((T, n, 14))
        obs = np.zeros((T, n, 29))
        rew = np.zeros((T, n), np.float32)
        term = np.zeros((T, n), np.uint8)
        trunc = np.zeros((T, n), np.uint8)
        succ = np.zeros((T, n), np.uint8)
        for i in range(n):
            env_rng = _Rec(np.random.RandomState(int(rng.randint(1 << 30))))
            feed = [(rng.normal(size=15), rng.normal(size=14)) for _ in range(5)]
            env = make_env(cls, 'large', iter(feed), env_rng, timing)
            rec.log.clear()
            env_rng.log.clear()
            ob, info = env.reset(options=dict(task_id=int(tasks[i])))
            g = [v for k, v in rec.log if k == 'uniform']
            noise[i] = [float(x) for x in g]  # init x, init y, goal x, goal y (add_noise order)
            draws = env_rng.log[-2:]  # the second reset_model: uniform(15), normal(14)
            assert draws[0][0] == 'uniform' and draws[1][0] == 'normal'
            body[i, :15] = draws[0][1]
            body[i, 15:] = draws[1][1]
            robs[i] = ob
            rgoal[i] = env.cur_goal_xy
            gstates[i] = np.concatenate(feed[-1])  # state after the 5 random steps
            gob[i] = info['goal']  # the reference's goal observation
            # post-physics states: half the envs walk onto the goal (success ->
            # terminated), the rest wander; every other coordinate random
            xy0 = np.array(env.get_xy())
            goal = np.array(env.cur_goal_xy)
            path = []
            for t in range(T):
                q = rng.normal(size=15)
                if i % 2 == 0:
                    q[:2] = xy0 + (goal - xy0) * min(1.0, (t + 1) / (10 + i % 7)) + rng.uniform(-0.2, 0.2, 2)
                else:
                    q[:2] = xy0 + rng.uniform(-2, 2, 2)
                path.append((q, rng.normal(size=14)))
            env._feed = iter(path)
            elapsed = 0
            for t in range(T):
                qpost[t, i], vpost[t, i] = path[t]
                o, r, te, tr, inf = env.step(np.zeros(8))
                elapsed += 1  # gymnasium TimeLimit
                tr = tr or elapsed >= max_steps
                obs[t, i] = o
                rew[t, i] = r
                term[t, i] = te
                trunc[t, i] = tr
                succ[t, i] = inf['success']
        p = f'{timing}_'
        out.update({p + 'task': tasks, p + 'noise': noise, p + 'body_draws': body, p + 'reset_obs': robs,
                    p + 'reset_goal': rgoal, p + 'goal_states': gstates, p + 'reset_goal_ob': gob,
                    p + 'qpos_post': qpost, p + 'qvel_post': vpost, p + 'obs': obs,
                    p + 'reward': rew, p + 'terminated': term, p + 'truncated': trunc, p + 'success': succ})
    out['max_episode_steps'] = np.array(max_steps, np.int32)
    out['src_sha256'] = np.array(sorted(f'{k} {v}' for k, v in _PROVENANCE.items()))
    out['ref_head'] = np.array(_ref_head())
    return out


def main():
    rng = np.random.RandomState(20261016)
    out = antmaze_golden(rng)
    np.savez_compressed(os.path.join(OUT, 'antmaze_golden.npz'), **out)
    print({k: v.shape for k, v in out.items()})
    for t in ('post', 'pre'):
        print(t, 'terminated', int(out[t + '_terminated'].sum()), 'success', int(out[t + '_success'].sum()),
              'truncated', int(out[t + '_truncated'].sum()))


if __name__ == '__main__':
    main()
