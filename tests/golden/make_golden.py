"""Generate the committed golden fixtures under tests/golden/ from the reference.

Run in the build container (where /root/reference exists):
    python tests/golden/make_golden.py

Nothing here runs on the GPU box and nothing from the reference is copied into
the repo: this script reads the reference source, executes the pure-Python /
NumPy pieces of it in-process (with tiny stand-ins for absent third-party
modules) and saves INPUT/OUTPUT vectors only.

Locomaze: ogbench/locomaze/maze.py imports mujoco at module top, so the module
cannot be imported here.  The methods that need no MuJoCo (xy_to_ij, ij_to_xy,
add_noise, compute_success, get_oracle_subgoal, set_tasks) are extracted from
the class body with `ast` and executed against a stub `self`; the maze maps
and task lists are read from the same source.
"""

import ast
import os
import re
import sys
import textwrap
import types

import numpy as np

REF = os.environ.get('OGBENCH_REF', '/root/reference')
OUT = os.path.dirname(os.path.abspath(__file__))


# ----------------------------------------------------------------- locomaze
def _maze_source():
    return open(os.path.join(REF, 'ogbench/locomaze/maze.py')).read()


def maze_tables():
    src = _maze_source()
    maps, tasks = {}, {}
    for name in ['arena', 'medium', 'large', 'giant', 'teleport']:
        m = re.search(r"self\._maze_type == '%s':\s*maze_map = (\[.*?\])\n" % name, src, re.S)
        maps[name] = np.array(ast.literal_eval(m.group(1)), np.int32)
        t = re.search(r"self\._maze_type == '%s':\s*tasks = (\[.*?\])\n" % name, src, re.S)
        tasks[name] = np.array(ast.literal_eval(t.group(1)), np.int32).reshape(-1, 4)
    return maps, tasks


def maze_methods():
    """Compile the MuJoCo-free MazeEnv methods of the reference into functions."""
    src = _maze_source()
    tree = ast.parse(src)
    fac = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == 'make_maze_env')
    cls = next(n for n in fac.body if isinstance(n, ast.ClassDef) and n.name == 'MazeEnv')
    want = {'xy_to_ij', 'ij_to_xy', 'add_noise', 'compute_success', 'get_oracle_subgoal', 'set_tasks'}
    fns = {}
    for node in cls.body:
        if isinstance(node, ast.FunctionDef) and node.name in want:
            code = textwrap.dedent(ast.get_source_segment(src, node))
            ns = {'np': np}
            exec(compile(code, f'<reference maze.py:{node.lineno}>', 'exec'), ns)
            fns[node.name] = ns[node.name]
    return fns


class _StubMaze:
    def __init__(self, maze_type, maps, fns, loco='point'):
        self._maze_type = maze_type
        self._maze_unit = 4.0
        self._offset_x = 4
        self._offset_y = 4
        self._noise = 1
        self._goal_tol = 1.0 if loco == 'point' else 0.5
        self._reward_task_id = None
        self.maze_map = maps[maze_type]
        self.cur_goal_xy = np.zeros(2)
        self._xy = np.zeros(2)
        for k, f in fns.items():
            setattr(self, k, types.MethodType(f, self))

    def get_xy(self):
        return self._xy.copy()


def locomaze_golden(rng):
    maps, tasks = maze_tables()
    fns = maze_methods()
    out = {}
    for name in maps:
        out[f'map_{name}'] = maps[name]
        out[f'tasks_{name}'] = tasks[name]
        stub = _StubMaze(name, maps, fns)
        stub.set_tasks()
        out[f'task_xy_{name}'] = np.array(
            [list(t['init_xy']) + list(t['goal_xy']) for t in stub.task_infos], np.float64)

    stub = _StubMaze('large', maps, fns)
    # xy_to_ij: truncation toward zero, including negative and boundary values.
    xs = np.concatenate([
        rng.uniform(-12, 50, 4000),
        np.array([-6.5, -6.0, -5.999999, -2.0, -2.0000000001, -1.9999999, 0.0, 1.999999, 2.0, 2.0000001,
                  -9.9, -10.0, 5.999, 6.0, 30.0, 41.99]),
    ])
    ys = np.concatenate([rng.uniform(-12, 38, 4000), rng.uniform(-8, 30, 16)])
    xy = np.stack([xs, ys], 1)
    out['xy2ij_in'] = xy
    out['xy2ij_out'] = np.array([stub.xy_to_ij(p) for p in xy], np.int32)
    # compute_success: np.linalg.norm(xy - goal) <= tol, with boundary cases
    # where fma and plain rounding disagree.
    n = 20000
    goal = rng.uniform(-4, 40, (n, 2))
    ang = rng.uniform(0, 2 * np.pi, n)
    rad = 1.0 + rng.normal(0, 1, n) * 1e-15
    rad[: n // 4] = rng.uniform(0.5, 1.5, n // 4)
    pos = goal + np.stack([np.cos(ang), np.sin(ang)], 1) * rad[:, None]
    succ = np.zeros(n, np.uint8)
    for i in range(n):
        stub._xy = pos[i]
        stub.cur_goal_xy = tuple(goal[i])
        succ[i] = stub.compute_success()
    out['succ_pos'] = pos
    out['succ_goal'] = goal
    out['succ_out'] = succ
    # reset arithmetic: add_noise(ij_to_xy(ij)) with injected np.random.uniform draws.
    saved = np.random.uniform
    try:
        for name in ['medium', 'large']:
            stub = _StubMaze(name, maps, fns)
            stub.set_tasks()
            draws = rng.uniform(-1, 1, (64, 4))
            res = np.zeros((64, 4))
            tids = (np.arange(64) % len(stub.task_infos)) + 1
            for i in range(64):
                it = iter(draws[i])
                np.random.uniform = lambda low=0.0, high=1.0, size=None, _it=it: next(_it)
                ti = stub.task_infos[tids[i] - 1]
                init_xy = stub.add_noise(stub.ij_to_xy(ti['init_ij']))
                goal_xy = stub.add_noise(stub.ij_to_xy(ti['goal_ij']))
                res[i] = [init_xy[0], init_xy[1], goal_xy[0], goal_xy[1]]
            out[f'reset_{name}_task'] = tids.astype(np.int32)
            out[f'reset_{name}_noise'] = draws
            out[f'reset_{name}_out'] = res
    finally:
        np.random.uniform = saved
    # get_oracle_subgoal on every (cell, cell) pair of the large and medium mazes
    for name in ['medium', 'large', 'giant']:
        stub = _StubMaze(name, maps, fns)
        H, W = maps[name].shape
        starts, goals, subs = [], [], []
        for si in range(H):
            for sj in range(W):
                for gi in range(H):
                    for gj in range(W):
                        if (si * W + sj + gi * 7 + gj) % 3:
                            continue
                        s_xy = np.array(stub.ij_to_xy((si, sj)), float) + rng.uniform(-1.5, 1.5, 2)
                        g_xy = np.array(stub.ij_to_xy((gi, gj)), float) + rng.uniform(-1.5, 1.5, 2)
                        sub, _ = stub.get_oracle_subgoal(s_xy, g_xy)
                        starts.append(s_xy)
                        goals.append(g_xy)
                        subs.append(sub)
        out[f'subgoal_{name}_start'] = np.array(starts)
        out[f'subgoal_{name}_goal'] = np.array(goals)
        out[f'subgoal_{name}_out'] = np.array(subs, np.float64)
    # free-space PointEnv step, float32 and float64 actions (point.py:68-71 with
    # mj_step an identity in free space): action = 0.2 * action; qpos + action.
    m = 4096
    q = np.stack([rng.choice([0.0, 4.0, 8.0, 12.0], m) + rng.uniform(-0.8, 0.8, m),
                  rng.choice([0.0, 8.0, 16.0], m) + rng.uniform(-0.8, 0.8, m)], 1)
    a32 = rng.uniform(-1, 1, (m, 2)).astype(np.float32)
    a64 = rng.uniform(-1, 1, (m, 2))
    out['free_qpos'] = q
    out['free_act32'] = a32
    out['free_act64'] = a64
    out['free_out32'] = q + 0.2 * a32
    out['free_out64'] = q + 0.2 * a64
    return out


def teleport_golden():
    """The teleport maze portal table (maze.py:149-161), read from the source."""
    src = _maze_source()
    m = re.search(r"self\._teleport_info = dict\((.*?)\n\s*\)", src, re.S)
    body = m.group(1)
    info = {}
    for key in ('teleport_in_ijs', 'teleport_out_ijs', 'teleport_radius'):
        v = re.search(key + r"=(\[.*?\]|[0-9.]+)", body, re.S).group(1)
        info[key] = ast.literal_eval(v)
    return info


def registry_golden():
    """max_episode_steps / kwargs of every locomaze + powderworld id."""
    src = open(os.path.join(REF, 'ogbench/locomaze/__init__.py')).read()
    src += open(os.path.join(REF, 'ogbench/powderworld/__init__.py')).read()
    calls = []

    def register(id, entry_point, max_episode_steps, kwargs):
        calls.append((id, max_episode_steps, dict(kwargs)))

    gym = types.ModuleType('gymnasium')
    gym.envs = types.ModuleType('gymnasium.envs')
    gym.envs.registration = types.ModuleType('gymnasium.envs.registration')
    gym.envs.registration.register = register
    sys.modules['gymnasium'] = gym
    sys.modules['gymnasium.envs'] = gym.envs
    sys.modules['gymnasium.envs.registration'] = gym.envs.registration
    exec(compile(src.replace('from gymnasium.envs.registration import register\n', ''), '<registry>', 'exec'),
         {'register': register})
    return calls


def main():
    rng = np.random.RandomState(20261015)
    lm = locomaze_golden(rng)
    np.savez_compressed(os.path.join(OUT, 'locomaze_golden.npz'), **lm)
    import json

    reg = [dict(id=i, max_episode_steps=m, kwargs=k) for i, m, k in registry_golden()]
    with open(os.path.join(OUT, 'registry_golden.json'), 'w') as f:
        json.dump(reg, f, indent=0, sort_keys=True)
    print('wrote', sorted(lm.keys())[:5], '...', len(reg), 'registry entries')
    with open(os.path.join(OUT, 'teleport_golden.json'), 'w') as f:
        json.dump(teleport_golden(), f, indent=0, sort_keys=True)
    for extra in ('make_golden_powder', 'make_golden_gc'):
        path = os.path.join(OUT, extra + '.py')
        if os.path.exists(path):
            ns = {'__name__': extra, '__file__': path}
            exec(compile(open(path).read(), path, 'exec'), ns)
            ns['main']()
            for fn in ('main_hgc', 'main_periodic', 'main_relabel', 'main_names', 'main_full'):
                if fn in ns:
                    ns[fn]()


if __name__ == '__main__':
    main()
