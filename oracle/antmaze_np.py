"""NumPy restatement of the antmaze wrapper -- TEST INFRASTRUCTURE ONLY (the
checker of ogbench_amd/csrc/antmaze.h and bench.py's cpu_baseline leg; never a
product path).

Follows the reference's MazeEnv.reset/step (ogbench/locomaze/maze.py:373-466)
and AntEnv.get_ob/reset_model/set_xy (ogbench/locomaze/ant.py:97-122) for
loco_env_type 'ant' over a batch, around caller-supplied post-physics states
(the ant's articulated dynamics are out of scope):
  ob = concat(qpos, qvel); success = ||qpos[:2] - goal|| <= 0.5 (maze.py:86,
  486-490; the 2-norm rounded as NumPy's BLAS does, sqrt(fma(dy, dy, dx*dx)));
  terminated = success & terminate_at_goal; reward = success (-1 for a
  single-task env); TimeLimit truncation at max_episode_steps; reset ob =
  qpos0 + uniform(-0.1, 0.1) with xy := init_xy, qvel = 0.1 * normal.
Pinned by tests/golden/antmaze_golden.npz (tests/test_antmaze_cpu.py).
"""

from fractions import Fraction

import numpy as np

QPOS0 = np.array([0, 0, 0.75, 1, 0, 0, 0] + [0] * 8, np.float64)  # ant.xml qpos0
GOAL_TOL = 0.5
# maze.py:322-329 (init_ij, goal_ij) of the large maze
LARGE_TASKS = np.array([[1, 1, 7, 10], [5, 4, 7, 1], [7, 4, 1, 10], [3, 8, 5, 4], [1, 1, 5, 4]])


def ij_to_xy(i, j):
    return j * 4.0 - 4, i * 4.0 - 4  # maze.py:558-562


def within(dx, dy, tol=GOAL_TOL):
    """sqrt(fma(dy, dy, dx*dx)) <= tol, exactly: the plain float expression
    decides every pair except those within 1e-12 of the boundary, which are
    rounded once through rationals."""
    dx = np.asarray(dx, np.float64)
    dy = np.asarray(dy, np.float64)
    r = np.sqrt(dx * dx + dy * dy)
    out = r <= tol
    for k in np.nonzero(np.abs(r - tol) <= 1e-12)[0]:
        s = float(Fraction(float(dy[k])) ** 2 + Fraction(float(dx[k] * dx[k])))
        out[k] = np.sqrt(s) <= tol
    return out


def reset_obs(task, noise, body_draws, tasks=LARGE_TASKS):
    """Batched MazeEnv.reset ob and goal: task [N] 1-based, noise [N,4]
    uniform(-1,1) add_noise draws, body_draws [N,29] reset_model draws."""
    t = tasks[np.asarray(task) - 1]
    ix, iy = ij_to_xy(t[:, 0], t[:, 1])
    gx, gy = ij_to_xy(t[:, 2], t[:, 3])
    init = np.stack([ix + noise[:, 0] * 4.0 / 4, iy + noise[:, 1] * 4.0 / 4], 1)
    goal = np.stack([gx + noise[:, 2] * 4.0 / 4, gy + noise[:, 3] * 4.0 / 4], 1)
    ob = np.concatenate([QPOS0 + body_draws[:, :15], 0.0 + 0.1 * body_draws[:, 15:]], 1)
    ob[:, :2] = init
    return ob, goal


def goal_obs(goal, goal_states):
    """info['goal'] of MazeEnv.reset (maze.py:407-418): the body state after
    the goal reset's random physics steps (given, [N,29]) with set_xy(goal_xy),
    as get_ob() concatenates it (ant.py:97-122)."""
    g = np.array(goal_states, np.float64, copy=True)
    g[:, :2] = goal
    return g


class Batch:
    """State of N antmaze envs between wrapper steps."""

    def __init__(self, task, noise, body_draws, max_steps=1000, timing='post', tasks=LARGE_TASKS):
        self.task = np.asarray(task).copy()
        self.tasks = tasks
        ob, self.goal = reset_obs(self.task, noise, body_draws, tasks)
        self.xy = ob[:, :2].copy()
        self.elapsed = np.zeros(len(self.task), np.int64)
        self.max_steps = max_steps
        self.timing = timing

    def step(self, qpos, qvel, auto_reset=False, rng=None):
        """One wrapper step on post-physics states; with auto_reset the ending
        envs are reset from `rng` draws (timing leg of bench.py only)."""
        obs = np.concatenate([qpos, qvel], 1)
        xy = self.xy if self.timing == 'pre' else qpos[:, :2]
        succ = within(xy[:, 0] - self.goal[:, 0], xy[:, 1] - self.goal[:, 1])
        self.elapsed += 1
        trunc = self.elapsed >= self.max_steps
        term = succ
        reward = succ.astype(np.float32)
        self.xy = qpos[:, :2].copy()
        if auto_reset:
            done = np.nonzero(term | trunc)[0]
            if len(done):
                ob, goal = reset_obs(self.task[done], rng.uniform(-1, 1, (len(done), 4)),
                                     np.concatenate([rng.uniform(-0.1, 0.1, (len(done), 15)),
                                                     rng.standard_normal((len(done), 14))], 1), self.tasks)
                obs[done] = ob
                self.goal[done] = goal
                self.xy[done] = ob[:, :2]
                self.elapsed[done] = 0
        return obs, reward, term, trunc, succ
