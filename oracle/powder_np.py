"""oracle/powder_np.py -- TEST INFRASTRUCTURE ONLY.

NumPy restatement of the powderworld env for the 'easy' element set
{plant, stone} (plus empty/wall), the checker for libogbx's powder kernels.
Pinned against tests/golden/powder_golden.npz (outputs of the reference's own
sim.py / powderworld_env.py).

State representation: per cell an element id and two flags,
  grav  = channel 2 (GravityInter; dynamic for stone),
  didg  = channel 8 (did-gravity).
For easy worlds every other channel of the reference's (9,H,W) float32 world
stays 0 (velocity, fluid momentum, ...), so the restatement is exact.

  element table          ogbench/powderworld/sim.py:15-37
  PWSim.forward          ogbench/powderworld/sim.py:363-380 (rule order :284-308)
  BehaviorStone          ogbench/powderworld/sim.py:574-590
  BehaviorGravity        ogbench/powderworld/sim.py:461-501
  Sand/Fluid/Ice/Water/Fire/Plant/Velocity: identities for easy worlds
  PWRenderer.render      ogbench/powderworld/sim.py:386-453
  PowderworldEnv         ogbench/powderworld/powderworld_env.py:21-476
"""

import numpy as np

DENSITY = np.array([1, 4, 3, 2, 0, 4, 4, 0, 4, 3, 3, 2, 2, 4, 2, 4, 3, 3, 3, 4, 3], np.int32)
GRAVITY = np.array([1, 0, 1, 1, 1, 0, 0, 1, 0, 1, 1, 1, 1, 0, 1, 0, 1, 1, 1, 0, 1], np.int32)
COLORS = np.array([
    [236, 240, 241], [108, 122, 137], [243, 194, 58], [75, 119, 190], [179, 157, 219], [202, 105, 36],
    [137, 196, 244], [249, 104, 14], [38, 194, 129], [38, 67, 72], [157, 41, 51], [176, 207, 120],
    [255, 179, 167], [191, 85, 236], [0, 229, 255], [61, 90, 254], [121, 85, 72], [56, 142, 60],
    [158, 157, 36], [198, 40, 40], [224, 64, 251]], np.float32)
EASY_ELEMS = [8, 9]  # plant, stone (powderworld_env.py:61-62)


def render_lut():
    """uint8(clip(color/255) * 255) in float32 (sim.py:402-453)."""
    c = COLORS / np.float32(255.0)
    img = (np.float32(1.0) - np.float32(0.0)) * c + np.float32(0.0) * c
    img = np.clip(img, 0, 1)
    return (img * np.float32(255)).astype(np.uint8)


def from_channels(world):
    """(9,H,W) reference world -> (ids, grav, didg) int arrays."""
    return world[0].astype(np.int32), world[2].astype(np.int32), world[8].astype(np.int32)


def forward(ids, grav, didg):
    """One PWSim.forward for an easy world (stone rule, then gravity)."""
    H, W = ids.shape
    stone = (ids == 9).astype(np.int32)
    # BehaviorStone: supports = stone at (r-1, c-1) + stone at (r-1, c+1), zero padded
    pad = np.zeros((H + 2, W + 2), np.int32)
    pad[1:-1, 1:-1] = stone
    sup = pad[0:H, 0:W] + pad[0:H, 2:W + 2]
    grav = np.where(stone == 1, (sup < 2).astype(np.int32), grav)
    # BehaviorGravity (periodic rolls along rows)
    didg = np.where(grav == 1, 0, didg)
    dens = DENSITY[ids]
    below = lambda a: np.roll(a, -1, axis=0)
    above = lambda a: np.roll(a, 1, axis=0)
    dbb = (dens[np.r_[1:H, 0]] - dens < 0) & (grav == 1) & (below(grav) == 1)
    overlap = dbb & above(dbb)
    dbb_real = dbb & ~overlap
    dba_real = above(dbb_real)
    new = []
    for a in (ids, grav, didg):
        b = np.where(dbb_real, below(a), np.where(dba_real, above(a), a))
        new.append(b)
    ids, grav, didg = new
    didg = np.where(dba_real, 1, didg)
    return ids, grav, didg


def paint(ids, grav, didg, elem, x, y, grid=4, brush=4):
    """powderworld_env.py:380-391: brush square of elem unless the cell is wall."""
    ry, rx = y * grid, x * grid
    m = np.zeros_like(ids, bool)
    m[ry:ry + brush, rx:rx + brush] = True
    m &= ids != 1
    ids = np.where(m, elem, ids)
    grav = np.where(m, GRAVITY[elem], grav)
    didg = np.where(m, 0, didg)
    return ids, grav, didg


def observe(ids, stage, elem, x, grid=4, brush=4):
    lut = render_lut()
    H, W = ids.shape
    ob = np.zeros((H, W, 6), np.uint8)
    ob[..., :3] = lut[ids]
    if stage == 1:
        ob[..., 3:] = lut[elem]
    elif stage == 2:
        ob[:, x * grid: x * grid + brush, 3:] = lut[elem]
    return ob


def error_count(ids, goal):
    match = np.zeros(ids.shape, bool)
    for dx, dy in [(0, 0), (1, 0), (-1, 0), (0, 1), (0, -1)]:
        match |= goal == np.roll(ids, (dy, dx), axis=(0, 1))
    return int((~match).sum())


class Env:
    """Single powderworld-easy env (task mode), draws injected by the caller."""

    def __init__(self, size, tol=32):
        self.size, self.tol = size, tol
        self.xy = (size - 4) // 4 + 1

    def blank(self):
        ids = np.zeros((self.size, self.size), np.int32)
        ids[0, :] = ids[-1, :] = ids[:, 0] = ids[:, -1] = 1
        return ids, GRAVITY[ids], np.zeros_like(ids)

    def reset(self, goal_world, elem_idx, x, y):
        ids, grav, didg = self.blank()
        ids, grav, didg = forward(ids, grav, didg)
        self.state = list(paint(ids, grav, didg, EASY_ELEMS[elem_idx], x, y))
        self.goal = goal_world
        self.stage, self.elem, self.x = 0, None, None
        return observe(self.state[0], 0, 0, 0)

    def step(self, action, draw=None):
        """draw: the np.random.randint value used when the action is invalid."""
        if self.stage == 0:
            self.elem = action if action < 2 else draw
        elif self.stage == 1:
            self.x = action if action < self.xy else draw
        else:
            y = action if action < self.xy else draw
            ids, grav, didg = forward(*self.state)
            self.state = list(paint(ids, grav, didg, EASY_ELEMS[self.elem], self.x, y))
        self.stage = (self.stage + 1) % 3
        elem = EASY_ELEMS[self.elem] if self.elem is not None else 0
        ob = observe(self.state[0], self.stage, elem, self.x if self.x is not None else 0)
        err = error_count(self.state[0], self.goal)
        success = err < self.tol
        return ob, float(success), success
