"""oracle/powder_full_np.py -- TEST INFRASTRUCTURE ONLY.

NumPy restatement of the full powderworld forward used by the medium (5
elements) and hard (8 elements) envs: every rule PWSim registers, on the
reference's (n, 9, H, W) float32 world with the three float32 rand fields of
the forward injected.  Pinned against tests/golden/powder_full_golden.npz
(outputs of the reference's own sim.py / powderworld_env.py).

  element table, rule order   ogbench/powderworld/sim.py:15-37, 284-308
  PWSim.forward               sim.py:363-380
  Stone / Gravity / Sand      sim.py:574-590, 461-501, 504-571
  FluidFlow                   sim.py:593-667
  Ice / Water / Fire / Plant  sim.py:670-823
  Velocity                    sim.py:919-982
  PWRenderer (velocity blend) sim.py:386-453

Float32 semantics follow the reference op by op (NumPy weak Python scalars,
in-place float64 round trips for the fire impulses).  The one reduction whose
order matters, the velocity blur (conv2d -> np.einsum over 9 taps), is summed
in the order of NumPy's baseline SSE3 einsum kernel (pinned by
tests/test_oracle_powder_full.py against the reference conv2d).
"""

import numpy as np

F = np.float32
EMPTY, WALL, SAND, WATER, GAS, WOOD, ICE, FIRE, PLANT, STONE, LAVA, ACID, DUST = range(13)
KANGAROO, LEMMING, BIRD, FISH, MOLE = 16, 18, 15, 14, 17
DENSITY = np.array([1, 4, 3, 2, 0, 4, 4, 0, 4, 3, 3, 2, 2, 4, 2, 4, 3, 3, 3, 4, 3], np.float32)
GRAVITY = np.array([1, 0, 1, 1, 1, 0, 0, 1, 0, 1, 1, 1, 1, 0, 1, 0, 1, 1, 1, 0, 1], np.float32)
ELEM_IDS = {5: [2, 3, 7, 8, 9], 8: [2, 3, 7, 8, 9, 4, 5, 6]}  # powderworld_env.py:57-60


def elem_vec(i):
    v = np.zeros(9, F)
    v[0], v[1], v[2] = i, DENSITY[i], GRAVITY[i]
    return v


def from_ids(ids):
    """(n, H, W) ids -> (n, 9, H, W) default element vectors (id_to_pw)."""
    ids = np.asarray(ids, np.int64)
    w = np.zeros((ids.shape[0], 9) + ids.shape[1:], F)
    w[:, 0] = ids
    w[:, 1] = DENSITY[ids]
    w[:, 2] = GRAVITY[ids]
    return w


# neighbours (periodic): value at (r, c) of the cell below / above / left / right
def dn(x):
    return np.roll(x, -1, axis=-2)


def up(x):
    return np.roll(x, 1, axis=-2)


def lf(x):
    return np.roll(x, 1, axis=-1)


def rt(x):
    return np.roll(x, -1, axis=-1)


def toward(d, x):
    """sim.py direction_func: 0 right, 1 below-right, 2 below, 3 below-left,
    4 left, 5 above-left, 6 above, 7 above-right."""
    return [rt, lambda a: rt(dn(a)), dn, lambda a: lf(dn(a)), lf, lambda a: lf(up(a)), up,
            lambda a: rt(up(a))][d](x)


def box_count(m):
    """3x3 zero-padded neighbourhood sum of an integer-valued float32 field."""
    m = np.asarray(m, F)
    H, W = m.shape[-2:]
    p = np.zeros(m.shape[:-2] + (H + 2, W + 2), F)
    p[..., 1:-1, 1:-1] = m
    s = np.zeros_like(m)
    for di in range(3):
        for dj in range(3):
            s = s + p[..., di:di + H, dj:dj + W]
    return s


def blur(v):
    """conv2d(v, ones(3,3)/18, padding=1) in NumPy's SSE3 einsum order."""
    H, W = v.shape[-2:]
    w = (np.ones(1, F) / 18)[0]
    p = np.zeros(v.shape[:-2] + (H + 2, W + 2), F)
    p[..., 1:-1, 1:-1] = v
    t = [p[..., di:di + H, dj:dj + W] * w for di in range(3) for dj in range(3)]
    l0 = (t[4] + t[0]) + t[8]
    return ((l0 + (t[5] + t[1])) + ((t[6] + t[2]) + (t[7] + t[3]))).astype(F)


def pick(sw, if_false, if_true):
    """interp: the switched cells take if_true (whole vectors)."""
    return np.where(sw[:, None] if sw.ndim == if_false.ndim - 1 else sw, if_true, if_false)


def is_id(w, *ids):
    out = np.zeros(w.shape[:1] + w.shape[2:], bool)
    for i in ids:
        out |= w[:, 0] == i
    return out


def set_elem(w, sw, i):
    return np.where(sw[:, None], elem_vec(i)[None, :, None, None], w)


def stone_rule(w):
    st = (w[:, 0] == STONE).astype(F)
    H, W = st.shape[-2:]
    p = np.zeros(st.shape[:-2] + (H + 2, W + 2), F)
    p[..., 1:-1, 1:-1] = st
    sup = p[..., 0:H, 0:W] + p[..., 0:H, 2:W + 2]
    w = w.copy()
    w[:, 2] = (1 - st) * w[:, 2] + st * (sup < 2)
    return w


def gravity_rule(w):
    w = w.copy()
    w[:, 8] = np.where(w[:, 2] == 1, F(0), w[:, 8])
    b = dn(w)
    mv = (b[:, 1] - w[:, 1] < 0) & (w[:, 2] == 1) & (b[:, 2] == 1)
    real = mv & ~up(mv)
    real_up = up(real)
    w = np.where(real[:, None], b, np.where(real_up[:, None], up(w), w))
    w[:, 8] = np.where(real_up, F(1), w[:, 8])
    return w


def sand_rule(w, rm):
    for to_left in (True, False):
        go, back = (lf, rt) if to_left else (rt, lf)
        bl = go(dn(w))
        ar = back(up(w))
        fall = (rm > 0.5) if to_left else (rm <= 0.5)
        fall_ar = back(up(fall))
        elem = is_id(w, SAND, DUST)
        elem_ar = is_id(ar, SAND, DUST)
        ndg = ~(w[:, 8] > 0)
        a = elem & ~(bl[:, 8] > 0) & fall & ((w[:, 1] - bl[:, 1]) > 0) & (bl[:, 2] == 1) & ndg
        b = elem_ar & ~(ar[:, 8] > 0) & fall_ar & ((ar[:, 1] - w[:, 1]) > 0) & (ar[:, 2] == 1) & ndg
        assert not (a & b).any(), 'both sand moves into one cell (needs dust; unreachable in the envs)'
        w = np.where(a[:, None], bl, np.where(b[:, None], ar, w))
    return w


FLUIDS = (EMPTY, WATER, GAS, LAVA, ACID)


def fluid_rule(w, rm):
    mom = np.zeros(w.shape[:1] + w.shape[2:], F)
    for to_left in (True, False):
        go, back = (lf, rt) if to_left else (rt, lf)
        fall = (rm + w[:, 6] + mom) > 0.5
        match = fall if to_left else ~fall
        side, other = go(w), back(w)
        air = is_id(w, KANGAROO, LEMMING)
        elem = is_id(w, *FLUIDS) | air
        mv = (match & elem & (~(w[:, 8] > 0) | air) & ((w[:, 1] - side[:, 1]) > 0) & (side[:, 2] == 1)
              & (w[:, 2] == 1))
        real = mv & ~back(mv)
        real_in = back(real)
        mom = (mom + real_in * (2 if to_left else -2)).astype(F)
        w = np.where(real[:, None], side, np.where(real_in[:, None], other, w))
    w = w.copy()
    w[:, 6] = np.where(is_id(w, *FLUIDS, KANGAROO, LEMMING), mom, w[:, 6])
    return w


def ice_rule(w, ri):
    melt = sum((w[:, 0] == i).astype(F) for i in (EMPTY, FIRE, LAVA, WATER))
    sw = (w[:, 0] == ICE) & (box_count(melt) > 1) & (ri < F(0.02))
    return set_elem(w, sw, WATER)


def water_rule(w, re):
    sw = (w[:, 0] == WATER) & (box_count((w[:, 0] == ICE).astype(F)) >= 3) & (re < F(0.05))
    return set_elem(w, sw, ICE)


def fire_rule(w, ri, re):
    w = w.copy()
    fl = (w[:, 0] == FIRE).astype(F) + (w[:, 0] == LAVA).astype(F)
    near = box_count(fl) > 0
    burn = ((is_id(w, WOOD) & (ri < F(0.05))) | (is_id(w, PLANT) & (ri < F(0.2))) | (is_id(w, GAS) & (ri < F(0.2)))
            | is_id(w, DUST) | (is_id(w, BIRD) & (ri < F(0.05)))
            | (is_id(w, FISH, LEMMING, KANGAROO, MOLE) & (ri < F(0.2)))) & near
    burn_ice = is_id(w, ICE) & (ri < F(0.2)) & near
    dust = is_id(w, DUST) & near
    # impulses away from a burning neighbour: 8 (30 for dust), float64 round trips
    for mag, m in ((8, burn & near), (30, dust)):
        v3, v4 = w[:, 3].astype(np.float64), w[:, 4].astype(np.float64)
        v4 = (v4 + mag * lf(m)).astype(F).astype(np.float64)        # left neighbour burns: pushed right
        v3 = (v3 + mag * up(m)).astype(F).astype(np.float64)        # above burns: pushed down
        v3 = (v3 - mag * dn(m)).astype(F).astype(np.float64)        # below burns: pushed up
        v4 = (v4 - mag * rt(m)).astype(F).astype(np.float64)        # right burns: pushed left
        w[:, 3], w[:, 4] = v3.astype(F), v4.astype(F)
    w = set_elem(w, burn, FIRE)
    w = set_elem(w, burn_ice, WATER)
    burnables = sum(is_id(w, i).astype(F) for i in (WOOD, PLANT, GAS, DUST, FISH, BIRD, KANGAROO, MOLE, LEMMING))
    nb = box_count(burnables)
    in_range = box_count(nb * fl + (w[:, 0] == LAVA).astype(F))
    w = set_elem(w, is_id(w, EMPTY) & (in_range > 0) & (ri < F(0.3)), FIRE)
    w = set_elem(w, is_id(w, FIRE) & (re < F(0.4)) & (nb == 0), EMPTY)
    return w


def plant_rule(w, ri):
    cnt = box_count((w[:, 0] == PLANT).astype(F))
    grow = is_id(w, WATER) & (ri < F(0.05))
    to_plant = grow & (cnt <= 3) & (cnt >= 1)
    to_empty = grow & (cnt > 3)
    wi = box_count((w[:, 0] == ICE).astype(F) + (w[:, 0] == WOOD).astype(F))
    to_plant = to_plant | ((wi > 0) & (ri < F(0.2)) & is_id(w, EMPTY) & (cnt > 0))
    return set_elem(set_elem(w, to_plant, PLANT), to_empty, EMPTY)


def velocity_rule(w):
    w = w.copy()
    inv2pi = F(1 / (2 * np.pi))
    for n in range(2):
        vy, vx = w[:, 3], w[:, 4]
        mag = np.sqrt(vy * vy + vx * vx)
        raw = inv2pi * np.arccos(vx / (mag + F(0.001)))
        ang = np.where(vy < 0, F(1) - raw, raw)
        bins = np.remainder(np.floor(ang * F(8) + F(0.5)), F(8))
        enough = (mag > (F(1.0) if n == 0 else F(2.0))) & (w[:, 0] != WALL)
        dirs = [toward(a, w) for a in range(8)]
        swaps = np.full(w.shape[:1] + w.shape[2:], -1.0)
        for a in range(8):
            m = (bins == a) & enough & (swaps == -1) & (toward(a, swaps) == -1) & (dirs[a][:, 0] == EMPTY)
            opp = toward((a + 4) % 8, m)
            swaps = np.where(m, a, swaps)
            swaps = np.where(opp, (a + 4) % 8, swaps)
        old = w[:, 3:5].copy()
        nw = np.where((swaps == -1)[:, None], w, 0)
        for a in range(8):
            nw = np.where((swaps == a)[:, None], dirs[a], nw)
        w = nw.astype(F)
        w[:, 3:5] = w[:, 3:5] * F(0.5) + old * F(0.5)
    w[:, 3:5] = w[:, 3:5] * F(0.95)
    for ch in (3, 4):
        w[:, ch] = blur(w[:, ch]) + w[:, ch] * F(0.5)
    return w


def forward(w, rand):
    """One PWSim.forward; rand = (rand_movement, rand_interact, rand_element),
    each float32 (n, H, W)."""
    rm, ri, re = (np.asarray(r, F) for r in rand)
    w = stone_rule(np.asarray(w, F))
    w = gravity_rule(w)
    w = sand_rule(w, rm)
    w = fluid_rule(w, rm)
    w = ice_rule(w, ri)
    w = water_rule(w, re)
    w = fire_rule(w, ri, re)
    w = plant_rule(w, ri)
    return velocity_rule(w)


def paint(w, elem_id, x, y, grid=4, brush=4):
    """powderworld_env.py:380-391 on an (n, 9, H, W) world."""
    H, W = w.shape[-2:]
    m = np.zeros((w.shape[0], H, W), bool)
    m[:, y * grid:y * grid + brush, x * grid:x * grid + brush] = True
    m &= w[:, 0] != WALL
    return set_elem(w, m, elem_id)


COLORS = np.array([
    [236, 240, 241], [108, 122, 137], [243, 194, 58], [75, 119, 190], [179, 157, 219], [202, 105, 36],
    [137, 196, 244], [249, 104, 14], [38, 194, 129], [38, 67, 72], [157, 41, 51], [176, 207, 120],
    [255, 179, 167], [191, 85, 236], [0, 229, 255], [61, 90, 254], [121, 85, 72], [56, 142, 60],
    [158, 157, 36], [198, 40, 40], [224, 64, 251]], np.float32) / np.float32(255.0)
VCOLOR = np.array([200, 100, 100], np.float32) / np.float32(255.0)


def render(w1):
    """PWRenderer.render of one (9, H, W) world -> (H, W, 3) uint8."""
    img = COLORS[w1[0].astype(int)].transpose(2, 0, 1)
    vy, vx = w1[3], w1[4]
    mag = np.sqrt(vy * vy + vx * vx)
    d = np.clip(mag / F(5), F(0), F(0.5))[None]
    img = (F(1) - d) * img + d * VCOLOR[:, None, None]
    img = np.clip(img, F(0), F(1))
    return (img.transpose(1, 2, 0) * F(255)).astype(np.uint8)


class Env:
    """One medium/hard PowderworldEnv (task mode) with every draw injected."""

    def __init__(self, num_elems, size=32):
        self.elems = ELEM_IDS[num_elems]
        self.size = size
        self.xy = (size - 4) // 4 + 1

    def blank(self):
        ids = np.zeros((1, self.size, self.size), np.int64)
        ids[:, 0, :] = ids[:, -1, :] = ids[:, :, 0] = ids[:, :, -1] = WALL
        return from_ids(ids)

    def replay(self, seq, rands):
        """Goal world: each semantic action = forward(rand) + paint."""
        w = self.blank()
        for (e, x, y), r in zip(seq, rands):
            w = paint(forward(w, [f[None] for f in r]), self.elems[e], x, y)
        return w

    def reset(self, goal_ids, elem, x, y, rand):
        self.goal = goal_ids
        self.w = paint(forward(self.blank(), [f[None] for f in rand]), self.elems[elem], x, y)
        self.stage, self.elem, self.x = 0, None, None
        return self.observe()

    def observe(self):
        ob = np.zeros((self.size, self.size, 6), np.uint8)
        ob[..., :3] = render(self.w[0])
        lut = (COLORS * np.float32(255.0)).astype(np.uint8)
        if self.stage == 1:
            ob[..., 3:] = lut[self.elems[self.elem]]
        elif self.stage == 2:
            ob[:, self.x * 4:self.x * 4 + 4, 3:] = lut[self.elems[self.elem]]
        return ob

    def step(self, action, rand, draw=None):
        n = len(self.elems)
        if self.stage == 0:
            self.elem = action if action < n else draw
        elif self.stage == 1:
            self.x = action if action < self.xy else draw
        else:
            y = action if action < self.xy else draw
            self.w = paint(forward(self.w, [f[None] for f in rand]), self.elems[self.elem], self.x, y)
        self.stage = (self.stage + 1) % 3
        return self.observe()

    def errors(self):
        cur = self.w[0, 0]
        match = np.zeros(cur.shape, bool)
        for dx, dy in [(0, 0), (1, 0), (-1, 0), (0, 1), (0, -1)]:
            match |= self.goal == np.roll(cur, (dy, dx), axis=(0, 1))
        return int((~match).sum())
