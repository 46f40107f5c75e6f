"""CPU: the algebra of the pointmaze solver's rank-one update
(ogbench_amd/csrc/point_contact.h, local_rank_one) restated in NumPy.

The lean contact loop solves the normal equations of a quadratic piece
(the active-edge set A of the three role slots, local frame: face normals
(-1, 0) and (0, -1), corner normal n, t = perp(n); edges n + t, n - t (weight
w) and n (weight 2w)).  When the solution shows exactly one edge e with the
wrong activity, the variant updates the solve by Sherman-Morrison instead of
rebuilding the piece:  u' = u - a rho H^-1 J / (1 + a J' H^-1 J),
a = +-c w, rho = J.u + kp (an opt-in variant, -DOGBX_RANK_ONE: measured
slower on gfx950 than rebuilding the piece, so the shipped build rebuilds).
This checks that formula against a rebuild of the
neighbouring piece for random slots, masks and flipped edges (every one of the
nine edges, adding and removing).  The GPU kernel itself is held to the oracle
by tests/test_locomaze_gpu.py."""

import numpy as np

M = 1114.0  # m + D_floor of the point model (order of magnitude is what matters)


def edges(n2):
    """J of the nine edges (slot-major: n+t, n-t, n) and their weight factors c."""
    ns = [np.array([-1.0, 0.0]), np.array([0.0, -1.0]), n2]
    J, c = [], []
    for n in ns:
        t = np.array([-n[1], n[0]])
        J += [n + t, n - t, n]
        c += [1.0, 1.0, 2.0]
    return np.array(J), np.array(c)


def solve(J, c, w, kp, act, mbv):
    """Normal equations of the piece `act` (bit e = edge e active)."""
    H = M * np.eye(2)
    r = mbv.copy()
    for e in range(9):
        if (act >> e) & 1:
            s = e // 3
            H += w[s] * c[e] * np.outer(J[e], J[e])
            r -= w[s] * c[e] * kp[s] * J[e]
    return np.linalg.solve(H, r), H


def rank_one(J, c, w, kp, act, e, u, H):
    s = e // 3
    a = (-1.0 if (act >> e) & 1 else 1.0) * c[e] * w[s]
    rho = J[e] @ u + kp[s]
    z = np.linalg.solve(H, J[e])
    return u - a * rho * z / (1.0 + a * (J[e] @ z))


def test_rank_one_matches_rebuild():
    rng = np.random.RandomState(0)
    worst = 0.0
    for trial in range(400):
        ang = rng.uniform(np.pi, 1.5 * np.pi)  # corner normal points away from (+h, +h)
        n2 = np.array([np.cos(ang), np.sin(ang)])
        J, c = edges(n2)
        w = rng.uniform(1500, 2100, 3) * (rng.rand(3) < 0.8)  # some slots invalid (w = 0)
        kp = rng.uniform(-200, 5, 3)
        mbv = rng.normal(0, 300, 2)
        act = int(rng.randint(0, 512))
        u, H = solve(J, c, w, kp, act, mbv)
        for e in range(9):
            if w[e // 3] == 0.0:
                continue
            got = rank_one(J, c, w, kp, act, e, u, H)
            ref, _ = solve(J, c, w, kp, act ^ (1 << e), mbv)
            err = np.abs(got - ref).max() / (1.0 + np.abs(ref).max())
            worst = max(worst, err)
    assert worst < 1e-12, worst


def test_the_removed_edge_keeps_the_denominator_positive():
    # removing an edge leaves M I + (the other edges): 1 - c w J' H^-1 J > 0
    rng = np.random.RandomState(1)
    for _ in range(200):
        n2 = -np.abs(rng.normal(size=2))
        n2 /= np.linalg.norm(n2)
        J, c = edges(n2)
        w = rng.uniform(0, 2100, 3)
        act = 511
        _, H = solve(J, c, w, np.zeros(3), act, np.zeros(2))
        for e in range(9):
            z = np.linalg.solve(H, J[e])
            assert 1.0 - c[e] * w[e // 3] * (J[e] @ z) > 0.0
