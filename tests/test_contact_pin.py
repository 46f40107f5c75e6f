"""CPU: the wall-contact model pinned independently of both implementations.

``tests/mjmodel_np.py`` restates MuJoCo's published constraint formulation for
the pointmaze sphere (solref -> B, K; the solimp power sigmoid; R from
diagApprox = (1 + mu^2) body_invweight0; aref = -B J.v - K imp pos; pyramid
edges of mju_makeFrame's contact frame; the exact minimiser by enumeration of
active edge sets; mj_RungeKutta) sharing no code with ``oracle/locomaze_ref.c``
or ``ogbench_amd/csrc/point_*.h``.  Here it is checked against two closed forms
(a straight one-face push-out and the symmetric inside corner, both solved by
hand piece by piece), and the C oracle is checked against it on contact
states spread over pointmaze-large.  tests/test_contact_pin_gpu.py holds the
GPU kernel to the same answers.
"""

import math
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import mjmodel_np as mj  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'locomaze_golden.npz')
TOL_CLOSED = 1e-12  # closed forms vs enumeration (and, on the GPU, vs the kernel)
TOL_MODEL = 1e-10   # the C oracle vs the enumeration model on general contact states


def maze_map():
    return np.load(GOLDEN)['map_large']


def cell_xy(i, j):
    return j * mj.MAZE_UNIT - mj.OFFSET, i * mj.MAZE_UNIT - mj.OFFSET


# pointmaze-large cells: (1, 6) has a wall on its -x side; (7, 6) has walls on
# its +x and +y sides (tests/golden map_large, maze.py:64-74)
PUSH_CELL = (1, 6)
CORNER_CELL = (7, 6)
DEPTHS = (1e-4, 5e-4, 0.002, 0.01, 0.05, 0.15, 0.3)
CORNER_DEPTHS = (5e-4, 0.002, 0.01, 0.05, 0.12, 0.19)


def pushout_cases():
    """(qpos, expected qpos) of the straight push-out from the -x wall of PUSH_CELL."""
    cx, cy = cell_xy(*PUSH_CELL)
    face = cx - mj.MAZE_UNIT / 2
    out = []
    for d in DEPTHS:
        x0 = face + mj.RADIUS - d
        s, _ = mj.pushout_1d(x0, face)
        out.append((np.array([x0, cy]), np.array([s, cy])))
    return out


def corner_cases():
    """(qpos, expected qpos) of the symmetric corner of CORNER_CELL (walls at +x, +y)."""
    cx, cy = cell_xy(*CORNER_CELL)
    out = []
    for d in CORNER_DEPTHS:
        p0 = mj.MAZE_UNIT / 2 - mj.RADIUS + d  # offset from the cell centre, both axes
        p, _ = mj.corner_symmetric(p0, mj.MAZE_UNIT / 2)
        out.append((np.array([cx + p0, cy + p0]), np.array([cx + p, cy + p])))
    return out


def random_contact_states(n, seed=0):
    """Centres in free cells of pointmaze-large within 1.6 of the cell centre
    per axis (penetration <= 0.3), keeping those touching a wall."""
    m = maze_map()
    boxes = mj.wall_boxes(m)
    free = np.argwhere(m == 0)
    rng = np.random.RandomState(seed)
    out = []
    while len(out) < n:
        i, j = free[rng.randint(len(free))]
        cx, cy = cell_xy(i, j)
        q = np.array([cx, cy]) + rng.uniform(-1.6, 1.6, 2)
        if len(mj.contacts(q, boxes)) > 1:
            out.append(q)
    return np.array(out)


def test_gain_constants():
    """The documented solref/solimp maps at the model's numbers."""
    B, K = mj.ref_gains()
    assert B == pytest.approx(2 / (0.95 * 0.04), rel=1e-15)
    assert K == pytest.approx(1 / (0.95 ** 2 * 0.04 ** 2), rel=1e-15)
    assert mj.impedance(0.0) == 0.9 and mj.impedance(-0.001) == 0.95 and mj.impedance(-0.3) == 0.95
    # power-2 sigmoid: midpoint 0.5 -> y = 0.5; x = 0.25 -> 2 x^2 = 0.125; x = 0.75 -> 1 - 2 (0.25)^2
    assert mj.impedance(-0.0005) == pytest.approx(0.925, rel=1e-15)
    assert mj.impedance(0.00025) == pytest.approx(0.9 + 0.125 * 0.05, rel=1e-15)
    assert mj.impedance(-0.00075) == pytest.approx(0.9 + 0.875 * 0.05, rel=1e-15)
    assert mj.body_invweight0() == pytest.approx(2 / (3 * mj.MASS), rel=1e-15)
    assert mj.MASS == pytest.approx(143.6755, abs=1e-4)
    # mju_makeFrame of a horizontal normal: one horizontal tangent, one vertical
    for n in ([1.0, 0, 0], [0, -1.0, 0], [0.6, 0.8, 0]):
        fr = mj.make_frame(n)
        assert np.allclose(fr @ fr.T, np.eye(3), atol=1e-15)
        assert sorted(np.round(np.abs(fr[1:, 2]), 12).tolist()) == [0.0, 1.0]


@pytest.mark.parametrize('k', range(len(DEPTHS)))
def test_pushout_closed_form_matches_enumeration(k):
    boxes = mj.wall_boxes(maze_map())
    q0, exp = pushout_cases()[k]
    got, v = mj.point_step(q0, boxes)
    assert np.abs(got - exp).max() <= TOL_CLOSED, (got, exp)
    assert got[1] == q0[1] and v[1] == 0.0  # no motion along the face
    assert got[0] > q0[0]  # pushed out of the wall


@pytest.mark.parametrize('k', range(len(CORNER_DEPTHS)))
def test_corner_closed_form_matches_enumeration(k):
    boxes = mj.wall_boxes(maze_map())
    q0, exp = corner_cases()[k]
    assert len(mj.contacts(q0, boxes)) == 3  # floor + two faces, no corner-box contact
    got, _ = mj.point_step(q0, boxes)
    assert np.abs(got - exp).max() <= TOL_CLOSED, (got, exp)
    assert abs((got[0] - q0[0]) - (got[1] - q0[1])) <= 1e-13  # symmetric
    assert got[0] < q0[0]


def test_pushout_recovers_equilibrium():
    """Sanity of the model's dynamics: a deep push-out moves the sphere back
    towards (not through) contact-free space within one env step."""
    boxes = mj.wall_boxes(maze_map())
    cx, cy = cell_xy(*PUSH_CELL)
    face = cx - mj.MAZE_UNIT / 2
    q0 = np.array([face + mj.RADIUS - 0.3, cy])
    q1, v1 = mj.point_step(q0, boxes)
    assert face + mj.RADIUS - 0.3 < q1[0] < face + mj.RADIUS + 0.5
    assert math.isfinite(v1[0])


def test_oracle_matches_mujoco_model():
    """oracle/locomaze_ref.c (Armijo Newton, 3x3-neighbourhood collider) vs the
    enumeration model (all wall boxes, explicit 3-D frames) on 150 contact states."""
    from oracle import locomaze as orc

    boxes = mj.wall_boxes(maze_map())
    q = random_contact_states(150)
    got, contact = orc.physics('large', q, np.zeros_like(q))
    assert contact.all()
    exp = np.array([mj.point_step(x, boxes)[0] for x in q])
    err = np.abs(got - exp).max()
    assert err <= TOL_MODEL, err


def test_oracle_matches_closed_forms():
    from oracle import locomaze as orc

    for q0, exp in pushout_cases() + corner_cases():
        got, contact = orc.physics('large', q0[None], np.zeros((1, 2)))
        assert contact[0] == 1
        assert np.abs(got[0] - exp).max() <= TOL_CLOSED, (q0, got[0], exp)
