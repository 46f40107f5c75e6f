"""Powderworld task tables (semantic action sequences whose replay defines the
goal worlds).  Restates PowderworldEnv.set_tasks for num_elems == 2
(ogbench/powderworld/powderworld_env.py:88-149); element indices refer to
_elem_names = ['plant', 'stone'] (powderworld_env.py:61-62).
"""

PLANT, STONE = 0, 1
EASY_TOL = 32


def _square(seq, elem, x, y, size):
    """Outline of a size x size square, in the reference's drawing order."""
    for i in range(size):
        seq.append((elem, x + i, y + size - 1))
    for i in range(size - 2, -1, -1):
        seq.append((elem, x, y + i))
    for i in range(size - 2, -1, -1):
        seq.append((elem, x + size - 1, y + i))
    for i in range(1, size - 1):
        seq.append((elem, x + i, y))


def _fill(seq, elem, pred=lambda x, y: True):
    for y in reversed(range(8)):
        for x in range(8):
            if pred(x, y):
                seq.append((elem, x, y))


def easy_task_sequences():
    """The 5 easy tasks: plant, stone, square, four squares, mosaic."""
    t1 = []
    _fill(t1, PLANT)
    t2 = []
    _fill(t2, PLANT)
    _fill(t2, STONE)
    t3 = []
    _fill(t3, PLANT)
    _square(t3, STONE, 1, 1, 6)
    t4 = []
    _fill(t4, PLANT)
    _fill(t4, STONE)
    for sx, sy in [(0, 0), (0, 5), (5, 0), (5, 5)]:
        _square(t4, PLANT, sx, sy, 3)
    t5 = []
    _fill(t5, PLANT)
    _fill(t5, STONE, lambda x, y: (x + y) % 2 == 0)
    return [t1, t2, t3, t4, t5]


EASY_TASK_NAMES = ['task1_plant', 'task2_stone', 'task3_square', 'task4_four_squares', 'task5_mosaic']


# ---------------------------------------------------------------- medium / hard
# Element indices into _elem_names (powderworld_env.py:57-60):
#   medium ['sand', 'water', 'fire', 'plant', 'stone'], hard adds ['gas', 'wood', 'ice'].
SAND, WATER, FIRE, M_PLANT, M_STONE, GAS, WOOD, ICE = range(8)


def medium_task_sequences():
    """powderworld_env.py:150-214 (num_elems == 5)."""
    t1 = []
    _square(t1, M_PLANT, 1, 1, 6)
    _square(t1, SAND, 0, 0, 8)
    _square(t1, M_STONE, 2, 2, 4)
    _square(t1, WATER, 3, 3, 2)
    t2 = []
    _fill(t2, WATER)
    _square(t2, M_PLANT, 0, 0, 8)
    t3 = []
    _square(t3, M_STONE, 0, 0, 8)
    for _ in range(32):
        t3 += [(SAND, 3, 1), (SAND, 4, 1)]
    t4 = [(M_PLANT, x, 6) for x in range(8)] + [(M_PLANT, x, 7) for x in range(8)]
    t4 += [(M_STONE, 0, y) for y in range(7, -1, -1)] + [(M_STONE, 7, y) for y in range(7, -1, -1)]
    t4 += [(M_STONE, x, 4) for x in range(1, 7)] + [(M_STONE, x, 3) for x in range(1, 7)]
    _square(t4, WATER, 2, 0, 3)
    _square(t4, WATER, 3, 0, 3)
    for _ in range(4):
        t4 += [(FIRE, 3, 7), (FIRE, 4, 7)]
    t5 = []
    _fill(t5, M_PLANT)
    for y in (4, 7):
        t5 += [(WATER, x, y) for x in range(8)]
    for _ in range(2):
        t5 += [(FIRE, x, 0) for x in range(8)]
    return [t1, t2, t3, t4, t5]


def hard_task_sequences():
    """powderworld_env.py:215-280 (num_elems == 8)."""
    t1 = []
    _fill(t1, SAND)
    t1 += [(SAND, x, 0) for x in range(8)] + [(WATER, x, 7) for x in range(8)]
    t1 += [(GAS, x, 7) for x in range(8)] + [(WATER, x, 7) for x in range(8)]
    t2 = []
    _square(t2, WOOD, 0, 0, 8)
    _square(t2, M_PLANT, 1, 1, 6)
    _square(t2, GAS, 2, 2, 4)
    for _ in range(3):
        t2 += [(FIRE, x, 0) for x in range(8)]
    t3 = [(ICE, x, 0) for x in range(8)]
    t3 += [(M_STONE, 2, y) for y in range(7, -1, -1)] + [(M_STONE, 5, y) for y in range(7, -1, -1)]
    for y in range(7, 0, -1):
        t3 += [(WATER, 3, y), (WATER, 4, y)]
    t3 += [(M_PLANT, 3, 3), (M_PLANT, 4, 3), (M_PLANT, 3, 4), (M_PLANT, 4, 4)]
    for y in range(7, 0, -1):
        t3 += [(GAS, 0, y), (GAS, 1, y), (GAS, 6, y), (GAS, 7, y)]
    t4 = []
    _square(t4, M_PLANT, 1, 4, 3)
    _square(t4, WOOD, 4, 4, 3)
    _square(t4, ICE, 1, 1, 3)
    _square(t4, M_PLANT, 4, 1, 3)
    for _ in range(10):
        _square(t4, M_PLANT, 4, 1, 3)
    t5 = []
    _fill(t5, WATER)
    _square(t5, M_PLANT, 3, 3, 2)
    for _ in range(4):
        _square(t5, M_STONE, 0, 0, 8)
    _square(t5, ICE, 3, 3, 2)
    return [t1, t2, t3, t4, t5]


MEDIUM_TASK_NAMES = ['task1_squares', 'task2_water_plant', 'task3_sandpile', 'task4_two_rooms', 'task5_elements']
MEDIUM_TOLS = [32, 64, 64, 64, 96]
HARD_TASK_NAMES = ['task1_bubbles', 'task2_firework', 'task3_three_rooms', 'task4_four_squares', 'task5_ice_plant']
HARD_TOLS = [96, 96, 96, 64, 96]


def task_sequences(num_elems):
    return {2: easy_task_sequences, 5: medium_task_sequences, 8: hard_task_sequences}[num_elems]()


def task_names(num_elems):
    return {2: EASY_TASK_NAMES, 5: MEDIUM_TASK_NAMES, 8: HARD_TASK_NAMES}[num_elems]


def task_tols(num_elems):
    return {2: [EASY_TOL] * 5, 5: MEDIUM_TOLS, 8: HARD_TOLS}[num_elems]
