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
