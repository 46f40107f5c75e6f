"""Minimal Gymnasium-compatible spaces (gymnasium is not a dependency).

Only what the batched envs expose: ``Box`` and ``Discrete`` with ``shape``,
``dtype``, ``low``/``high``/``n``, ``contains`` and ``sample``.  Mirrors the
fields the reference reads (ogbench/locomaze/maze.py:198,218;
ogbench/powderworld/powderworld_env.py:75-77).
"""

from __future__ import annotations

import numpy as np


class Box:
    def __init__(self, low, high, shape, dtype):
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)
        self.low = np.full(self.shape, low, dtype=self.dtype)
        self.high = np.full(self.shape, high, dtype=self.dtype)

    def sample(self, rng=None):
        rng = np.random if rng is None else rng
        if np.issubdtype(self.dtype, np.integer):
            return rng.randint(self.low, self.high.astype(np.int64) + 1).astype(self.dtype)
        low = np.where(np.isfinite(self.low), self.low, -1.0)
        high = np.where(np.isfinite(self.high), self.high, 1.0)
        return rng.uniform(low, high, self.shape).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return f'Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})'


class Discrete:
    def __init__(self, n):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.dtype(np.int64)

    def sample(self, rng=None):
        rng = np.random if rng is None else rng
        return int(rng.randint(self.n))

    def contains(self, x):
        return 0 <= int(x) < self.n

    def __repr__(self):
        return f'Discrete({self.n})'
