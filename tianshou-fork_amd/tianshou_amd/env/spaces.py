"""Minimal gym-style spaces (gymnasium is not a dependency of this package)."""
import numpy as np


class Box:
    def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
        shape = tuple(shape) if shape is not None else np.shape(low)
        self.shape, self.dtype = shape, np.dtype(dtype)
        self.low = np.full(shape, low, self.dtype)
        self.high = np.full(shape, high, self.dtype)
        self.np_random = np.random.default_rng(seed)

    def seed(self, seed=None):
        self.np_random = np.random.default_rng(seed)
        return [seed]

    def sample(self):
        lo = np.where(np.isfinite(self.low), self.low, -1.0)
        hi = np.where(np.isfinite(self.high), self.high, 1.0)
        return self.np_random.uniform(lo, hi).astype(self.dtype)

    def __repr__(self):
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"


class Discrete:
    def __init__(self, n, seed=None):
        self.n, self.shape, self.dtype = int(n), (), np.dtype(np.int64)
        self.np_random = np.random.default_rng(seed)

    def seed(self, seed=None):
        self.np_random = np.random.default_rng(seed)
        return [seed]

    def sample(self):
        return int(self.np_random.integers(self.n))

    def __repr__(self):
        return f"Discrete({self.n})"
