"""Minimal stand-in for ``gymnasium.spaces.Box`` (gymnasium is not installed in this image).

Only what the reference and rsl_rl touch: ``shape``, ``dtype``, ``low``/``high``, ``sample()`` and
``gym.spaces.flatdim`` (``flatdim`` below)."""
from __future__ import annotations

import numpy as np


class Box:
    def __init__(self, low, high, shape, dtype=np.float32):
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)
        self.low = np.full(self.shape, low, dtype=self.dtype)
        self.high = np.full(self.shape, high, dtype=self.dtype)

    def sample(self, rng: np.random.Generator | None = None):
        rng = rng or np.random.default_rng()
        lo = np.where(np.isfinite(self.low), self.low, -1.0)
        hi = np.where(np.isfinite(self.high), self.high, 1.0)
        return rng.uniform(lo, hi).astype(self.dtype)

    def __repr__(self) -> str:
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"


class Dict(dict):
    """``gymnasium.spaces.Dict`` stand-in: a plain mapping of named spaces."""


def flatdim(space) -> int:
    if isinstance(space, Box):
        return int(np.prod(space.shape))
    if isinstance(space, Dict):
        return sum(flatdim(s) for s in space.values())
    raise TypeError(f"unsupported space {space!r}")
