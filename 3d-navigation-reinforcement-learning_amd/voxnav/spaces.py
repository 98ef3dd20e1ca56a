"""Minimal stand-ins for gymnasium.spaces (gymnasium is optional).

Only what GridAgent exposes (envs/CubicEnv.py:56-62): ``Discrete(6)`` and an
80-float ``Box``.  If gymnasium is importable its classes are used instead.
"""
from __future__ import annotations

import numpy as np

try:  # pragma: no cover - exercised only where gymnasium is installed
    from gymnasium import Env as EnvBase  # type: ignore
    from gymnasium.spaces import Box, Discrete  # type: ignore
    HAVE_GYMNASIUM = True
except Exception:  # noqa: BLE001
    HAVE_GYMNASIUM = False

    class EnvBase:
        """Stand-in for ``gymnasium.Env`` (the reference subclasses it,
        envs/CubicEnv.py:15): with gymnasium installed, GridAgent is a real
        ``gymnasium.Env`` and passes SB3's ``check_env``
        (train/Grid_Train.py:138-147)."""
        metadata = {"render_modes": []}
        render_mode = None
        spec = None

        @property
        def unwrapped(self):
            return self


    class Discrete:
        def __init__(self, n: int, seed=None):
            self.n = int(n)
            self.shape = ()
            self.dtype = np.int64
            self._rng = np.random.default_rng(seed)

        def sample(self):
            return int(self._rng.integers(self.n))

        def contains(self, x) -> bool:
            try:
                return 0 <= int(x) < self.n
            except (TypeError, ValueError):
                return False

        def __repr__(self):
            return f"Discrete({self.n})"

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
            self.dtype = np.dtype(dtype)
            lo = np.asarray(low, dtype=self.dtype)
            hi = np.asarray(high, dtype=self.dtype)
            if shape is not None:
                lo = np.broadcast_to(lo, shape).astype(self.dtype)
                hi = np.broadcast_to(hi, shape).astype(self.dtype)
            self.low, self.high = lo, hi
            self.shape = tuple(lo.shape)
            self._rng = np.random.default_rng(seed)

        def sample(self):
            return self._rng.uniform(self.low, self.high).astype(self.dtype)

        def contains(self, x) -> bool:
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def __repr__(self):
            return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"
