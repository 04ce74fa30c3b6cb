"""gym.Env / gym.spaces when gym is importable, else minimal stand-ins with the
same attributes (gym is not installed in this image)."""
import numpy as np

try:  # pragma: no cover - gym absent here
    import gym as _gym
    from gym.spaces import Box, Dict, Discrete, MultiDiscrete  # noqa: F401
    GymEnvBase = _gym.Env
except Exception:  # noqa: BLE001
    _gym = None

    class GymEnvBase(object):
        """Stand-in for gym.Env."""

    class Box(object):
        def __init__(self, low, high, dtype=np.float32, shape=None):
            self.low = np.asarray(low)
            self.high = np.asarray(high)
            self.dtype = np.dtype(dtype)
            self.shape = self.low.shape if shape is None else tuple(shape)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def __repr__(self):
            return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"

    class Discrete(object):
        def __init__(self, n):
            self.n = int(n)
            self.shape = ()
            self.dtype = np.dtype(np.int64)

        def contains(self, x):
            return 0 <= int(x) < self.n

        def __repr__(self):
            return f"Discrete({self.n})"

    class MultiDiscrete(object):
        def __init__(self, nvec):
            self.nvec = np.asarray(nvec, dtype=np.int64)
            self.shape = self.nvec.shape
            self.dtype = np.dtype(np.int64)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all((x >= 0) & (x < self.nvec)))

        def __repr__(self):
            return f"MultiDiscrete({self.nvec.tolist()[:4]}{'...' if self.nvec.size > 4 else ''})"

    class Dict(object):
        def __init__(self, spaces):
            self.spaces = dict(spaces)

        def __getitem__(self, k):
            return self.spaces[k]

        def __repr__(self):
            return "Dict(" + ", ".join(f"{k}: {v}" for k, v in self.spaces.items()) + ")"

HAVE_GYM = _gym is not None
