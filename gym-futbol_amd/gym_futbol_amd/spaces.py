"""Spaces of the registered envs.

gym (0.17.1 in the reference's environment) is not a dependency: when it is
importable its `gym.spaces` classes are used, otherwise these duck-typed
stand-ins with the same constructor arguments, attributes (`n`, `nvec`, `low`,
`high`, `shape`, `dtype`, `spaces`) and `sample()` / `contains()` / `seed()`.
"""
import numpy as np

try:  # pragma: no cover - gym absent in this image
    from gym import spaces as _gym_spaces  # type: ignore
except Exception:  # noqa: BLE001
    _gym_spaces = None


class Space:
    def __init__(self, shape=None, dtype=None):
        self.shape = None if shape is None else tuple(shape)
        self.dtype = None if dtype is None else np.dtype(dtype)
        self.np_random = np.random.RandomState()

    def seed(self, seed=None):
        self.np_random = np.random.RandomState(seed)
        return [seed]


class Discrete(Space):
    def __init__(self, n):
        super().__init__((), np.int64)
        self.n = int(n)

    def sample(self):
        return int(self.np_random.randint(self.n))

    def contains(self, x):
        try:
            x = int(x)
        except (TypeError, ValueError):
            return False
        return 0 <= x < self.n

    def __repr__(self):
        return "Discrete(%d)" % self.n


class MultiDiscrete(Space):
    def __init__(self, nvec):
        self.nvec = np.asarray(nvec, dtype=np.int64)
        super().__init__(self.nvec.shape, np.int64)

    def sample(self):
        # gym 0.17: (np_random.random_sample(nvec.shape) * nvec).astype(dtype)
        return (self.np_random.random_sample(self.nvec.shape) * self.nvec).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all((0 <= x) & (x < self.nvec)))

    def __repr__(self):
        return "MultiDiscrete(%s)" % self.nvec


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32):
        dtype = np.dtype(dtype)
        if shape is None:
            low = np.asarray(low, dtype=dtype)
            shape = low.shape
        self.low = np.broadcast_to(np.asarray(low, dtype=dtype), shape).copy()
        self.high = np.broadcast_to(np.asarray(high, dtype=dtype), shape).copy()
        super().__init__(shape, dtype)

    def sample(self):
        return self.np_random.uniform(self.low, self.high).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all((x >= self.low) & (x <= self.high)))

    def __repr__(self):
        return "Box(%s, %s)" % (self.shape, self.dtype)


class Tuple(Space):
    def __init__(self, spaces):
        self.spaces = tuple(spaces)
        super().__init__(None, None)

    def sample(self):
        return tuple(s.sample() for s in self.spaces)

    def contains(self, x):
        return isinstance(x, (tuple, list)) and len(x) == len(self.spaces) and all(
            s.contains(v) for s, v in zip(self.spaces, x))

    def seed(self, seed=None):
        for i, s in enumerate(self.spaces):
            s.seed(None if seed is None else seed + i)
        return [seed]

    def __repr__(self):
        return "Tuple(%s)" % (self.spaces,)


if _gym_spaces is not None:  # pragma: no cover
    Discrete, MultiDiscrete, Box, Tuple = (_gym_spaces.Discrete, _gym_spaces.MultiDiscrete, _gym_spaces.Box,
                                           _gym_spaces.Tuple)


def v1_action_space(n):
    """envs_v1/futbol_env.py:78-79"""
    return MultiDiscrete([5, 5] * n)


def v1_observation_space(n):
    """envs_v1/futbol_env.py:86-91"""
    k = 4 * (1 + 2 * n)
    return Box(low=np.array([-1.0] * k, dtype=np.float32), high=np.array([1.0] * k, dtype=np.float32),
               dtype=np.float32)


def v0_action_space(action_as_int=True):
    """envs/futbol_env.py:156-163"""
    return Discrete(16) if action_as_int else Tuple((Discrete(4), Discrete(4)))


def v0_observation_space(length=105, width=68, player_speed=12, shoot_speed=20):
    """envs/futbol_env.py:172-179"""
    low = np.array([[0, 0, -length, -width, 0]] * 6, dtype=np.float64)
    high = np.array([[length, width, length, width, player_speed]] * 4
                    + [[length, width, length, width, shoot_speed], [10, 10, 10, 10, 10]], dtype=np.float64)
    return Box(low=low, high=high, dtype=np.float64)
