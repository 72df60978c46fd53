"""Minimal stand-ins for third-party modules the reference imports but this container lacks.

Used ONLY by ``tools/gen_goldens.py`` in the build container to import the read-only
reference at /root/reference and record golden vectors.  Nothing here ships to the GPU
box's product path, and no reference source is copied: these stubs replace *third-party*
packages (numba, gymnasium, h5py, ...), never reference modules.

* ``numba.njit`` is the identity, so the reference's @njit kernels (e.g. ``_gae_return``,
  tianshou/policy/base.py:453-497) run as Python under NumPy 2.2 promotion rules -- the
  semantics SURVEY.md §8a A5-bits pins.
* gymnasium gets just the Space/Box/Discrete/Env/Wrapper surface the reference touches.
"""
import importlib.machinery
import sys
import types

import numpy as np


def _module(name, **attrs):
    m = types.ModuleType(name)
    m.__spec__ = importlib.machinery.ModuleSpec(name, None)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


class _Inert:
    def __init__(self, *a, **k):
        pass

    def __getattr__(self, name):
        return lambda *a, **k: None


def _njit(*args, **kwargs):
    if args and callable(args[0]) and not kwargs:
        return args[0]
    return lambda fn: fn


class Space:
    def __init__(self, shape=None, dtype=None, seed=None):
        self.shape = shape
        self.dtype = dtype
        self.np_random = np.random.default_rng(seed)

    def seed(self, seed=None):
        self.np_random = np.random.default_rng(seed)
        return [seed]


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
        shape = tuple(shape) if shape is not None else np.shape(low)
        super().__init__(shape, np.dtype(dtype), seed)
        self.low = np.full(shape, low, dtype)
        self.high = np.full(shape, high, dtype)

    def sample(self):
        return self.np_random.uniform(self.low, self.high).astype(self.dtype)


class Discrete(Space):
    def __init__(self, n, seed=None):
        super().__init__((), np.int64, seed)
        self.n = n

    def sample(self):
        return int(self.np_random.integers(self.n))


class _OtherSpace(Space):
    pass


class Env:
    metadata = {}
    reward_range = (-float("inf"), float("inf"))
    spec = None

    def reset(self, seed=None, options=None):
        self.np_random = np.random.default_rng(seed)

    def close(self):
        pass


class Wrapper(Env):
    def __init__(self, env):
        self.env = env


class _Graph:
    def __init__(self, *a, **k):
        self.nodes = {}

    def add_nodes_from(self, nodes):
        for n in nodes:
            self.nodes[n] = {}


def install():
    if "numba" in sys.modules and getattr(sys.modules["numba"], "_tsrl_stub", False):
        return
    _module("numba", njit=_njit, _tsrl_stub=True)
    _module("h5py", File=_Inert, Dataset=_Inert, Group=_Inert)
    spaces = _module("gymnasium.spaces", Space=Space, Box=Box, Discrete=Discrete,
                     MultiDiscrete=_OtherSpace, MultiBinary=_OtherSpace, Dict=_OtherSpace,
                     Tuple=_OtherSpace)
    spaces.__path__ = []
    _module("gymnasium.spaces.discrete", Discrete=Discrete)
    wrappers = _module("gymnasium.wrappers", TimeLimit=Wrapper)
    _module("gymnasium", Env=Env, Space=Space, Wrapper=Wrapper, ActionWrapper=Wrapper,
            spaces=spaces, wrappers=wrappers, __version__="0.29.1")
    _module("pettingzoo", __version__="1.24.0")
    _module("pettingzoo.utils")
    _module("pettingzoo.utils.env", AECEnv=_Inert)
    _module("pettingzoo.utils.wrappers", BaseWrapper=_Inert)
    for name in ("tensorboard", "tensorboard.backend", "tensorboard.backend.event_processing"):
        _module(name)
    _module("tensorboard.backend.event_processing.event_accumulator", EventAccumulator=_Inert)
    _module("torch.utils.tensorboard", SummaryWriter=_Inert)
    _module("jsonargparse", set_docstring_parse_options=lambda **k: None, CLI=_Inert)
    _module("networkx", Graph=_Graph)


def import_reference(path="/root/reference"):
    install()
    if path not in sys.path:
        sys.path.insert(0, path)
    import tianshou  # noqa: F401
    return tianshou
