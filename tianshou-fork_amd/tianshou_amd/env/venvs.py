"""DummyVectorEnv (tianshou/env/venvs.py:15-418 with worker/dummy.py): host envs stepped
sequentially in this process, results stacked into [N, ...] arrays -- the path every
non-device env takes through the Collector (collector.py:258-361, the generic loop of
data/collector.py).  Synchronous only (``wait_num`` / ``timeout`` are not supported)."""
from typing import Any, Callable, List, Optional, Union

import numpy as np


class DummyVectorEnv:
    is_async = False

    def __init__(self, env_fns: List[Callable[[], Any]], wait_num: Optional[int] = None,
                 timeout: Optional[float] = None) -> None:
        assert wait_num is None and timeout is None, "DummyVectorEnv is synchronous"
        self.envs = [fn() for fn in env_fns]
        self.env_num = len(self.envs)
        self.is_closed = False

    def __len__(self) -> int:
        return self.env_num

    # per-env attributes as lists (venvs.py:187-206: get_env_attr)
    @property
    def action_space(self) -> list:
        return [e.action_space for e in self.envs]

    @property
    def observation_space(self) -> list:
        return [e.observation_space for e in self.envs]

    def get_env_attr(self, key: str, id=None) -> list:
        return [getattr(self.envs[i], key) for i in self._wrap_id(id)]

    def _wrap_id(self, id: Optional[Union[int, List[int], np.ndarray]]) -> List[int]:
        if id is None:
            return list(range(self.env_num))
        return [int(i) for i in np.atleast_1d(id)]

    def _assert_is_not_closed(self) -> None:
        assert not self.is_closed, \
            f"Methods of {self.__class__.__name__} cannot be called after close."

    def reset(self, id=None, **kwargs):
        """venvs.py:260-297: stacked obs and the list of per-env info dicts."""
        self._assert_is_not_closed()
        rets = [self.envs[i].reset(**kwargs) for i in self._wrap_id(id)]
        assert isinstance(rets[0], (tuple, list)) and len(rets[0]) == 2 and \
            isinstance(rets[0][1], dict)
        obs_list = [r[0] for r in rets]
        if isinstance(obs_list[0], tuple):
            raise TypeError("Tuple observation space is not supported. ",
                            "Please change it to array or dict space")
        try:
            obs = np.stack(obs_list)
        except ValueError:  # different len(obs)
            obs = np.array(obs_list, dtype=object)
        return obs, [r[1] for r in rets]

    def step(self, action: np.ndarray, id=None):
        """venvs.py:299-381: (obs, rew, terminated, truncated, info) stacked over the envs,
        info[i]["env_id"] = the env's index."""
        self._assert_is_not_closed()
        ids = self._wrap_id(id)
        assert len(action) == len(ids)
        result = []
        for a, j in zip(action, ids):
            ret = self.envs[j].step(a)
            ret[-1]["env_id"] = j
            result.append(ret)
        obs_list, rew_list, term_list, trunc_list, info_list = tuple(zip(*result))
        try:
            obs_stack = np.stack(obs_list)
        except ValueError:
            obs_stack = np.array(obs_list, dtype=object)
        return (obs_stack, np.stack(rew_list), np.stack(term_list), np.stack(trunc_list),
                np.stack(info_list))

    def seed(self, seed: Optional[Union[int, List[int]]] = None) -> list:
        """venvs.py:383-403 + worker/dummy.py:40-46: int -> [seed + i]; each env's action
        space is seeded, then env.seed(s) or, for gymnasium-style envs, env.reset(seed=s)."""
        self._assert_is_not_closed()
        if seed is None:
            seed_list = [None] * self.env_num
        elif isinstance(seed, int):
            seed_list = [seed + i for i in range(self.env_num)]
        else:
            seed_list = list(seed)
        out = []
        for env, s in zip(self.envs, seed_list):
            env.action_space.seed(s)
            fn = getattr(env, "seed", None)
            if callable(fn):
                out.append(fn(s))
            else:
                env.reset(seed=s)
                out.append([s])
        return out

    def render(self, **kwargs: Any) -> list:
        return [getattr(e, "render", lambda **k: None)(**kwargs) for e in self.envs]

    def close(self) -> None:
        self._assert_is_not_closed()
        for e in self.envs:
            e.close()
        self.is_closed = True
