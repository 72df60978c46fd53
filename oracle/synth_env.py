"""ORACLE (test infrastructure only) -- NumPy restatement of the synthetic env.

Only ``tests/``, ``__graft_entry__.smoke()``, ``bench.py``'s cpu_baseline leg and
``tools/gen_goldens.py`` may import this module.  The product path
(``tianshou_amd.env.SyntheticVectorEnv``) computes the same function on the GPU in
``csrc/env.hip``; this file is the checker.

Spec (made concrete here; identical on CPU and HIP):

* ``sm(x)`` = splitmix64 finaliser of ``x + 0x9E3779B97F4A7C15`` (all arithmetic mod 2**64).
* key of (env e, episode j, time t): ``k = sm(sm(sm(sm(seed) ^ e) ^ j) ^ t)``.
* Box obs[d]  = ``(sm(k + d*G) >> 40) * 2**-23 - 1``  (f32-exact, in [-1, 1)), G = 0x9E3779B97F4A7C15.
* u8 obs[i]   = ``sm(k + i*G) & 0xFF`` (Atari-shaped 4x84x84, flattened index i).
* rew         = ``(sm(k ^ 0xD1B54A32D192ED03) >> 40) * 2**-24``  (exact in f32 and f64).
* Episode length L.  ``reset`` of env e: j += 1 (j starts at -1), t = (e % L if j == 0 else 0),
  returns obs(e, j, t).  ``step``: t += 1, returns obs(e, j, t), rew(e, j, t),
  terminated = (t >= L) and e even, truncated = (t >= L) and e odd.  Actions are ignored,
  except by the action-coupled variant (``act_coef`` c != 0, Box only): a step's obs[d] is
  ``f32(box_obs[d] + f32(c * a[d % A]))`` for the env's (remapped) f32 action row a.

The reference drives this through its own ``DummyVectorEnv``/``Collector``
(``tianshou/env/venvs.py:300-381``, ``tianshou/data/collector.py:258-361``) when
``tools/gen_goldens.py`` builds the collector goldens.
"""
import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
GAMMA = np.uint64(0x9E3779B97F4A7C15)
REW_SALT = np.uint64(0xD1B54A32D192ED03)
_C1 = np.uint64(0xBF58476D1CE4E5B9)
_C2 = np.uint64(0x94D049BB133111EB)


def sm(x):
    """splitmix64 step: mix(x + GAMMA); numpy uint64 arithmetic wraps mod 2**64."""
    with np.errstate(over="ignore"):
        z = np.asarray(x, dtype=np.uint64) + GAMMA
        z = (z ^ (z >> np.uint64(30))) * _C1
        z = (z ^ (z >> np.uint64(27))) * _C2
        return z ^ (z >> np.uint64(31))


def key(seed, e, j, t):
    s = sm(np.uint64(seed))
    e = np.asarray(e).astype(np.uint64)
    j = np.asarray(j).astype(np.int64).astype(np.uint64)
    t = np.asarray(t).astype(np.int64).astype(np.uint64)
    return sm(sm(sm(s ^ e) ^ j) ^ t)


def box_obs(k, dim):
    """k: uint64[...]; returns f32[..., dim]."""
    with np.errstate(over="ignore"):
        d = np.arange(dim, dtype=np.uint64) * GAMMA
        h = sm(k[..., None] + d)
    return ((h >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -23)
            - np.float32(1.0)).astype(np.float32)


def u8_obs(k, shape):
    n = int(np.prod(shape))
    with np.errstate(over="ignore"):
        i = np.arange(n, dtype=np.uint64) * GAMMA
        h = sm(k[..., None] + i)
    return (h & np.uint64(0xFF)).astype(np.uint8).reshape(k.shape + tuple(shape))


def u8_obs_stacked(seed, e, j, t, t0, shape):
    """frame_stack mode (shape = (S, *frame)): frame q is the u8 frame of time
    max(t - (S-1-q), t0), t0 the episode's first step (gymnasium FrameStack over a one-frame
    env; a reset repeats its first frame)."""
    S, frame = shape[0], tuple(shape[1:])
    e, j, t, t0 = (np.asarray(a, np.int64) for a in (e, j, t, t0))
    out = [u8_obs(key(seed, e, j, np.maximum(t - (S - 1 - q), t0)), frame) for q in range(S)]
    return np.stack(out, axis=e.ndim)


def reward(k):
    h = sm(k ^ REW_SALT)
    return (h >> np.uint64(40)).astype(np.float64) * (2.0 ** -24)


class SynthVecEnvNP:
    """Vectorised NumPy version (all envs in one object), used as the CPU port."""

    def __init__(self, num_envs, obs_shape, act_dim, ep_len, seed=0, u8=False, frame_stack=1,
                 act_coef=0.0):
        self.num_envs, self.obs_shape, self.act_dim = num_envs, tuple(obs_shape), act_dim
        self.ep_len, self.seed, self.u8 = ep_len, seed, u8
        self.frame_stack = frame_stack
        self.act_coef = np.float32(act_coef)
        self.j = np.full(num_envs, -1, np.int64)
        self.t = np.zeros(num_envs, np.int64)

    def _obs(self, ids):
        k = key(self.seed, ids, self.j[ids], self.t[ids])
        if self.u8 and self.frame_stack > 1:
            t0 = np.where(self.j[ids] == 0, ids % self.ep_len, 0)
            return u8_obs_stacked(self.seed, ids, self.j[ids], self.t[ids], t0, self.obs_shape)
        if self.u8:
            return u8_obs(k, self.obs_shape)
        return box_obs(k, int(np.prod(self.obs_shape))).reshape((len(ids),) + self.obs_shape)

    def reset(self, ids=None):
        ids = np.arange(self.num_envs) if ids is None else np.asarray(ids, np.int64)
        self.j[ids] += 1
        self.t[ids] = np.where(self.j[ids] == 0, ids % self.ep_len, 0)
        return self._obs(ids)

    def step(self, ids=None, action=None):
        ids = np.arange(self.num_envs) if ids is None else np.asarray(ids, np.int64)
        self.t[ids] += 1
        k = key(self.seed, ids, self.j[ids], self.t[ids])
        obs = self._obs(ids)
        if self.act_coef != 0:
            a = np.asarray(action, np.float32).reshape(len(ids), self.act_dim)
            D = obs.shape[-1]
            ca = (self.act_coef * a[:, np.arange(D) % self.act_dim]).astype(np.float32)
            obs = (obs + ca).astype(np.float32)
        rew = reward(k)
        done = self.t[ids] >= self.ep_len
        term = done & (ids % 2 == 0)
        trunc = done & (ids % 2 == 1)
        return obs, rew, term, trunc
