"""ORACLE (test infrastructure only) -- the replay-buffer rows the reference would store for
the headline collect (BASELINE config 3: the synthetic Box env, 4096 envs x 2048 steps,
VectorEnvNormObs), rebuilt from the env's closed form and the reference's own obs_rms
trajectory (``tests/golden/rms_fullT.npz``, written by ``tools/gen_goldens.py
gen_rms_fullT`` from the reference VectorEnvNormObs).

Only ``tests/`` may import this module.

What the reference stores (collector.py:282-356, venv_wrappers.py:77-99,
statistics.py:88-92):

* step s of env e: ``obs_next`` = norm(raw step row, the statistic right after that step's
  update);
* ``obs`` of step 0 = norm(raw reset row, the statistic after the initial reset); of step
  s > 0: the previous step's ``obs_next`` (the same normalised row), unless the env finished
  at step s - 1, then norm(raw reset row, the statistic after that step's reset update);
* norm(x) = clip((x - mean) / sqrt(var + eps), -10, 10) in f32 (NEP 50: the Python-float eps
  is weak, every operand f32).
"""
import numpy as np

from oracle import synth_env

EPS = np.finfo(np.float32).eps.item()


def norm_f32(x, mean, var, eps=EPS, clip=10.0):
    """RunningMeanStd.norm (statistics.py:88-92) on f32 rows."""
    x = np.asarray(x, np.float32)
    y = (x - np.asarray(mean, np.float32)) / np.sqrt(np.asarray(var, np.float32) + eps)
    assert y.dtype == np.float32
    return np.clip(y, -clip, clip)


def step_coords(e, s, L):
    """(episode j, time t) of env e after its step s (0-based) in a fresh collect: episodes of
    L steps, the first starting at phase e % L (oracle/synth_env.py)."""
    e, s = np.asarray(e, np.int64), np.asarray(s, np.int64)
    q = e % L + s + 1
    later = q > L
    r = q - L
    j = np.where(later, 1 + (r - 1) // L, 0)
    t = np.where(later, (r - 1) % L + 1, q)
    return j, t


def rebuild_rows(z, envs, seed=0):
    """(obs, obs_next) f32 [len(envs), T, D]: the reference's buffer rows of ``envs``."""
    T, D, L = int(z["T"]), int(z["D"]), int(z["L"])
    envs = np.asarray(envs, np.int64)
    sm, sv = z["step_mean"], z["step_var"]        # [T + 1, D]: 0 = after the initial reset
    rm, rv = z["reset_mean"], z["reset_var"]      # [T, D]: after step s's reset update
    s = np.arange(T, dtype=np.int64)
    ee, ss = np.meshgrid(envs, s, indexing="ij")
    j, t = step_coords(ee, ss, L)
    raw = synth_env.box_obs(synth_env.key(seed, ee, j, t), D)       # [n, T, D]
    obs_next = norm_f32(raw, sm[1:][None], sv[1:][None])
    obs = np.empty_like(obs_next)
    k0 = synth_env.key(seed, envs, np.zeros_like(envs), envs % L)
    obs[:, 0] = norm_f32(synth_env.box_obs(k0, D), sm[0], sv[0])
    obs[:, 1:] = obs_next[:, :-1]
    done = t == L
    for a, b in zip(*np.nonzero(done[:, :-1])):   # env a finished at step b: reset row
        kr = synth_env.key(seed, envs[a:a + 1], j[a:a + 1, b] + 1, np.zeros(1, np.int64))
        obs[a, b + 1] = norm_f32(synth_env.box_obs(kr, D)[0], rm[b], rv[b])
    return obs, obs_next


def done_ids(z, s):
    """Envs that finished at step s in the reference run."""
    p = z["done_ptr"]
    return z["done_ids"][p[s]:p[s + 1]]
