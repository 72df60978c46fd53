"""CartPole-v1 (BASELINE config 1: test/discrete/test_ppo.py's task), restated.

gymnasium is not installed here, so its ``CartPole-v1`` (classic_control/cartpole.py behind
``TimeLimit(max_episode_steps=500)``) is restated from its published dynamics; gymnasium
parity is therefore UNPINNED (no gymnasium output exists in this container to compare
with).  The reference's Collector / PPOPolicy are driven by this same class when
tools/gen_goldens.py records the config-1 goldens, so the tianshou side of the path is
pinned.

* ``CartPoleEnv``       -- host env with the gymnasium API (reset(seed) -> (obs, info),
                           step(a) -> (obs, rew, terminated, truncated, info)): f64 state,
                           Euler integration, x / theta thresholds, reward 1 per step, the
                           episode truncated at 500 steps; resets draw U(-0.05, 0.05)^4 from
                           ``np.random.default_rng(seed)`` (gymnasium's seeding.np_random is
                           Generator(PCG64(SeedSequence(seed)))).  Drives the Collector's
                           generic host-env path through ``DummyVectorEnv``.
* ``CartPoleVectorEnv`` -- the same dynamics for N envs in HBM (csrc/cartpole.hip, f64,
                           no FMA contraction), for the fused device collect path; resets
                           draw from a counter hash (splitmix64 of (seed, env, episode)) --
                           oracle/cartpole.py restates it.
"""
import math
from typing import Optional

import numpy as np
import torch

from tianshou_amd import _C
from tianshou_amd.env.spaces import Box, Discrete
from tianshou_amd.env.synthetic import DeviceVectorEnv

GRAVITY = 9.8
MASSCART = 1.0
MASSPOLE = 0.1
TOTAL_MASS = MASSPOLE + MASSCART
LENGTH = 0.5  # half the pole's length
POLEMASS_LENGTH = MASSPOLE * LENGTH
FORCE_MAG = 10.0
TAU = 0.02
THETA_THRESHOLD = 12 * 2 * math.pi / 360
X_THRESHOLD = 2.4
MAX_EPISODE_STEPS = 500  # CartPole-v1 registration


def _spaces():
    high = np.array([X_THRESHOLD * 2, np.finfo(np.float32).max, THETA_THRESHOLD * 2,
                     np.finfo(np.float32).max], dtype=np.float32)
    return Box(-high, high, dtype=np.float32), Discrete(2)


class CartPoleEnv:
    """One CartPole-v1 env (gymnasium API, TimeLimit included)."""

    metadata = {"render_modes": []}

    def __init__(self, max_episode_steps: int = MAX_EPISODE_STEPS, render_mode=None):
        self.observation_space, self.action_space = _spaces()
        self.max_episode_steps = max_episode_steps
        self.np_random = None
        self.state = None
        self.steps_beyond_terminated = None
        self._elapsed_steps = None

    def reset(self, seed: Optional[int] = None, options=None):
        if seed is not None or self.np_random is None:
            self.np_random = np.random.default_rng(seed)
        self.state = self.np_random.uniform(low=-0.05, high=0.05, size=(4,))
        self.steps_beyond_terminated = None
        self._elapsed_steps = 0
        return np.array(self.state, dtype=np.float32), {}

    def step(self, action):
        assert self.state is not None, "Call reset before using step method."
        a = int(action)
        assert a in (0, 1), f"{action!r} invalid"
        x, x_dot, theta, theta_dot = (float(v) for v in self.state)
        force = FORCE_MAG if a == 1 else -FORCE_MAG
        costheta = math.cos(theta)
        sintheta = math.sin(theta)
        temp = (force + POLEMASS_LENGTH * (theta_dot * theta_dot) * sintheta) / TOTAL_MASS
        thetaacc = (GRAVITY * sintheta - costheta * temp) / (
            LENGTH * (4.0 / 3.0 - MASSPOLE * (costheta * costheta) / TOTAL_MASS))
        xacc = temp - POLEMASS_LENGTH * thetaacc * costheta / TOTAL_MASS
        x = x + TAU * x_dot
        x_dot = x_dot + TAU * xacc
        theta = theta + TAU * theta_dot
        theta_dot = theta_dot + TAU * thetaacc
        self.state = np.array((x, x_dot, theta, theta_dot), dtype=np.float64)
        terminated = bool(x < -X_THRESHOLD or x > X_THRESHOLD or theta < -THETA_THRESHOLD
                          or theta > THETA_THRESHOLD)
        if not terminated:
            reward = 1.0
        elif self.steps_beyond_terminated is None:
            self.steps_beyond_terminated = 0
            reward = 1.0
        else:
            self.steps_beyond_terminated += 1
            reward = 0.0
        self._elapsed_steps += 1
        truncated = self._elapsed_steps >= self.max_episode_steps
        return np.array(self.state, dtype=np.float32), reward, terminated, truncated, {}

    def close(self) -> None:
        pass


class CartPoleVectorEnv(DeviceVectorEnv):
    """N CartPole-v1 envs stepped by one HIP kernel (state f64 [N, 4] in HBM).  Actions are
    the Discrete(2) indices of the policy; obs f32 [N, 4]; rew f64; the Collector's fused
    device path drives it (no obs normalisation)."""

    def __init__(self, num_envs: int, seed: int = 0, device=None,
                 max_episode_steps: int = MAX_EPISODE_STEPS):
        self.env_num = int(num_envs)
        self.obs_shape = (4,)
        self.obs_numel = 4
        self.u8 = False
        self.seed_ = int(seed)
        self.max_episode_steps = int(max_episode_steps)
        self.device = torch.device(device) if device is not None else \
            torch.device("cuda", torch.cuda.current_device())
        self.observation_space, self.action_space = _spaces()
        self.state = torch.zeros((self.env_num, 4), dtype=torch.float64, device=self.device)
        self.ep_j = torch.full((self.env_num,), -1, dtype=torch.int64, device=self.device)
        self.ep_t = torch.zeros(self.env_num, dtype=torch.int64, device=self.device)
        self.obs_torch_dtype = torch.float32
        self.nblk = 0

    supports_step_reset = False

    def nblk_for(self, k: int) -> int:
        return 0

    def alloc_obs(self, k: int) -> torch.Tensor:
        return torch.empty((k, 4), dtype=torch.float32, device=self.device)

    def alloc_partials(self, k: int):
        return None

    def _step_raw(self, ids, k, obs_out, rew_out, term_out, trunc_out, partials=None,
                  action=None) -> None:
        assert action is not None, "CartPoleVectorEnv.step needs actions"
        act = action.reshape(-1)
        if act.dtype != torch.int64:
            act = act.to(torch.int64)
        _C.check(_C.lib().tsrl_cartpole_step(
            _C.ptr(ids), k, _C.ptr(act.contiguous()), self.max_episode_steps,
            _C.ptr(self.state), _C.ptr(self.ep_t), _C.ptr(obs_out), _C.ptr(rew_out),
            _C.ptr(term_out), _C.ptr(trunc_out), _C.stream_ptr(self.device)),
            "tsrl_cartpole_step")

    def _reset_raw(self, ids, mask, k, obs_out, partials=None) -> None:
        _C.check(_C.lib().tsrl_cartpole_reset(
            _C.ptr(ids), _C.ptr(mask), k, self.seed_, _C.ptr(self.state), _C.ptr(self.ep_j),
            _C.ptr(self.ep_t), _C.ptr(obs_out), _C.stream_ptr(self.device)),
            "tsrl_cartpole_reset")

    def step(self, action, id=None):
        ids, k = self._ids(id)
        obs = self.alloc_obs(k)
        rew = torch.empty(k, dtype=torch.float64, device=self.device)
        term = torch.empty(k, dtype=torch.bool, device=self.device)
        trunc = torch.empty(k, dtype=torch.bool, device=self.device)
        act = torch.as_tensor(np.asarray(action) if not isinstance(action, torch.Tensor)
                              else action, device=self.device)
        self._step_raw(ids, k, obs, rew, term, trunc, None, act)
        env_id = ids if ids is not None else torch.arange(k, device=self.device)
        return obs, rew, term, trunc, {"env_id": env_id}
