"""ORACLE (test infrastructure only) -- NumPy/Python restatement of the device CartPole-v1
env (tianshou_amd/env/cartpole.py CartPoleVectorEnv, csrc/cartpole.hip).

Only ``tests/`` may import this module.  Dynamics: gymnasium's classic_control cartpole.py
(Euler, force +-10, thresholds x 2.4 / theta 12 deg) + TimeLimit(500), in f64 with Python's
math.sin/cos (glibc); resets draw U(-0.05, 0.05)^4 from the counter hash
``u_i = (sm(key ^ (i+1)) >> 11) * 2^-53``, key = sm(sm(sm(seed) ^ env) ^ episode)
(oracle/synth_env.py's splitmix64).  gymnasium parity of the dynamics is unpinned (gymnasium
is absent); the host CartPoleEnv that drove the reference goldens runs the same formulas.
"""
import math

import numpy as np

from oracle.synth_env import sm

THETA = 12 * 2 * math.pi / 360


class CartPoleHashVecNP:
    def __init__(self, num_envs, seed=0, max_steps=500):
        self.n, self.seed, self.max_steps = num_envs, seed, max_steps
        self.state = np.zeros((num_envs, 4))
        self.j = np.full(num_envs, -1, np.int64)
        self.t = np.zeros(num_envs, np.int64)

    def reset(self, ids=None):
        ids = np.arange(self.n) if ids is None else np.asarray(ids, np.int64)
        for e in ids:
            self.j[e] += 1
            self.t[e] = 0
            key = sm(sm(sm(np.uint64(self.seed)) ^ np.uint64(e)) ^ np.uint64(self.j[e]))
            for i in range(4):
                u = float(sm(key ^ np.uint64(i + 1)) >> np.uint64(11)) * (1.0 / 9007199254740992.0)
                self.state[e, i] = -0.05 + (0.05 - -0.05) * u
        return self.state[ids].astype(np.float32)

    def step(self, act, ids=None):
        ids = np.arange(self.n) if ids is None else np.asarray(ids, np.int64)
        obs = np.zeros((len(ids), 4), np.float32)
        rew = np.zeros(len(ids))
        term = np.zeros(len(ids), bool)
        trunc = np.zeros(len(ids), bool)
        for r, e in enumerate(ids):
            x, x_dot, theta, theta_dot = (float(v) for v in self.state[e])
            was = x < -2.4 or x > 2.4 or theta < -THETA or theta > THETA
            force = 10.0 if int(act[r]) == 1 else -10.0
            ct, st = math.cos(theta), math.sin(theta)
            temp = (force + 0.05 * (theta_dot * theta_dot) * st) / 1.1
            thetaacc = (9.8 * st - ct * temp) / (0.5 * (4.0 / 3.0 - 0.1 * (ct * ct) / 1.1))
            xacc = temp - 0.05 * thetaacc * ct / 1.1
            x = x + 0.02 * x_dot
            x_dot = x_dot + 0.02 * xacc
            theta = theta + 0.02 * theta_dot
            theta_dot = theta_dot + 0.02 * thetaacc
            self.state[e] = (x, x_dot, theta, theta_dot)
            self.t[e] += 1
            obs[r] = self.state[e].astype(np.float32)
            rew[r] = 0.0 if was else 1.0
            term[r] = x < -2.4 or x > 2.4 or theta < -THETA or theta > THETA
            trunc[r] = self.t[e] >= self.max_steps
        return obs, rew, term, trunc
