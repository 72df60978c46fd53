"""Run-to-run spread of the action-coupled collect's obs_rms.

The action-coupled synthetic env (SyntheticVectorEnv(act_coef=c), the general fused collect
path: env after the actor) sums its obs_rms column moments as f64 atomic adds, whose order
varies from run to run.  This runs the same seeded collect (4096 envs x T steps, Box 376/17,
headline networks) R times in one process and reports how far obs_rms and the stored rows
move between runs (max |d| / |value|), next to the quantised env's exact int64 moments
(identical bits every run).

    python tools/coupled_spread.py [--T 256] [--reps 3] [--act-coef 0.05]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "tianshou-fork_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def one(E, T, D, A, act_coef, dev):
    from tianshou_amd.data import Collector, VectorReplayBuffer
    from tianshou_amd.env import SyntheticVectorEnv, VectorEnvNormObs
    from tianshou_amd.policy import PPOPolicy
    from tianshou_amd.utils.models import fixed_std_normal, get_actor_critic, init_and_get_optim
    torch.manual_seed(0)
    np.random.seed(0)
    env = VectorEnvNormObs(SyntheticVectorEnv(E, (D,), A, ep_len=1000, device=dev,
                                              act_coef=act_coef))
    actor, critic = get_actor_critic((D,), (64, 64), (A,), dev)
    actor, critic = actor.to(dev), critic.to(dev)
    optim = init_and_get_optim(actor, critic, 3e-4)
    policy = PPOPolicy(actor, critic, optim, fixed_std_normal, action_space=env.action_space,
                       reward_normalization=True, action_bound_method="clip").to(dev)
    buf = VectorReplayBuffer(E * T, E, device=dev)
    coll = Collector(policy, env, buf)
    torch.manual_seed(1)
    coll.collect(n_step=E * T)
    rms = env.get_obs_rms()
    rows = buf._meta.obs_next[:: max(1, (E * T) // 65536)][:, :D].cpu().numpy()
    return np.asarray(rms.mean), np.asarray(rms.var), rows, coll._step_on


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--E", type=int, default=4096)
    ap.add_argument("--T", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--act-coef", type=float, default=0.05)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    out = {}
    for coef in (a.act_coef, 0.0):
        runs = [one(a.E, a.T, 376, 17, coef, dev) for _ in range(a.reps)]

        def spread(i):
            base = runs[0][i].astype(np.float64)
            d = max(float(np.abs(r[i].astype(np.float64) - base).max()) for r in runs[1:])
            rel = max(float((np.abs(r[i].astype(np.float64) - base) /
                             np.maximum(np.abs(base), 1e-30)).max()) for r in runs[1:])
            same = all(np.array_equal(r[i], runs[0][i]) for r in runs[1:])
            return {"bit_identical": same, "max_abs_diff": d, "max_rel_diff": rel}
        out[f"act_coef={coef}"] = {"fused_step": bool(runs[0][3]), "obs_rms_mean": spread(0),
                                   "obs_rms_var": spread(1), "obs_next_rows": spread(2)}
    print(json.dumps({"envs": a.E, "steps": a.T, "reps": a.reps, "spread": out}, indent=1))


if __name__ == "__main__":
    main()
