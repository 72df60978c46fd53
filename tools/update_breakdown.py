"""Wall-time breakdown of one bench iteration (collect / process_fn / learn epochs) with a
device synchronisation around each part.  Same setup as bench.py.

    python tools/update_breakdown.py [--iters 3]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tianshou-fork_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--T", type=int, default=2048)
    a = ap.parse_args()
    from tianshou_amd.data import Collector, VectorReplayBuffer
    from tianshou_amd.env import SyntheticVectorEnv, VectorEnvNormObs
    from tianshou_amd.policy import PPOPolicy
    from tianshou_amd.utils.models import fixed_std_normal, get_actor_critic, init_and_get_optim
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    E, T, D, A = a.envs, a.T, 376, 17
    n = E * T
    env = VectorEnvNormObs(SyntheticVectorEnv(E, (D,), A, ep_len=1000, device=dev))
    actor, critic = get_actor_critic((D,), (64, 64), (A,), dev)
    actor, critic = actor.to(dev), critic.to(dev)  # before the optimiser: fused + capturable Adam
    optim = init_and_get_optim(actor, critic, 3e-4)
    pol = PPOPolicy(actor, critic, optim, fixed_std_normal, action_space=env.action_space,
                    max_grad_norm=0.5, vf_coef=0.25, ent_coef=0.0, reward_normalization=True,
                    perm_device=True).to(dev)
    buf = VectorReplayBuffer(n, E, device=dev)
    coll = Collector(pol, env, buf)
    tm = {}

    def timed(name, fn, *args, **kw):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn(*args, **kw)
        torch.cuda.synchronize()
        tm[name] = tm.get(name, 0.0) + time.perf_counter() - t0
        return out

    for it in range(a.iters + 1):
        if it == 1:
            tm.clear()
        timed("collect", coll.collect, n_step=n)
        batch, idx = buf.sample(0)
        batch = timed("process_fn", pol.process_fn, batch, buf, idx)
        timed("learn", pol.learn, batch, batch_size=n // 32, repeat=4)
        coll.reset_buffer(keep_statistics=True)
    for k, v in tm.items():
        print(f"{k:12s} {v / a.iters * 1e3:8.1f} ms", flush=True)
    print("graph learn:", pol._learn_graph is not None)
    opt = pol.optim
    print("ready:", pol._graph_ready(), "graph_learn", pol.graph_learn, "dp", pol.dp.active,
          "recompute", pol._recompute_adv, "capturable", opt.defaults.get("capturable"),
          "nstate", len(opt.state),
          "missing", sum(1 for g in opt.param_groups for p in g["params"] if p not in opt.state))


if __name__ == "__main__":
    main()
