"""Worker for tests/test_gpu_a_dist.py: one rank of a 2-rank data-parallel PPO update on
cuda:0 over the gloo backend (RCCL needs one GPU per rank; gloo carries device tensors).

    python tests/dist_worker.py RANK WORLD PORT OUTDIR
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tianshou-fork_amd"))


def make_data(n, D, A, dev, seed=7):
    import torch
    g = torch.Generator().manual_seed(seed)
    obs = torch.randn(n, D, generator=g)
    act = torch.randn(n, A, generator=g)
    logp_old = torch.randn(n, generator=g) * 0.2 - A * 1.2
    adv = torch.randn(n, generator=g) * 2 + 0.3
    ret = torch.randn(n, generator=g)
    v_s = ret + torch.randn(n, generator=g) * 0.3
    return {k: v.to(dev) for k, v in dict(obs=obs, act=act, logp_old=logp_old, adv=adv,
                                            returns=ret, v_s=v_s).items()}


def build_policy(D, A, dev):
    import torch
    from tianshou_amd.env import Box
    from tianshou_amd.policy import PPOPolicy
    from tianshou_amd.utils.models import fixed_std_normal, get_actor_critic, init_and_get_optim
    torch.manual_seed(0)
    actor, critic = get_actor_critic((D,), (64, 64), (A,), dev)
    optim = init_and_get_optim(actor, critic, 3e-4)
    return PPOPolicy(actor, critic, optim, fixed_std_normal, action_space=Box(-1.0, 1.0, (A,)),
                     max_grad_norm=0.5, vf_coef=0.25, ent_coef=0.01,
                     advantage_normalization=True).to(dev)


def main():
    rank, world, port, outdir = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    import numpy as np
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = port
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    from tianshou_amd.data import Batch, Collector, VectorReplayBuffer
    from tianshou_amd.env import SyntheticVectorEnv, VectorEnvNormObs
    n, D, A = 4096, 23, 5
    data = make_data(n, D, A, dev)
    sl = slice(rank * n // world, (rank + 1) * n // world)
    policy = build_policy(D, A, dev)
    np.random.seed(0)  # one global np.random stream (dp_permutation="global")
    batch = Batch(**{k: v[sl].contiguous() for k, v in data.items()})
    res = policy.learn(batch, batch_size=n // world, repeat=1)
    sd = {k: v.cpu() for k, v in policy.state_dict().items()}
    # several global minibatches over 2 repeats: the reference's Batch.split of the GLOBAL
    # batch (dp_permutation="global": the same np.random stream on every rank)
    policy2 = build_policy(D, A, dev)
    np.random.seed(0)
    res2 = policy2.learn(batch, batch_size=256, repeat=2)
    sd2 = {k: v.cpu() for k, v in policy2.state_dict().items()}
    # obs_rms kept global across ranks (sync_obs_rms): different env shards per rank
    E, T = 32, 24
    env = VectorEnvNormObs(SyntheticVectorEnv(E, (D,), A, ep_len=9, seed=rank, device=dev))
    buf = VectorReplayBuffer(E * T, E, device=dev)
    coll = Collector(policy, env, buf, sync_obs_rms=True)
    coll.collect(n_step=E * T)
    rms = env.get_obs_rms()
    torch.save(dict(sd=sd, loss=torch.tensor(res["loss"]), sd2=sd2,
                    loss2=torch.tensor([res2[k] for k in ("loss", "loss/clip", "loss/vf",
                                                          "loss/ent")]),
                    rms_mean=torch.as_tensor(rms.mean),
                    rms_var=torch.as_tensor(rms.var), rms_count=torch.tensor(rms.count)),
               os.path.join(outdir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
