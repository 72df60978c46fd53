"""Op-level attribution (torch.profiler) of one collector step and one PPO minibatch of the
bench workload.  GPU only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tianshou-fork_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402


def main():
    from tianshou_amd.data import Collector, VectorReplayBuffer
    from tianshou_amd.env import SyntheticVectorEnv, VectorEnvNormObs
    from tianshou_amd.policy import PPOPolicy
    from tianshou_amd.utils.models import fixed_std_normal, get_actor_critic, init_and_get_optim
    dev = torch.device("cuda", 0)
    E, T, D, A = 4096, int(os.environ.get("T", "64")), 376, 17
    env = VectorEnvNormObs(SyntheticVectorEnv(E, (D,), A, ep_len=1000, device=dev))
    actor, critic = get_actor_critic((D,), (64, 64), (A,), dev)
    optim = init_and_get_optim(actor, critic, 3e-4)
    policy = PPOPolicy(actor, critic, optim, fixed_std_normal, action_space=env.action_space,
                       max_grad_norm=0.5, vf_coef=0.25, ent_coef=0.0, reward_normalization=True,
                       perm_device=True).to(dev)
    buf = VectorReplayBuffer(E * T, E, device=dev)
    c = Collector(policy, env, buf)
    c.collect(n_step=E * T)
    policy.update(0, buf, batch_size=E * T // 4, repeat=1)
    c.reset_buffer(keep_statistics=True)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                 record_shapes=True) as prof:
        c.collect(n_step=E * 8)
        torch.cuda.synchronize()
    print("=== collect 8 steps")
    print(prof.key_averages(group_by_input_shape=True).table(
        sort_by="cuda_time_total", row_limit=25, max_name_column_width=60))
    c.reset_buffer()
    c.collect(n_step=E * T)
    batch, idx = buf.sample(0)
    batch = policy.process_fn(batch, buf, idx)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                 record_shapes=True) as prof:
        policy.learn(batch, batch_size=E * T // 4, repeat=1)
        torch.cuda.synchronize()
    print("=== learn 4 minibatches of", E * T // 4)
    print(prof.key_averages(group_by_input_shape=True).table(
        sort_by="cuda_time_total", row_limit=40, max_name_column_width=60))


if __name__ == "__main__":
    main()
