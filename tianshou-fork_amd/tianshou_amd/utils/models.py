"""Model factories matching tianshou/utils/models.py:34-97."""
from typing import Sequence

import numpy as np
import torch
from torch import nn
from torch.distributions import Independent, Normal

from tianshou_amd.utils.net import ActorCritic, ActorProb, Critic, Net


def get_actor_critic(state_shape, hidden_sizes: Sequence[int], action_shape, device="cpu"):
    net_a = Net(state_shape, hidden_sizes=hidden_sizes, activation=nn.Tanh, device=device)
    actor = ActorProb(net_a, action_shape, unbounded=True, device=device)
    net_c = Net(state_shape, hidden_sizes=hidden_sizes, activation=nn.Tanh, device=device)
    critic = Critic(net_c, device=device)
    return actor, critic


def init_actor_critic(actor: nn.Module, critic: nn.Module) -> ActorCritic:
    actor_critic = ActorCritic(actor, critic)
    torch.nn.init.constant_(actor.sigma_param, -0.5)
    for m in actor_critic.modules():
        if isinstance(m, torch.nn.Linear):
            torch.nn.init.orthogonal_(m.weight, gain=np.sqrt(2))
            torch.nn.init.zeros_(m.bias)
    if hasattr(actor, "mu"):
        for m in actor.mu.modules():
            if isinstance(m, torch.nn.Linear):
                torch.nn.init.zeros_(m.bias)
                m.weight.data.copy_(0.01 * m.weight.data)
    return actor_critic


def init_and_get_optim(actor, critic, lr: float, optim_class=None):
    """models.py:77-93.  Default optimiser: Adam, fused single-kernel form on the GPU (same
    update rule; the foreach form launches ~10 kernels per step over 14 small tensors), and
    capturable (step counts on device) so PPO epochs can be replayed from a HIP graph."""
    actor_critic = init_actor_critic(actor, critic)
    if optim_class is None:
        on_gpu = next(actor_critic.parameters()).is_cuda
        if on_gpu:
            return torch.optim.Adam(actor_critic.parameters(), lr=lr, fused=True,
                                    capturable=True)
        return torch.optim.Adam(actor_critic.parameters(), lr=lr)
    return optim_class(actor_critic.parameters(), lr=lr)


def fixed_std_normal(*logits):
    return Independent(Normal(*logits), 1)
