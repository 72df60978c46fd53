"""TRPOPolicy (tianshou/policy/modelfree/trpo.py:12-160): NPG's direction with the step
size of the KL bound and a backtracking line search (trpo.py:74-160).  process_fn is NPG's
(device path); the line-search decisions use rank-averaged KL and loss under data
parallelism, so every rank accepts the same step."""
import warnings
from typing import Any, Callable, Dict, List

import torch
from torch.distributions import kl_divergence

from tianshou_amd.data.batch import Batch, split_indices
from tianshou_amd.policy.npg import NPGPolicy


class TRPOPolicy(NPGPolicy):
    def __init__(self, actor: torch.nn.Module, critic: torch.nn.Module,
                 optim: torch.optim.Optimizer, dist_fn: Callable, max_kl: float = 0.01,
                 backtrack_coeff: float = 0.8, max_backtracks: int = 10,
                 **kwargs: Any) -> None:
        super().__init__(actor, critic, optim, dist_fn, **kwargs)
        self._max_backtracks = max_backtracks
        self._delta = max_kl
        self._backtrack_coeff = backtrack_coeff

    def _surrogate(self, dist, minibatch: Batch) -> torch.Tensor:
        """-(ratio * adv).mean() (trpo.py:80-87)."""
        ratio = (dist.log_prob(minibatch.act) - minibatch.logp_old).exp().float()
        ratio = ratio.reshape(ratio.size(0), -1).transpose(0, 1)
        return -(ratio * minibatch.adv).mean()

    def learn(self, batch: Batch, batch_size: int, repeat: int, **kwargs: Any
              ) -> Dict[str, List[float]]:
        self._require_equal_shards(len(batch), next(self.critic.parameters()).device, "learn")
        actor_losses, vf_losses, step_sizes, kls = [], [], [], []
        for _ in range(repeat):
            for part in split_indices(len(batch), batch_size, True, True):
                minibatch = batch[part]
                dist = self(minibatch).dist
                actor_loss = self._surrogate(dist, minibatch)
                direction, flat_kl_grad, old_dist = self._natural_direction(
                    minibatch, dist, actor_loss)
                # largest step inside the KL bound (trpo.py:103-110)
                step_size = torch.sqrt(2 * self._delta / (
                    direction * self._MVP(direction, flat_kl_grad)).sum(0, keepdim=True))
                loss_ref = self._mean_over_ranks(actor_loss.detach().clone())
                with torch.no_grad():
                    flat_params = torch.cat([p.data.view(-1) for p in self.actor.parameters()])
                    for i in range(self._max_backtracks):
                        new_flat_params = flat_params + step_size * direction
                        self._set_from_flat_params(self.actor, new_flat_params)
                        new_dist = self(minibatch).dist
                        new_actor_loss = self._surrogate(new_dist, minibatch)
                        kl = kl_divergence(old_dist, new_dist).mean()
                        both = self._mean_over_ranks(torch.stack([kl, new_actor_loss]))
                        kl_ok, loss_down = (both[0] < self._delta), (both[1] < loss_ref)
                        if bool(kl_ok) and bool(loss_down):
                            if i > 0:
                                warnings.warn(f"Backtracking to step {i}.")
                            break
                        elif i < self._max_backtracks - 1:
                            step_size = step_size * self._backtrack_coeff
                        else:
                            self._set_from_flat_params(self.actor, new_flat_params)
                            step_size = torch.tensor([0.0])
                            warnings.warn("Line search failed! It seems hyperparamters"
                                          " are poor and need to be changed.")
                vf_loss = self._critic_steps(minibatch)
                actor_losses.append(actor_loss.detach())
                vf_losses.append(vf_loss.detach())
                step_sizes.append(step_size.detach().reshape(()).to(kl.device))
                kls.append(kl.detach())
        return self._read_lists({"loss/actor": actor_losses, "loss/vf": vf_losses,
                                 "step_size": step_sizes, "kl": kls})
