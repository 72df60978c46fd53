"""NPGPolicy (tianshou/policy/modelfree/npg.py:14-181).

process_fn is the A2C/PPO device path (critic values, GAE, logp_old on the fused kernels,
policy/fused_eval.py) followed by the whole-batch advantage normalisation of npg.py:68-79
(torch unbiased std, no epsilon).  learn keeps the reference's algorithm on device tensors:
the vanilla policy gradient, the KL Hessian-vector products by double backward, 10 conjugate
gradient steps, the fixed natural-gradient step and ``optim_critic_iters`` critic steps
(npg.py:81-130, 132-181).

Data parallel (one process per GPU, env-sharded batches of equal size): every quantity that
is a mean over the minibatch is averaged over the ranks before it is used -- the flat actor
gradient, every Hessian-vector product, the critic gradients and the logged KL / losses -- so
all ranks take the identical step (the one a single process would take on the union of the
ranks' minibatches).
"""
from typing import Any, Callable, Dict, List

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn
from torch.distributions import kl_divergence

from tianshou_amd.data.batch import Batch, split_indices
from tianshou_amd.policy.a2c import A2CPolicy
from tianshou_amd.policy.fused_eval import FusedEvalMixin


class NPGPolicy(FusedEvalMixin, A2CPolicy):
    def __init__(self, actor: torch.nn.Module, critic: torch.nn.Module,
                 optim: torch.optim.Optimizer, dist_fn: Callable,
                 advantage_normalization: bool = True, optim_critic_iters: int = 5,
                 actor_step_size: float = 0.5, fused_mlp: bool = True, **kwargs: Any) -> None:
        super().__init__(actor, critic, optim, dist_fn, **kwargs)
        del self._weight_vf, self._weight_ent, self._grad_norm
        self._norm_adv = advantage_normalization
        self._optim_critic_iters = optim_critic_iters
        self._step_size = actor_step_size
        # adjusts Hessian-vector product calculation for numerical stability
        self._damping = 0.1
        self._init_fused_eval(actor, critic, dist_fn, fused_mlp)

    # -- process_fn -------------------------------------------------------------------------
    def process_fn(self, batch: Batch, buffer, indices: np.ndarray) -> Batch:
        """npg.py:68-79."""
        self._pending_logp = None
        batch = super().process_fn(batch, buffer, indices)
        batch.logp_old = self._logp_old(batch)
        if self._norm_adv:
            batch.adv = self._normalize_adv(batch.adv)
        return batch

    def _normalize_adv(self, adv: torch.Tensor) -> torch.Tensor:
        """(adv - mean) / std over the whole batch (all ranks' batches under data
        parallelism; moments from one all-reduce of (n, sum, sum of squares) in f64)."""
        if not self.dp.active:
            return (adv - adv.mean()) / adv.std()
        a = adv.double()
        m = torch.stack([torch.tensor(float(a.numel()), dtype=torch.float64, device=a.device),
                         a.sum(), (a * a).sum()])
        self.dp.all_reduce_(m)
        n, s, ss = m[0], m[1], m[2]
        mean = s / n
        std = ((ss - n * mean * mean) / (n - 1)).clamp_min(0).sqrt()
        return ((a - mean) / std).to(adv.dtype)

    # -- learn ------------------------------------------------------------------------------
    def _actor_loss(self, minibatch: Batch):
        """dist, log pi(act|obs) and the vanilla policy-gradient loss (npg.py:88-93)."""
        dist = self(minibatch).dist
        log_prob = dist.log_prob(minibatch.act)
        log_prob = log_prob.reshape(log_prob.size(0), -1).transpose(0, 1)
        return dist, -(log_prob * minibatch.adv).mean()

    def _mean_over_ranks(self, t: torch.Tensor) -> torch.Tensor:
        if self.dp.active:
            self.dp.all_reduce_(t)
            t.div_(self.dp.world)
        return t

    def _natural_direction(self, minibatch: Batch, dist, actor_loss):
        """Search direction -F^-1 g and the KL gradient graph (npg.py:94-106)."""
        flat_grads = self._get_flat_grad(actor_loss, self.actor, retain_graph=True).detach()
        self._mean_over_ranks(flat_grads)
        with torch.no_grad():
            old_dist = self(minibatch).dist
        kl = kl_divergence(old_dist, dist).mean()
        flat_kl_grad = self._get_flat_grad(kl, self.actor, create_graph=True)
        direction = -self._conjugate_gradients(flat_grads, flat_kl_grad, nsteps=10)
        return direction, flat_kl_grad, old_dist

    def _critic_steps(self, minibatch: Batch) -> torch.Tensor:
        """npg.py:117-123."""
        vf_loss = None
        for _ in range(self._optim_critic_iters):
            value = self.critic(minibatch.obs).flatten()
            vf_loss = F.mse_loss(minibatch.returns, value)
            self.optim.zero_grad()
            vf_loss.backward()
            self.dp.all_reduce_grads_(self.critic.parameters(), average=True)
            self.optim.step()
        return vf_loss

    def learn(self, batch: Batch, batch_size: int, repeat: int, **kwargs: Any
              ) -> Dict[str, List[float]]:
        self._require_equal_shards(len(batch), next(self.critic.parameters()).device, "learn")
        actor_losses, vf_losses, kls = [], [], []
        for _ in range(repeat):
            for part in split_indices(len(batch), batch_size, True, True):
                minibatch = batch[part]
                dist, actor_loss = self._actor_loss(minibatch)
                direction, _, old_dist = self._natural_direction(minibatch, dist, actor_loss)
                with torch.no_grad():
                    flat_params = torch.cat([p.data.view(-1) for p in self.actor.parameters()])
                    self._set_from_flat_params(self.actor,
                                               flat_params + self._step_size * direction)
                    new_dist = self(minibatch).dist
                    kl = kl_divergence(old_dist, new_dist).mean()
                vf_loss = self._critic_steps(minibatch)
                actor_losses.append(actor_loss.detach())
                vf_losses.append(vf_loss.detach())
                kls.append(kl.detach())
        return self._read_lists({"loss/actor": actor_losses, "loss/vf": vf_losses, "kl": kls})

    def _read_lists(self, lists: Dict[str, list]) -> Dict[str, List[float]]:
        """One device->host copy for every logged value (the reference .item()s each)."""
        out = {}
        for k, v in lists.items():
            if not v:
                out[k] = []
                continue
            t = torch.stack([x.reshape(()).float() for x in v])
            out[k] = self._mean_over_ranks(t).cpu().tolist()
        return out

    # -- npg.py:132-181 ---------------------------------------------------------------------
    def _MVP(self, v: torch.Tensor, flat_kl_grad: torch.Tensor) -> torch.Tensor:
        """Fisher(KL Hessian)-vector product + damping."""
        kl_v = (flat_kl_grad * v).sum()
        flat_kl_grad_grad = self._get_flat_grad(kl_v, self.actor, retain_graph=True).detach()
        self._mean_over_ranks(flat_kl_grad_grad)
        return flat_kl_grad_grad + v * self._damping

    def _conjugate_gradients(self, minibatch: torch.Tensor, flat_kl_grad: torch.Tensor,
                             nsteps: int = 10, residual_tol: float = 1e-10) -> torch.Tensor:
        x = torch.zeros_like(minibatch)
        r, p = minibatch.clone(), minibatch.clone()
        # r = b - MVP(x) with x = 0
        rdotr = r.dot(r)
        for _ in range(nsteps):
            z = self._MVP(p, flat_kl_grad)
            alpha = rdotr / p.dot(z)
            x += alpha * p
            r -= alpha * z
            new_rdotr = r.dot(r)
            if new_rdotr < residual_tol:
                break
            p = r + new_rdotr / rdotr * p
            rdotr = new_rdotr
        return x

    def _get_flat_grad(self, y: torch.Tensor, model: nn.Module, **kwargs: Any) -> torch.Tensor:
        grads = torch.autograd.grad(y, model.parameters(), **kwargs)
        return torch.cat([grad.reshape(-1) for grad in grads])

    def _set_from_flat_params(self, model: nn.Module, flat_params: torch.Tensor) -> nn.Module:
        prev_ind = 0
        for param in model.parameters():
            flat_size = int(np.prod(list(param.size())))
            param.data.copy_(flat_params[prev_ind:prev_ind + flat_size].view(param.size()))
            prev_ind += flat_size
        return model
