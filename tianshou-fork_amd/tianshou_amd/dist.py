"""Env-sharded data parallelism over torch.distributed (backend "nccl" = RCCL on ROCm).

Each rank owns a disjoint shard of the vector envs (weak scaling: per-GPU work fixed).
Rollout collection and GAE are rank-local (episode segments never cross ranks, SURVEY.md
§8e).  The exchanges are the reference semantics of ONE global minibatch made of every
rank's local minibatch: advantage moments (sum, sum of squares), the loss partial sums,
the flattened gradients (one all-reduce per minibatch), the obs_rms batch moments per env
step, and the ret_rms partials per update.
"""
from typing import Iterable, Optional

import torch
import torch.distributed as dist


class DataParallel:
    # True: run the collective code path even with a single rank (all-reduces over a
    # one-rank RCCL communicator are identities) -- bench.py --force-dp, used by the GPU test
    # that rehearses the N>1 path on a one-GPU box.
    force = False

    def __init__(self, group=None) -> None:
        self.group = group
        self.enabled = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if self.enabled else 1
        self.rank = dist.get_rank(group) if self.enabled else 0
        self._flat = None

    @property
    def active(self) -> bool:
        return self.enabled and (self.world > 1 or DataParallel.force)

    @property
    def capturable(self) -> bool:
        """Collectives of this group can be captured into a HIP graph (RCCL); gloo cannot."""
        return self.enabled and dist.get_backend(self.group) == "nccl"

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.active:
            dist.all_reduce(t, group=self.group)
        return t

    def all_gather_cat(self, t: torch.Tensor) -> torch.Tensor:
        """Concatenate equally-shaped tensors of every rank in rank order."""
        if not self.active:
            return t
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t.contiguous(), group=self.group)
        return torch.cat(out)

    def broadcast_params_(self, params: Iterable[torch.nn.Parameter], src: int = 0) -> None:
        """Make every rank's replica rank ``src``'s (one bucketed broadcast): data-parallel
        learning keeps identical replicas by applying the same all-reduced step, which needs
        identical starting parameters whatever seed each rank built its networks with."""
        if not self.active:
            return
        ps = [p for p in params]
        if not ps:
            return
        flat = torch.cat([p.detach().reshape(-1) for p in ps])
        dist.broadcast(flat, src=src, group=self.group)
        o = 0
        with torch.no_grad():
            for p in ps:
                p.copy_(flat[o:o + p.numel()].view_as(p))
                o += p.numel()

    def all_reduce_grads_(self, params: Iterable[torch.nn.Parameter],
                          average: bool = False) -> None:
        """One bucketed all-reduce of every gradient.  SUM by default (the fused PPO loss
        already divides each rank's contribution by the global minibatch size); ``average``
        for losses that are per-rank means."""
        if not self.active:
            return
        grads = [p.grad for p in params if p.grad is not None]
        if not grads:
            return
        n = sum(g.numel() for g in grads)
        if self._flat is None or self._flat.numel() != n or self._flat.device != grads[0].device:
            self._flat = torch.empty(n, dtype=grads[0].dtype, device=grads[0].device)
        torch.cat([g.reshape(-1) for g in grads], out=self._flat)
        dist.all_reduce(self._flat, group=self.group)
        if average:
            self._flat.div_(self.world)
        o = 0
        for g in grads:
            g.copy_(self._flat[o:o + g.numel()].view_as(g))
            o += g.numel()


_DEFAULT: Optional[DataParallel] = None


def default_dp() -> DataParallel:
    global _DEFAULT
    if _DEFAULT is None or (not _DEFAULT.enabled and dist.is_available()
                            and dist.is_initialized()):
        _DEFAULT = DataParallel()
    return _DEFAULT
