"""Device evaluation shared by the on-policy policies whose process_fn needs logp_old next to
the critic values: PPOPolicy (ppo.py:87-97) and NPGPolicy/TRPOPolicy (npg.py:68-79).

For the get_actor_critic networks (Gaussian ActorProb with state-independent log-std) one
pass of the fused MLP kernels (policy/fused_mlp.py) yields V(s) and log pi(act|s) together;
V(s') reuses V(s) of the next row of the same env.  Categorical policies get the fused
Categorical log-prob kernel (tsrl_cat_logp) on the torch actor output.
"""
from typing import Optional

import torch
from torch.distributions import Independent, Normal

from tianshou_amd import _C
from tianshou_amd.policy import fused_mlp as _fmlp
from tianshou_amd.utils.net import ActorProb, DiscreteActor, DiscreteCritic


def _is_fixed_std_normal(dist_fn) -> bool:
    try:
        d = dist_fn(torch.zeros(1, 2), torch.ones(1, 2))
    except Exception:
        return False
    return isinstance(d, Independent) and isinstance(d.base_dist, Normal) and \
        d.reinterpreted_batch_ndims == 1


def cat_mode(dist_fn) -> Optional[int]:
    """0 when dist_fn(x) is Categorical(logits=x), 1 when Categorical(probs=x), else None."""
    x = torch.tensor([[0.2, 0.6, 0.2]])
    try:
        d = dist_fn(x)
    except Exception:
        return None
    if not isinstance(d, torch.distributions.Categorical):
        return None
    if torch.allclose(d.probs, x / x.sum(-1, keepdim=True)):
        return 1
    if torch.allclose(d.probs, torch.softmax(x, -1)):
        return 0
    return None


def cat_logp(x: torch.Tensor, act: torch.Tensor, mode: int) -> torch.Tensor:
    """Categorical(...).log_prob(act) of dist_fn input rows x (tsrl_cat_logp)."""
    x = x.detach().float().contiguous()
    act = act.reshape(-1).to(torch.int64).contiguous()
    out = torch.empty(x.shape[0], dtype=torch.float32, device=x.device)
    _C.check(_C.lib().tsrl_cat_logp(_C.ptr(x), _C.ptr(act), x.shape[0], x.shape[1], int(mode),
                                    _C.ptr(out), _C.stream_ptr(x.device)), "tsrl_cat_logp")
    return out


class FusedEvalMixin:
    """Mixed into an A2CPolicy subclass: detection of the fused paths, the fused
    ``_eval_values`` override and ``_logp_old``."""

    def _init_fused_eval(self, actor, critic, dist_fn, fused_mlp: bool = True) -> None:
        self._fused = isinstance(actor, ActorProb) and not actor._c_sigma and \
            _is_fixed_std_normal(dist_fn)
        self._gauss_dist = self._fused
        # Categorical policies: the fused log-prob / loss kernels (tsrl_cat_*), torch nets
        self._cat = cat_mode(dist_fn) if not self._fused else None
        # the get_actor_critic MLPs as fused HIP kernels (policy/fused_mlp.py)
        self._mlp = None
        self._pending_logp = None
        # one preprocess net under both heads (examples/atari/atari_ppo.py:104-125 shares the
        # features_only DQN trunk): the trunk runs once per row for V(s) and the actor output
        self._shared_trunk = isinstance(actor, DiscreteActor) and \
            isinstance(critic, DiscreteCritic) and actor.preprocess is critic.preprocess
        if self._fused and fused_mlp:
            layers = _fmlp.match(actor, critic)
            if layers is not None:
                self._mlp = _fmlp.FusedActorCritic(layers, self._actor_critic.parameters())

    def _logp_old(self, batch) -> torch.Tensor:
        """log pi_old(act|obs) of every row (after _compute_returns, which may have produced
        it already on the fused path)."""
        with torch.no_grad():
            if self._pending_logp is not None:
                out = self._pending_logp
            elif self._fused:
                out = self._logp_fused(batch.obs, batch.act)
            elif self._cat is not None and isinstance(batch.obs, torch.Tensor) and \
                    batch.obs.is_cuda:
                out = self._logp_cat(batch.obs, batch.act)
            else:
                n = len(batch.act)
                parts = [self(batch[s:e]).dist.log_prob(batch.act[s:e])
                         for s, e in self._chunks(n)]
                out = torch.cat(parts) if parts else torch.empty(0)
        self._pending_logp = None
        return out

    def _eval_values(self, batch, obs, obs_next, buffer, indices):
        """Fused path: one layer-1 pass over obs gives V(s) and logp_old together (the latter
        kept for process_fn).  V(s') reuses V(s) of the next row of the same env whenever the
        buffer was filled by the Collector (``buffer.obs_chain``: the stored obs of step t+1 is
        the stored obs_next of step t unless the episode ended at t), so only the episode-end
        and segment-end rows are evaluated on obs_next; the values are bit-identical to a full
        evaluation because every row's arithmetic is independent of the other rows."""
        if self._cat is not None and self._shared_trunk and obs.is_cuda:
            return self._eval_values_shared(batch, obs, obs_next, buffer, indices)
        if self._mlp is None or not obs.is_cuda or obs.dtype != torch.float32 or obs.dim() != 2:
            return super()._eval_values(batch, obs, obs_next, buffer, indices)
        # rows must be contiguous, not the whole tensor: the buffer's padded storage views
        # (128-byte row pitch) are read in place (a .contiguous() here copied 12.6 GB)
        if obs.stride(-1) != 1 or obs.stride(0) < obs.shape[1]:
            obs = obs.contiguous()
        if obs_next.stride(-1) != 1 or obs_next.stride(0) < obs_next.shape[1]:
            obs_next = obs_next.contiguous()
        n = obs.shape[0]
        act = torch.as_tensor(batch.act, device=obs.device).to(torch.float32).reshape(n, -1)
        v_s, logp = self._mlp.evaluate(obs, act.contiguous())
        self._pending_logp = logp
        row_len, _ = self._gae_layout(buffer, indices)
        if row_len and getattr(buffer, "obs_chain", False) and n % row_len == 0:
            done = torch.as_tensor(batch.done, device=obs.device).bool().reshape(n).clone()
            done[row_len - 1::row_len] = True
            rows = done.nonzero().flatten()
            v_s_ = torch.roll(v_s, -1)
            if rows.numel():
                vals, _ = self._mlp.evaluate(obs_next, None, rows)
                v_s_[rows] = vals
        else:
            v_s_, _ = self._mlp.evaluate(obs_next)
        return v_s, v_s_

    def _logp_fused(self, obs: torch.Tensor, act: torch.Tensor) -> torch.Tensor:
        dev = act.device
        n = len(act)
        act = act.reshape(n, -1).contiguous()
        A = act.shape[1]
        out = torch.empty(n, dtype=torch.float32, device=dev)
        log_std = self.actor.sigma_param.detach().reshape(-1).contiguous()
        L = _C.lib()
        for s, e in self._chunks(n):
            mu = self.actor.forward_mu(obs[s:e]).contiguous()
            _C.check(L.tsrl_gauss_logp(_C.ptr(mu), _C.ptr(log_std), _C.ptr(act[s:e]), e - s, A,
                                       _C.ptr(out[s:e]), _C.stream_ptr(dev)), "tsrl_gauss_logp")
        return out

    def _trunk_heads(self, obs: torch.Tensor, rows: Optional[torch.Tensor] = None):
        """(actor output, V) of a shared-trunk DiscreteActor / DiscreteCritic pair with ONE
        trunk pass: actor.forward (utils/net.py DiscreteActor, discrete.py:52-71) and
        critic.forward (discrete.py:111-121) both start with preprocess(obs, None) on the same
        module, so the features are computed once and fed to both heads.  Forward values are
        those of the two separate passes; in backward the two heads' feature gradients are
        summed before the trunk instead of after it (float summation order only).  rows: the
        minibatch is obs[rows], read in place when the trunk can (DQN.reads_rows)."""
        if rows is not None:
            h, _ = self.actor.preprocess(obs, None, rows=rows)
        else:
            h, _ = self.actor.preprocess(obs, None)
        x = self.actor.last(h)
        if self.actor.softmax_output:
            x = torch.softmax(x, dim=-1)
        return x, self.critic.last(h).flatten()

    def _eval_values_shared(self, batch, obs, obs_next, buffer, indices):
        """Shared-trunk process_fn evaluation: V(s) and logp_old (kept for _logp_old) from one
        trunk pass per row; V(s') from V(s) when the buffer's obs_next rows are batch rows."""
        n = obs.shape[0]
        dev = obs.device
        v_s = torch.empty(n, dtype=torch.float32, device=dev)
        logp = torch.empty(n, dtype=torch.float32, device=dev)
        act = torch.as_tensor(batch.act, device=dev).reshape(n)
        for s, e in self._chunks(n, obs[0].numel() if n else 1):
            x, v = self._trunk_heads(obs[s:e])
            v_s[s:e] = v
            logp[s:e] = cat_logp(x, act[s:e], self._cat)
        self._pending_logp = logp
        p = self._next_positions(buffer, indices, dev)
        return v_s, (v_s[p] if p is not None else self._values(obs_next))

    def _logp_cat(self, obs: torch.Tensor, act: torch.Tensor) -> torch.Tensor:
        n = obs.shape[0]
        out = torch.empty(n, dtype=torch.float32, device=obs.device)
        act = torch.as_tensor(act, device=obs.device).reshape(n)
        for s, e in self._chunks(n, obs[0].numel() if n else 1):
            x, _ = self.actor(obs[s:e])
            out[s:e] = cat_logp(x, act[s:e], self._cat)
        return out

