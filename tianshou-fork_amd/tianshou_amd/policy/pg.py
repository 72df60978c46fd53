"""PGPolicy (tianshou/policy/modelfree/pg.py:20-171)."""
from typing import Any, Callable, Dict, List, Literal, Optional

import numpy as np
import torch

from tianshou_amd.data.batch import Batch, split_indices
from tianshou_amd.policy.base import BasePolicy
from tianshou_amd.utils.statistics import DeviceScalarRMS


def make_dist(dist_fn, logits, validate: bool = False):
    """dist_fn(*logits), by default without torch.distributions argument validation: its
    checks are device reductions followed by a host-side ``if not valid.all()`` -- a
    device->host sync per construction, i.e. per collector step.  The reference validates
    (invalid parameters raise ValueError); ``validate=True`` (``PGPolicy(validate_args=True)``)
    keeps that behaviour at the cost of the sync, otherwise invalid parameters surface as NaN
    losses.  The global default is restored afterwards either way."""
    if validate:
        return dist_fn(*logits) if isinstance(logits, tuple) else dist_fn(logits)
    prev = torch.distributions.Distribution._validate_args
    torch.distributions.Distribution.set_default_validate_args(False)
    try:
        return dist_fn(*logits) if isinstance(logits, tuple) else dist_fn(logits)
    finally:
        torch.distributions.Distribution.set_default_validate_args(prev)


def _gumbel_ok(dist) -> bool:
    """A plain torch Categorical over [batch, A] f32 logits on the GPU."""
    if type(dist) is not torch.distributions.Categorical:
        return False
    lg = dist.logits
    return lg.is_cuda and lg.dim() == 2 and lg.dtype == torch.float32


def gumbel_sample(logits: torch.Tensor) -> torch.Tensor:
    """Categorical(logits).sample() in one HIP pass (tsrl_cat_gumbel_argmax): argmax of
    logits + Gumbel noise from torch.rand_like (torch's seeded, graph-capturable stream).
    Same distribution as torch's softmax + multinomial, one launch instead of ~14."""
    from tianshou_amd import _C
    lg = logits.contiguous()
    u = torch.rand_like(lg)
    out = torch.empty(lg.shape[0], dtype=torch.int64, device=lg.device)
    _C.check(_C.lib().tsrl_cat_gumbel_argmax(_C.ptr(lg), _C.ptr(u), lg.shape[0], lg.shape[1],
                                             _C.ptr(out), _C.stream_ptr(lg.device)),
             "tsrl_cat_gumbel_argmax")
    return out


class PGPolicy(BasePolicy):
    # Categorical collector steps sample through gumbel_sample (False: dist.sample())
    fused_cat_sample = True

    def __init__(self, model: torch.nn.Module, optim: torch.optim.Optimizer,
                 dist_fn: Callable[..., torch.distributions.Distribution],
                 discount_factor: float = 0.99, reward_normalization: bool = False,
                 action_scaling: bool = True,
                 action_bound_method: Optional[Literal["clip", "tanh"]] = "clip",
                 deterministic_eval: bool = False, validate_args: bool = False,
                 **kwargs: Any) -> None:
        super().__init__(action_scaling=action_scaling, action_bound_method=action_bound_method,
                         **kwargs)
        self.actor = model
        self.optim = optim
        self.dist_fn = dist_fn
        assert 0.0 <= discount_factor <= 1.0, "discount factor should be in [0, 1]"
        self._gamma = discount_factor
        self._rew_norm = reward_normalization
        self._ret_rms = None
        self._eps = 1e-8
        self._deterministic_eval = deterministic_eval
        # torch.distributions argument checks as in the reference (ValueError on invalid
        # parameters; one host sync per distribution), off by default (see make_dist)
        self.validate_args = validate_args

    @property
    def ret_rms(self) -> DeviceScalarRMS:
        """Running mean/std of the returns, kept in HBM (pg.py:82)."""
        if self._ret_rms is None:
            dev = next(self.parameters()).device
            self._ret_rms = DeviceScalarRMS(dev)
        return self._ret_rms

    # -- fused collector step (policy/fused_act.py) ------------------------------------------
    def prepare_fused_act(self) -> bool:
        """True when the collector may run this policy's act + map_action as the fused
        kernel (Gaussian ActorProb of the get_actor_critic shape, Box actions); packs the
        current first-layer weight."""
        if not getattr(self, "_gauss_dist", False) or not self._is_box_action():
            return False
        fa = getattr(self, "_fused_act", None)
        if fa is None:
            from tianshou_amd.policy.fused_act import FusedGaussAct, match_actor
            layers = match_actor(self.actor)
            fa = FusedGaussAct(layers) if layers is not None else False
            self._fused_act = fa
        if fa is False or not next(self.actor.parameters()).is_cuda:
            return False
        fa.rng = getattr(self, "fused_act_rng", "device")
        fa.pack()
        return True

    def fused_act(self, obs, act_out, remap_out, ctr=None) -> None:
        sample = not (self._deterministic_eval and not self.training)
        low_high = self._low_high(obs.device) if self.action_scaling else None
        self._fused_act(obs, act_out, remap_out, sample, self.action_bound_method, low_high,
                        ctr)

    def fused_collect_fill(self, c, ctr) -> bool:
        """Fill the actor fields of the fused collect step (csrc/collect.hip) after
        prepare_fused_act(); False if this policy's act must stay a separate launch."""
        fa = getattr(self, "_fused_act", None)
        if not fa:
            return False
        sample = not (self._deterministic_eval and not self.training)
        dev = fa.L["w1"].weight.device
        low_high = self._low_high(dev) if self.action_scaling else None
        return fa.fill_collect(c, sample, self.action_bound_method, low_high, ctr)

    def _get_deterministic_action(self, logits):
        if self.action_type == "discrete":
            return logits.argmax(-1)
        return logits[0]

    def forward(self, batch: Batch, state=None, **kwargs: Any) -> Batch:
        """pg.py:133-171."""
        if getattr(self, "_gauss_dist", False):
            # ActorProb with state-independent sigma + Independent(Normal): sigma is
            # exp(sigma_param) broadcast (continuous.py:229-233) and dist.sample() is
            # torch.normal(mu, sigma) = standard normal * sigma + mu; written out directly,
            # because torch.normal's tensor-std path checks std >= 0 with a host sync.
            mu = self.actor.forward_mu(batch.obs)
            sigma = self.actor.sigma_param.view(1, -1).exp().expand_as(mu)
            dist = make_dist(self.dist_fn, (mu, sigma), self.validate_args)
            if self._deterministic_eval and not self.training:
                act = mu
            else:
                act = torch.randn_like(mu).mul_(sigma).add_(mu)
            return Batch(logits=(mu, sigma), act=act, state=state, dist=dist)
        logits, hidden = self.actor(batch.obs, state=state, info=batch.get("info", {}))
        dist = make_dist(self.dist_fn, logits, self.validate_args)
        if self._deterministic_eval and not self.training:
            act = self._get_deterministic_action(logits)
        elif self.fused_cat_sample and _gumbel_ok(dist):
            act = gumbel_sample(dist.logits)
        else:
            act = dist.sample()
        return Batch(logits=logits, act=act, state=hidden, dist=dist)

    def process_fn(self, batch, buffer, indices):
        """pg.py:87-126: Monte-Carlo returns (GAE with lambda = 1, v_s_ = ret_rms.mean)."""
        n = len(indices)
        v_s_ = np.full(n, self.ret_rms.mean)
        ret, _ = self.compute_episodic_return(batch, buffer, indices, v_s_=v_s_, gamma=self._gamma,
                                              gae_lambda=1.0)
        if self._rew_norm:
            batch.returns = (ret - self.ret_rms.mean) / np.sqrt(self.ret_rms.var + self._eps)
            r = torch.as_tensor(ret, device=self.ret_rms.state.device)
            bm, bv, bc = r.mean(), r.var(unbiased=False), float(len(r))
            st = self.ret_rms.state
            delta = bm - st[0]
            tot = st[2] + bc
            m2 = st[1] * st[2] + bv * bc + delta ** 2 * st[2] * bc / tot
            st.copy_(torch.stack([st[0] + delta * bc / tot, m2 / tot, tot]))
        else:
            batch.returns = ret
        return batch

    def learn(self, batch: Batch, batch_size: int, repeat: int, **kwargs: Any
              ) -> Dict[str, List[float]]:
        losses = []
        for _ in range(repeat):
            for part in split_indices(len(batch), batch_size, True, True):
                minibatch = batch[part]
                self.optim.zero_grad()
                result = self(minibatch)
                dist = result.dist
                act = torch.as_tensor(minibatch.act, device=result.act.device)
                ret = torch.as_tensor(minibatch.returns, device=result.act.device,
                                      dtype=torch.float32)
                log_prob = dist.log_prob(act).reshape(len(ret), -1).transpose(0, 1)
                loss = -(log_prob * ret).mean()
                loss.backward()
                self.optim.step()
                losses.append(loss.detach())
        return {"loss": [float(x) for x in torch.stack(losses).cpu()] if losses else []}
