"""Collector policy step of the MuJoCo Gaussian actor as one HIP kernel.

``policy(batch).act`` + ``policy.map_action`` of collector.py:286-303 (pg.py:133-171,
base.py:183-215) for the actor of utils/models.py:34-97 (two Tanh layers of 64, unbounded
``Linear(64, A)`` mu head, state-independent log-std) is one launch of
``tsrl_gauss_policy_act`` after a standard-normal draw of the noise; torch would run ~12
kernels (three GEMMs, tanh, exp, broadcast, randn, mul, add, clamp, scaling).  The noise is
drawn with torch's generator exactly as ``torch.randn_like(mu)`` would (same shape, same
stream), so the sampled actions equal ``randn * sigma + mu`` of the torch path up to the
GEMM summation order.
"""
from typing import Optional

import torch

from tianshou_amd import _C
from tianshou_amd.policy.fused_mlp import MAX_ACT, _seq, _trunk

_BOUND = {None: 0, "clip": 1, "tanh": 2}


def match_actor(actor) -> Optional[dict]:
    from tianshou_amd.utils.net import ActorProb
    if not isinstance(actor, ActorProb) or actor._c_sigma or not actor._unbounded:
        return None
    l1 = getattr(actor.preprocess, "model", None)
    D = getattr(getattr(l1, "model", [None])[0], "in_features", None) if l1 is not None else None
    if not isinstance(D, int):
        return None
    tr = _trunk(actor.preprocess, D)
    mu = _seq(actor.mu)
    if tr is None or mu is None or len(mu) != 1 or not isinstance(mu[0], torch.nn.Linear):
        return None
    head = mu[0]
    if head.in_features != 64 or not 0 < head.out_features <= MAX_ACT or head.bias is None:
        return None
    if actor.sigma_param.numel() != head.out_features:
        return None
    return {"w1": tr[0], "w2": tr[1], "w3": head, "sigma": actor.sigma_param, "D": D,
            "A": head.out_features}


class FusedGaussAct:
    def __init__(self, layers: dict) -> None:
        self.L = layers
        self.D, self.A = layers["D"], layers["A"]
        self.packed = None
        self.packed_c = None  # layer-1 layout of the fused collect step (tsrl_collect_pack_w1)
        self._eps = None
        # "device": noise drawn in-kernel from a counter hash seeded from torch's CPU
        # generator at each pack() (reproducible under torch.manual_seed); "torch": noise
        # from torch.randn on the GPU stream (the torch path's exact noise, one extra launch)
        self.rng = "device"
        self._seed = None
        self._ctr = None      # own [2] counter pair when the caller passes none
        self._parity = 0

    def pack(self) -> None:
        """Pack the first-layer weight (call after every parameter update; the collector
        does it at the start of each collect)."""
        w = self.L["w1"].weight
        lib = _C.lib()
        n = int(lib.tsrl_policy_pack_floats(self.D))
        if self.packed is None or self.packed.numel() != n or self.packed.device != w.device:
            self.packed = torch.empty(n, dtype=torch.float32, device=w.device)
        _C.check(lib.tsrl_policy_pack_l1(_C.ptr(w.detach()), self.D, _C.ptr(self.packed),
                                         _C.stream_ptr(w.device)), "tsrl_policy_pack_l1")
        if self.D <= 512:
            nc = int(lib.tsrl_collect_pack_floats(self.D))
            if self.packed_c is None or self.packed_c.numel() != nc or \
                    self.packed_c.device != w.device:
                self.packed_c = torch.empty(nc, dtype=torch.float32, device=w.device)
            _C.check(lib.tsrl_collect_pack_w1(_C.ptr(w.detach()), self.D, _C.ptr(self.packed_c),
                                              _C.stream_ptr(w.device)), "tsrl_collect_pack_w1")
        if self.rng == "device":
            # one seed per policy, drawn at the first pack from torch's CPU generator: steps
            # replayed from HIP graphs carry the seed captured with them, so a per-collect
            # reseed would give eager and replayed steps different streams; fresh noise comes
            # from the collector's step counters, which never repeat
            if self._seed is None:
                self._seed = int(torch.randint(0, 2 ** 62, (1,)).item())
            if self._ctr is None or self._ctr.device != w.device:
                self._ctr = torch.zeros(2, dtype=torch.int64, device=w.device)
            self._ctr.zero_()
            self._parity = 0

    def fill_collect(self, c, sample: bool, bound_method, low_high, ctr) -> bool:
        """Actor fields of a ``tsrl_collect_args`` (the fused collect step, csrc/collect.hip):
        the same operands and noise stream as the ``tsrl_gauss_policy_act_rng`` launch of
        ``__call__``.  False when that step cannot run this actor (torch-generator noise, or
        an observation dim beyond its 512 columns)."""
        if self.packed_c is None or (sample and self.rng != "device"):
            return False
        L = self.L
        low, high = low_high if low_high is not None else (None, None)
        c.w1p = _C.ptr(self.packed_c)
        c.b1 = _C.ptr(L["w1"].bias.detach())
        c.w2 = _C.ptr(L["w2"].weight.detach())
        c.b2 = _C.ptr(L["w2"].bias.detach())
        c.w3 = _C.ptr(L["w3"].weight.detach())
        c.b3 = _C.ptr(L["w3"].bias.detach())
        c.log_std = _C.ptr(L["sigma"].detach())
        c.act_dim = self.A
        c.sample = int(bool(sample))
        c.act_seed = int(self._seed or 0)
        c.rng_ctr = _C.ptr(ctr[0]) if sample else None
        c.rng_next = _C.ptr(ctr[1]) if sample else None
        c.bound_method = _BOUND[bound_method]
        c.low, c.high = _C.ptr(low), _C.ptr(high)
        return True

    def __call__(self, obs: torch.Tensor, act_out: torch.Tensor, remap_out: torch.Tensor,
                 sample: bool, bound_method, low_high, ctr=None) -> None:
        """ctr: optional (in, out) device int64 words of the noise step counter (the
        collector passes its ping-pong slots); default: this object's own pair."""
        L, lib = self.L, _C.lib()
        n = obs.shape[0]
        low, high = low_high if low_high is not None else (None, None)
        if sample and self.rng == "device":
            if ctr is None:
                ctr = (self._ctr[self._parity:self._parity + 1],
                       self._ctr[1 - self._parity:2 - self._parity])
                self._parity ^= 1
            _C.check(lib.tsrl_gauss_policy_act_rng(
                _C.ptr(obs), obs.stride(0), n, self.D, _C.ptr(self.packed),
                _C.ptr(L["w1"].bias.detach()), _C.ptr(L["w2"].weight.detach()),
                _C.ptr(L["w2"].bias.detach()), _C.ptr(L["w3"].weight.detach()),
                _C.ptr(L["w3"].bias.detach()), _C.ptr(L["sigma"].detach()), self.A,
                self._seed, _C.ptr(ctr[0]), _C.ptr(ctr[1]),
                _BOUND[bound_method], _C.ptr(low), _C.ptr(high), _C.ptr(act_out),
                _C.ptr(remap_out), _C.stream_ptr(obs.device)), "tsrl_gauss_policy_act_rng")
            return
        eps = None
        if sample:
            if self._eps is None or self._eps.shape[0] < n or self._eps.device != obs.device:
                self._eps = torch.empty(n, self.A, device=obs.device)
            eps = self._eps[:n]
            eps.normal_()
        _C.check(lib.tsrl_gauss_policy_act(
            _C.ptr(obs), obs.stride(0), n, self.D, _C.ptr(self.packed),
            _C.ptr(L["w1"].bias.detach()), _C.ptr(L["w2"].weight.detach()),
            _C.ptr(L["w2"].bias.detach()), _C.ptr(L["w3"].weight.detach()),
            _C.ptr(L["w3"].bias.detach()), _C.ptr(L["sigma"].detach()), self.A,
            _C.ptr(eps), _BOUND[bound_method], _C.ptr(low), _C.ptr(high), _C.ptr(act_out),
            _C.ptr(remap_out), _C.stream_ptr(obs.device)), "tsrl_gauss_policy_act")
