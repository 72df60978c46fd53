"""BasePolicy (tianshou/policy/base.py:24-335) with the GAE of compute_episodic_return
running as the tsrl_gae HIP kernel."""
from typing import Any, Dict, Literal, Optional, Tuple, Union

import numpy as np
import torch
from torch import nn

from tianshou_amd import _C
from tianshou_amd.data.batch import Batch
from tianshou_amd.env.spaces import Box, Discrete


def _dev_of(*xs):
    for x in xs:
        if isinstance(x, torch.Tensor) and x.device.type == "cuda":
            return x.device
    return torch.device("cuda", torch.cuda.current_device())


# Optional timing hook: called as GAE_HOOK("start"|"end", n) around every tsrl_gae launch
# (bench.py records HIP events on the launch stream through it).
GAE_HOOK = None


def gae_device(v_s: torch.Tensor, v_s_: torch.Tensor, rew: torch.Tensor, term: torch.Tensor,
               trunc: torch.Tensor, gamma: float, gae_lambda: float, row_len: int = 0,
               end_extra: Optional[torch.Tensor] = None, value_scale: Optional[torch.Tensor] = None,
               want_f32: bool = True, want_f64: bool = False,
               ret_partials: Optional[torch.Tensor] = None):
    """Launch tsrl_gae on device tensors.  Returns (adv32, ret32, adv64, ret64) (None where
    not requested).  In rew_norm mode (value_scale given) ret32 is normalised by the scale
    (a2c.py:110-111) and ret64 is the unnormalised return."""
    n = rew.numel()
    dev = rew.device
    adv32 = torch.empty(n, dtype=torch.float32, device=dev) if want_f32 else None
    ret32 = torch.empty(n, dtype=torch.float32, device=dev) if want_f32 else None
    adv64 = torch.empty(n, dtype=torch.float64, device=dev) if want_f64 else None
    ret64 = torch.empty(n, dtype=torch.float64, device=dev) if want_f64 else None
    L = _C.lib()
    ws_bytes = int(L.tsrl_gae_workspace_bytes(n, row_len))
    ws = torch.empty(max(ws_bytes, 8), dtype=torch.uint8, device=dev) if ws_bytes else None
    args = (_C.ptr(v_s), _C.ptr(v_s_), _C.ptr(rew), _C.ptr(term), _C.ptr(trunc),
            _C.ptr(end_extra), n, row_len, _C.ptr(value_scale), float(gamma),
            float(gae_lambda), _C.ptr(adv32), _C.ptr(ret32), _C.ptr(adv64), _C.ptr(ret64),
            _C.ptr(ret_partials), _C.ptr(ws), ws_bytes, _C.stream_ptr(dev))
    fn = L.tsrl_gae
    if GAE_HOOK is not None:
        GAE_HOOK("start", n)
    rc = fn(*args)
    if GAE_HOOK is not None:
        GAE_HOOK("end", n)
    _C.check(rc, "tsrl_gae")
    return adv32, ret32, adv64, ret64


def _as_dev(x, dev, dtype=None):
    t = x if isinstance(x, torch.Tensor) else torch.as_tensor(np.asarray(x))
    t = t.to(dev)
    if dtype is not None:
        t = t.to(dtype)
    return t.reshape(-1).contiguous()


class BasePolicy(nn.Module):
    def __init__(self, observation_space=None, action_space=None, action_scaling: bool = False,
                 action_bound_method: Optional[Literal["clip", "tanh"]] = None,
                 lr_scheduler=None) -> None:
        if action_bound_method is not None:
            assert action_bound_method in ("clip", "tanh")
        if isinstance(action_space, list):
            action_space = action_space[0]
        if action_scaling and not isinstance(action_space, Box):
            raise ValueError(f"action_scaling can only be True when action_space is Box but "
                             f"got: {action_space}")
        super().__init__()
        self.observation_space = observation_space
        self.action_space = action_space
        if isinstance(action_space, Discrete) or hasattr(action_space, "n"):
            self.action_type = "discrete"
        elif isinstance(action_space, Box) or hasattr(action_space, "low"):
            self.action_type = "continuous"
        self.agent_id = 0
        self.updating = False
        self.action_scaling = action_scaling
        self.action_bound_method = action_bound_method
        self.lr_scheduler = lr_scheduler
        self._act_low_high = {}

    def set_agent_id(self, agent_id: int) -> None:
        self.agent_id = agent_id

    def exploration_noise(self, act, batch):
        return act

    def soft_update(self, tgt: nn.Module, src: nn.Module, tau: float) -> None:
        for tp, sp in zip(tgt.parameters(), src.parameters()):
            tp.data.copy_(tau * sp.data + (1 - tau) * tp.data)

    def forward(self, batch: Batch, state=None, **kwargs) -> Batch:
        raise NotImplementedError

    def _is_box_action(self) -> bool:
        return isinstance(self.action_space, Box) or (
            hasattr(self.action_space, "low") and not hasattr(self.action_space, "n"))

    def _low_high(self, device):
        key = str(device)
        if key not in self._act_low_high:
            low = torch.as_tensor(self.action_space.low, dtype=torch.float32, device=device)
            high = torch.as_tensor(self.action_space.high, dtype=torch.float32, device=device)
            self._act_low_high[key] = (low, high)
        return self._act_low_high[key]

    def map_action(self, act):
        """base.py:183-215: bound to [-1, 1] (clip / tanh), then scale to [low, high].
        Device tensors stay on device (the reference's [-1, 1] assert would need a
        device->host sync; it holds by construction after clip/tanh)."""
        if not self._is_box_action():
            return act
        if isinstance(act, torch.Tensor):
            if self.action_bound_method == "clip":
                act = act.clamp(-1.0, 1.0)
            elif self.action_bound_method == "tanh":
                act = torch.tanh(act)
            if self.action_scaling:
                low, high = self._low_high(act.device)
                act = low + (high - low) * (act + 1.0) / 2.0
            return act
        if isinstance(act, np.ndarray):
            if self.action_bound_method == "clip":
                act = np.clip(act, -1.0, 1.0)
            elif self.action_bound_method == "tanh":
                act = np.tanh(act)
            if self.action_scaling:
                assert np.min(act) >= -1.0 and np.max(act) <= 1.0, \
                    "action scaling only accepts raw action range = [-1, 1]"
                low, high = self.action_space.low, self.action_space.high
                act = low + (high - low) * (act + 1.0) / 2.0
        return act

    def map_action_inverse(self, act):
        is_box = isinstance(self.action_space, Box)
        if not is_box:
            return act
        if isinstance(act, torch.Tensor):
            if self.action_scaling:
                low, high = self._low_high(act.device)
                act = ((act - low) * 2.0) / (high - low) - 1.0
            if self.action_bound_method == "tanh":
                act = (torch.log(1.0 + act) - torch.log(1.0 - act)) / 2.0
            return act
        act = np.asarray(act)
        if self.action_scaling:
            low, high = self.action_space.low, self.action_space.high
            act = ((act - low) * 2.0) / (high - low) - 1.0
        if self.action_bound_method == "tanh":
            act = (np.log(1.0 + act) - np.log(1.0 - act)) / 2.0
        return act

    def process_fn(self, batch, buffer, indices):
        return batch

    def learn(self, batch, **kwargs) -> Dict[str, Any]:
        raise NotImplementedError

    def post_process_fn(self, batch, buffer, indices) -> None:
        if hasattr(buffer, "update_weight") and hasattr(batch, "weight"):
            buffer.update_weight(indices, batch.weight)

    def update(self, sample_size: int, buffer, **kwargs: Any) -> Dict[str, Any]:
        """base.py:288-315."""
        if buffer is None:
            return {}
        batch, indices = buffer.sample(sample_size)
        self.updating = True
        batch = self.process_fn(batch, buffer, indices)
        result = self.learn(batch, **kwargs)
        self.post_process_fn(batch, buffer, indices)
        if self.lr_scheduler is not None:
            self.lr_scheduler.step()
        self.updating = False
        return result

    @staticmethod
    def value_mask(buffer, indices: np.ndarray):
        """base.py:317-335: ~buffer.terminated[indices]."""
        t = buffer.terminated[torch.as_tensor(np.asarray(indices), device=buffer.device)]
        return ~t

    @staticmethod
    def compute_episodic_return(batch: Batch, buffer, indices: np.ndarray, v_s_=None,
                                v_s=None, gamma: float = 0.99, gae_lambda: float = 0.95
                                ) -> Tuple[Any, Any]:
        """base.py:337-384 on the GPU.  Any index order is accepted (general 3-phase scan,
        end flags forced at ``np.isin(indices, buffer.unfinished_index())``).  Returns f64
        (returns, advantage): NumPy when the inputs were NumPy, device tensors otherwise."""
        numpy_out = not any(isinstance(x, torch.Tensor) for x in (batch.rew, v_s_, v_s))
        dev = _dev_of(batch.rew, v_s_, v_s)
        rew = _as_dev(batch.rew, dev, torch.float64)
        n = rew.numel()
        term = _as_dev(batch.terminated, dev).bool().to(torch.uint8)
        trunc = _as_dev(batch.truncated, dev).bool().to(torch.uint8)
        if v_s_ is None:
            assert np.isclose(gae_lambda, 1.0)
            v_s_ = torch.zeros(n, dtype=torch.float64, device=dev)
        else:
            v_s_ = _as_dev(v_s_, dev)
        if v_s is None:  # base.py:377: v_s = roll(v_s_ * value_mask, 1)
            v_s = torch.roll(v_s_ * (term == 0).to(v_s_.dtype), 1)
        else:
            v_s = _as_dev(v_s, dev)
        unfinished = buffer.unfinished_index()
        extra = torch.as_tensor(np.isin(np.asarray(indices), unfinished).astype(np.uint8),
                                device=dev)
        if v_s.dtype == torch.float32 and v_s_.dtype == torch.float32:
            adv32, ret32, adv, ret = gae_device(v_s, v_s_, rew, term, trunc, gamma,
                                                gae_lambda, 0, extra, None, want_f32=False,
                                                want_f64=True)
        else:
            vs64, vn64 = v_s.to(torch.float64).contiguous(), v_s_.to(torch.float64).contiguous()
            adv = torch.empty(n, dtype=torch.float64, device=dev)
            ret = torch.empty(n, dtype=torch.float64, device=dev)
            L = _C.lib()
            ws_bytes = int(L.tsrl_gae_workspace_bytes(n, 0))
            ws = torch.empty(max(ws_bytes, 8), dtype=torch.uint8, device=dev)
            _C.check(L.tsrl_gae_f64v(_C.ptr(vs64), _C.ptr(vn64), _C.ptr(rew), _C.ptr(term),
                                     _C.ptr(trunc), _C.ptr(extra), n, 0, float(gamma),
                                     float(gae_lambda), _C.ptr(adv), _C.ptr(ret), _C.ptr(ws),
                                     ws_bytes, _C.stream_ptr(dev)), "tsrl_gae_f64v")
        if numpy_out:
            return ret.cpu().numpy(), adv.cpu().numpy()
        return ret, adv

    @staticmethod
    def compute_nstep_return(batch: Batch, buffer, indice: np.ndarray, target_q_fn,
                             gamma: float = 0.99, n_step: int = 1, rew_norm: bool = False
                             ) -> Batch:
        """base.py:386-440 with _nstep_return (base.py:500-524) as tsrl_nstep_return: the
        terminal rows next^(n_step-1)(indice) come from tsrl_ring_step_index on device (one
        host copy for ``target_q_fn``, which takes NumPy indices as in the reference); the
        discounted n-step sum, the episode-end truncation, the value mask and the
        gamma^k bootstrap run in one kernel in the reference's f64 operation order."""
        assert not rew_norm, \
            "Reward normalization in computing n-step returns is unsupported now."
        bsz = len(indice)
        dev = buffer._ensure_device()
        it = buffer._index_tensor(indice)
        terminal = buffer._step_dev(it, -(n_step - 1)) if n_step > 1 else \
            buffer._step_dev(it, 0)
        with torch.no_grad():
            target_q_torch = target_q_fn(buffer, terminal.cpu().numpy())  # (bsz, ?)
        tq = target_q_torch.reshape(bsz, -1)
        f64 = tq.dtype == torch.float64
        tq_dev = tq.to(device=dev, dtype=torch.float64 if f64 else torch.float32).contiguous()
        out = torch.empty_like(tq_dev)
        m = buffer._meta
        done, last, lengths = buffer._ring_dev()
        _C.check(_C.lib().tsrl_nstep_return(
            _C.ptr(m.rew), _C.ptr(done), _C.ptr(m.terminated), _C.ptr(last), _C.ptr(lengths),
            buffer._ring.size, buffer.buffer_num, _C.ptr(it), bsz, int(n_step), float(gamma),
            _C.ptr(tq_dev), tq_dev.shape[1] if bsz else 1, int(f64), _C.ptr(out),
            _C.stream_ptr(dev)), "tsrl_nstep_return")
        batch.returns = out.to(device=target_q_torch.device, dtype=target_q_torch.dtype)
        if hasattr(batch, "weight"):  # prio buffer update
            batch.weight = torch.as_tensor(batch.weight).to(device=target_q_torch.device,
                                                            dtype=target_q_torch.dtype)
        return batch
