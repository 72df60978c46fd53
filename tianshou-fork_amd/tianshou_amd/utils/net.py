"""Actor/critic networks with the reference's module layout, so ``state_dict()`` keys match
tianshou 0.5.1 checkpoints (utils/net/common.py:56-285, continuous.py:87-235,
discrete.py:12-121).  The GEMMs run through PyTorch-ROCm (hipBLASLt) on the GPU."""
from typing import Any, Dict, Optional, Sequence, Tuple, Type, Union

import numpy as np
import torch
from torch import nn

from tianshou_amd import _C

SIGMA_MIN = -20
SIGMA_MAX = 2


def sum_rows(x: torch.Tensor) -> torch.Tensor:
    """x.sum(0) for a [rows, cols] f32 HIP tensor through tsrl_sum_rows_f32 (torch's
    reduction of a [262144, 17] gradient took 0.34 ms; this one reads it at HBM rate)."""
    x = x.contiguous()
    rows, cols = x.shape[0], int(x[0].numel()) if x.dim() > 1 else 1
    out = torch.empty(x.shape[1:], dtype=x.dtype, device=x.device)
    L = _C.lib()
    wsb = int(L.tsrl_sum_rows_workspace_bytes(rows, cols))
    ws = torch.empty(max(wsb, 4), dtype=torch.uint8, device=x.device) if wsb else None
    _C.check(L.tsrl_sum_rows_f32(_C.ptr(x), rows, cols, _C.ptr(out), _C.ptr(ws), wsb,
                                 _C.stream_ptr(x.device)), "tsrl_sum_rows_f32")
    return out


def _split_factor(rows: int) -> int:
    """Split-K factor for the weight-gradient GEMM dW = dY^T X over `rows` minibatch rows."""
    for s in (256, 128, 64, 32, 16):
        if rows % s == 0 and rows // s >= 512:
            return s
    return 1


class _LinearFn(torch.autograd.Function):
    """y = x W^T + b.  The backward's weight gradient reduces over the minibatch rows
    (K = 262144 in the benchmark): as a single GEMM that leaves a handful of output tiles for
    256 CUs (hipBLASLt measured 0.75 ms for [64 x 262144] x [262144 x 376] on MI355X), so it
    is split over K in a batched GEMM and the partial products are summed (0.14 ms)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        if bias is not None:
            return torch.addmm(bias, x, weight.t())
        return x @ weight.t()

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        gx = gw = gb = None
        if torch.is_grad_enabled():
            # backward of a create_graph pass (NPG/TRPO's KL Hessian-vector products): only
            # differentiable torch ops, so the double backward sees the whole graph
            if ctx.needs_input_grad[0]:
                gx = gy @ weight
            if ctx.needs_input_grad[1]:
                gw = gy.t() @ x
            if ctx.has_bias and ctx.needs_input_grad[2]:
                gb = gy.sum(0)
            return gx, gw, gb
        if ctx.needs_input_grad[0]:
            gx = gy @ weight
        if ctx.needs_input_grad[1]:
            s = _split_factor(x.shape[0])
            if s > 1 and x.is_cuda:
                part = torch.bmm(gy.reshape(s, -1, gy.shape[1]).transpose(1, 2),
                                 x.reshape(s, -1, x.shape[1]))
                gw = sum_rows(part.reshape(s, -1)).view_as(weight)
            else:
                gw = gy.t() @ x
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = sum_rows(gy) if gy.is_cuda else gy.sum(0)
        return gx, gw, gb


class Linear(nn.Linear):
    """nn.Linear (same parameters / state_dict keys) with the split-K weight gradient."""

    def forward(self, x):
        if x.dim() != 2:
            return super().forward(x)
        return _LinearFn.apply(x, self.weight, self.bias)


def miniblock(input_size, output_size=0, norm_layer=None, activation=None,
              linear_layer: Type[nn.Linear] = Linear):
    layers = [linear_layer(input_size, output_size)]
    if norm_layer is not None:
        layers += [norm_layer(output_size)]
    if activation is not None:
        layers += [activation()]
    return layers


class MLP(nn.Module):
    """MLP backbone (common.py:56-150): Linear/activation stack in ``self.model``."""

    def __init__(self, input_dim: int, output_dim: int = 0, hidden_sizes: Sequence[int] = (),
                 norm_layer=None, activation=nn.ReLU, device=None,
                 linear_layer: Type[nn.Linear] = Linear, flatten_input: bool = True):
        super().__init__()
        self.device = device
        sizes = [input_dim] + list(hidden_sizes)
        acts = activation if isinstance(activation, (list, tuple)) else \
            [activation] * len(hidden_sizes)
        norms = norm_layer if isinstance(norm_layer, (list, tuple)) else \
            [norm_layer] * len(hidden_sizes)
        model = []
        for i, (din, dout) in enumerate(zip(sizes[:-1], sizes[1:])):
            model += miniblock(din, dout, norms[i], acts[i], linear_layer)
        if output_dim > 0:
            model += [linear_layer(sizes[-1], output_dim)]
        self.output_dim = output_dim or sizes[-1]
        self.model = nn.Sequential(*model)
        self.flatten_input = flatten_input

    def forward(self, obs):
        obs = torch.as_tensor(obs, device=self.device, dtype=torch.float32)
        if self.flatten_input:
            obs = obs.flatten(1)
        return self.model(obs)


class Net(nn.Module):
    """common.py:161-285 (no dueling / atoms / concat beyond what PPO uses)."""

    def __init__(self, state_shape, action_shape=0, hidden_sizes: Sequence[int] = (),
                 norm_layer=None, activation=nn.ReLU, device="cpu", softmax: bool = False,
                 concat: bool = False, num_atoms: int = 1, linear_layer=Linear):
        super().__init__()
        self.device = device
        self.softmax = softmax
        self.num_atoms = num_atoms
        input_dim = int(np.prod(state_shape))
        action_dim = int(np.prod(action_shape)) * num_atoms
        if concat:
            input_dim += action_dim
        output_dim = action_dim if not concat else 0
        self.model = MLP(input_dim, output_dim, hidden_sizes, norm_layer, activation, device,
                         linear_layer)
        self.output_dim = self.model.output_dim

    def forward(self, obs, state: Any = None, **kwargs):
        logits = self.model(obs)
        if self.num_atoms > 1:
            logits = logits.view(logits.shape[0], -1, self.num_atoms)
        if self.softmax:
            logits = torch.softmax(logits, dim=-1)
        return logits, state


def _module_device(m: nn.Module):
    try:
        return next(m.parameters()).device
    except StopIteration:
        return None


class _PreprocessWrapper(nn.Module):
    """continuous.py:13-30: the preprocess net is registered under two names."""

    def __init__(self, preprocess_net: nn.Module, device=None):
        super().__init__()
        device = device if device else _module_device(preprocess_net)
        preprocess_net.to(device)
        self.device = device
        self.preprocess_net = preprocess_net
        self.preprocess = preprocess_net


class ActorProb(_PreprocessWrapper):
    """Gaussian actor (continuous.py:153-235).  With ``conditioned_sigma=False`` the log-std
    ``sigma_param`` is state-independent, which is what the fused HIP PPO loss consumes."""

    def __init__(self, preprocess_net, action_shape, hidden_sizes=(), max_action=1.0,
                 device="cpu", unbounded=False, conditioned_sigma=False,
                 preprocess_net_output_dim=None):
        super().__init__(preprocess_net, device=device)
        if unbounded:
            max_action = 1.0
        self.output_dim = int(np.prod(action_shape))
        input_dim = getattr(preprocess_net, "output_dim", preprocess_net_output_dim)
        self.mu = MLP(input_dim, self.output_dim, hidden_sizes, device=self.device)
        self._c_sigma = conditioned_sigma
        if conditioned_sigma:
            self.sigma = MLP(input_dim, self.output_dim, hidden_sizes, device=self.device)
        else:
            self.sigma_param = nn.Parameter(torch.zeros(self.output_dim, 1))
        self.max_action = max_action
        self._unbounded = unbounded

    def forward_mu(self, obs):
        logits, _ = self.preprocess(obs, None)
        mu = self.mu(logits)
        if not self._unbounded:
            mu = self.max_action * torch.tanh(mu)
        return mu

    def forward(self, obs, state=None, info: Dict[str, Any] = {}):
        logits, hidden = self.preprocess(obs, state)
        mu = self.mu(logits)
        if not self._unbounded:
            mu = self.max_action * torch.tanh(mu)
        if self._c_sigma:
            sigma = torch.clamp(self.sigma(logits), min=SIGMA_MIN, max=SIGMA_MAX).exp()
        else:
            shape = [1] * len(mu.shape)
            shape[1] = -1
            sigma = (self.sigma_param.view(shape) + torch.zeros_like(mu)).exp()
        return (mu, sigma), state


class Critic(_PreprocessWrapper):
    """V(s) head (continuous.py:87-150)."""

    def __init__(self, preprocess_net, hidden_sizes=(), device=None,
                 preprocess_net_output_dim=None, linear_layer=Linear, flatten_input=True):
        super().__init__(preprocess_net, device=device)
        self.output_dim = 1
        input_dim = getattr(preprocess_net, "output_dim", preprocess_net_output_dim)
        self.last = MLP(input_dim, 1, hidden_sizes, device=self.device,
                        linear_layer=linear_layer, flatten_input=flatten_input)

    def forward(self, obs, act=None, info: Dict[str, Any] = {}):
        obs = torch.as_tensor(obs, device=self.device, dtype=torch.float32).flatten(1)
        if act is not None:
            act = torch.as_tensor(act, device=self.device, dtype=torch.float32).flatten(1)
            obs = torch.cat([obs, act], dim=1)
        logits, _ = self.preprocess(obs)
        return self.last(logits)


class DiscreteActor(nn.Module):
    """Softmax actor (utils/net/discrete.py:12-71): preprocess -> MLP -> softmax unless
    softmax_output=False.  Module layout (``preprocess``, ``last``) as the reference's, so
    state_dicts interchange."""

    def __init__(self, preprocess_net, action_shape, hidden_sizes=(), softmax_output=True,
                 preprocess_net_output_dim=None, device="cpu"):
        super().__init__()
        self.device = device
        self.preprocess = preprocess_net
        self.output_dim = int(np.prod(action_shape))
        input_dim = getattr(preprocess_net, "output_dim", preprocess_net_output_dim)
        self.last = MLP(input_dim, self.output_dim, hidden_sizes, device=self.device)
        self.softmax_output = softmax_output

    def forward(self, obs, state=None, info: Dict[str, Any] = {}):
        logits, hidden = self.preprocess(obs, state)
        logits = self.last(logits)
        if self.softmax_output:
            logits = torch.softmax(logits, dim=-1)
        return logits, hidden


class DiscreteCritic(nn.Module):
    """V(s) head of discrete-action policies (utils/net/discrete.py:74-121): the observation
    goes to the preprocess net unchanged (a conv trunk sees its frame stack)."""

    def __init__(self, preprocess_net, hidden_sizes=(), last_size: int = 1,
                 preprocess_net_output_dim=None, device="cpu"):
        super().__init__()
        self.device = device
        self.preprocess = preprocess_net
        self.output_dim = last_size
        input_dim = getattr(preprocess_net, "output_dim", preprocess_net_output_dim)
        self.last = MLP(input_dim, last_size, hidden_sizes, device=self.device)

    def forward(self, obs, **kwargs: Any):
        logits, _ = self.preprocess(obs, state=kwargs.get("state", None))
        return self.last(logits)


class ActorCritic(nn.Module):
    """common.py:364-377."""

    def __init__(self, actor: nn.Module, critic: nn.Module) -> None:
        super().__init__()
        self.actor = actor
        self.critic = critic


def build_actor_critic_from_state(state: Dict[str, torch.Tensor], device="cpu"):
    """Rebuild get_actor_critic-shaped (Tanh MLP) actor/critic from a policy state_dict."""
    w0 = state["actor.preprocess_net.model.model.0.weight"]
    hidden = []
    i = 0
    while f"actor.preprocess_net.model.model.{i}.weight" in state:
        hidden.append(state[f"actor.preprocess_net.model.model.{i}.weight"].shape[0])
        i += 2
    obs_dim = w0.shape[1]
    act_dim = state["actor.mu.model.0.weight"].shape[0]
    from tianshou_amd.utils.models import get_actor_critic
    actor, critic = get_actor_critic((obs_dim,), hidden, (act_dim,), device)
    ac = ActorCritic(actor, critic)
    ac.load_state_dict({k: v for k, v in state.items()
                        if k.startswith("actor.") or k.startswith("critic.")}, strict=False)
    return actor.to(device), critic.to(device)
