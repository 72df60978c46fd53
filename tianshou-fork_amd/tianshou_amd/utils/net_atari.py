"""Atari network of the reference's PPO example (examples/atari/atari_network.py:10-80):
the Nature-DQN conv trunk over a uint8 4x84x84 frame stack scaled by 1/255
(``scale_obs``, :18-30) with orthogonal ``layer_init`` (:10-15), used as the shared
``features_only`` trunk of the actor and critic (examples/atari/atari_ppo.py:104-125).

The convolutions and the two linear layers run on MIOpen / hipBLASLt through PyTorch-ROCm
(the conv trunk is MFMA-bound library work); the PPO loss around it is the
fused tsrl_ppo_cat kernel (policy/ppo.py).  The conv weights and the scaled input are kept
channels_last (NHWC): MIOpen's NHWC f32 kernels measured 7.1 vs 8.8 ms per 8192-row
minibatch forward+backward on MI355X (tools/atari_trunk_bench.py); values are the same
function of the same weights (summation order only), and state_dict() holds the same
tensors."""
from typing import Any, Dict, Optional, Sequence

import numpy as np
import torch
from torch import nn

from tianshou_amd import _C
from tianshou_amd.utils.net import sum_rows


def frames_to_f32_nhwc(obs: torch.Tensor, lut: torch.Tensor) -> torch.Tensor:
    """uint8 [n, c, h, w] frame stacks -> f32 [n, c, h, w] in channels_last memory, each byte
    mapped through ``lut`` (tsrl_frames_to_f32_nhwc: one HBM pass instead of torch's layout
    copy + dtype conversion + division)."""
    assert obs.dtype == torch.uint8 and obs.dim() == 4 and obs.is_cuda
    obs = obs.contiguous()
    n, c, h, w = obs.shape
    out = torch.empty((n, h, w, c), dtype=torch.float32, device=obs.device)
    _C.check(_C.lib().tsrl_frames_to_f32_nhwc(_C.ptr(obs), n, c, h * w, _C.ptr(lut),
                                              _C.ptr(out), _C.stream_ptr(obs.device)),
             "tsrl_frames_to_f32_nhwc")
    return out.permute(0, 3, 1, 2)


def _gather(t: torch.Tensor, rows: torch.Tensor) -> torch.Tensor:
    from tianshou_amd.data.batch import gather_rows
    return gather_rows(t, rows)


def conv1_u8(obs: torch.Tensor, conv: nn.Conv2d, scale: float,
             rows: Optional[torch.Tensor] = None) -> torch.Tensor:
    """relu(conv(obs / scale)) of the trunk's first layer straight from uint8 frame stacks
    [n, 4, 84, 84] (tsrl_dqn_conv1_fwd: bytes as exact bf16 operands, the weight split into
    three bf16 planes; f32 GEMM error).  Returns [n, 32, 20, 20] in channels_last memory.
    rows (int64, on the device): the output rows are obs[rows], read in place."""
    obs = obs.contiguous()
    if rows is not None:
        rows = rows.to(torch.int64).contiguous()
    n = obs.shape[0] if rows is None else rows.numel()
    w = conv.weight.detach()
    if not (w.is_cuda and w.dtype == torch.float32 and w.device == obs.device):
        raise _C.TsrlError("conv1_u8: the conv weight must be an f32 tensor on the frames' "
                           "device")
    out = torch.empty((n, 20, 20, 32), dtype=torch.float32, device=obs.device)
    b = conv.bias.detach() if conv.bias is not None else None
    # the weight is addressed through its strides (channels_last needs no copy)
    _C.check(_C.lib().tsrl_dqn_conv1_fwd(_C.ptr(obs), n, _C.ptr(rows) if rows is not None
                                         else None, w.data_ptr(), *w.stride(),
                                         _C.ptr(b) if b is not None else None, float(scale), 1,
                                         _C.ptr(out), _C.stream_ptr(obs.device)),
             "tsrl_dqn_conv1_fwd")
    return out.permute(0, 3, 1, 2)


# conv1's weight/bias gradient from the uint8 frames (tsrl_dqn_conv1_wgrad); False: MIOpen over
# the scaled f32 frames (tsrl_frames_to_f32_nhwc)
CONV1_WGRAD_U8 = True


def conv1_u8_wgrad(obs: torch.Tensor, gy_nhwc: torch.Tensor, weight: torch.Tensor,
                   scale: float, bias: bool, rows: Optional[torch.Tensor] = None):
    """(dW1, db1 or None) of relu-masked gradient rows gy [n, 20, 20, 32] (NHWC) w.r.t.
    conv(obs / scale, W1) + b1, straight from the uint8 frames (tsrl_dqn_conv1_wgrad); with
    rows, gradient row s belongs to frame stack obs[rows[s]]."""
    if rows is not None:
        rows = rows.to(torch.int64).contiguous()
    n = obs.shape[0] if rows is None else rows.numel()
    dev = obs.device
    lib = _C.lib()
    gw = torch.empty((32, 4, 8, 8), dtype=torch.float32, device=dev)
    gb = torch.empty(32, dtype=torch.float32, device=dev) if bias else None
    ws = torch.empty(max(1, (int(lib.tsrl_dqn_conv1_wgrad_workspace_bytes(n)) + 3) // 4),
                     dtype=torch.float32, device=dev)
    gy_nhwc = gy_nhwc.contiguous()
    _C.check(lib.tsrl_dqn_conv1_wgrad(_C.ptr(obs.contiguous()), n,
                                      _C.ptr(rows) if rows is not None else None,
                                      _C.ptr(gy_nhwc), float(scale),
                                      _C.ptr(gw), _C.ptr(gb) if gb is not None else None,
                                      _C.ptr(ws), ws.numel() * 4, _C.stream_ptr(dev)),
             "tsrl_dqn_conv1_wgrad")
    if weight.is_contiguous(memory_format=torch.channels_last) and not weight.is_contiguous():
        gw = gw.contiguous(memory_format=torch.channels_last)
    return gw, gb


class _Conv1U8(torch.autograd.Function):
    """conv1 + ReLU from uint8 frames (forward: tsrl_dqn_conv1_fwd).  Backward: the ReLU
    mask, then the weight and bias gradients straight from the frames (tsrl_dqn_conv1_wgrad;
    with CONV1_WGRAD_U8 off, MIOpen over the scaled f32 frames of tsrl_frames_to_f32_nhwc);
    the frames themselves need no gradient."""

    @staticmethod
    def forward(ctx, obs, rows, weight, bias, conv, lut, scale):
        z = conv1_u8(obs, conv, scale, rows)
        ctx.save_for_backward(obs, rows, weight, z)
        ctx.lut = lut
        ctx.scale = scale
        ctx.has_bias = bias is not None
        return z

    @staticmethod
    def backward(ctx, gz):
        obs, rows, weight, z = ctx.saved_tensors
        gy = torch.ops.aten.threshold_backward(gz, z, 0.0)
        if CONV1_WGRAD_U8:
            gw, gb = conv1_u8_wgrad(obs, _nhwc(gy), weight, ctx.scale, ctx.has_bias, rows)
            return None, None, gw, gb, None, None, None
        x = frames_to_f32_nhwc(obs if rows is None else _gather(obs, rows), ctx.lut)
        _, gw, gb = torch.ops.aten.convolution_backward(
            gy, x, weight, [weight.shape[0]] if ctx.has_bias else None, (4, 4), (0, 0), (1, 1),
            False, (0, 0), 1, (False, True, ctx.has_bias))
        return None, None, gw, gb, None, None, None


def bias_relu_(y: torch.Tensor, bias: Optional[torch.Tensor]) -> torch.Tensor:
    """relu(y + bias) in place for a channels_last [n, C, h, w] f32 activation on the GPU
    (tsrl_bias_relu_rows: one pass); other tensors take torch's add + relu."""
    n, C = y.shape[0], y.shape[1]
    if (y.is_cuda and y.dtype == torch.float32 and C % 4 == 0 and y.dim() == 4 and
            y.is_contiguous(memory_format=torch.channels_last) and y.data_ptr() % 16 == 0 and
            (bias is None or (bias.is_contiguous() and bias.data_ptr() % 16 == 0))):
        _C.check(_C.lib().tsrl_bias_relu_rows(
            y.data_ptr(), bias.data_ptr() if bias is not None else None,
            n * y.shape[2] * y.shape[3], C, _C.stream_ptr(y.device)), "tsrl_bias_relu_rows")
        return y
    if bias is not None:
        y = y.add_(bias.view(1, -1, 1, 1))
    return torch.relu_(y)


RELU_BWD_FUSED = True


def relu_bwd_bias(gz: torch.Tensor, z: torch.Tensor, want_bias: bool):
    """(gy, gb): gy = (z > 0) * gz and, when want_bias, gb = gy summed over (n, h, w), in one
    pass over channels_last f32 [n, C, h, w] activations on the GPU (tsrl_relu_bwd_rows; f64
    fold of per-workgroup partials).  Other tensors take threshold_backward and return
    gb = None, leaving the bias gradient to convolution_backward."""
    C = z.shape[1] if z.dim() == 4 else 0
    c4 = C // 4
    cl = torch.channels_last
    if (RELU_BWD_FUSED and z.is_cuda and z.dtype == torch.float32 and gz.dtype == torch.float32
            and z.dim() == 4 and gz.shape == z.shape and C % 4 == 0 and 0 < C <= 1024 and
            (c4 & (c4 - 1)) == 0 and z.is_contiguous(memory_format=cl) and
            gz.is_contiguous(memory_format=cl) and z.data_ptr() % 16 == 0 and
            gz.data_ptr() % 16 == 0):
        rows = z.shape[0] * z.shape[2] * z.shape[3]
        gy = torch.empty_like(z, memory_format=cl)
        gb = ws = None
        nb = 0
        if want_bias:
            gb = torch.empty(C, dtype=torch.float32, device=z.device)
            nb = int(_C.lib().tsrl_relu_bwd_rows_workspace_bytes(rows, C))
            ws = torch.empty(max(nb, 16), dtype=torch.uint8, device=z.device)
        _C.check(_C.lib().tsrl_relu_bwd_rows(
            gz.data_ptr(), z.data_ptr(), gy.data_ptr(), rows, C,
            gb.data_ptr() if gb is not None else None, ws.data_ptr() if ws is not None else None,
            nb, _C.stream_ptr(z.device)), "tsrl_relu_bwd_rows")
        return gy, gb
    return torch.ops.aten.threshold_backward(gz, z, 0.0), None


class _ConvBiasReLU(torch.autograd.Function):
    """Conv2d + ReLU with the bias add and the ReLU as one pass (bias_relu_) after the library
    convolution run without bias.  Backward: the ReLU mask, then the library's data / weight /
    bias gradients (the same calls as autograd of Conv2d + ReLU)."""

    @staticmethod
    def forward(ctx, x, weight, bias, conv):
        z = bias_relu_(torch.nn.functional.conv2d(x, weight, None, conv.stride, conv.padding,
                                                  conv.dilation, conv.groups), bias)
        ctx.save_for_backward(x, weight, z)
        ctx.conv = conv
        ctx.has_bias = bias is not None
        return z

    @staticmethod
    def backward(ctx, gz):
        x, weight, z = ctx.saved_tensors
        cv = ctx.conv
        gy, gb = relu_bwd_bias(gz, z, ctx.has_bias)
        lib_bias = ctx.has_bias and gb is None
        gx, gw, gb2 = torch.ops.aten.convolution_backward(
            gy, x, weight, [weight.shape[0]] if lib_bias else None, cv.stride, cv.padding,
            cv.dilation, False, (0, 0), cv.groups,
            (ctx.needs_input_grad[0], True, lib_bias))
        return gx, gw, gb if gb is not None else gb2, None


class _FlattenLinear(torch.autograd.Function):
    """Flatten + Linear over a channels_last [n, C, h, w] activation without the NCHW copy that
    Flatten needs: the Linear runs on the NHWC rows (a view) against its weight with the input
    features permuted to (h, w, C) order -- the same products, summed in another order -- and
    the input gradient comes back as a channels_last view.  Backward: the bias gradient is one
    HIP column sum (tsrl_sum_rows_f32; torch's reduction took 23 us per 8192 rows), and the
    (h, w, C)-ordered weight gradient goes straight into an existing ``weight.grad`` (added)
    or into the flat-bucket slot FlatAdam.release_grads() published (written, and made the
    .grad) through a permuted view -- one strided pass instead of the (C, h, w) reshape copy
    plus autograd's accumulation or hand-over copy (round 6) -- when the weight has no
    gradient hooks."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        n, C, H, W = x.shape
        O = weight.shape[0]
        xf = x.permute(0, 2, 3, 1).reshape(n, H * W * C)
        wp = weight.view(O, C, H, W).permute(0, 2, 3, 1).reshape(O, H * W * C)
        ctx.save_for_backward(xf, wp)
        ctx.weight = weight
        ctx.shape = (n, C, H, W)
        ctx.has_bias = bias is not None
        return torch.nn.functional.linear(xf, wp, bias)

    @staticmethod
    def _grad_slot(weight: torch.Tensor, O: int, C: int, H: int, W: int):
        """(g, fresh): the gradient tensor the weight gradient may be written into directly
        (a plain dense .grad, no hooks on the weight) and whether it is to be overwritten --
        the flat-bucket slot FlatAdam.release_grads() published while .grad is None -- rather
        than accumulated into; (None, False) when autograd must take it."""
        g, fresh = weight.grad, False
        if g is None:
            g, fresh = getattr(weight, "_tsrl_flat_slot", None), True
        if (g is None or g.requires_grad or not g.is_cuda or g.dtype != weight.dtype or
                g.shape != weight.shape or not g.is_contiguous() or weight._backward_hooks or
                getattr(weight, "_post_accumulate_grad_hooks", None)):
            return None, False
        return g, fresh

    @staticmethod
    def backward(ctx, gy):
        xf, wp = ctx.saved_tensors
        n, C, H, W = ctx.shape
        O = wp.shape[0]
        gx = (gy @ wp).view(n, H, W, C).permute(0, 3, 1, 2) if ctx.needs_input_grad[0] else None
        gw = gb = None
        if torch.is_grad_enabled():
            # double backward: differentiable torch ops only
            if ctx.needs_input_grad[1]:
                gw = (gy.t() @ xf).view(O, H, W, C).permute(0, 3, 1, 2).reshape(O, C * H * W)
            if ctx.has_bias and ctx.needs_input_grad[2]:
                gb = gy.sum(0)
            return gx, gw, gb
        if ctx.needs_input_grad[1]:
            g_hwc = gy.t() @ xf
            g, fresh = _FlattenLinear._grad_slot(ctx.weight, O, C, H, W)
            if g is None:
                gw = g_hwc.view(O, H, W, C).permute(0, 3, 1, 2).reshape(O, C * H * W)
            else:
                slot = g.view(O, C, H, W).permute(0, 2, 3, 1)
                if fresh:
                    slot.copy_(g_hwc.view(O, H, W, C))
                    ctx.weight.grad = g  # the slot now holds this backward's gradient
                else:
                    slot.add_(g_hwc.view(O, H, W, C))
        if ctx.has_bias and ctx.needs_input_grad[2]:
            gb = sum_rows(gy) if gy.is_cuda else gy.sum(0)
        return gx, gw, gb


def _run_rest(rest: nn.Module, h: torch.Tensor) -> torch.Tensor:
    """The layers after the fused first block; a leading zero-padding Conv2d + ReLU pair runs
    as _ConvBiasReLU."""
    if (len(rest) >= 2 and isinstance(rest[0], nn.Conv2d) and isinstance(rest[1], nn.ReLU) and
            rest[0].padding_mode == "zeros" and isinstance(rest[0].padding, tuple) and
            h.is_cuda):
        cv = rest[0]
        h = _ConvBiasReLU.apply(h, cv.weight, cv.bias, cv)
        return rest[2:](h)
    return rest(h)


def _nhwc(t: torch.Tensor) -> torch.Tensor:
    """The [n, h, w, c] contiguous tensor behind an [n, c, h, w] channels_last tensor (a copy
    only when it is not channels_last)."""
    return t.permute(0, 2, 3, 1).contiguous()


class _Conv12U8(torch.autograd.Function):
    """conv1 + ReLU + conv2 + ReLU from uint8 frames.  Forward: tsrl_dqn_conv1_fwd, MIOpen
    conv2, ReLU.  Backward: ReLU mask of conv2, MIOpen weight/bias gradient of conv2, the
    conv2 data gradient with conv1's ReLU mask fused (tsrl_dqn_conv2_dgrad), then conv1's
    weight/bias gradient straight from the frames (tsrl_dqn_conv1_wgrad)."""

    @staticmethod
    def forward(ctx, obs, rows, w1, b1, w2, b2, conv1, conv2, lut, scale):
        z1 = conv1_u8(obs, conv1, scale, rows)
        z2 = bias_relu_(torch.nn.functional.conv2d(z1, w2, None, conv2.stride), b2)
        ctx.save_for_backward(obs, rows, w1, w2, z1, z2)
        ctx.lut = lut
        ctx.scale = scale
        ctx.bias = (b1 is not None, b2 is not None)
        return z2

    @staticmethod
    def backward(ctx, gz2):
        obs, rows, w1, w2, z1, z2 = ctx.saved_tensors
        n = z1.shape[0]
        gy2, gb2 = relu_bwd_bias(gz2, z2, ctx.bias[1])
        gy2 = gy2.contiguous(memory_format=torch.channels_last)
        lib_bias = ctx.bias[1] and gb2 is None
        _, gw2, gb2_ = torch.ops.aten.convolution_backward(
            gy2, z1, w2, [w2.shape[0]] if lib_bias else None, (2, 2), (0, 0), (1, 1), False,
            (0, 0), 1, (False, True, lib_bias))
        if gb2 is None:
            gb2 = gb2_
        gy1 = torch.empty((n, 20, 20, 32), dtype=torch.float32, device=obs.device)
        g2 = _nhwc(gy2)
        _C.check(_C.lib().tsrl_dqn_conv2_dgrad(_C.ptr(g2), n, w2.data_ptr(), *w2.stride(),
                                               _C.ptr(_nhwc(z1)), _C.ptr(gy1),
                                               _C.stream_ptr(obs.device)),
                 "tsrl_dqn_conv2_dgrad")
        if CONV1_WGRAD_U8:
            gw1, gb1 = conv1_u8_wgrad(obs, gy1, w1, ctx.scale, ctx.bias[0], rows)
        else:
            x = frames_to_f32_nhwc(obs if rows is None else _gather(obs, rows), ctx.lut)
            _, gw1, gb1 = torch.ops.aten.convolution_backward(
                gy1.permute(0, 3, 1, 2), x, w1, [w1.shape[0]] if ctx.bias[0] else None, (4, 4),
                (0, 0), (1, 1), False, (0, 0), 1, (False, True, ctx.bias[0]))
        return None, None, gw1, gb1, gw2, gb2, None, None, None, None


def layer_init(layer: nn.Module, std: float = np.sqrt(2), bias_const: float = 0.0):
    torch.nn.init.orthogonal_(layer.weight, std)
    torch.nn.init.constant_(layer.bias, bias_const)
    return layer


class DQN(nn.Module):
    """Conv(c,32,8,4)-ReLU-Conv(32,64,4,2)-ReLU-Conv(64,64,3,1)-ReLU-Flatten, then either the
    Q head (Linear 512 - ReLU - Linear A) or, with ``features_only``, an optional
    Linear(., output_dim)-ReLU projection."""

    def __init__(self, c: int, h: int, w: int, action_shape: Sequence[int], device="cpu",
                 features_only: bool = False, output_dim: Optional[int] = None,
                 layer_init=lambda x: x, scale: float = 255.0,
                 channels_last: bool = True) -> None:
        super().__init__()
        self.device = device
        self.scale = scale
        self.net = nn.Sequential(
            layer_init(nn.Conv2d(c, 32, kernel_size=8, stride=4)), nn.ReLU(inplace=True),
            layer_init(nn.Conv2d(32, 64, kernel_size=4, stride=2)), nn.ReLU(inplace=True),
            layer_init(nn.Conv2d(64, 64, kernel_size=3, stride=1)), nn.ReLU(inplace=True),
            nn.Flatten())
        with torch.no_grad():
            self.output_dim = int(np.prod(self.net(torch.zeros(1, c, h, w)).shape[1:]))
        if not features_only:
            self.net = nn.Sequential(self.net, layer_init(nn.Linear(self.output_dim, 512)),
                                     nn.ReLU(inplace=True),
                                     layer_init(nn.Linear(512, int(np.prod(action_shape)))))
            self.output_dim = int(np.prod(action_shape))
        elif output_dim is not None:
            self.net = nn.Sequential(self.net, layer_init(nn.Linear(self.output_dim, output_dim)),
                                     nn.ReLU(inplace=True))
            self.output_dim = output_dim
        self.channels_last = channels_last
        if channels_last:
            self.net.to(memory_format=torch.channels_last)
        # uint8 frame stacks on the GPU enter through the hand-written first layer
        # (conv1_u8); False keeps MIOpen for it
        self.fused_conv1 = True
        self._conv1_split = None

    def _scale_lut(self, dev) -> torch.Tensor:
        """The 256 scaled byte values, divided on the host: f32 division there is
        bit-identical to scale_obs's f64 division + f32 cast for every byte (torch's GPU
        division by a scalar multiplies by the reciprocal instead, which is not)."""
        key = (str(dev), float(self.scale))
        lut = getattr(self, "_lut", None)
        if lut is None or lut[0] != key:
            t = (torch.arange(256, dtype=torch.uint8) / self.scale).to(torch.float32)
            self._lut = lut = (key, t.to(dev).contiguous())
        return lut[1]

    def _conv1_parts(self):
        """(conv1, conv2 or None, rest of the conv stack, outer layers after it) when the
        trunk starts with Conv2d(4, 32, 8, stride 4) + ReLU over 84x84 frames (conv2 when it
        is followed by the Nature-DQN Conv2d(32, 64, 4, stride 2) + ReLU), else None."""
        if self._conv1_split is None:
            outer = None
            seq = self.net
            if len(seq) and isinstance(seq[0], nn.Sequential):
                outer, seq = self.net, self.net[0]
            conv = seq[0] if len(seq) > 1 else None
            ok = isinstance(conv, nn.Conv2d) and isinstance(seq[1], nn.ReLU) and \
                conv.in_channels == 4 and conv.out_channels == 32 and \
                conv.kernel_size == (8, 8) and conv.stride == (4, 4) and \
                conv.padding == (0, 0) and conv.dilation == (1, 1) and conv.groups == 1 and \
                conv.padding_mode == "zeros"
            conv2 = seq[2] if ok and len(seq) > 3 else None
            ok2 = isinstance(conv2, nn.Conv2d) and isinstance(seq[3], nn.ReLU) and \
                conv2.in_channels == 32 and conv2.out_channels == 64 and \
                conv2.kernel_size == (4, 4) and conv2.stride == (2, 2) and \
                conv2.padding == (0, 0) and conv2.dilation == (1, 1) and \
                conv2.groups == 1 and conv2.padding_mode == "zeros"
            self._conv1_split = (conv, conv2 if ok2 else None, seq[4:] if ok2 else seq[2:],
                                 outer[1:] if outer is not None else None) if ok else False
        return self._conv1_split or None

    def reads_rows(self, obs) -> bool:
        """Whether forward(obs, rows=...) reads obs[rows] in place (the uint8 first-layer
        path on a contiguous frame-stack batch) instead of needing the rows gathered."""
        return (self.fused_conv1 and self._conv1_parts() is not None and
                isinstance(obs, torch.Tensor) and obs.dim() == 4 and
                obs.dtype == torch.uint8 and obs.is_cuda and obs.is_contiguous() and
                tuple(obs.shape[1:]) == (4, 84, 84) and bool(self.scale) and
                obs.data_ptr() % 4 == 0)

    def forward(self, obs, state: Any = None, info: Dict[str, Any] = {},
                rows: Optional[torch.Tensor] = None):
        """atari_network.py:84-90.  rows (int64 device indices, this repo's extension):
        the output rows are those of obs[rows]; the uint8 first-layer kernels read them in
        place (round 6: no gathered copy of the minibatch's frame stacks), any other path
        gathers them first."""
        obs = torch.as_tensor(obs, device=self.device)
        if rows is not None and not self.reads_rows(obs):
            obs, rows = _gather(obs, rows), None
        parts = self._conv1_parts() if self.fused_conv1 else None
        if parts is not None and obs.dim() == 4 and obs.dtype == torch.uint8 and obs.is_cuda \
                and tuple(obs.shape[1:]) == (4, 84, 84) and self.scale and \
                obs.data_ptr() % 4 == 0:
            conv, conv2, rest, outer = parts
            lut = self._scale_lut(obs.device)
            if conv2 is not None:
                h = _Conv12U8.apply(obs.contiguous(), rows, conv.weight, conv.bias, conv2.weight,
                                    conv2.bias, conv, conv2, lut, float(self.scale))
            else:
                h = _Conv1U8.apply(obs.contiguous(), rows, conv.weight, conv.bias, conv, lut,
                                   float(self.scale))
            if (outer is not None and len(rest) and isinstance(rest[-1], nn.Flatten) and
                    rest[-1].start_dim == 1 and rest[-1].end_dim == -1 and len(outer) and
                    isinstance(outer[0], nn.Linear)):
                h = _run_rest(rest[:-1], h)
                if h.dim() == 4 and h.is_contiguous(memory_format=torch.channels_last):
                    h = _FlattenLinear.apply(h, outer[0].weight, outer[0].bias)
                else:
                    h = outer[0](h.flatten(1))
                return outer[1:](h), state
            h = _run_rest(rest, h)
            return (outer(h) if outer is not None else h), state
        if self.channels_last and obs.dim() == 4 and obs.dtype == torch.uint8 and \
                obs.is_cuda and self.scale:
            return self.net(frames_to_f32_nhwc(obs, self._scale_lut(obs.device))), state
        if self.channels_last and obs.dim() == 4:
            obs = obs.contiguous(memory_format=torch.channels_last)  # 1-byte frames
        # scale_obs (atari_network.py:18-30) divides the frames in f64 and the trunk casts to
        # f32 (:84): uint8 frames go through the same host-divided table as the NHWC path (a
        # GPU division by the scalar multiplies by its reciprocal, which is not bit-identical),
        # so the memory layout is the only difference between the two paths
        if obs.dtype == torch.uint8 and self.scale:
            x = self._scale_lut(obs.device)[obs.long()]
        else:
            x = (obs / self.scale).to(torch.float32) if self.scale else obs.to(torch.float32)
        return self.net(x), state
