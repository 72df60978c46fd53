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

    def forward(self, obs, state: Any = None, info: Dict[str, Any] = {}):
        obs = torch.as_tensor(obs, device=self.device)
        if self.channels_last and obs.dim() == 4 and obs.dtype == torch.uint8 and \
                obs.is_cuda and self.scale:
            return self.net(frames_to_f32_nhwc(obs, self._scale_lut(obs.device))), state
        if self.channels_last and obs.dim() == 4:
            obs = obs.contiguous(memory_format=torch.channels_last)  # 1-byte frames
        # scale_obs (atari_network.py:18-30) divides the frames in f64 and the trunk casts to
        # f32 (:84); other inputs (host tensors, non-u8 frames) take torch's division
        x = (obs / self.scale).to(torch.float32) if self.scale else obs.to(torch.float32)
        return self.net(x), state
