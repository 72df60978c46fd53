"""SegmentTree (tianshou/data/utils/segtree.py:7-137) resident in HBM.

The f64 sum tree lives in one device tensor (binary heap of 2 * bound nodes, leaves at
[bound, bound + size)); its three numba kernels are HIP kernels (csrc/replay.hip):
``tsrl_segtree_set`` (leaves, last duplicate wins, then every ancestor = left + right),
``tsrl_segtree_reduce`` (the reference's summation order) and ``tsrl_segtree_prefix_idx``.

The public methods keep the reference's host-facing contract (NumPy in, NumPy / float out,
the same assertions).  The ``*_dev`` methods take and return device tensors without any
host synchronisation; the prioritized buffers use those.
"""
from typing import Optional, Union

import numpy as np
import torch

from tianshou_amd import _C


def _default_device():
    return torch.device("cuda", torch.cuda.current_device())


class SegmentTree:
    def __init__(self, size: int, device=None) -> None:
        bound = 1
        while bound < size:
            bound *= 2
        self._size = int(size)
        self._bound = bound
        self.device = torch.device(device) if device is not None else _default_device()
        self._value = torch.zeros(2 * bound, dtype=torch.float64, device=self.device)
        # leaf -> winning position scratch of tsrl_segtree_set (kept all -1 between calls)
        self._win = torch.full((max(self._size, 1),), -1, dtype=torch.int32, device=self.device)

    def __len__(self) -> int:
        return self._size

    # -- host API (segtree.py:33-85) ------------------------------------------------------------
    def _node_index(self, index):
        """index + bound with NumPy's range rules on the 2*bound node array."""
        j = np.asarray(index, dtype=np.int64) + self._bound
        n = 2 * self._bound
        if np.any(j >= n) or np.any(j < -n):
            raise IndexError(f"index out of bounds for a tree of {n} nodes")
        return j % n

    def __getitem__(self, index: Union[int, np.ndarray]) -> Union[float, np.ndarray]:
        j = self._node_index(index)
        vals = self._value[torch.as_tensor(j.reshape(-1), device=self.device)].cpu().numpy()
        return vals.reshape(j.shape) if j.ndim else vals[0]

    def __setitem__(self, index: Union[int, np.ndarray], value: Union[float, np.ndarray]) -> None:
        if isinstance(index, (int, np.integer)):
            index, value = np.array([index]), np.array([value])
        index = np.asarray(index, dtype=np.int64).reshape(-1)
        assert np.all(0 <= index) and np.all(index < self._size)
        value = np.array(np.broadcast_to(np.asarray(value, dtype=np.float64), index.shape))
        self.set_dev(torch.as_tensor(index, device=self.device),
                     torch.as_tensor(value, device=self.device))

    def reduce(self, start: int = 0, end: Optional[int] = None) -> float:
        """Sum of value[start:end] (segtree.py:56-64)."""
        if start == 0 and end is None:
            return float(self._value[1].item())
        return float(self.reduce_dev(start, end).item())

    def get_prefix_sum_idx(self, value: Union[float, np.ndarray]) -> Union[int, np.ndarray]:
        """Minimum index i with value <= sum(arr[:i+1]) (segtree.py:66-85)."""
        total = float(self._value[1].item())
        assert np.all(np.asarray(value) >= 0.0) and np.all(np.asarray(value) < total)
        single = not isinstance(value, np.ndarray)
        arr = np.array([value]) if single else value
        if arr.dtype not in (np.float32, np.float64):
            arr = arr.astype(np.float64)
        out = self.prefix_dev(torch.as_tensor(np.ascontiguousarray(arr).reshape(-1),
                                              device=self.device)).cpu().numpy()
        return int(out[0]) if single else out.reshape(arr.shape)

    # -- device API ---------------------------------------------------------------------------
    def set_dev(self, idx: torch.Tensor, values: torch.Tensor) -> None:
        """tree[idx] = values (values: [k] f64, or one f64 element broadcast), then the
        ancestors; ``idx`` must lie in [0, size) (not checked on device)."""
        idx = idx.reshape(-1).to(device=self.device, dtype=torch.int64).contiguous()
        values = values.reshape(-1).to(device=self.device, dtype=torch.float64).contiguous()
        k = idx.numel()
        if k == 0:
            return
        stride = 1 if values.numel() == k else 0
        assert stride == 1 or values.numel() == 1
        _C.check(_C.lib().tsrl_segtree_set(
            _C.ptr(self._value), self._bound, _C.ptr(idx), _C.ptr(values), stride, k,
            _C.ptr(self._win), _C.stream_ptr(self.device)), "tsrl_segtree_set")

    def get_dev(self, idx: torch.Tensor) -> torch.Tensor:
        return self._value[idx.reshape(-1).to(self.device) + self._bound]

    def reduce_dev(self, start: int = 0, end: Optional[int] = None) -> torch.Tensor:
        """0-dim device f64 tensor of the reference's _reduce (root for the whole range)."""
        if start == 0 and end is None:
            return self._value[1]
        if end is None:
            end = self._size
        if end < 0:
            end += self._size
        out = torch.empty((), dtype=torch.float64, device=self.device)
        _C.check(_C.lib().tsrl_segtree_reduce(_C.ptr(self._value), self._bound, int(start),
                                              int(end), _C.ptr(out), _C.stream_ptr(self.device)),
                 "tsrl_segtree_reduce")
        return out

    def prefix_dev(self, values: torch.Tensor) -> torch.Tensor:
        """Device int64 indices of _get_prefix_sum_idx for f64 / f32 device values."""
        values = values.reshape(-1).to(self.device).contiguous()
        if values.dtype not in (torch.float32, torch.float64):
            values = values.to(torch.float64)
        out = torch.empty(values.numel(), dtype=torch.int64, device=self.device)
        _C.check(_C.lib().tsrl_segtree_prefix_idx(
            _C.ptr(self._value), self._bound, _C.ptr(values),
            int(values.dtype == torch.float64), values.numel(), _C.ptr(out),
            _C.stream_ptr(self.device)), "tsrl_segtree_prefix_idx")
        return out
