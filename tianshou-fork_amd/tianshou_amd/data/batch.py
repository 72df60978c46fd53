"""Batch: dict-of-arrays container (tianshou/data/batch.py), restricted to what the on-policy
path uses -- attribute access, fancy indexing (row gathers run through libtsrl on device),
scatter, ``split`` (batch.py:896-912) and conversions.  Values may be HIP tensors or NumPy
arrays; nested dicts become nested Batches.
"""
from typing import Any, Dict, Iterator, Optional, Union

import numpy as np
import torch

from tianshou_amd import _C


def _is_index_array(index) -> bool:
    return isinstance(index, (np.ndarray, list, torch.Tensor))


def gather_rows(t: torch.Tensor, index) -> torch.Tensor:
    """t[index] for a HIP tensor, through tsrl_gather_rows (rows of t.shape[1:])."""
    if not isinstance(index, torch.Tensor):
        index = torch.as_tensor(np.asarray(index, dtype=np.int64), device=t.device)
    elif index.dtype != torch.int64 or index.device != t.device:
        index = index.to(device=t.device, dtype=torch.int64)
    index = index.contiguous()
    k = index.numel()
    out = torch.empty((k,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    if k == 0:
        return out
    row_bytes = t.element_size() * (t[0].numel() if t.dim() > 1 else 1)
    if t.dim() >= 2 and t[0].is_contiguous() and t.stride(0) > t[0].numel():
        # rows of a padded storage (VectorReplayBuffer pads wide f32 observation rows to a
        # 128-byte multiple): gathered in place, no copy of the storage
        _C.check(_C.lib().tsrl_gather_rows_pitched(
            _C.ptr_rows(t), t.stride(0) * t.element_size(), row_bytes, _C.ptr(index), k,
            _C.ptr(out), _C.stream_ptr()), "tsrl_gather_rows")
        return out
    src = t if t.is_contiguous() else t.contiguous()
    _C.check(_C.lib().tsrl_gather_rows(_C.ptr(src), row_bytes, _C.ptr(index), k, _C.ptr(out),
                                       _C.stream_ptr()), "tsrl_gather_rows")
    return out


def _index_value(v, index):
    if isinstance(v, Batch):
        return v[index]
    if isinstance(v, torch.Tensor):
        if _is_index_array(index) and v.device.type == "cuda" and v.dim() >= 1:
            if isinstance(index, torch.Tensor) and index.dtype == torch.bool:
                return v[index.to(v.device)]
            if not isinstance(index, torch.Tensor):
                arr = np.asarray(index)
                if arr.dtype == bool:
                    return v[torch.as_tensor(arr, device=v.device)]
            return gather_rows(v, index)
        if isinstance(index, np.ndarray):
            index = torch.as_tensor(index, device=v.device)
        return v[index]
    if isinstance(v, np.ndarray):
        if isinstance(index, torch.Tensor):
            index = index.cpu().numpy()
        return v[index]
    return v


def _stack_dicts(seq) -> "Batch":
    """Batch.stack of a sequence of dicts (batch.py:_parse_value for a list / object array
    of dicts, e.g. the per-env info dicts a host vector env returns): keys present in every
    dict are stacked."""
    keys = set(seq[0].keys())
    for d in seq[1:]:
        keys &= set(d.keys())
    out = {}
    for k in sorted(keys):
        vals = [d[k] for d in seq]
        if all(isinstance(x, dict) for x in vals):
            out[k] = _stack_dicts(vals)
        else:
            out[k] = np.stack([np.asarray(x) for x in vals])
    return Batch(out)


def _parse(v):
    if isinstance(v, dict):
        return Batch(v)
    if isinstance(v, np.ndarray) and v.dtype == object and v.ndim == 1 and len(v) and \
            all(isinstance(x, dict) for x in v):
        return _stack_dicts(list(v))
    if isinstance(v, (list, tuple)) and len(v) and all(isinstance(x, dict) for x in v):
        return _stack_dicts(list(v))
    if isinstance(v, (list, tuple)) and not isinstance(v, Batch):
        if any(isinstance(x, torch.Tensor) for x in v):
            return v  # e.g. logits=(mu, sigma) of a Gaussian actor
        try:
            return np.asarray(v)
        except ValueError:
            return np.asarray(v, dtype=object)
    return v


class Batch:
    """Minimal tianshou Batch."""

    def __init__(self, batch_dict: Optional[Union[dict, "Batch"]] = None, **kwargs: Any):
        if isinstance(batch_dict, Batch):
            batch_dict = batch_dict.__dict__
        for k, v in {**(batch_dict or {}), **kwargs}.items():
            self.__dict__[k] = _parse(v)

    # -- mapping surface ------------------------------------------------------------------
    def keys(self):
        return self.__dict__.keys()

    def values(self):
        return self.__dict__.values()

    def items(self):
        return self.__dict__.items()

    def get(self, key, default=None):
        return self.__dict__.get(key, default)

    def pop(self, key, default=None):
        return self.__dict__.pop(key, default)

    def __contains__(self, key) -> bool:
        return key in self.__dict__

    def __setattr__(self, key: str, value: Any) -> None:
        self.__dict__[key] = _parse(value)

    def __getitem__(self, index):
        if isinstance(index, str):
            return self.__dict__[index]
        return Batch({k: _index_value(v, index) for k, v in self.__dict__.items()
                      if not (isinstance(v, Batch) and v.is_empty())},
                     **{k: Batch() for k, v in self.__dict__.items()
                        if isinstance(v, Batch) and v.is_empty()})

    def __setitem__(self, index, value) -> None:
        if isinstance(index, str):
            self.__dict__[index] = _parse(value)
            return
        value = value if isinstance(value, Batch) else Batch(value)
        for k, v in value.items():
            dst = self.__dict__.get(k)
            if dst is None:
                continue
            if isinstance(dst, Batch):
                dst[index] = v
            elif isinstance(dst, torch.Tensor):
                idx = index
                if not isinstance(idx, (torch.Tensor, slice, int)):
                    idx = torch.as_tensor(np.asarray(idx), device=dst.device)
                dst[idx] = torch.as_tensor(v, device=dst.device, dtype=dst.dtype)
            else:
                dst[index] = v

    def __len__(self) -> int:
        lens = []
        for v in self.__dict__.values():
            if isinstance(v, Batch):
                if v.is_empty():
                    continue
                lens.append(len(v))
            elif isinstance(v, (np.ndarray, torch.Tensor)) and v.ndim > 0:
                lens.append(v.shape[0])
        if not lens:
            raise TypeError(f"Object {self} has no len()")
        return min(lens)

    def __iter__(self) -> Iterator["Batch"]:
        for i in range(len(self)):
            yield self[i]

    def __repr__(self) -> str:
        inner = ", ".join(f"{k}: {getattr(v, 'shape', v)}" for k, v in self.__dict__.items())
        return f"Batch({inner})"

    def is_empty(self, recurse: bool = False) -> bool:
        if not self.__dict__:
            return True
        if recurse:
            return all(isinstance(v, Batch) and v.is_empty(True) for v in self.__dict__.values())
        return False

    def update(self, batch=None, **kwargs) -> None:
        for k, v in {**(dict(batch.items()) if batch is not None else {}), **kwargs}.items():
            self.__dict__[k] = _parse(v)

    # -- conversions ------------------------------------------------------------------------
    def to_torch(self, dtype=None, device="cpu") -> "Batch":
        for k, v in self.__dict__.items():
            if isinstance(v, Batch):
                v.to_torch(dtype, device)
            elif isinstance(v, (np.ndarray, torch.Tensor)):
                t = torch.as_tensor(v, device=device)
                self.__dict__[k] = t.to(dtype) if dtype is not None else t
        return self

    def to_numpy(self) -> "Batch":
        for k, v in self.__dict__.items():
            if isinstance(v, Batch):
                v.to_numpy()
            elif isinstance(v, torch.Tensor):
                self.__dict__[k] = v.detach().cpu().numpy()
        return self

    # -- minibatches ------------------------------------------------------------------------
    def split(self, size: int, shuffle: bool = True, merge_last: bool = False,
              indices=None) -> Iterator["Batch"]:
        """Batch.split (batch.py:896-912): np.random.permutation order when shuffling, the
        last chunk merged when ``merge_last`` and idx + 2*size >= length."""
        for part in split_indices(len(self), size, shuffle, merge_last, indices):
            yield self[part]


def split_indices(length: int, size: int, shuffle: bool = True, merge_last: bool = False,
                  indices=None):
    """The index arrays Batch.split would use (same RNG consumption: one
    ``np.random.permutation(length)`` call from the global legacy RandomState)."""
    if size == -1:
        size = length
    assert 1 <= size  # size can be greater than length, return whole batch
    if indices is None:
        indices = np.random.permutation(length) if shuffle else np.arange(length)
    merge_last = merge_last and length % size > 0
    parts = []
    for idx in range(0, length, size):
        if merge_last and idx + size + size >= length:
            parts.append(indices[idx:])
            break
        parts.append(indices[idx:idx + size])
    return parts


def to_numpy(x):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    if isinstance(x, Batch):
        return Batch(x).to_numpy()
    return np.asarray(x) if x is not None else np.array(None, dtype=object)


def to_torch(x, dtype=None, device="cpu"):
    if isinstance(x, Batch):
        return Batch(x).to_torch(dtype, device)
    t = torch.as_tensor(x, device=device)
    return t.to(dtype) if dtype is not None else t


def to_torch_as(x, y: torch.Tensor) -> torch.Tensor:
    return to_torch(x, dtype=y.dtype, device=y.device)
