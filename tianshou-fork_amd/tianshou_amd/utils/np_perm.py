"""``np.random.permutation(n)`` of the global legacy RandomState, bit-exact, on the device.

Batch.split (tianshou/data/batch.py:896-912) shuffles every PPO repeat with
``np.random.permutation(length)`` (ppo.py:106-107).  NumPy runs that as one sequential
Fisher-Yates over MT19937 words: 0.2-0.3 s of single-threaded host time at 8.4M indices,
plus a 67 MB host-to-device copy.  Here the work is split (csrc/perm.hip):

* ``tsrl_np_shuffle_draws_mt`` (host C++, no HIP call, releases the GIL through ctypes): the
  MT19937 stream and the masked rejection loop, advancing a copy of the global state that is
  written back with ``np.random.set_state`` -- the global RandomState ends exactly where
  NumPy's own call would leave it.  Sequential below 2^21 elements (~10 ms at 8.4M on the
  MI355X box host); above, host threads (MT19937 jump-ahead + chunk-parallel rejection, exact:
  csrc/np_perm_mt.cpp), ~30 ms instead of 75 ms at 67M -- the global permutation of an 8-rank
  update;
* ``tsrl_shuffle_apply`` (device): the swap sequence resolved in parallel from the draws.

``prefetch(n, count)`` starts a host thread that computes the draws of the next ``count``
permutations while the caller does other work (the collect phase of the next iteration).  A
prefetched permutation is only used if the global state is still the one it was computed
from; otherwise it is discarded and recomputed, so results never depend on timing.
"""
import ctypes
import os
import threading
from typing import List, Optional

import numpy as np
import torch

from tianshou_amd import _C


def _state_key():
    st = np.random.get_state(legacy=True)
    if st[0] != "MT19937":
        raise TypeError(f"global RandomState uses {st[0]}, expected MT19937")
    return st


# host threads for the draws of large permutations (tsrl_np_shuffle_draws_mt; below 2^21
# elements it runs the sequential loop)
THREADS = int(os.environ.get("TSRL_PERM_THREADS", "0")) or min(16, os.cpu_count() or 1)


def _draws(key: np.ndarray, pos: int, n: int, out: np.ndarray):
    """Fill out[:n] with the shuffle draws; return the advanced (key, pos)."""
    key = np.ascontiguousarray(key, dtype=np.uint32).copy()
    cpos = ctypes.c_int32(int(pos))
    _C.check(_C.lib().tsrl_np_shuffle_draws_mt(key.ctypes.data, ctypes.addressof(cpos), int(n),
                                               out.ctypes.data if n > 0 else None, THREADS),
             "tsrl_np_shuffle_draws_mt")
    return key, cpos.value


class _Prefetch:
    def __init__(self, n: int, count: int, key: np.ndarray, pos: int):
        self.n = n
        self.start = (key.copy(), int(pos))
        # pinned host buffers allocated here (caller thread): the worker makes no HIP call
        self.bufs = [torch.empty(max(n, 1), dtype=torch.int32, pin_memory=True)
                     for _ in range(count)]
        self.states: List = [None] * count
        self.ready = [threading.Event() for _ in range(count)]
        self.error: Optional[BaseException] = None
        self.thread = threading.Thread(target=self._run, name="tsrl-np-perm", daemon=True)
        self.thread.start()

    def _run(self):
        try:
            key, pos = self.start
            for i, b in enumerate(self.bufs):
                key, pos = _draws(key, pos, self.n, b.numpy().view(np.uint32))
                self.states[i] = (key, pos)
                self.ready[i].set()
        except BaseException as e:  # surfaced to the consumer
            self.error = e
            for ev in self.ready:
                ev.set()

    def wait(self, i: int):
        """Block until permutation i's draws exist (not the later ones)."""
        self.ready[i].wait()
        if self.error is not None:
            raise self.error

class LegacyPermutation:
    """Callable: ``perm(n, device) -> int64 device tensor`` equal to
    ``np.random.permutation(n)``, consuming the global legacy RandomState identically."""

    def __init__(self):
        self._pf: Optional[_Prefetch] = None
        self._pf_next = 0
        self._ws = {}  # per (device, stream): a workspace is only reused in its stream's order

    # -- device side ----------------------------------------------------------------------
    def _apply(self, host_draws: torch.Tensor, n: int, device) -> torch.Tensor:
        out = torch.empty(n, dtype=torch.int64, device=device)
        if n == 0:
            return out
        L = _C.lib()
        wsb = int(L.tsrl_shuffle_apply_workspace_bytes(n))
        wkey = (out.device, torch.cuda.current_stream(out.device).cuda_stream)
        ws = self._ws.get(wkey)
        if ws is None or ws.numel() < wsb:
            ws = self._ws[wkey] = torch.empty(wsb, dtype=torch.uint8, device=device)
        d = torch.empty(n, dtype=torch.int32, device=device)
        d.copy_(host_draws[:n], non_blocking=host_draws.is_pinned())
        _C.check(L.tsrl_shuffle_apply(_C.ptr(d), n, _C.ptr(out), _C.ptr(ws), wsb,
                                      _C.stream_ptr(out.device)), "tsrl_shuffle_apply")
        return out

    # -- host stream ----------------------------------------------------------------------
    def __call__(self, n: int, device, stream=None) -> torch.Tensor:
        """The permutation as an int64 tensor on ``device``.  With ``stream`` the copy and the
        device resolution are enqueued there (the caller orders its own stream after it and
        owns the tensor's cross-stream lifetime); otherwise on the current stream."""
        st = _state_key()
        pf = self._pf
        if pf is not None and pf.n == n and self._pf_next < len(pf.bufs):
            i = self._pf_next
            pf.wait(i)
            want = pf.start if i == 0 else pf.states[i - 1]
            if int(st[2]) == want[1] and np.array_equal(st[1], want[0]):
                key, pos = pf.states[i]
                np.random.set_state(("MT19937", key, pos, st[3], st[4]))
                self._pf_next += 1
                return self._apply_on(pf.bufs[i], n, device, stream)
        self._drop()
        buf = torch.empty(max(n, 1), dtype=torch.int32, pin_memory=True)
        key, pos = _draws(st[1], st[2], n, buf.numpy().view(np.uint32))
        np.random.set_state(("MT19937", key, pos, st[3], st[4]))
        return self._apply_on(buf, n, device, stream)

    def _apply_on(self, buf, n, device, stream):
        if stream is None:
            return self._apply(buf, n, device)
        with torch.cuda.stream(stream):
            return self._apply(buf, n, device)

    def next_ready(self, n: int) -> bool:
        """True if the next call with size ``n`` would not wait for host draws."""
        pf = self._pf
        if pf is None or pf.n != n or self._pf_next >= len(pf.bufs):
            return False
        return pf.ready[self._pf_next].is_set()

    def prefetch(self, n: int, count: int) -> None:
        """Start computing the draws of the next ``count`` permutations of size ``n`` from
        the current global state, in a background host thread."""
        self._drop()
        if count <= 0 or n <= 1:
            return
        st = _state_key()
        self._pf = _Prefetch(n, count, np.asarray(st[1]), int(st[2]))
        self._pf_next = 0

    def _drop(self):
        if self._pf is not None:
            self._pf.thread.join()
        self._pf = None
        self._pf_next = 0


_GLOBAL = LegacyPermutation()


def np_permutation(n: int, device) -> torch.Tensor:
    """Module-level convenience over one shared LegacyPermutation."""
    return _GLOBAL(n, device)
