"""Env-sharded data parallelism over torch.distributed (backend "nccl" = RCCL on ROCm).

Each rank owns a disjoint shard of the vector envs (weak scaling: per-GPU work fixed).
Rollout collection and GAE are rank-local (episode segments never cross ranks, SURVEY.md
§8e).  The exchanges are the reference semantics of ONE global minibatch made of every
rank's local minibatch: advantage moments (sum, sum of squares), the loss partial sums,
the flattened gradients (one all-reduce per minibatch), the obs_rms batch moments per env
step, and the ret_rms partials per update.
"""
from collections import defaultdict
from typing import Dict, Iterable, Optional

import torch
import torch.distributed as dist


class CollectiveLog:
    """What the data-parallel path exchanged, by kind ("obs_rms", "grad", "adv_moments",
    "loss_sums", "ret_rms", "perm_check", "param_broadcast", ...): logical call counts --
    a collective captured into a HIP graph counts once per REPLAY of that graph, not at
    capture -- and the payload (elements, dtype, bytes) of the last call.  bench.py reports
    it per iteration at N > 1 and times each kind at its payload (``probe_collectives``)."""

    def __init__(self) -> None:
        self.calls: Dict[str, int] = defaultdict(int)
        self.payload: Dict[str, tuple] = {}
        self._capture: Optional[Dict[str, int]] = None

    def note(self, kind: str, t: torch.Tensor, op: str) -> None:
        self.payload[kind] = (op, t.numel(), str(t.dtype).replace("torch.", ""),
                              t.numel() * t.element_size())
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            if self._capture is None:
                self._capture = defaultdict(int)
            self._capture[kind] += 1
        else:
            self.calls[kind] += 1

    def capture_begin(self) -> None:
        self._capture = defaultdict(int)

    def capture_end(self) -> Dict[str, int]:
        """The collectives recorded since capture_begin (the graph's tally)."""
        tally, self._capture = dict(self._capture or {}), None
        return tally

    def replayed(self, tally: Optional[Dict[str, int]]) -> None:
        for k, v in (tally or {}).items():
            self.calls[k] += v

    def reset(self) -> None:
        self.calls = defaultdict(int)


LOG = CollectiveLog()


class DataParallel:
    # True: run the collective code path even with a single rank (all-reduces over a
    # one-rank RCCL communicator are identities) -- bench.py --force-dp, used by the GPU test
    # that rehearses the N>1 path on a one-GPU box.
    force = False

    def __init__(self, group=None) -> None:
        self.group = group
        self.enabled = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if self.enabled else 1
        self.rank = dist.get_rank(group) if self.enabled else 0
        self._flat = None

    @property
    def active(self) -> bool:
        return self.enabled and (self.world > 1 or DataParallel.force)

    @property
    def capturable(self) -> bool:
        """Collectives of this group can be captured into a HIP graph (RCCL); gloo cannot."""
        return self.enabled and dist.get_backend(self.group) == "nccl"

    def all_reduce_(self, t: torch.Tensor, kind: str = "other") -> torch.Tensor:
        if self.active:
            LOG.note(kind, t, "all_reduce")
            dist.all_reduce(t, group=self.group)
        return t

    def all_gather_cat(self, t: torch.Tensor, kind: str = "other",
                       ragged: bool = False) -> torch.Tensor:
        """Concatenate the 1-D (or equally-shaped) tensors of every rank in rank order.
        ``ragged``: the ranks' lengths may differ (e.g. per-workgroup partials of unequal env
        shards): the lengths are exchanged first (one small all-gather, kind "shape", and a
        host read), every rank's tensor is padded to the longest and the padding dropped."""
        if not self.active:
            return t
        t = t.contiguous()
        if ragged:
            n = torch.tensor([t.numel()], dtype=torch.int64, device=t.device)
            LOG.note("shape", n, "all_gather")
            ns = [torch.empty_like(n) for _ in range(self.world)]
            dist.all_gather(ns, n, group=self.group)
            ns = [int(x) for x in torch.cat(ns).cpu()]
            m = max(ns)
            if m != t.numel() or len(set(ns)) > 1:
                pad = torch.zeros(m, dtype=t.dtype, device=t.device)
                pad[:t.numel()] = t.reshape(-1)
                LOG.note(kind, pad, "all_gather")
                out = [torch.empty_like(pad) for _ in range(self.world)]
                dist.all_gather(out, pad, group=self.group)
                return torch.cat([o[:k] for o, k in zip(out, ns)])
        LOG.note(kind, t, "all_gather")
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        return torch.cat(out)

    def all_gather_known(self, t: torch.Tensor, lengths, kind: str = "other") -> torch.Tensor:
        """all_gather_cat of 1-D tensors whose per-rank lengths every rank already knows
        (``lengths[r]`` = rank r's numel, e.g. from the once-per-update shard table): each
        rank pads to the longest, no length exchange and no host read."""
        if not self.active:
            return t
        lengths = [int(k) for k in lengths]
        assert lengths[self.rank] == t.numel(), (lengths, t.numel())
        m = max(lengths)
        if len(set(lengths)) == 1:
            return self.all_gather_cat(t, kind)
        pad = torch.zeros(m, dtype=t.dtype, device=t.device)
        pad[:t.numel()] = t.reshape(-1)
        LOG.note(kind, pad, "all_gather")
        out = [torch.empty_like(pad) for _ in range(self.world)]
        dist.all_gather(out, pad, group=self.group)
        return torch.cat([o[:k] for o, k in zip(out, lengths)])

    def broadcast_params_(self, params: Iterable[torch.nn.Parameter], src: int = 0) -> None:
        """Make every rank's replica rank ``src``'s (one bucketed broadcast): data-parallel
        learning keeps identical replicas by applying the same all-reduced step, which needs
        identical starting parameters whatever seed each rank built its networks with."""
        if not self.active:
            return
        ps = [p for p in params]
        if not ps:
            return
        flat = torch.cat([p.detach().reshape(-1) for p in ps])
        LOG.note("param_broadcast", flat, "broadcast")
        dist.broadcast(flat, src=src, group=self.group)
        o = 0
        with torch.no_grad():
            for p in ps:
                p.copy_(flat[o:o + p.numel()].view_as(p))
                o += p.numel()

    def all_reduce_grads_(self, params: Iterable[torch.nn.Parameter],
                          average: bool = False) -> None:
        """One bucketed all-reduce of every gradient.  SUM by default (the fused PPO loss
        already divides each rank's contribution by the global minibatch size); ``average``
        for losses that are per-rank means."""
        if not self.active:
            return
        grads = [p.grad for p in params if p.grad is not None]
        if not grads:
            return
        n = sum(g.numel() for g in grads)
        if self._flat is None or self._flat.numel() != n or self._flat.device != grads[0].device:
            self._flat = torch.empty(n, dtype=grads[0].dtype, device=grads[0].device)
        torch.cat([g.reshape(-1) for g in grads], out=self._flat)
        LOG.note("grad", self._flat, "all_reduce")
        dist.all_reduce(self._flat, group=self.group)
        if average:
            self._flat.div_(self.world)
        o = 0
        for g in grads:
            g.copy_(self._flat[o:o + g.numel()].view_as(g))
            o += g.numel()


_DEFAULT: Optional[DataParallel] = None


def default_dp() -> DataParallel:
    global _DEFAULT
    if _DEFAULT is None or (not _DEFAULT.enabled and dist.is_available()
                            and dist.is_initialized()):
        _DEFAULT = DataParallel()
    return _DEFAULT


def param_hash(params: Iterable[torch.Tensor]) -> torch.Tensor:
    """An int64 device hash of the parameters' bit patterns (position-weighted, so a swap
    or a one-bit change moves it): equal on every rank iff the replicas agree (bench.py
    compares its all-reduced MAX and MIN)."""
    h = None
    for i, p in enumerate(params):
        # every one of the 32 bits (the sign too) as a value in [0, 2^32); times a weight
        # < 2^31 it stays below 2^63
        bits = p.detach().reshape(-1).contiguous().view(torch.int32).to(torch.int64)
        w = torch.arange(bits.numel(), device=bits.device, dtype=torch.int64) * 2654435761 \
            + (i + 1) * 97
        v = ((bits & 0xFFFFFFFF) * (w % 2147483647 + 1)).remainder(2305843009213693951).sum()
        h = v if h is None else (h * 31 + v).remainder(2305843009213693951)
    return h


def probe_collectives(dp: DataParallel, reps: int = 30) -> Dict[str, dict]:
    """Mean HIP-event time of each logged collective kind at its logged payload: `reps`
    collectives issued eagerly, and the same `reps` captured in one HIP graph and replayed
    (how the collect steps and the small-minibatch learn epochs issue them)."""
    out = {}
    if not dp.active:
        return out
    dev = torch.device("cuda", torch.cuda.current_device())
    for kind, (op, numel, dtype, nbytes) in sorted(LOG.payload.items()):
        if op != "all_reduce":
            out[kind] = dict(op=op, numel=numel, dtype=dtype, bytes=nbytes)
            continue
        t = torch.zeros(numel, dtype=getattr(torch, dtype), device=dev)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(3):
            dist.all_reduce(t, group=dp.group)
        dist.barrier(group=dp.group)
        torch.cuda.synchronize()
        s.record()
        for _ in range(reps):
            dist.all_reduce(t, group=dp.group)
        e.record()
        torch.cuda.synchronize()
        eager_us = s.elapsed_time(e) * 1e3 / reps
        graph_us = None
        try:
            g = torch.cuda.CUDAGraph()
            from tianshou_amd.utils.capture import graph_capture
            with graph_capture(g):
                for _ in range(reps):
                    dist.all_reduce(t, group=dp.group)
            g.replay()
            dist.barrier(group=dp.group)
            torch.cuda.synchronize()
            s.record()
            g.replay()
            e.record()
            torch.cuda.synchronize()
            graph_us = s.elapsed_time(e) * 1e3 / reps
        except RuntimeError:
            torch.cuda.synchronize()
        out[kind] = dict(op=op, numel=numel, dtype=dtype, bytes=nbytes,
                         eager_us=round(eager_us, 2),
                         graph_us=None if graph_us is None else round(graph_us, 2))
    return out
