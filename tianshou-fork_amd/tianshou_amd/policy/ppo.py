"""PPOPolicy (tianshou/policy/modelfree/ppo.py:13-162).

For the Gaussian actor with state-independent log-std (ActorProb + Independent(Normal, 1),
the MuJoCo/Box configuration of utils/models.py:34-97) the minibatch loss runs as the fused
``tsrl_ppo_gauss_*`` kernels: the minibatch rows are addressed through the permutation
index (no per-key minibatch copies except the obs rows the MLP GEMMs read), the clipped
surrogate / value / entropy terms and their gradients come out of one pass, and the loss
values are accumulated on device (no per-minibatch .item() syncs; the returned lists are
read back once at the end).  Other actor/dist combinations run the reference's torch
formulation on the GPU.
"""
import contextlib
import os
from typing import Any, Callable, Dict, List, Optional

import numpy as np
import torch
from torch import nn

from tianshou_amd import _C
from tianshou_amd.data.batch import Batch, gather_rows, split_indices
from tianshou_amd.dist import LOG
from tianshou_amd.utils.capture import graph_capture
from tianshou_amd.policy.a2c import A2CPolicy
from tianshou_amd.policy.flat_adam import FlatAdam
from tianshou_amd.policy.fused_eval import FusedEvalMixin, cat_logp, cat_mode  # noqa: F401
from tianshou_amd.utils.np_perm import LegacyPermutation

# a shared uint8 conv trunk reads each minibatch's frame stacks in place from the whole batch
# (DQN.forward(..., rows=idx)); TSRL_TRUNK_ROWS=0: gather them into a minibatch copy first
TRUNK_ROWS = os.environ.get("TSRL_TRUNK_ROWS", "1") != "0"


def split_bounds(length: int, size: int, merge_last: bool):
    """[start, end) of every Batch.split chunk (batch.py:896-912)."""
    if size == -1:
        size = length
    assert 1 <= size
    merge_last = merge_last and length % size > 0
    out = []
    for idx in range(0, length, size):
        if merge_last and idx + size + size >= length:
            out.append((idx, length))
            break
        out.append((idx, min(idx + size, length)))
    return out


class _GaussPPOLoss(torch.autograd.Function):
    """Fused forward+backward: the kernels produce the loss terms and the gradients w.r.t.
    mu, log-std and value in one pass; backward just scales them by the incoming grad."""

    @staticmethod
    def forward(ctx, mu, sigma_param, value, ctx_args):
        (act, logp_old, adv, ret, v_s, idx, params, dp) = ctx_args
        L = _C.lib()
        s = _C.stream_ptr(mu.device)
        mu = mu.contiguous()
        value = value.contiguous()
        log_std = sigma_param.detach().reshape(-1).contiguous()
        B, A = mu.shape
        nblk = int(L.tsrl_ppo_num_partials(B))
        dev = mu.device
        adv_sums = None
        if params.norm_adv:
            pa = torch.empty(nblk * 2, dtype=torch.float64, device=dev)
            _C.check(L.tsrl_adv_moments(_C.ptr(adv), _C.ptr(idx), B, _C.ptr(pa), s),
                     "tsrl_adv_moments")
            adv_sums = torch.empty(2, dtype=torch.float64, device=dev)
            _C.check(L.tsrl_reduce_partials(_C.ptr(pa), nblk, 2, _C.ptr(adv_sums), s),
                     "tsrl_reduce_partials")
            dp.all_reduce_(adv_sums, kind="adv_moments")
        grad_mu = torch.empty_like(mu)
        grad_value = torch.empty_like(value)
        partials = torch.empty(nblk * (4 + A), dtype=torch.float64, device=dev)
        _C.check(L.tsrl_ppo_gauss_fwd_bwd(
            _C.ptr(mu.detach()), _C.ptr(log_std), _C.ptr(value.detach()), _C.ptr(act),
            _C.ptr(logp_old), _C.ptr(adv), _C.ptr(ret), _C.ptr(v_s), _C.ptr(idx), B, A,
            _C.ptr(adv_sums), params, _C.ptr(grad_mu), _C.ptr(grad_value), _C.ptr(partials),
            s), "tsrl_ppo_gauss_fwd_bwd")
        sums = torch.empty(4 + A, dtype=torch.float64, device=dev)
        _C.check(L.tsrl_reduce_partials(_C.ptr(partials), nblk, 4 + A, _C.ptr(sums), s),
                 "tsrl_reduce_partials")
        dp.all_reduce_(sums, kind="loss_sums")
        terms = torch.empty(4, dtype=torch.float32, device=dev)
        grad_ls = torch.empty(A, dtype=torch.float32, device=dev)
        _C.check(L.tsrl_ppo_gauss_finalize(_C.ptr(sums), A, _C.ptr(log_std), params,
                                           _C.ptr(terms), _C.ptr(grad_ls), s),
                 "tsrl_ppo_gauss_finalize")
        ctx.save_for_backward(grad_mu, grad_value, grad_ls)
        ctx.sp_shape = sigma_param.shape
        loss = terms[0].clone()
        ctx.mark_non_differentiable(terms)
        return loss, terms

    @staticmethod
    def backward(ctx, g_loss, g_terms):
        grad_mu, grad_value, grad_ls = ctx.saved_tensors
        return (grad_mu * g_loss, (grad_ls * g_loss).reshape(ctx.sp_shape),
                grad_value * g_loss, None)


class _CatPPOLoss(torch.autograd.Function):
    """Fused forward+backward of the Categorical PPO loss (tsrl_ppo_cat_*): x is the dist_fn
    input (logits or probs) of the minibatch rows."""

    @staticmethod
    def forward(ctx, x, value, ctx_args):
        (act, logp_old, adv, ret, v_s, idx, params, dp, mode) = ctx_args
        L = _C.lib()
        s = _C.stream_ptr(x.device)
        x = x.detach().float().contiguous()
        value = value.detach().contiguous()
        B, A = x.shape
        nblk = int(L.tsrl_ppo_num_partials(B))
        dev = x.device
        adv_sums = None
        if params.norm_adv:
            pa = torch.empty(nblk * 2, dtype=torch.float64, device=dev)
            _C.check(L.tsrl_adv_moments(_C.ptr(adv), _C.ptr(idx), B, _C.ptr(pa), s),
                     "tsrl_adv_moments")
            adv_sums = torch.empty(2, dtype=torch.float64, device=dev)
            _C.check(L.tsrl_reduce_partials(_C.ptr(pa), nblk, 2, _C.ptr(adv_sums), s),
                     "tsrl_reduce_partials")
            dp.all_reduce_(adv_sums, kind="adv_moments")
        grad_x = torch.empty_like(x)
        grad_value = torch.empty_like(value)
        partials = torch.empty(nblk * 4, dtype=torch.float64, device=dev)
        _C.check(L.tsrl_ppo_cat_fwd_bwd(
            _C.ptr(x), _C.ptr(value), _C.ptr(act), _C.ptr(logp_old), _C.ptr(adv), _C.ptr(ret),
            _C.ptr(v_s), _C.ptr(idx), B, A, int(mode), _C.ptr(adv_sums), params,
            _C.ptr(grad_x), _C.ptr(grad_value), _C.ptr(partials), s), "tsrl_ppo_cat_fwd_bwd")
        sums = torch.empty(4, dtype=torch.float64, device=dev)
        _C.check(L.tsrl_reduce_partials(_C.ptr(partials), nblk, 4, _C.ptr(sums), s),
                 "tsrl_reduce_partials")
        dp.all_reduce_(sums, kind="loss_sums")
        terms = torch.empty(4, dtype=torch.float32, device=dev)
        _C.check(L.tsrl_ppo_cat_finalize(_C.ptr(sums), params, _C.ptr(terms), s),
                 "tsrl_ppo_cat_finalize")
        ctx.save_for_backward(grad_x, grad_value)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the terms output
        loss = terms[0].clone()
        ctx.mark_non_differentiable(terms)
        return loss, terms

    @staticmethod
    def backward(ctx, g_loss, g_terms):
        grad_x, grad_value = ctx.saved_tensors
        if g_loss is None:
            return None, None, None
        if _is_unit_seed(g_loss):
            # loss.backward(UNIT): the gradients are the kernel's as they are (x * 1.0 is x)
            return grad_x, grad_value, None
        return grad_x * g_loss, grad_value * g_loss, None


_UNIT = {}


def _unit_seed(dev: torch.device) -> torch.Tensor:
    """A constant f32 1.0 on dev, the seed gradient of the Categorical minibatch's
    loss.backward(): it spares autograd's ones_like fill, and _CatPPOLoss recognises it and
    skips two scaling passes (round 6).  Never written."""
    t = _UNIT.get(dev)
    if t is None:
        t = _UNIT[dev] = torch.ones((), dtype=torch.float32, device=dev)
    return t


def _is_unit_seed(g: torch.Tensor) -> bool:
    t = _UNIT.get(g.device)
    return t is not None and g.dim() == 0 and g.data_ptr() == t.data_ptr()


class PPOPolicy(FusedEvalMixin, A2CPolicy):
    def __init__(self, actor: torch.nn.Module, critic: torch.nn.Module,
                 optim: torch.optim.Optimizer, dist_fn: Callable, eps_clip: float = 0.2,
                 dual_clip: Optional[float] = None, value_clip: bool = False,
                 advantage_normalization: bool = True, recompute_advantage: bool = False,
                 perm_device: bool = False, fused_mlp: bool = True, **kwargs: Any) -> None:
        super().__init__(actor, critic, optim, dist_fn, **kwargs)
        self._eps_clip = eps_clip
        assert dual_clip is None or dual_clip > 1.0, \
            "Dual-clip PPO parameter should greater than 1.0."
        self._dual_clip = dual_clip
        self._value_clip = value_clip
        self._norm_adv = advantage_normalization
        self._recompute_adv = recompute_advantage
        # perm_device=False: minibatch order from np.random.permutation (the reference's
        # global RandomState stream, bit-exact: MT19937 draws on the host, the shuffle
        # resolved on the device, the next update's draws prefetched in a host thread --
        # utils/np_perm.py); True: torch.randperm on the GPU.
        self.perm_device = perm_device
        self._np_perm = LegacyPermutation()
        self._plan_stream = None
        self._np_perm_used, self._np_perm_n = False, 0
        self._dp_shards = (0, 0)  # (this rank's first global row, global rows) of learn()
        # data-parallel minibatch composition (see _minibatch_plan): "global" = the
        # reference's split of the global batch, "local" = every rank splits its own rows
        self.dp_permutation = "global"
        self._bounds_cache = None
        self._graph_failed = False
        # sort_minibatch=True: the rows of every minibatch are visited in ascending buffer
        # order (same minibatch SETS as Batch.split over the permutation; only the order of
        # rows inside a minibatch -- i.e. the float summation order -- changes).  The fused
        # kernels gather rows through the index, and ascending order measured ~4 % faster
        # per minibatch at 262144 x 376 (tools/mlp_kernel_bench.py --sorted).
        self.sort_minibatch = False
        # fused paths (policy/fused_eval.py): Gaussian / Categorical detection, and the whole
        # minibatch (MLP forward, loss, backward) as three HIP kernels when the networks have
        # the get_actor_critic shape (policy/fused_mlp.py); fused_mlp=False keeps the torch
        # layers + fused loss kernel.
        self._init_fused_eval(actor, critic, dist_fn, fused_mlp)
        # graph_learn=True replays whole epochs of the fused minibatch step from a captured
        # HIP graph; None (default) = only for minibatches below GRAPH_LEARN_MAX_ROWS.  Large
        # minibatches launch eagerly: with ~15 launches per 0.75 ms minibatch the host stays
        # far ahead of the GPU, and eager launches measured 100 ms per update vs 105 ms for
        # graph replay (bench.py, MI355X, 4096x2048: graph nodes cost more per kernel); small
        # ones (config 2: 2048 rows, ~50 us of GPU work) are host-bound without the graph.
        self.graph_learn = None
        self._learn_graph = None
        # clip_grad_norm_ + Adam as one HIP pass over flat parameter storage (csrc/optim.hip)
        self.fused_adam = True
        self._cat_adam: Optional[FlatAdam] = None
        self._cat_warm = False

    def _params(self, b_global: float) -> _C.PPOParams:
        p = _C.PPOParams()
        p.eps_clip = float(self._eps_clip)
        p.dual_clip = float(self._dual_clip) if self._dual_clip else 0.0
        p.vf_coef = float(self._weight_vf)
        p.ent_coef = float(self._weight_ent)
        p.adv_eps = float(self._eps)
        p.b_global = float(b_global)
        p.value_clip = int(bool(self._value_clip))
        p.norm_adv = int(bool(self._norm_adv))
        return p

    # -- process_fn -------------------------------------------------------------------------
    def process_fn(self, batch: Batch, buffer, indices: np.ndarray) -> Batch:
        """ppo.py:87-97."""
        if self._recompute_adv:
            self._buffer, self._indices = buffer, indices
        self._pending_logp = None
        batch = self._compute_returns(batch, buffer, indices)
        batch.act = torch.as_tensor(batch.act, device=batch.v_s.device).to(batch.v_s.dtype)
        batch.logp_old = self._logp_old(batch)
        return batch

    # -- learn ----------------------------------------------------------------------------------
    def _permutation(self, n: int, dev, batch_size: Optional[int] = None):
        if self.perm_device:
            if self.sort_minibatch and batch_size:
                # Minibatch k = the rows whose position in a uniform permutation falls in
                # chunk k; the inverse of a uniform permutation is uniform, so the chunk label
                # of row r is randperm(n)[r] // size (the merged last chunk clamps).  One stable
                # 8-bit-key sort then lists every chunk's rows in ascending order.
                bounds = split_bounds(n, batch_size, merge_last=True)
                if len(bounds) <= 256:
                    lab = torch.div(torch.randperm(n, device=dev), batch_size,
                                    rounding_mode="floor").clamp_(max=len(bounds) - 1)
                    return torch.sort(lab.to(torch.uint8), stable=True).indices
            perm = torch.randperm(n, device=dev)
        else:
            perm = self._np_perm(n, dev)
            self._np_perm_used = True
            self._np_perm_n = n
        if self.sort_minibatch and batch_size:
            bounds = split_bounds(n, batch_size, merge_last=True)
            sizes = {e - s for s, e in bounds}
            if len(sizes) == 1:
                perm = perm.view(len(bounds), -1).sort(dim=1).values.reshape(-1)
            else:
                perm = torch.cat([perm[s:e].sort().values for s, e in bounds])
        return perm

    def learn(self, batch: Batch, batch_size: int, repeat: int, **kwargs: Any
              ) -> Dict[str, List[float]]:
        self._np_perm_used = False
        out = self._learn(batch, batch_size, repeat)
        if self._np_perm_used:
            # the next update's np.random.permutation draws, computed while it collects
            self._np_perm.prefetch(self._np_perm_n, repeat)
        return out

    def _learn(self, batch: Batch, batch_size: int, repeat: int) -> Dict[str, List[float]]:
        if not self._fused:
            if self._cat is not None and isinstance(batch.obs, torch.Tensor) and \
                    batch.obs.is_cuda:
                return self._learn_cat(batch, batch_size, repeat)
            return self._learn_generic(batch, batch_size, repeat)
        dev = batch.v_s.device
        n = len(batch.v_s)
        terms = []
        f32 = dict(device=dev, dtype=torch.float32)
        mlp_ok = self._mlp is not None and batch.obs.is_cuda and \
            batch.obs.dtype == torch.float32 and batch.obs.dim() == 2
        if not self._global_perm(n, dev, mlp_ok):
            self._require_equal_shards(n, dev, "learn")
        plans = self._plan_pipeline(n, dev, batch_size, repeat, mlp_ok)
        for step in range(repeat):
            if self._recompute_adv and step > 0:
                batch = self._compute_returns(batch, self._buffer, self._indices)
            act = batch.act.reshape(n, -1).contiguous()
            logp_old = batch.logp_old.reshape(-1).to(**f32).contiguous()
            adv = batch.adv.reshape(-1).to(**f32).contiguous()
            ret = batch.returns.reshape(-1).to(**f32).contiguous()
            v_s = batch.v_s.reshape(-1).to(**f32).contiguous()
            perm, chunks = plans(step)
            if mlp_ok and self.fused_adam and self._mlp.bind_adam(self.optim):
                self._mlp.set_lr()
            obs_all = self._mlp.rows(batch.obs) if mlp_ok else None
            if mlp_ok and self._use_graph(batch_size) and self._graph_ready(chunks):
                t = self._epoch_graph(obs_all, (act, logp_old, adv, ret, v_s), perm, chunks,
                                      first=(step == 0))
                if t is not None:
                    terms.append(t)
                    continue
            adv_mom = None
            if mlp_ok and self._norm_adv:
                bounds, max_seg = self._dev_bounds(chunks, dev)
                adv_mom = self._mlp.epoch_adv_moments(adv, perm, bounds, max_seg, self.dp)
            fused_opt = mlp_ok and self._mlp.adam_bound(self.optim)
            if fused_opt:
                self._mlp.split_w1()  # later minibatches get the planes from the Adam pass
            for k, (s, e, b_glob) in enumerate(chunks):
                idx = perm[s:e]
                params = self._params(b_glob)
                if mlp_ok:
                    t = self._mlp.minibatch(obs_all, idx, e - s, act, logp_old, adv, ret, v_s,
                                            params, self.dp,
                                            adv_sums=None if adv_mom is None else adv_mom[k],
                                            split_w=not fused_opt)
                    self._opt_step(last=(k == len(chunks) - 1))
                    terms.append(t)
                    continue
                obs_mb = gather_rows(batch.obs, idx)
                mu = self.actor.forward_mu(obs_mb)
                value = self.critic(obs_mb).flatten()
                loss, t = _GaussPPOLoss.apply(mu, self.actor.sigma_param, value,
                                              (act, logp_old, adv, ret, v_s, idx, params,
                                               self.dp))
                self.optim.zero_grad()
                loss.backward()
                self.dp.all_reduce_grads_(self._actor_critic.parameters())
                if self._grad_norm:
                    nn.utils.clip_grad_norm_(self._actor_critic.parameters(),
                                             max_norm=self._grad_norm)
                self.optim.step()
                terms.append(t)
        vals = torch.cat([t.reshape(-1, 4) for t in terms]).cpu().numpy() if terms else \
            np.zeros((0, 4), np.float32)
        if self._mlp is not None:
            self._mlp.check_handoff()
        return {"loss": vals[:, 0].tolist(), "loss/clip": vals[:, 1].tolist(),
                "loss/vf": vals[:, 2].tolist(), "loss/ent": vals[:, 3].tolist()}

    # -- minibatch plan (Batch.split over a permutation; data-parallel shares) ----------------
    def _minibatch_plan(self, n: int, dev, batch_size: int, allow_global: bool = False):
        """(idx, [(start, end, b_global)]): minibatch k = rows idx[start:end] of this rank,
        b_global = the size of the global minibatch (the loss divides by it).

        Single process: Batch.split(batch_size, shuffle=True, merge_last=True) over one
        permutation (batch.py:896-912).  Data parallel, ``dp_permutation == "global"``: the
        reference's split of the GLOBAL batch -- every rank draws the same
        np.random.permutation(N) of the N = sum of every rank's n rows (identical global
        RandomState on every rank; rank r owns global rows [n_0 + ... + n_{r-1}, ... + n_r),
        the env-major order of one VectorReplayBuffer over all ranks' envs -- shards may be
        unequal) with global minibatches of world * batch_size rows, and keeps its own rows
        of each, in permutation order.  ``"local"``: each rank splits its own n rows
        (weak scaling: the sequential host draws stay O(n) per rank)."""
        return self._take_plan(self._issue_plan(n, dev, batch_size, allow_global, None), dev)

    def _plan_pipeline(self, n: int, dev, batch_size: int, repeat: int, allow_global: bool):
        """plans(k) -> repeat k's (idx, chunks).  With the np.random permutation on a HIP
        device, each repeat's permutation (pinned draws -> device copy -> swap resolution ->
        this rank's share) is enqueued on a side stream, and the next repeat's too as soon as
        its prefetched host draws exist, so the copy and the resolution overlap the previous
        repeat's minibatches instead of serialising with them.  The global RandomState is
        consumed in the same order as repeat sequential calls."""
        if self.perm_device or dev.type != "cuda":
            return lambda k: self._minibatch_plan(n, dev, batch_size, allow_global)
        if self._plan_stream is None or self._plan_stream.device != dev:
            self._plan_stream = torch.cuda.Stream(dev)
        side = self._plan_stream
        issued = {}

        def plans(k):
            if k not in issued:
                issued[k] = self._issue_plan(n, dev, batch_size, allow_global, side)
            # the permutation size: the global row count (known after the first plan's
            # shard-size exchange) or this rank's n
            pn = self._np_perm_n if self._global_perm(n, dev, allow_global) else n
            if k + 1 < repeat and k + 1 not in issued and self._np_perm.next_ready(pn):
                issued[k + 1] = self._issue_plan(n, dev, batch_size, allow_global, side)
            return self._take_plan(issued.pop(k), dev)
        return plans

    def _global_perm(self, n: int, dev, allow_global: bool) -> bool:
        W = self.dp.world if self.dp.active else 1
        return W > 1 and allow_global and self.dp_permutation == "global" and \
            not self.perm_device

    def _issue_plan(self, n: int, dev, batch_size: int, allow_global: bool, stream):
        """Enqueue one repeat's minibatch plan on ``stream`` (None: the current stream) and
        return it pending; _take_plan orders the current stream after it.  No host
        synchronisation here (beyond the once-per-learn() check of the ranks' RandomStates,
        which also exchanges the shard sizes): the data-parallel share selection is a
        compaction by prefix sum whose size is known (this rank owns exactly n of the global
        rows), and the per-minibatch share counts travel back to pinned host memory behind an
        event."""
        W = self.dp.world if self.dp.active else 1
        ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
        cuda = dev.type == "cuda"
        if self._global_perm(n, dev, allow_global):
            if not self._np_perm_used:  # once per learn(): every rank holds the same stream
                # (the shard table of this update's process_fn: no second exchange)
                tab = self._learn_shards(n, dev)
                if not tab["hash_equal"]:
                    raise RuntimeError(
                        "dp_permutation='global' needs the same global np.random state on "
                        "every rank (seed np.random identically, or set "
                        "dp_permutation='local')")
                sizes = tab["n"]
                self._dp_shards = (sum(sizes[:self.dp.rank]), sum(sizes))
            lo, N = self._dp_shards
            B = batch_size * W
            gb = split_bounds(N, B, merge_last=True)
            self._np_perm_used = True
            self._np_perm_n = N
            ends = torch.tensor([ge - 1 for _, ge in gb], dtype=torch.int64)
            with ctx:
                perm_g = self._np_perm(N, dev)
                mine = (perm_g >= lo) & (perm_g < lo + n)
                cs = torch.cumsum(mine, 0)
                # this rank's rows in permutation order: row perm_g[p] - lo goes to slot
                # cs[p] - 1; every other position writes the spare slot n
                tgt = cs.sub(1).masked_fill_(~mine, n)
                idx = torch.empty(n + 1, dtype=torch.int64, device=dev)
                idx.scatter_(0, tgt, perm_g.sub_(lo))
                cum_dev = cs[ends.to(dev, non_blocking=True)]
                cum = torch.empty(len(gb), dtype=torch.int64, pin_memory=cuda)
                cum.copy_(cum_dev, non_blocking=cuda)
                ev = torch.cuda.Event() if cuda else None
                if ev is not None:
                    ev.record()
            return {"idx": idx[:n], "cum": cum, "gb": gb, "ev": ev}
        with ctx:
            perm = self._permutation(n, dev, batch_size)
            ev = torch.cuda.Event() if cuda else None
            if ev is not None:
                ev.record()
        return {"idx": perm, "ev": ev,
                "chunks": [(s, e, (e - s) * W) for s, e in split_bounds(n, batch_size, True)]}

    def _take_plan(self, rec, dev):
        if rec["ev"] is not None:
            cur = torch.cuda.current_stream(dev)
            cur.wait_event(rec["ev"])
            rec["idx"].record_stream(cur)
        if "chunks" in rec:
            return rec["idx"], rec["chunks"]
        if rec["ev"] is not None:
            rec["ev"].synchronize()  # the share counts (pinned host): long done by now
        chunks, o = [], 0
        for (gs, ge), c in zip(rec["gb"], rec["cum"].tolist()):
            chunks.append((o, c, ge - gs))
            o = c
        return rec["idx"], chunks

    def _dev_bounds(self, chunks, dev):
        """Device int64 [n_minibatch + 1] start offsets of the chunks (cached per plan)."""
        key = tuple((s, e) for s, e, _ in chunks)
        c = self._bounds_cache
        if c is None or c[0] != key or c[1].device != dev:
            host = torch.tensor([s for s, _, _ in chunks] + [chunks[-1][1]],
                                dtype=torch.int64).pin_memory()
            t = torch.empty(len(host), dtype=torch.int64, device=dev)
            t.copy_(host, non_blocking=True)
            c = self._bounds_cache = (key, t, max(e - s for s, e, _ in chunks), host)
        return c[1], c[2]

    def _opt_step(self, last: bool = True) -> None:
        """clip_grad_norm_ + optim.step() of ppo.py:143-151: one fused HIP pass
        (tsrl_clip_adam) when the optimiser is a plain Adam over the fused MLP's parameters
        -- it also re-splits the first-layer weights for the next minibatch, and leaves the
        clipped gradients in .grad only after an epoch's last minibatch (the next minibatch
        overwrites them otherwise) -- torch's otherwise."""
        if self._mlp is not None and self._mlp.adam_bound(self.optim):
            self._mlp.clip_adam(self._grad_norm, scale_grads=last, split_w1=True)
            return
        if self._grad_norm:
            nn.utils.clip_grad_norm_(self._actor_critic.parameters(), max_norm=self._grad_norm)
        self.optim.step()

    # -- HIP-graph replay of whole epochs ------------------------------------------------------
    GRAPH_LEARN_MAX_ROWS = 65536

    def _use_graph(self, batch_size: int) -> bool:
        if self.graph_learn is None:
            return batch_size < self.GRAPH_LEARN_MAX_ROWS
        return bool(self.graph_learn)

    def _graph_ready(self, chunks) -> bool:
        """An epoch of fused minibatches can be captured once and replayed: a static plan
        (single process, or data parallel with per-rank splits and a capturable backend --
        the RCCL all-reduces are then graph nodes), no advantage recomputation, and a
        capturable optimiser whose state already exists (the first update runs eagerly)."""
        if self.graph_learn is False or self._recompute_adv or self._graph_failed:
            return False
        if self.dp.active:
            static = self.dp_permutation == "local" or self.dp.world == 1 or self.perm_device
            if not (static and self.dp.capturable):
                return False
        opt = self.optim
        for flat in (self._mlp, self._cat_adam):
            if flat is not None and flat.adam_bound(opt):
                return True
        if not opt.defaults.get("capturable", False) or len(opt.state) == 0:
            return False
        return all(p in opt.state for g in opt.param_groups for p in g["params"])

    def _epoch_graph(self, obs_all, arrays, perm, chunks, first: bool):
        """One epoch (the epoch's advantage moments, then every minibatch of the plan:
        forward, loss, backward, clip_grad_norm_, optimiser step) as a replay of a captured
        HIP graph.  The per-update arrays and the permutation are copied into static buffers
        the graph reads, the learning rate is a device word (FusedActorCritic.set_lr);
        returns the [n_minibatch, 4] loss terms, or None if the capture failed (the caller
        then runs the epoch eagerly, and later epochs do too)."""
        n = perm.numel()
        flat_opt = self._mlp.adam_bound(self.optim)
        # the flat Adam pass reads lr from a device word (set_lr), so a schedule needs no
        # re-capture; any other (capturable torch) optimiser bakes the float lr into the
        # captured step, so the lrs are part of the key and a schedule step re-captures
        lrs = None if flat_opt else tuple(float(g["lr"]) for g in self.optim.param_groups)
        key = (n, tuple(chunks), obs_all.data_ptr(), tuple(obs_all.shape),
               tuple(a.shape for a in arrays), self._mlp.flat_grad is not None and
               self._mlp.flat_grad.data_ptr(), flat_opt, lrs)
        st = self._learn_graph
        if st is None or st["key"] != key:
            st = None
            self._learn_graph = None
            dev = perm.device
            static = [torch.empty_like(a) for a in arrays]
            sperm = torch.empty(n, dtype=torch.int64, device=dev)
            sterms = torch.empty(len(chunks), 4, dtype=torch.float32, device=dev)
            for d, a in zip(static, arrays):
                d.copy_(a)
            sperm.copy_(perm)
            bounds, max_seg = self._dev_bounds(chunks, dev)
            sbounds = bounds.clone()
            self._mlp.bind_grads()
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            LOG.capture_begin()
            try:
                with graph_capture(graph):
                    mom = None
                    if self._norm_adv:
                        mom = self._mlp.epoch_adv_moments(static[2], sperm, sbounds, max_seg,
                                                          self.dp)
                    fused_opt = self._mlp.adam_bound(self.optim)
                    if fused_opt:
                        self._mlp.split_w1()
                    for i, (s, e, b_glob) in enumerate(chunks):
                        t = self._mlp.minibatch(obs_all, sperm[s:e], e - s, *static,
                                                self._params(b_glob), self.dp,
                                                adv_sums=None if mom is None else mom[i],
                                                split_w=not fused_opt, terms_out=sterms[i])
                        self._opt_step(last=(i == len(chunks) - 1))
                        if t.data_ptr() != sterms[i].data_ptr():  # data parallel: reduced
                            sterms[i].copy_(t)
            except RuntimeError as err:  # e.g. a collective backend that cannot be captured
                import warnings
                warnings.warn(f"learn-graph capture failed, running epochs eagerly: {err}")
                self._graph_failed = True
                torch.cuda.synchronize()
                return None
            st = dict(key=key, graph=graph, static=static, perm=sperm, terms=sterms,
                      bounds=sbounds, tally=LOG.capture_end())
            self._learn_graph = st
            first = False  # static arrays already hold this update's data
        if first:
            for d, a in zip(st["static"], arrays):
                d.copy_(a)
        st["perm"].copy_(perm)
        st["graph"].replay()
        LOG.replayed(st["tally"])
        return st["terms"].clone()

    def _learn_cat(self, batch: Batch, batch_size: int, repeat: int
                   ) -> Dict[str, List[float]]:
        """ppo.py:99-162 for Categorical policies: torch actor/critic (MLP or conv trunk on
        MIOpen/hipBLASLt), minibatch rows gathered once through the permutation, the loss and
        its gradient w.r.t. the dist_fn input from the fused tsrl_ppo_cat kernel.  With a
        plain Adam the gradients live in one flat bucket and clip_grad_norm_ + Adam.step() are
        one HIP pass (policy/flat_adam.py); epochs after the first eager one then replay from
        a captured HIP graph (small minibatches -- test_ppo.py's 64 rows -- are otherwise
        bound by ~40 host launches each)."""
        dev = batch.v_s.device
        n = len(batch.v_s)
        terms = []
        f32 = dict(device=dev, dtype=torch.float32)
        fa = self._cat_flat_adam()
        self._require_equal_shards(n, dev, "learn")
        for step in range(repeat):
            if self._recompute_adv and step > 0:
                batch = self._compute_returns(batch, self._buffer, self._indices)
            act = torch.as_tensor(batch.act, device=dev).reshape(n).to(torch.int64).contiguous()
            arrays = (act, batch.logp_old.reshape(-1).to(**f32).contiguous(),
                      batch.adv.reshape(-1).to(**f32).contiguous(),
                      batch.returns.reshape(-1).to(**f32).contiguous(),
                      batch.v_s.reshape(-1).to(**f32).contiguous())
            perm = self._permutation(n, dev)
            chunks = [(s, e, (e - s) * self.dp.world)
                      for s, e in split_bounds(n, batch_size, merge_last=True)]
            if fa is not None:
                fa.set_lr()
                # conv trunks (MIOpen) stay eager unless graph_learn=True
                graph = self._use_graph(batch_size) and (batch.obs.dim() == 2 or
                                                         self.graph_learn is True)
                if self._cat_warm and graph and self._graph_ready(chunks):
                    t = self._cat_epoch_graph(fa, batch.obs, arrays, perm, chunks,
                                              first=(step == 0))
                    if t is not None:
                        terms.append(t)
                        continue
            for k, (s, e, b_glob) in enumerate(chunks):
                terms.append(self._cat_minibatch(fa, batch.obs, perm[s:e], b_glob, arrays,
                                                 last=(k == len(chunks) - 1)))
            self._cat_warm = True
        vals = torch.cat([t.reshape(-1, 4) for t in terms]).cpu().numpy() if terms else \
            np.zeros((0, 4), np.float32)
        if fa is not None:
            fa.check_handoff()
        return {"loss": vals[:, 0].tolist(), "loss/clip": vals[:, 1].tolist(),
                "loss/vf": vals[:, 2].tolist(), "loss/ent": vals[:, 3].tolist()}

    def _cat_flat_adam(self) -> Optional[FlatAdam]:
        """The flat gradient / Adam storage of the actor-critic parameters when the optimiser
        is a plain Adam over exactly them (None otherwise: torch's optimiser runs)."""
        if not self.fused_adam:
            return None
        fa = self._cat_adam
        if fa is None:
            fa = self._cat_adam = FlatAdam(self._actor_critic.parameters())
        return fa if fa.bind_adam(self.optim) else None

    def _cat_minibatch(self, fa: Optional[FlatAdam], obs: torch.Tensor, idx: torch.Tensor,
                       b_glob: int, arrays, last: bool) -> torch.Tensor:
        """One Categorical minibatch (ppo.py:107-151): forward, fused loss, backward,
        gradient all-reduce, clip_grad_norm_ + Adam.step(); returns the [4] loss terms."""
        pre = self.actor.preprocess if self._shared_trunk else None
        if TRUNK_ROWS and pre is not None and hasattr(pre, "reads_rows") and pre.reads_rows(obs):
            # the trunk's uint8 kernels read the minibatch's frame stacks in place (round 6)
            x, value = self._trunk_heads(obs, rows=idx)
        elif self._shared_trunk:
            x, value = self._trunk_heads(gather_rows(obs, idx))
        else:
            obs_mb = gather_rows(obs, idx)
            x, _ = self.actor(obs_mb)
            value = self.critic(obs_mb).flatten()
        loss, t = _CatPPOLoss.apply(x, value, (*arrays, idx, self._params(b_glob), self.dp,
                                               self._cat))
        if fa is not None:
            # eager: autograd hands over each gradient and one pass gathers them into the flat
            # bucket; under graph capture it accumulates into the zeroed bucket in place
            gather = loss.is_cuda and not torch.cuda.is_current_stream_capturing()
            if gather:
                fa.release_grads()
            else:
                fa.zero_grad()
            loss.backward(_unit_seed(loss.device))
            if gather:
                fa.gather_grads()
            self.dp.all_reduce_(fa.flat_grad, kind="grad")
            fa.clip_adam(self._grad_norm, scale_grads=last)
            return t
        self.optim.zero_grad()
        loss.backward()
        self.dp.all_reduce_grads_(self._actor_critic.parameters())
        if self._grad_norm:
            nn.utils.clip_grad_norm_(self._actor_critic.parameters(), max_norm=self._grad_norm)
        self.optim.step()
        return t

    def _cat_epoch_graph(self, fa: FlatAdam, obs, arrays, perm, chunks, first: bool):
        """One Categorical epoch replayed from a captured HIP graph (the torch forward /
        autograd backward, the fused loss kernels and the flat Adam pass of every minibatch).
        Static copies of the per-update arrays and the permutation feed it, and of the obs
        rows when they are small (≤ 64 MB: a buffer whose sample returns fresh rows every
        update -- CartPoleVectorEnv's -- would otherwise re-capture the graph every update,
        ~100 ms each, round 6); larger obs rows are read in place (their address is part of
        the key).  None if the capture failed."""
        n = perm.numel()
        static_obs = obs.numel() * obs.element_size() <= (64 << 20)
        key = (n, tuple(chunks), "static" if static_obs else obs.data_ptr(), tuple(obs.shape),
               obs.dtype, tuple(a.shape for a in arrays), fa.flat_grad.data_ptr(),
               tuple(p.data_ptr() for p in fa.params))
        st = self._learn_graph
        if st is None or st["key"] != key:
            self._learn_graph = None
            dev = perm.device
            static = [a.clone() for a in arrays]
            sobs = obs.clone() if static_obs else obs
            sperm = perm.clone()
            sterms = torch.empty(len(chunks), 4, dtype=torch.float32, device=dev)
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            LOG.capture_begin()
            try:
                with graph_capture(graph):
                    for i, (s, e, b_glob) in enumerate(chunks):
                        t = self._cat_minibatch(fa, sobs, sperm[s:e], b_glob, static,
                                                last=(i == len(chunks) - 1))
                        sterms[i].copy_(t)
            except RuntimeError as err:
                import warnings
                warnings.warn(f"learn-graph capture failed, running epochs eagerly: {err}")
                self._graph_failed = True
                torch.cuda.synchronize()
                return None
            st = self._learn_graph = dict(key=key, graph=graph, static=static, perm=sperm,
                                          terms=sterms, tally=LOG.capture_end(),
                                          obs=sobs if static_obs else None)
            first = False
        if first:
            for d, a in zip(st["static"], arrays):
                d.copy_(a)
            if st["obs"] is not None and st["obs"].data_ptr() != obs.data_ptr():
                st["obs"].copy_(obs)
        st["perm"].copy_(perm)
        st["graph"].replay()
        LOG.replayed(st["tally"])
        return st["terms"].clone()

    def _learn_generic(self, batch: Batch, batch_size: int, repeat: int
                       ) -> Dict[str, List[float]]:
        """ppo.py:99-162 as written, on device tensors."""
        self._require_equal_shards(len(batch), next(self.critic.parameters()).device, "learn")
        losses, clip_losses, vf_losses, ent_losses = [], [], [], []
        for step in range(repeat):
            if self._recompute_adv and step > 0:
                batch = self._compute_returns(batch, self._buffer, self._indices)
            for part in split_indices(len(batch), batch_size, True, True):
                minibatch = batch[part]
                dist = self(minibatch).dist
                adv = minibatch.adv
                if self._norm_adv:
                    if self.dp.active:
                        # moments of the GLOBAL minibatch (every rank's share): torch's
                        # unbiased std from the all-reduced (count, sum, sum of squares)
                        a64 = adv.detach().double()
                        m = torch.stack([a64.new_tensor(float(a64.numel())), a64.sum(),
                                         (a64 * a64).sum()])
                        self.dp.all_reduce_(m, kind="adv_moments")
                        cnt, s1, s2 = m[0], m[1], m[2]
                        mean = (s1 / cnt).to(adv.dtype)
                        std = ((s2 - s1 * s1 / cnt) / (cnt - 1)).clamp_(min=0).sqrt_() \
                            .to(adv.dtype)
                    else:
                        mean, std = adv.mean(), adv.std()
                    adv = (adv - mean) / (std + self._eps)
                ratio = (dist.log_prob(minibatch.act) - minibatch.logp_old).exp().float()
                ratio = ratio.reshape(ratio.size(0), -1).transpose(0, 1)
                surr1 = ratio * adv
                surr2 = ratio.clamp(1.0 - self._eps_clip, 1.0 + self._eps_clip) * adv
                if self._dual_clip:
                    clip1 = torch.min(surr1, surr2)
                    clip2 = torch.max(clip1, self._dual_clip * adv)
                    clip_loss = -torch.where(adv < 0, clip2, clip1).mean()
                else:
                    clip_loss = -torch.min(surr1, surr2).mean()
                value = self.critic(minibatch.obs).flatten()
                if self._value_clip:
                    v_clip = minibatch.v_s + (value - minibatch.v_s).clamp(-self._eps_clip,
                                                                           self._eps_clip)
                    vf_loss = torch.max((minibatch.returns - value).pow(2),
                                        (minibatch.returns - v_clip).pow(2)).mean()
                else:
                    vf_loss = (minibatch.returns - value).pow(2).mean()
                ent_loss = dist.entropy().mean()
                loss = clip_loss + self._weight_vf * vf_loss - self._weight_ent * ent_loss
                self.optim.zero_grad()
                loss.backward()
                self.dp.all_reduce_grads_(self._actor_critic.parameters(), average=True)
                if self._grad_norm:
                    nn.utils.clip_grad_norm_(self._actor_critic.parameters(),
                                             max_norm=self._grad_norm)
                self.optim.step()
                terms4 = torch.stack([loss.detach(), clip_loss.detach(), vf_loss.detach(),
                                      ent_loss.detach()]).float()
                if self.dp.active:  # equal per-rank shares: global mean = mean over ranks
                    self.dp.all_reduce_(terms4, kind="loss_sums")
                    terms4 /= self.dp.world
                losses.append(terms4[0])
                clip_losses.append(terms4[1])
                vf_losses.append(terms4[2])
                ent_losses.append(terms4[3])
        out = {}
        for k, v in (("loss", losses), ("loss/clip", clip_losses), ("loss/vf", vf_losses),
                     ("loss/ent", ent_losses)):
            out[k] = torch.stack(v).cpu().tolist() if v else []
        return out
