"""One PPO minibatch of the MuJoCo actor/critic shape through the fused MLP kernels.

The networks of tianshou/utils/models.py:34-97 (``get_actor_critic``: two
``Net(D, (64, 64), Tanh)`` trunks, an unbounded ``ActorProb`` mu head ``Linear(64, A)`` with a
state-independent log-std, a ``Critic`` head ``Linear(64, 1)``) are run as three HIP kernels per
minibatch instead of ~60 framework ops (include/tsrl.h, csrc/mlp.hip):

1. ``tsrl_mlp_l1_fwd``  first layers of both nets, rows read through the minibatch index,
2. ``tsrl_ppo_tail``    layers 2-3, the PPO loss (ppo.py:121-142) and its backward,
3. ``tsrl_mlp_dw``      first-layer weight/bias gradients.

The gradients land in one flat buffer that the parameters' ``.grad`` views point into, so the
data-parallel all-reduce is a single call and torch's (fused) Adam and ``clip_grad_norm_``
consume them unchanged (ppo.py:143-151).  Every gradient element is overwritten each
minibatch, which is what ``optim.zero_grad()`` + ``loss.backward()`` amount to.
"""
import os
from typing import Dict, Optional

import torch
from torch import nn

from tianshou_amd import _C
from tianshou_amd.policy.flat_adam import FlatAdam

HIDDEN = 64
MAX_ACT = 32
# first-layer forward on the bf16 matrix cores with the exact 3-way operand split
# (tsrl_mlp_l1_fwd_x6, f32-level error); False: the f32-input MFMA kernel (tsrl_mlp_l1_fwd)
L1_X6 = True
# the tail's reduction launch runs on a second stream beside tsrl_mlp_dw (TSRL_TAIL_OVERLAP=0:
# one stream)
TAIL_OVERLAP = os.environ.get("TSRL_TAIL_OVERLAP", "1") != "0"
# process_fn's evaluation as one launch per call, layer 1 and the evaluation fused
# (tsrl_ppo_eval_fused; TSRL_EVAL_FUSED=0: tsrl_mlp_l1_fwd_x6 + tsrl_ppo_eval per 2M-row chunk)
EVAL_FUSED = os.environ.get("TSRL_EVAL_FUSED", "1") != "0"
# minibatches of at most this many rows run the actor's and the critic's tail kernels on the
# two streams side by side (each tail then fills at most half of a 256-CU device:
# ceil(rows / 16 / 8) workgroups <= 128); TSRL_TAIL_SPLIT=0 keeps them on one stream,
# TSRL_TAIL_SPLIT_ROWS moves the threshold
TAIL_SPLIT_ROWS = int(os.environ.get("TSRL_TAIL_SPLIT_ROWS", "16384")) \
    if os.environ.get("TSRL_TAIL_SPLIT", "1") != "0" else 0


def _seq(mlp) -> Optional[list]:
    model = getattr(mlp, "model", None)
    return list(model) if isinstance(model, nn.Sequential) else None


def _trunk(net, D: int) -> Optional[list]:
    """[Linear(D,64), Tanh, Linear(64,64), Tanh] of a utils.net.Net, else None."""
    if getattr(net, "softmax", False) or getattr(net, "num_atoms", 1) != 1:
        return None
    mods = _seq(getattr(net, "model", None))
    if mods is None or len(mods) != 4:
        return None
    l1, a1, l2, a2 = mods
    if not (isinstance(l1, nn.Linear) and isinstance(l2, nn.Linear) and isinstance(a1, nn.Tanh)
            and isinstance(a2, nn.Tanh)):
        return None
    if l1.in_features != D or l1.out_features != HIDDEN or l2.in_features != HIDDEN or \
            l2.out_features != HIDDEN or l1.bias is None or l2.bias is None:
        return None
    return [l1, l2]


def match(actor, critic) -> Optional[Dict[str, nn.Linear]]:
    """The layers of a get_actor_critic-shaped actor/critic pair, or None."""
    from tianshou_amd.utils.net import ActorProb, Critic
    if not isinstance(actor, ActorProb) or not isinstance(critic, Critic):
        return None
    if actor._c_sigma or not actor._unbounded:
        return None
    l1 = getattr(actor.preprocess, "model", None)
    D = getattr(getattr(l1, "model", [None])[0], "in_features", None) if l1 is not None else None
    if not isinstance(D, int) or (D % 4 != 0 and not L1_X6):
        return None  # D % 4 != 0 runs on zero-padded rows (FusedActorCritic.rows), x6 only
    ta, tc = _trunk(actor.preprocess, D), _trunk(critic.preprocess, D)
    mu, last = _seq(actor.mu), _seq(critic.last)
    if ta is None or tc is None or mu is None or last is None or len(mu) != 1 or len(last) != 1:
        return None
    (h_a,), (h_c,) = mu, last
    if not (isinstance(h_a, nn.Linear) and isinstance(h_c, nn.Linear)):
        return None
    if h_a.in_features != HIDDEN or not 0 < h_a.out_features <= MAX_ACT or h_a.bias is None:
        return None
    if h_c.in_features != HIDDEN or h_c.out_features != 1 or h_c.bias is None:
        return None
    if actor.sigma_param.numel() != h_a.out_features:
        return None
    return {"w1a": ta[0], "w2a": ta[1], "w3a": h_a, "w1c": tc[0], "w2c": tc[1], "w3c": h_c,
            "D": D, "A": h_a.out_features, "sigma": actor.sigma_param}


class FusedActorCritic(FlatAdam):
    # data-parallel: the minibatch's loss partial sums ride after the flat gradients, so a
    # single all-reduce per minibatch carries both
    BUCKET_TAIL = 4 + MAX_ACT

    def __init__(self, layers: Dict, params) -> None:
        super().__init__(params)
        self.L = layers
        self.D = layers["D"]
        self.Dp = (self.D + 3) // 4 * 4  # row stride the kernels read (16-byte rows)
        self.A = layers["A"]
        self._bufs: Dict[str, torch.Tensor] = {}

    def _grads_bound(self) -> None:
        L = self.L
        g = lambda m: _C.ptr(m.grad)  # noqa: E731
        self._tail_grads = _C.TailGrads(
            g(L["w2a"].weight), g(L["w2a"].bias), g(L["w2c"].weight), g(L["w2c"].bias),
            g(L["w3a"].weight), g(L["w3a"].bias), g(L["w3c"].weight), g(L["w3c"].bias))
        self._tail_w = _C.TailWeights(
            _C.ptr(L["w2a"].weight), _C.ptr(L["w2a"].bias), _C.ptr(L["w2c"].weight),
            _C.ptr(L["w2c"].bias), _C.ptr(L["w3a"].weight), _C.ptr(L["w3a"].bias),
            _C.ptr(L["w3c"].weight), _C.ptr(L["w3c"].bias), _C.ptr(L["sigma"]))

    def clip_adam(self, max_norm: Optional[float], scale_grads: bool = True,
                  split_w1: bool = False) -> None:
        """FlatAdam.clip_adam; ``split_w1`` re-splits the updated first-layer weights into
        the bf16x6 planes the next minibatch's layer-1 kernels read (no split_w launch)."""
        sp = None
        if split_w1 and L1_X6:
            ws = self._buf("w1split", (int(_C.lib().tsrl_mlp_split_bytes(self.D)) + 3) // 4)
            sp = _C.W1Split(_C.ptr(ws), self.flat_offset(self.L["w1a"].weight),
                            self.flat_offset(self.L["w1c"].weight), self.D,
                            (self.D + 31) // 32 * 32)
        super().clip_adam(max_norm, scale_grads, sp)

    def _weights(self) -> "_C.TailWeights":
        L = self.L
        return _C.TailWeights(
            _C.ptr(L["w2a"].weight.detach()), _C.ptr(L["w2a"].bias.detach()),
            _C.ptr(L["w2c"].weight.detach()), _C.ptr(L["w2c"].bias.detach()),
            _C.ptr(L["w3a"].weight.detach()), _C.ptr(L["w3a"].bias.detach()),
            _C.ptr(L["w3c"].weight.detach()), _C.ptr(L["w3c"].bias.detach()),
            _C.ptr(L["sigma"].detach()))

    def _l1_fwd(self, xp, ldx, ip, m, out, frag_out: int, split: bool = True) -> None:
        """Layer 1 of both nets for m rows (X at xp, rows through ip when given)."""
        L, lib = self.L, _C.lib()
        s = _C.stream_ptr(self.params[0].device)
        D = self.D
        if L1_X6:
            ws = self._buf("w1split", (int(lib.tsrl_mlp_split_bytes(D)) + 3) // 4)
            if split:
                _C.check(lib.tsrl_mlp_split_w(_C.ptr(L["w1a"].weight), _C.ptr(L["w1c"].weight),
                                              D, _C.ptr(ws), s), "tsrl_mlp_split_w")
            _C.check(lib.tsrl_mlp_l1_fwd_x6(xp, ldx, ip, m, D, _C.ptr(ws),
                                            _C.ptr(L["w1a"].bias), _C.ptr(L["w1c"].bias), 1,
                                            out, frag_out, s), "tsrl_mlp_l1_fwd_x6")
            return
        _C.check(lib.tsrl_mlp_l1_fwd(xp, ldx, ip, m, D, _C.ptr(L["w1a"].weight),
                                     _C.ptr(L["w1a"].bias), _C.ptr(L["w1c"].weight),
                                     _C.ptr(L["w1c"].bias), 1, out, frag_out, s),
                 "tsrl_mlp_l1_fwd")

    def split_w1(self) -> None:
        """Split the current first-layer weights into the bf16x6 planes (tsrl_mlp_split_w)."""
        if not L1_X6:
            return
        L, lib = self.L, _C.lib()
        ws = self._buf("w1split", (int(lib.tsrl_mlp_split_bytes(self.D)) + 3) // 4)
        _C.check(lib.tsrl_mlp_split_w(_C.ptr(L["w1a"].weight), _C.ptr(L["w1c"].weight), self.D,
                                      _C.ptr(ws), _C.stream_ptr(self.params[0].device)),
                 "tsrl_mlp_split_w")

    def rows(self, obs: torch.Tensor, key: str = "xpad") -> torch.Tensor:
        """The observation rows as the kernels read them (row pitch = ``stride(0)``, the
        kernels' ldx): obs itself when its rows are contiguous, 16-byte aligned and at least
        roundup(D, 4) floats apart -- a padded VectorReplayBuffer storage view included (no
        copy; the kernels read no column past roundup(D, 4)) -- else a zero-padded
        [n, roundup(D, 4)] copy in a persistent buffer (stable address: the captured learn
        graph reads it)."""
        if (obs.dim() == 2 and obs.stride(1) == 1 and obs.stride(0) >= self.Dp and
                obs.stride(0) % 4 == 0 and obs.data_ptr() % 16 == 0 and obs.shape[0] > 0):
            return obs
        if self.Dp == self.D:
            return obs.contiguous()
        n = obs.shape[0]
        b = self._buf(key, n * self.Dp)[:n * self.Dp].view(n, self.Dp)
        b[:, self.D:].zero_()
        b[:, :self.D].copy_(obs)
        return b

    # -- forward-only evaluation (process_fn) ---------------------------------------------------
    EVAL_CHUNK = 1 << 21

    def evaluate(self, obs: torch.Tensor, act: Optional[torch.Tensor] = None,
                 idx: Optional[torch.Tensor] = None):
        """Critic values of the rows obs[idx] (all rows when idx is None) and, with act, the
        Gaussian log-prob of act[row] (a2c.py:83-100, ppo.py:95-96).  Per-row results do not
        depend on the chunking or on the other rows."""
        L, lib = self.L, _C.lib()
        dev = obs.device
        s = _C.stream_ptr(dev)
        D, A = self.D, self.A
        assert obs.dim() == 2 and obs.shape[1] == D
        obs = self.rows(obs, "xpad_eval")
        ldx = obs.stride(0)
        n = obs.shape[0] if idx is None else idx.numel()
        values = torch.empty(n, dtype=torch.float32, device=dev)
        logp = torch.empty(n, dtype=torch.float32, device=dev) if act is not None else None
        w = self._weights()
        if L1_X6 and EVAL_FUSED:
            # layer 1 + the evaluation in one launch over all rows (tsrl_ppo_eval_fused):
            # no layer-1 activations in memory, so no chunking either
            self.split_w1()
            ws = self._buf("w1split", (int(lib.tsrl_mlp_split_bytes(D)) + 3) // 4)
            nb = int(lib.tsrl_ppo_eval_fused_workspace_bytes())
            evw = self._buf("eval_ws", (nb + 3) // 4)
            _C.check(lib.tsrl_ppo_eval_fused(
                obs.data_ptr(), ldx, None if idx is None else idx.data_ptr(), n, D, _C.ptr(ws),
                _C.ptr(L["w1a"].bias), _C.ptr(L["w1c"].bias), w, A,
                None if act is None else act.data_ptr(), values.data_ptr(),
                None if logp is None else logp.data_ptr(), _C.ptr(evw), nb, s),
                "tsrl_ppo_eval_fused")
            return values, logp
        for s0 in range(0, n, self.EVAL_CHUNK):
            e0 = min(n, s0 + self.EVAL_CHUNK)
            m = e0 - s0
            h1 = self._buf("eval_h1", int(lib.tsrl_mlp_frag_floats(m)))
            if idx is None:
                xp, ip = obs.data_ptr() + s0 * ldx * 4, None
            else:
                xp, ip = obs.data_ptr(), idx.data_ptr() + s0 * 8
            self._l1_fwd(xp, ldx, ip, m, _C.ptr(h1), 1, split=(s0 == 0))
            ap = None
            if act is not None:
                ap = act.data_ptr() + s0 * A * 4
            _C.check(lib.tsrl_ppo_eval(_C.ptr(h1), m, w, A, ap, values.data_ptr() + s0 * 4,
                                       logp.data_ptr() + s0 * 4 if logp is not None else None,
                                       s), "tsrl_ppo_eval")
        return values, logp

    def _buf(self, key: str, numel: int, dtype=torch.float32) -> torch.Tensor:
        b = self._bufs.get(key)
        if b is None or b.numel() < numel or b.dtype != dtype:
            b = torch.empty(max(numel, 1), dtype=dtype, device=self.params[0].device)
            self._bufs[key] = b
        return b

    # -- advantage moments of a whole epoch ------------------------------------------------------
    def epoch_adv_moments(self, adv: torch.Tensor, idx: torch.Tensor, bounds: torch.Tensor,
                          max_seg: int, dp) -> torch.Tensor:
        """[n_minibatch, 2] f64 (sum adv, sum adv^2) of every minibatch of the epoch
        (bounds = device int64 [n_minibatch + 1] into idx), summed over the data-parallel
        ranks with ONE all-reduce per epoch (ppo.py:109-113 normalises per minibatch)."""
        lib = _C.lib()
        nseg = bounds.numel() - 1
        parts = int(lib.tsrl_adv_moments_seg_parts(max_seg))
        pa = self._buf("adv_seg_part", nseg * parts * 2, torch.float64)
        out = self._buf("adv_seg", nseg * 2, torch.float64)[:nseg * 2].view(nseg, 2)
        _C.check(lib.tsrl_adv_moments_seg(_C.ptr(adv), _C.ptr(idx), _C.ptr(bounds), nseg,
                                          max_seg, _C.ptr(pa), _C.ptr(out),
                                          _C.stream_ptr(adv.device)), "tsrl_adv_moments_seg")
        dp.all_reduce_(out, kind="adv_moments")
        return out

    # -- one minibatch --------------------------------------------------------------------------
    def minibatch(self, obs: torch.Tensor, idx: Optional[torch.Tensor], b: int,
                  act: torch.Tensor, logp_old: torch.Tensor, adv: torch.Tensor,
                  ret: torch.Tensor, v_s: torch.Tensor, params: "_C.PPOParams", dp,
                  adv_sums: Optional[torch.Tensor] = None, split_w: bool = True,
                  terms_out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Gradients of the minibatch loss into the parameters' .grad; returns the device
        tensor [loss, clip, vf, ent] (ppo.py:140-142).  ``obs`` are the rows of ``rows()``;
        ``adv_sums`` = this minibatch's row of epoch_adv_moments (computed here when None).
        Under data parallelism ONE all-reduce carries the gradients and the loss sums; a rank
        whose share of the global minibatch is empty (b == 0) contributes zeros.
        ``split_w=False``: the bf16x6 planes of W1 are already current (split_w1(), or the
        previous clip_adam(split_w1=True)).  ``terms_out``: a float32 [4] device tensor the
        single-process loss finalisation writes into (a captured epoch's per-minibatch row: no
        copy node per minibatch)."""
        self.bind_grads()
        L, lib = self.L, _C.lib()
        dev = obs.device
        s = _C.stream_ptr(dev)
        D, A = self.D, self.A
        assert obs.dim() == 2 and obs.stride(1) == 1 and obs.stride(0) >= self.Dp
        ldx = obs.stride(0)
        assert act.shape[-1] == A and act.is_contiguous()
        assert obs.shape[0] < 2 ** 32, "tsrl_mlp_dw: row indices must be < 2^32"
        ip = _C.ptr(idx) if idx is not None else None
        if b == 0:
            return self._empty_minibatch(params, dp, adv_sums)
        # advantage moments of the (global) minibatch
        if params.norm_adv and adv_sums is None:
            nblk = int(lib.tsrl_ppo_num_partials(b))
            pa = self._buf("adv_part", 2 * nblk, torch.float64)
            _C.check(lib.tsrl_adv_moments(_C.ptr(adv), ip, b, _C.ptr(pa), s), "tsrl_adv_moments")
            adv_sums = self._buf("adv_sums", 2, torch.float64)[:2]
            _C.check(lib.tsrl_reduce_partials(_C.ptr(pa), nblk, 2, _C.ptr(adv_sums), s),
                     "tsrl_reduce_partials")
            dp.all_reduce_(adv_sums, kind="adv_moments")
        h1 = self._buf("h1", int(lib.tsrl_mlp_frag_floats(b)))
        self._l1_fwd(_C.ptr_rows(obs), ldx, ip, b, _C.ptr(h1), 1, split=split_w)
        dz1 = self._buf("dz1", b * 2 * 64)
        sums = self._buf("sums", 4 + A, torch.float64)[:4 + A]
        wsb = int(lib.tsrl_ppo_tail_workspace_bytes(b))
        ws = self._buf("tail_ws", wsb, torch.uint8)
        args = (_C.ptr(h1), b, ip, self._tail_w, A, _C.ptr(act), _C.ptr(logp_old), _C.ptr(adv),
                _C.ptr(ret), _C.ptr(v_s), _C.ptr(adv_sums) if adv_sums is not None else None,
                params, _C.ptr(dz1), self._tail_grads, _C.ptr(sums), _C.ptr(ws), wsb)
        # single process: the loss finalisation rides the tail's reduction launch
        terms = None if dp.active else (
            terms_out if terms_out is not None else torch.empty(4, dtype=torch.float32,
                                                                device=dev))
        fin = (None, None, None) if terms is None else (
            _C.ptr(L["sigma"]), _C.ptr(terms), _C.ptr(L["sigma"].grad))
        side = self._side_stream(dev)
        if side is None:
            _C.check(lib.tsrl_ppo_tail_stage(*args, *fin, 3, s), "tsrl_ppo_tail_stage")
        else:
            cur = torch.cuda.current_stream(dev)
            if b <= TAIL_SPLIT_ROWS:
                # small minibatches: each net's tail fills at most half the CUs, so the
                # critic's runs on the second stream beside the actor's
                side.wait_stream(cur)
                _C.check(lib.tsrl_ppo_tail_stage(*args, *fin, 4, s), "tsrl_ppo_tail_stage")
                _C.check(lib.tsrl_ppo_tail_stage(*args, *fin, 8, side.cuda_stream),
                         "tsrl_ppo_tail_stage")
                cur.wait_stream(side)
            else:
                _C.check(lib.tsrl_ppo_tail_stage(*args, *fin, 1, s), "tsrl_ppo_tail_stage")
            # the tail's reduction only reads the tail kernels' slabs and dw only their dz1:
            # the reduction runs on a second stream beside the first-layer weight gradients
            side.wait_stream(cur)
            _C.check(lib.tsrl_ppo_tail_stage(*args, *fin, 2, side.cuda_stream),
                     "tsrl_ppo_tail_stage")
        wsb2 = int(lib.tsrl_mlp_dw_workspace_bytes(b, D))
        ws2 = self._buf("dw_ws", wsb2, torch.uint8)
        _C.check(lib.tsrl_mlp_dw(
            _C.ptr(dz1), _C.ptr_rows(obs), ldx, ip, b, D, _C.ptr(L["w1a"].weight.grad),
            _C.ptr(L["w1a"].bias.grad), _C.ptr(L["w1c"].weight.grad),
            _C.ptr(L["w1c"].bias.grad), _C.ptr(ws2), wsb2, s), "tsrl_mlp_dw")
        if side is not None:
            cur.wait_stream(side)
        if terms is not None:
            return terms
        return self._reduce_finalize(sums, params, dp)

    def _side_stream(self, dev) -> Optional[torch.cuda.Stream]:
        """The second stream of the tail/dw overlap (None when TSRL_TAIL_OVERLAP=0)."""
        if not TAIL_OVERLAP:
            return None
        st = getattr(self, "_side", None)
        if st is None or st.device != dev:
            st = self._side = torch.cuda.Stream(device=dev)
        return st

    def _empty_minibatch(self, params, dp, adv_sums) -> torch.Tensor:
        sums = self._buf("sums", 4 + self.A, torch.float64)[:4 + self.A]
        sums.zero_()
        self._flat.zero_()
        return self._reduce_finalize(sums, params, dp)

    def _reduce_finalize(self, sums: torch.Tensor, params, dp) -> torch.Tensor:
        """One all-reduce of [flat grads | loss sums] (sums travel as f32 in the bucket
        tail), then the loss terms and the log-std gradient from the global sums."""
        L, lib = self.L, _C.lib()
        dev = sums.device
        if dp.active:
            P, k = self._flat.numel(), sums.numel()
            bucket = self._bucket[:P + k]
            bucket[P:].copy_(sums)
            dp.all_reduce_(bucket, kind="grad")
            sums.copy_(bucket[P:])
        terms = torch.empty(4, dtype=torch.float32, device=dev)
        _C.check(lib.tsrl_ppo_gauss_finalize(
            _C.ptr(sums), self.A, _C.ptr(L["sigma"]), params, _C.ptr(terms),
            _C.ptr(L["sigma"].grad), _C.stream_ptr(dev)), "tsrl_ppo_gauss_finalize")
        return terms
