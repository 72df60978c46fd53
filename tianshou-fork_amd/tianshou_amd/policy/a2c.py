"""A2CPolicy (tianshou/policy/modelfree/a2c.py:14-160): critic values + GAE on device."""
import zlib
from typing import Any, Callable, Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from tianshou_amd import _C
from tianshou_amd.data.batch import Batch, split_indices
from tianshou_amd.dist import default_dp
from tianshou_amd.policy.base import gae_device
from tianshou_amd.policy.pg import PGPolicy
from tianshou_amd.utils.net import ActorCritic

# Critic/actor evaluation chunk for process_fn.  The reference chunks by max_batchsize
# (default 256, a2c.py:86-90) to bound host memory; per-row results do not depend on the
# chunking, and 288 GB of HBM makes 2M-row chunks cheap.
EVAL_CHUNK = 1 << 21


class A2CPolicy(PGPolicy):
    def __init__(self, actor: torch.nn.Module, critic: torch.nn.Module,
                 optim: torch.optim.Optimizer, dist_fn: Callable, vf_coef: float = 0.5,
                 ent_coef: float = 0.01, max_grad_norm: Optional[float] = None,
                 gae_lambda: float = 0.95, max_batchsize: int = 256, **kwargs: Any) -> None:
        super().__init__(actor, optim, dist_fn, **kwargs)
        self.critic = critic
        assert 0.0 <= gae_lambda <= 1.0, "GAE lambda should be in [0, 1]."
        self._lambda = gae_lambda
        self._weight_vf = vf_coef
        self._weight_ent = ent_coef
        self._grad_norm = max_grad_norm
        self._batch = max_batchsize
        self._actor_critic = ActorCritic(self.actor, self.critic)
        self.dp = default_dp()

    # -- process_fn -------------------------------------------------------------------------
    def process_fn(self, batch: Batch, buffer, indices: np.ndarray) -> Batch:
        batch = self._compute_returns(batch, buffer, indices)
        batch.act = torch.as_tensor(batch.act, device=batch.v_s.device).to(batch.v_s.dtype)
        return batch

    def _chunks(self, n: int, row_numel: int = 1):
        """Evaluation chunks: at most EVAL_CHUNK rows and 2**30 input elements per chunk (a
        conv trunk's activations are ~2x its uint8 frame stack per row in f32), rounded down
        to a power of two: the Nature-DQN trunk ran 0.385 us/row at the 38043-row chunk that
        the element bound gives for 4x84x84 frames and 0.306 at 32768 (MIOpen kernel choice,
        tools/atari_eval_chunk_probe.py)."""
        c = min(EVAL_CHUNK, (1 << 30) // max(int(row_numel), 1))
        c = max(self._batch, 1 << (max(c, 1).bit_length() - 1))
        return [(s, min(s + c, n)) for s in range(0, n, c)]

    def _values(self, obs: torch.Tensor) -> torch.Tensor:
        n = len(obs)
        out = torch.empty(n, dtype=torch.float32, device=obs.device)
        for s, e in self._chunks(n, obs[0].numel() if n else 1):
            out[s:e] = self.critic(obs[s:e]).flatten()
        return out

    def _eval_values(self, batch, obs, obs_next, buffer, indices):
        """V(s) and V(s') of a2c.py:86-93 (V(s') read from V(s) when obs_next rows are
        rows of obs, see _next_positions)."""
        v_s = self._values(obs)
        p = self._next_positions(buffer, indices, obs.device)
        return v_s, (v_s[p] if p is not None else self._values(obs_next))

    @staticmethod
    def _next_positions(buffer, indices, dev) -> Optional[torch.Tensor]:
        """Buffers that do not store obs_next (ignore_obs_next) return
        ``obs_next[i] = get(next(indices[i]), "obs")`` (base.py:380-381): byte for byte the
        ``obs`` row of the batch position j with ``indices[j] == next(indices[i])`` (stacked
        the same way, manager.py:279-297).  Returns those positions when every next-row is in
        the batch (always for sample(0)), else None.  Per-row critic outputs do not depend on
        the other rows, so ``V(obs_next) = V(obs)[p]``."""
        if getattr(buffer, "_save_obs_next", True) or not hasattr(buffer, "_step_dev") or \
                indices is None:
            return None
        idx = np.asarray(indices, np.int64).reshape(-1)
        n = len(idx)
        if n == 0:
            return None
        it = torch.as_tensor(idx % buffer.maxsize, device=dev)
        nxt = buffer._step_dev(it, -1)
        pos = torch.full((buffer.maxsize,), -1, dtype=torch.int64, device=dev)
        pos[it] = torch.arange(n, device=dev)
        p = pos[nxt]
        if bool((p < 0).any()):
            return None
        return p

    @staticmethod
    def _gae_layout(buffer, indices):
        """(row_len, end_extra): row_len > 0 when ``indices`` is the buffer's sample(0) order
        with equal per-env chunks (each env's chunk ends at its unfinished/done row, so every
        row_len-th element closes a segment); otherwise the reference's
        ``np.isin(indices, buffer.unfinished_index())`` mask on device."""
        ring = getattr(buffer, "_ring", None)
        if ring is not None and indices is getattr(buffer, "_last_sample0", None):
            row_len, _ = ring.chunk_layout()
            if row_len:
                return row_len, None
        mask = np.isin(np.asarray(indices), buffer.unfinished_index()).astype(np.uint8)
        return 0, torch.as_tensor(mask, device=buffer.device)

    def _sync_replicas(self) -> None:
        """Data parallel: rank 0's parameters on every rank before the first update (the
        process_fn evaluation and every later step then run on identical replicas)."""
        if self.dp.active and not getattr(self, "_replicas_synced", False):
            self.dp.broadcast_params_(self._actor_critic.parameters())
            self._replicas_synced = True

    def _shard_table(self, n: int, row_len: int, dev) -> dict:
        """Data parallel: every rank's row count, GAE row length and global np.random state
        hash, exchanged with ONE all-gather of three int64 per rank and one host read.
        process_fn makes it (``fresh``) and the update's learn() consumes it, so an update
        reads the shard layout from the host once: the ret_rms partial counts of every rank
        follow from it (no ragged length exchange), learn() checks the shared RandomState and
        whether the shards are equal with it."""
        st = np.random.get_state()
        h = zlib.crc32(np.ascontiguousarray(st[1]).tobytes() + int(st[2]).to_bytes(4, "little"))
        W = self.dp.world
        hs = self.dp.all_gather_cat(torch.tensor([h, n, row_len], dtype=torch.int64,
                                                 device=dev), kind="shard_table")
        hs = hs.view(W, 3).cpu()
        t = {"hash_equal": bool((hs[:, 0] == hs[0, 0]).all()), "n": hs[:, 1].tolist(),
             "row_len": hs[:, 2].tolist(), "n_local": n, "fresh": True}
        assert t["n"][self.dp.rank] == n
        self._shards = t
        return t

    def _learn_shards(self, n: int, dev) -> dict:
        """The shard table for this learn(): process_fn's of the same update if there is one,
        else a new exchange (learn() called on its own).  Consumed here: the next update makes
        its own."""
        t = getattr(self, "_shards", None)
        if t is None or not t["fresh"]:
            t = self._shard_table(n, 0, dev)
        elif t["n_local"] != n:
            raise RuntimeError(f"learn() got {n} rows, this update's process_fn "
                               f"{t['n_local']}")
        t["fresh"] = False
        return t

    def _require_equal_shards(self, n: int, dev, path: str) -> None:
        """Local minibatch splits (``split_indices`` over this rank's rows, b_global =
        world x local size) need every rank to hold the same row count: otherwise the ranks
        run different numbers of minibatches and their per-minibatch all-reduces stop
        matching (a hang, or mixed payloads).  Raise instead."""
        if not self.dp.active or self.dp.world == 1:
            return
        t = self._learn_shards(n, dev)
        if len(set(t["n"])) > 1:
            raise ValueError(
                f"{type(self).__name__}.{path}: unequal data-parallel shards {t['n']} rows per "
                f"rank; only the fused-MLP PPO update with dp_permutation='global' splits the "
                f"global batch -- give every rank the same number of envs and steps")

    def _compute_returns(self, batch: Batch, buffer, indices: np.ndarray) -> Batch:
        self._sync_replicas()
        obs = torch.as_tensor(batch.obs)
        dev = next(self.critic.parameters()).device
        obs = obs.to(dev)
        obs_next = torch.as_tensor(batch.obs_next).to(dev)
        with torch.no_grad():
            v_s, v_s_ = self._eval_values(batch, obs, obs_next, buffer, indices)
        batch.v_s = v_s
        rew = torch.as_tensor(batch.rew).to(dev, torch.float64).contiguous()
        term = torch.as_tensor(batch.terminated).to(dev).bool().contiguous()
        trunc = torch.as_tensor(batch.truncated).to(dev).bool().contiguous()
        row_len, extra = self._gae_layout(buffer, indices)
        n = len(v_s)
        tab = self._shard_table(n, row_len, dev) if self.dp.active else None
        if self._rew_norm:
            st = self.ret_rms.state
            scale = (st[1:2] + self._eps).sqrt()
            num = _C.lib().tsrl_gae_num_partials
            nparts = int(num(n, row_len))
            partials = torch.empty(max(nparts, 1) * 3, dtype=torch.float64, device=dev)
            adv, ret, _, _ = gae_device(v_s, v_s_, rew, term, trunc, self._gamma, self._lambda,
                                        row_len, extra, scale, ret_partials=partials)
            if self.dp.active:  # every rank folds every rank's partials in rank order
                # (unequal env shards give unequal partial counts, known from the table)
                counts = [3 * int(num(nr, rl)) for nr, rl in zip(tab["n"], tab["row_len"])]
                partials = self.dp.all_gather_known(partials[:nparts * 3], counts,
                                                    kind="ret_rms")
                nparts = partials.numel() // 3
            self.ret_rms.update_from_partials(partials, nparts)
        else:
            adv, ret, _, _ = gae_device(v_s, v_s_, rew, term, trunc, self._gamma, self._lambda,
                                        row_len, extra)
        batch.returns = ret
        batch.adv = adv
        return batch

    def learn(self, batch: Batch, batch_size: int, repeat: int, **kwargs: Any
              ) -> Dict[str, List[float]]:
        """a2c.py:119-160 (generic torch path on device)."""
        self._require_equal_shards(len(batch), next(self.critic.parameters()).device, "learn")
        losses, actor_losses, vf_losses, ent_losses = [], [], [], []
        for _ in range(repeat):
            for part in split_indices(len(batch), batch_size, True, True):
                minibatch = batch[part]
                dist = self(minibatch).dist
                log_prob = dist.log_prob(minibatch.act)
                log_prob = log_prob.reshape(len(minibatch.adv), -1).transpose(0, 1)
                actor_loss = -(log_prob * minibatch.adv).mean()
                value = self.critic(minibatch.obs).flatten()
                vf_loss = F.mse_loss(minibatch.returns, value)
                ent_loss = dist.entropy().mean()
                loss = actor_loss + self._weight_vf * vf_loss - self._weight_ent * ent_loss
                self.optim.zero_grad()
                loss.backward()
                self.dp.all_reduce_grads_(self._actor_critic.parameters(), average=True)
                if self._grad_norm:
                    nn.utils.clip_grad_norm_(self._actor_critic.parameters(),
                                             max_norm=self._grad_norm)
                self.optim.step()
                actor_losses.append(actor_loss.detach())
                vf_losses.append(vf_loss.detach())
                ent_losses.append(ent_loss.detach())
                losses.append(loss.detach())
        out = {}
        for k, v in (("loss", losses), ("loss/actor", actor_losses), ("loss/vf", vf_losses),
                     ("loss/ent", ent_losses)):
            out[k] = torch.stack(v).cpu().tolist() if v else []
        return out
