"""Collector (tianshou/data/collector.py:21-402) on device.

Two paths behind the reference API:

* fused (a ``DeviceVectorEnv``, optionally wrapped in ``VectorEnvNormObs``, no
  ``preprocess_fn``): every vector step is policy forward -> map_action -> env kernel (raw obs
  + column partials) -> obs_rms merge -> one ``tsrl_buffer_add`` launch that writes obs, act,
  rew, flags, env_id, the NORMALISED obs_next (into the buffer and into the live obs) and the
  episode statistics -> masked reset kernel for done envs (+ its obs_rms merge and
  normalisation).  No host<->device synchronisation inside an n_step collect; the returned
  statistics are gathered once at the end.
* generic (any other env): the reference's loop, with the buffer still in HBM.
"""
import ctypes
import time
import warnings
from typing import Any, Callable, Dict, Optional

import numpy as np
import torch

from tianshou_amd import _C
from tianshou_amd.data.batch import Batch
from tianshou_amd.data.buffer import ReplayBuffer, VectorReplayBuffer
from tianshou_amd.dist import LOG
from tianshou_amd.utils.capture import graph_capture
from tianshou_amd.env.synthetic import DeviceVectorEnv
from tianshou_amd.env.wrappers import VectorEnvNormObs


def _empty_data() -> Batch:
    return Batch(obs={}, act={}, rew={}, terminated={}, truncated={}, done={}, obs_next={},
                 info={}, policy={})


class Collector:
    def __init__(self, policy, env, buffer: Optional[ReplayBuffer] = None,
                 preprocess_fn: Optional[Callable[..., Batch]] = None,
                 exploration_noise: bool = False, sync_obs_rms: bool = True) -> None:
        """``sync_obs_rms`` (data-parallel runs only; default True): keep ONE global
        VectorEnvNormObs statistic across ranks -- the reference's single wrapper over all
        envs -- with one all-reduce of the step+reset batch moments per env step (captured
        into the collect HIP graphs when the backend is RCCL; eager steps over gloo).  False:
        each rank's env shard normalises with its own running statistics."""
        self.env = env
        self.env_num = len(env)
        self.exploration_noise = exploration_noise
        self.policy = policy
        self.preprocess_fn = preprocess_fn
        self._action_space = env.action_space
        self._norm = env if isinstance(env, VectorEnvNormObs) else None
        self._base = env.venv if self._norm is not None else env
        self._fused = isinstance(self._base, DeviceVectorEnv) and preprocess_fn is None
        self.device = getattr(self._base, "device", None)
        self._assign_buffer(buffer)
        if getattr(self.buffer, "_prioritized", False):
            # prioritized buffers initialise a priority per added row (prio.py:50-57): the
            # generic path's buffer.add does that; the fused step writes rows directly
            self._fused = False
        self._scratch = None
        # vector steps per captured HIP graph (0 disables graph replay of the fused step)
        self.graph_steps = 64
        self._graphs = {}  # captured collect graphs by step count
        # run the policy step as the fused HIP kernel when the policy offers one
        self.use_fused_act = True
        self._fused_act_on = False
        # one launch per vector step (csrc/collect.hip) when env, normalisation and actor
        # allow it; _pending = the buffer add of the previous step, run by the next step's
        # launch or by _flush()
        self.use_fused_step = True
        self._step_on = False
        # CollectArgs of the last fused step whose obs_rms merge is still deferred (None: none)
        self._rms_chain = None
        self._rms_step = 0  # index of the next deferred launch in its chain
        self._pending = None
        # exact_obs_rms on the fused step with the action-independent env: the reference's
        # f32 statistic of step i runs on a second graph branch while the step launches go on,
        # its env rows computed this many launches ahead (csrc/collect.hip E; 0: the serial
        # form, one tsrl_rms_exact_update between launches)
        self.exact_pipeline = 5
        # statistics launches in flight at once (side streams); with groups of 2 one branch
        # (a group's workgroups already fill the room beside the step launches)
        self.exact_branches = 2
        # steps per statistics launch (tsrl_rms_exact_stats_n; <= exact_pipeline - 1): one
        # cross-branch graph edge per group.  Headline shape, collect per 2048 steps
        # (profiles/r05_xpipe_ab.log): depth 2 / group 1 / 2 branches 79 ms, depth 4 / group 2
        # 69, depth 5 / group 2 65, depth 6 / group 2 69, group 3 86, serial 142
        self.exact_group = 2
        self._xp_streams = None
        self._xp_keep = []
        from tianshou_amd.dist import default_dp
        self.dp = default_dp()
        if sync_obs_rms and self.dp.active and self._norm is not None:
            self._norm.obs_rms.sync_with(self.dp)
            if not self.dp.capturable:
                self.graph_steps = 0
        self.reset(False)

    def _assign_buffer(self, buffer) -> None:
        if buffer is None:
            buffer = VectorReplayBuffer(self.env_num, self.env_num, device=self.device)
        elif type(buffer) is ReplayBuffer or (isinstance(buffer, ReplayBuffer)
                                              and buffer.buffer_num == 1 and self.env_num > 1):
            if self.env_num > 1:
                raise TypeError(
                    f"Cannot use ReplayBuffer(size={buffer.maxsize}, ...) to collect "
                    f"{self.env_num} envs,\n\tplease use VectorReplayBuffer(total_size="
                    f"{buffer.maxsize}, buffer_num={self.env_num}, ...) instead.")
        else:
            assert buffer.buffer_num >= self.env_num
        if buffer.device is None and self.device is not None:
            buffer.device = self.device
        self.buffer = buffer

    # -- resets ---------------------------------------------------------------------------------
    def reset(self, reset_buffer: bool = True,
              gym_reset_kwargs: Optional[Dict[str, Any]] = None) -> None:
        self.data = _empty_data()
        self.reset_env(gym_reset_kwargs)
        if reset_buffer:
            self.reset_buffer()
        self.reset_stat()

    def reset_stat(self) -> None:
        self.collect_step, self.collect_episode, self.collect_time = 0, 0, 0.0

    def reset_buffer(self, keep_statistics: bool = False) -> None:
        self.buffer.reset(keep_statistics=keep_statistics)

    def _alloc_scratch(self) -> None:
        if self._scratch is not None:
            return
        b, N = self._base, self.env_num
        dev = b.device
        self._scratch = dict(
            cur=b.alloc_obs(N) if b.u8 else torch.empty((N,) + b.obs_shape, device=dev),
            raw=b.alloc_obs(N),
            reset_raw=b.alloc_obs(N),
            rew=torch.empty(N, dtype=torch.float64, device=dev),
            term=torch.empty(N, dtype=torch.bool, device=dev),
            trunc=torch.empty(N, dtype=torch.bool, device=dev),
            done=torch.empty(N, dtype=torch.bool, device=dev),
            part=b.alloc_partials(N),
            part2=b.alloc_partials(N),
            env_id=torch.arange(N, device=dev),
        )
        act_shape, act_dtype = self._act_spec()
        nblk = b.nblk_for(N)
        self._scratch["blk_done"] = torch.zeros(max(nblk, 1), dtype=torch.float64, device=dev)
        # ping-pong step counters [slot][ring cursor, noise counter]: step i reads slot i%2
        # and writes slot (i+1)%2, so graph-captured steps need no atomics or extra launches
        self._scratch["step_ctr"] = torch.zeros((2, 2), dtype=torch.int64, device=dev)
        self._parity = 0
        self._scratch["act"] = torch.empty((N,) + act_shape, dtype=act_dtype, device=dev)
        self._scratch["act_remap"] = torch.empty((N,) + act_shape, dtype=act_dtype, device=dev)

    def reset_env(self, gym_reset_kwargs: Optional[Dict[str, Any]] = None) -> None:
        if not self._fused:
            gym_reset_kwargs = gym_reset_kwargs or {}
            obs, info = self.env.reset(**gym_reset_kwargs)
            if self.preprocess_fn:
                processed = self.preprocess_fn(obs=obs, info=info,
                                               env_id=np.arange(self.env_num))
                obs = processed.get("obs", obs)
                info = processed.get("info", info)
            self.data.info = info
            self.data.obs = obs
            return
        self._alloc_scratch()
        s, b, N = self._scratch, self._base, self.env_num
        b._reset_raw(None, None, N, s["raw"], s["part"])
        self._finish_obs(s["raw"], s["cur"], s["part"], None, N)
        self.data.obs = s["cur"]
        self.data.info = Batch(env_id=s["env_id"])

    def _finish_obs(self, raw, cur, partials, mask, k) -> None:
        """obs_rms update + normalisation of (masked) raw rows into ``cur``."""
        if self._norm is not None and not self._base.u8:
            rms = self._norm.obs_rms
            if self._norm.update_obs_rms:
                if rms.exact:
                    rms.exact_update(raw[:k], None if mask is None else mask[:k])
                else:
                    rms.merge_partials(partials, self._base.nblk_for(k), mask, k)
            rms.norm_rows(raw.reshape(k, -1), cur.reshape(k, -1), mask)
        elif mask is None:
            cur.copy_(raw)
        else:
            m = mask.view((k,) + (1,) * (raw.dim() - 1))
            torch.where(m, raw, cur, out=cur)

    # -- collect ----------------------------------------------------------------------------------
    def collect(self, n_step: Optional[int] = None, n_episode: Optional[int] = None,
                random: bool = False, render: Optional[float] = None, no_grad: bool = True,
                gym_reset_kwargs: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
        assert not self.env.is_async, "Please use AsyncCollector if using async venv."
        if n_step is not None:
            assert n_episode is None, (
                f"Only one of n_step or n_episode is allowed in Collector."
                f"collect, got n_step={n_step}, n_episode={n_episode}.")
            assert n_step > 0
            if not n_step % self.env_num == 0:
                warnings.warn(
                    f"n_step={n_step} is not a multiple of #env ({self.env_num}), "
                    "which may cause extra transitions collected into the buffer.")
        elif n_episode is not None:
            assert n_episode > 0
        else:
            raise TypeError("Please specify at least one (either n_step or n_episode) "
                            "in AsyncCollector.collect().")
        start_time = time.time()
        if self._fused:
            step_count, episode_count, rews, lens, idxs = self._collect_fused(
                n_step, n_episode, random, no_grad)
        else:
            step_count, episode_count, rews, lens, idxs = self._collect_generic(
                n_step, n_episode, random, render, no_grad, gym_reset_kwargs)
        self.collect_step += step_count
        self.collect_episode += episode_count
        self.collect_time += max(time.time() - start_time, 1e-9)
        if n_episode:
            self.data = _empty_data()
            self.reset_env()
        if episode_count > 0:
            rew_mean, rew_std = rews.mean(), rews.std()
            len_mean, len_std = lens.mean(), lens.std()
        else:
            rews, lens, idxs = np.array([]), np.array([], int), np.array([], int)
            rew_mean = rew_std = len_mean = len_std = 0
        return {"n/ep": episode_count, "n/st": step_count, "rews": rews, "lens": lens,
                "idxs": idxs, "rew": rew_mean, "len": len_mean, "rew_std": rew_std,
                "len_std": len_std}

    def _policy_act(self, obs, info, random: bool, no_grad: bool, k: int, ids=None):
        if random:
            # collector.py:262-266: one sample per READY env from that env's own space
            ids = range(k) if ids is None else ids
            try:
                acts = [self._action_space[i].sample() for i in ids]
            except TypeError:
                acts = [self._action_space.sample() for _ in range(k)]
            act = torch.as_tensor(np.asarray(acts), device=self.device)
            if hasattr(self.policy, "map_action_inverse"):
                act = self.policy.map_action_inverse(act)
            return act, Batch()
        data = Batch(obs=obs, info=info)
        if no_grad:
            with torch.no_grad():
                result = self.policy(data, None)
        else:
            result = self.policy(data, None)
        act = result.act
        if self.exploration_noise:
            act = self.policy.exploration_noise(act, data)
        policy = result.get("policy", Batch())
        return act, policy

    def _noise_active(self) -> bool:
        """exploration_noise=True with a policy that keeps BasePolicy.exploration_noise (the
        identity, base.py:121-133; every on-policy algorithm, e.g. examples/atari/atari_ppo.py's
        Collector(..., exploration_noise=True)) changes nothing, so such steps stay eligible
        for the fused act kernel and HIP-graph replay."""
        if not self.exploration_noise:
            return False
        from tianshou_amd.policy.base import BasePolicy
        return type(self.policy).exploration_noise is not BasePolicy.exploration_noise

    # -- fused device path ------------------------------------------------------------------
    def _act_spec(self):
        act_space = self._action_space
        if isinstance(act_space, (list, tuple)):  # host vector envs: one space per env
            act_space = act_space[0]
        if hasattr(act_space, "n"):
            return (), torch.int64
        return tuple(act_space.shape), torch.float32

    def _fused_step_ok(self, n_step, kk) -> bool:
        """The one-launch step (tsrl_collect_box_step) applies: n_step collects over every env
        of a SyntheticVectorEnv with Box rows under an updating VectorEnvNormObs, and the
        fused Gaussian act."""
        from tianshou_amd.env.synthetic import SyntheticVectorEnv
        b, norm = self._base, self._norm
        if not (self.use_fused_step and self._fused_act_on and n_step is not None
                and kk == self.env_num == self.buffer.buffer_num):
            return False
        if not isinstance(b, SyntheticVectorEnv) or b.u8 or norm is None or \
                not norm.update_obs_rms:
            return False
        D = b.obs_numel
        if D > 512 or self._act_spec()[1] != torch.float32:
            return False
        # the exact int64 obs_rms moments (csrc/collect.hip D): a row adds <= 2^46 to a
        # column's sum of squares, so the rows summed into one totals slot -- every rank's
        # after the data-parallel all-reduce -- must stay <= 2^17
        rms = norm.obs_rms
        world = rms.dp.world if (rms.dp is not None and rms.dp.active) else 1
        if kk * world > 1 << 17 and b.act_coef == 0.0:
            return False
        if b.act_coef != 0.0 and self._act_spec()[0] != (b.act_dim,):
            return False
        buf = self.buffer
        buf._alloc_storage(b.obs_shape, b.obs_torch_dtype, *self._act_spec())
        m = buf._meta
        if getattr(buf, "stack_num", 1) != 1 or m.obs.dtype != torch.float32 or \
                m.obs[0].numel() != D:
            return False
        sc = self._scratch["step_ctr"]
        return bool(self.policy.fused_collect_fill(_C.CollectArgs(), (sc[0, 1:2], sc[1, 1:2])))

    def _fused_box_step(self, cur, kk, add_kw, xp=None) -> None:
        """One vector step as one launch: the pending add of the previous step, policy act,
        env step + auto-reset, both obs_rms updates (csrc/collect.hip).  This step's add is
        left pending for the next launch or _flush().  ``xp``: launch i of a pipelined exact
        chain (see _xpipe_steps): dict(i, stats_prev, spec, rows, reset_rows)."""
        s, b, buf = self._scratch, self._base, self.buffer
        rms = self._norm.obs_rms
        rms.ensure_snapshot()
        ws = s.get("collect_ws")
        if ws is None:
            nbytes = int(_C.lib().tsrl_collect_workspace_bytes(kk, b.obs_numel))
            ws = s["collect_ws"] = torch.zeros(nbytes, dtype=torch.uint8, device=b.device)
        p, sc = self._parity, s["step_ctr"]
        c = _C.CollectArgs()
        if self._pending is not None:
            c.add = self._pending
        c.k, c.dim, c.cur = kk, b.obs_numel, _C.ptr(cur)
        # this step's stored obs rows come from the launch itself (the live obs never
        # round-trips through HBM between fused steps); the adds then copy no obs
        c.obs_dst, c.obs_offset = _C.ptr_rows(buf._meta.obs), _C.ptr(buf._dev["offset"])
        c.obs_pitch = buf._meta.obs.stride(0)  # padded storage rows (buffer.py obs_storage)
        c.obs_rel_dev = _C.ptr(add_kw.get("rel_dev"))
        c.obs_uniform_rel = int(add_kw.get("uniform_rel", 0))
        assert self.policy.fused_collect_fill(c, (sc[p, 1:2], sc[1 - p, 1:2]))
        c.act, c.act_remap = _C.ptr(s["act"]), _C.ptr(s["act_remap"])
        c.env_seed, c.ep_len = b.seed_, b.ep_len
        c.act_coef = b.act_coef  # != 0: the action-coupled env (env after the actor, f64 moments)
        c.ep_j, c.ep_t = _C.ptr(b.ep_j), _C.ptr(b.ep_t)
        c.raw, c.reset_raw = _C.ptr(s["raw"]), _C.ptr(s["reset_raw"])
        c.rew, c.term, c.trunc, c.done = (_C.ptr(s[x]) for x in ("rew", "term", "trunc", "done"))
        c.workspace = _C.ptr(ws)
        c.mean, c.var, c.count = _C.ptr(rms.mean_t), _C.ptr(rms.var_t), _C.ptr(rms.count_t)
        c.snap_mean, c.snap_var = _C.ptr(rms.snap_mean_t), _C.ptr(rms.snap_var_t)
        dp = rms.dp is not None and rms.dp.active
        obs_next, reset_src = s["raw"], s["reset_raw"]
        if xp is not None:
            # pipelined exact obs_rms: merge step i - 1's batch moments in the prologue, write
            # the spec env's rows of step i + d, read this step's rows from the ring slot
            c.xpipe, c.rms_step = 1, xp["i"]
            c.xstats = _C.ptr(xp["stats_prev"])
            if xp["spec"] is not None:
                sj, st_, sraw, sreset, sdone = xp["spec"]
                c.spec_j, c.spec_t = _C.ptr(sj), _C.ptr(st_)
                c.spec_raw, c.spec_reset_raw, c.spec_done = (_C.ptr(sraw), _C.ptr(sreset),
                                                             _C.ptr(sdone))
            obs_next, reset_src = xp["rows"], xp["reset_rows"]
        elif rms.exact:
            # the launch computes no moments; the exact f32 update runs after it (below)
            c.no_moments = 1
        if xp is None:
            c.rms_step = 0 if rms.exact else self._rms_step
        _C.check(_C.lib().tsrl_collect_box_step(c, _C.stream_ptr(b.device)),
                 "tsrl_collect_box_step")
        if dp and not rms.exact:
            # the step's exact integer moments summed over the ranks (one all-reduce per env
            # step, a graph node under RCCL); the next launch merges the GLOBAL batch, as the
            # reference's single VectorEnvNormObs over every env shard (venv_wrappers.py:93-99)
            # (the slot carries its own step-row count, so unequal env shards merge right)
            off = int(_C.lib().tsrl_collect_totals_offset(self._rms_step))
            n = 4 * b.obs_numel + 2
            rms.dp.all_reduce_(ws[off:off + 8 * n].view(torch.float64 if b.act_coef
                                                        else torch.int64), kind="obs_rms")
        # deferred merge: the next launch (or _flush's tsrl_collect_rms_finalize) merges this
        # step's obs_rms moments
        self._rms_chain = None if rms.exact else c
        self._rms_step = 0 if rms.exact else self._rms_step + 1
        if rms.exact and xp is None:
            # both updates from the raw step / reset rows the launch wrote, in the
            # reference's f32 arithmetic
            rms.exact_update(s["raw"][:kk], None, s["reset_raw"][:kk], s["done"][:kk],
                             snapshot=True)
        self._pending = buf._launch_add(
            ids=None, k=kk, obs=None, act=s["act"], obs_next=obs_next, cur_obs=cur, norm=rms,
            norm_snapshot=True, reset_src=reset_src, reset_mask=s["done"], reset_norm=rms,
            rew=s["rew"], term=s["term"], trunc=s["trunc"], launch=False, **add_kw)
        self._parity ^= 1
        return c

    # -- pipelined exact obs_rms (csrc/collect.hip E) ---------------------------------------------
    def _xpipe_ok(self) -> bool:
        """exact_obs_rms on the one-launch step with the action-independent env (rows of a
        multiple of 4 floats, one process): its f32 statistic can run beside the launches."""
        if not (self.exact_pipeline and self._step_on and self._norm is not None):
            return False
        rms, b = self._norm.obs_rms, self._base
        return bool(rms.exact and b.act_coef == 0.0 and b.obs_numel % 4 == 0
                    and not (rms.dp is not None and rms.dp.active))

    def _xpipe_scratch(self) -> None:
        """Ring of d + 2 slots (a step's env rows, reset rows, done flags, batch moments),
        the spec env counters and the side streams of the statistics branches."""
        s, b = self._scratch, self._base
        d = int(self.exact_pipeline)
        nsl, k, D, dev = d + 2, self.env_num, b.obs_numel, b.device
        if s.get("xp_raw") is None or s["xp_raw"].shape[0] != nsl:
            s["xp_raw"] = torch.empty((nsl, k, D), device=dev)
            s["xp_reset"] = torch.empty((nsl, k, D), device=dev)
            s["xp_done"] = torch.zeros((nsl, k), dtype=torch.uint8, device=dev)
            nb = -(-int(_C.lib().tsrl_rms_exact_stats_bytes(D)) // 256) * 256
            s["xp_stats"] = torch.zeros((nsl, nb), dtype=torch.uint8, device=dev)
            s["xp_spec"] = torch.zeros((2, k), dtype=torch.int64, device=dev)
        nbr = max(1, min(int(self.exact_branches), d))
        if self._xpipe_group() > 1:
            nbr = 1  # a group's workgroups already fill the room beside the step launches
        if self._xp_streams is None or len(self._xp_streams) != nbr:
            self._xp_streams = [torch.cuda.Stream(device=dev) for _ in range(nbr)]

    def _xpipe_steps(self, G: int, sc) -> None:
        """G fused steps with the exact statistic pipelined (inside a graph capture): the spec
        env computes step j's rows d launches before launch j + 1 needs their statistic; the
        statistics of m = exact_group consecutive steps run as ONE tsrl_rms_exact_stats_n
        launch (on side stream q % exact_branches for group q) after the launch (or the
        head's tsrl_collect_spec_step) that wrote the group's last rows; launch j + 1 waits
        for its group (one cross-branch graph edge per group, not per step) and merges step
        j's; tsrl_collect_xpipe_finalize merges the last step's, then _flush runs its add."""
        s, b = self._scratch, self._base
        lib = _C.lib()
        d, m = int(self.exact_pipeline), self._xpipe_group()
        nsl, k, D = d + 2, self.env_num, b.obs_numel
        main = torch.cuda.current_stream(b.device)
        raw, rst, dn, st, spec = (s[x] for x in ("xp_raw", "xp_reset", "xp_done", "xp_stats",
                                                 "xp_spec"))
        ev_group = {}
        # the events outlive the capture (destroyed before the next one begins, not inside it)
        keep = self._xp_keep

        def spec_of(j):
            return spec[0], spec[1], raw[j % nsl], rst[j % nsl], dn[j % nsl]

        def group_stats(q):  # the rows of group q's steps are written (on main)
            steps = range(m * q, min(m * q + m, G))
            ev = torch.cuda.Event()
            ev.record(main)
            side = self._xp_streams[q % len(self._xp_streams)]
            side.wait_event(ev)
            keep.append(ev)
            n = len(steps)
            arr = lambda ts: (ctypes.c_void_p * n)(*[_C.ptr(t) for t in ts])  # noqa: E731
            _C.check(lib.tsrl_rms_exact_stats_n(
                n, arr([raw[j % nsl] for j in steps]), arr([rst[j % nsl] for j in steps]),
                arr([dn[j % nsl] for j in steps]), k, D, arr([st[j % nsl] for j in steps]),
                side.cuda_stream), "tsrl_rms_exact_stats_n")
            ev_group[q] = torch.cuda.Event()
            ev_group[q].record(side)
            keep.append(ev_group[q])

        def rows_written(j):  # step j's rows now exist: launch its group once complete
            if j == G - 1 or (j + 1) % m == 0:
                group_stats(j // m)

        for j in range(min(d, G)):
            c = _C.CollectArgs()
            c.k, c.dim, c.env_seed, c.ep_len = k, D, b.seed_, b.ep_len
            c.ep_j, c.ep_t = _C.ptr(b.ep_j), _C.ptr(b.ep_t)
            c.spec_j, c.spec_t, c.spec_raw, c.spec_reset_raw, c.spec_done = (
                _C.ptr(x) for x in spec_of(j))
            _C.check(lib.tsrl_collect_spec_step(c, int(j == 0), main.cuda_stream),
                     "tsrl_collect_spec_step")
            rows_written(j)
        c = None
        for i in range(G):
            if i > 0 and (i - 1) % m == 0:  # the group of step i - 1 (later members: waited)
                main.wait_event(ev_group[(i - 1) // m])
            xp = dict(i=i, stats_prev=st[(i - 1) % nsl] if i > 0 else None,
                      spec=spec_of(i + d) if i + d < G else None, rows=raw[i % nsl],
                      reset_rows=rst[i % nsl])
            c = self._fused_box_step(self._scratch["cur"], k, dict(
                rel_dev=sc[i % 2, 0:1], rel_next=sc[(i + 1) % 2, 0:1]), xp=xp)
            if i + d < G:
                rows_written(i + d)
        if (G - 1) % m == 0:  # the last step opens its group: no launch waited for it
            main.wait_event(ev_group[(G - 1) // m])
        c.xstats = _C.ptr(st[(G - 1) % nsl])
        _C.check(lib.tsrl_collect_xpipe_finalize(c, main.cuda_stream),
                 "tsrl_collect_xpipe_finalize")
        self._flush()
        for side in self._xp_streams[:min(len(self._xp_streams), -(-G // m))]:  # join forks
            ev = torch.cuda.Event()
            ev.record(side)
            main.wait_event(ev)
            keep.append(ev)

    def _xpipe_group(self) -> int:
        """Steps per statistics launch: the group's last rows must exist d launches before
        its first step's statistic is merged, so m <= d - 1 (m = 1 below depth 2), and one
        tsrl_rms_exact_stats_n launch carries at most tsrl_rms_exact_stats_max_steps() steps."""
        return max(1, min(int(self.exact_group), int(self.exact_pipeline) - 1,
                          int(_C.lib().tsrl_rms_exact_stats_max_steps())))

    def _flush(self) -> None:
        """Run the pending buffer add of the last fused step (tsrl_buffer_add), after merging
        that step's deferred obs_rms moments (tsrl_collect_rms_finalize)."""
        if self._rms_chain is not None:
            c, self._rms_chain = self._rms_chain, None
            self._rms_step = 0
            _C.check(_C.lib().tsrl_collect_rms_finalize(c, _C.stream_ptr(self.buffer.device)),
                     "tsrl_collect_rms_finalize")
        if self._pending is not None:
            a, self._pending = self._pending, None
            _C.check(_C.lib().tsrl_buffer_add(a, _C.stream_ptr(self.buffer.device)),
                     "tsrl_buffer_add")

    def _device_step(self, cur, kk, ids_t, random, no_grad, add_kw) -> None:
        """All device work of one vector step: policy -> map_action -> env kernel (+ column
        partials) -> obs_rms merge -> buffer add (+ fused obs_next normalisation) -> masked
        reset (+ merge + normalisation).  No host synchronisation, so the sequence can be
        captured in a HIP graph."""
        if self._step_on and not random and ids_t is None and kk == self.env_num:
            self._fused_box_step(cur, kk, add_kw)
            return
        self._flush()
        s, b, buf = self._scratch, self._base, self.buffer
        act_shape, act_dtype = self._act_spec()
        if self._fused_act_on and not random:
            # policy forward + sampling + map_action as one kernel (policy/fused_act.py)
            act, action_remap = s["act"][:kk], s["act_remap"][:kk]
            p = self._parity
            sc = s["step_ctr"]
            self.policy.fused_act(cur, act, action_remap, (sc[p, 1:2], sc[1 - p, 1:2]))
        else:
            info = Batch(env_id=s["env_id"][:kk] if ids_t is None else ids_t)
            act, _policy = self._policy_act(cur, info, random, no_grad, kk)
            act = act.to(act_dtype).reshape((kk,) + act_shape).contiguous()
            action_remap = self.policy.map_action(act)
        raw, rew = s["raw"][:kk], s["rew"][:kk]
        term, trunc, done = s["term"][:kk], s["trunc"][:kk], s["done"][:kk]
        norm_obj = self._norm
        if ids_t is None and not b.u8 and getattr(b, "supports_step_reset", False):
            # step + auto-reset (one env launch), both obs_rms updates (one launch; data
            # parallel: + one all-reduce), buffer add with the step/reset normalisation and
            # the ring advance (one launch)
            upd = norm_obj is not None and norm_obj.update_obs_rms
            blk = s["blk_done"]
            b._step_reset_raw(kk, raw, s["reset_raw"][:kk], rew, term, trunc, done,
                              s["part"] if upd else None, s["part2"] if upd else None,
                              blk if upd else None, action=action_remap)
            rms = norm_obj.obs_rms if norm_obj is not None else None
            if upd and rms.exact:
                rms.exact_update(raw, None, s["reset_raw"][:kk], done, snapshot=True)
            elif upd:
                rms.merge2(s["part"], s["part2"], blk, b.nblk_for(kk), kk)
            kw = dict(add_kw)
            buf._launch_add(ids=None, k=kk, obs=cur, act=act, obs_next=raw, cur_obs=cur,
                            norm=rms, norm_snapshot=upd, reset_src=s["reset_raw"][:kk],
                            reset_mask=done, reset_norm=rms, rew=rew, term=term, trunc=trunc,
                            **kw)
            self._parity ^= 1
            return
        b._step_raw(ids_t, kk, raw, rew, term, trunc, s["part"], action_remap)
        norm = None
        if self._norm is not None and not b.u8:
            if self._norm.update_obs_rms:
                if self._norm.obs_rms.exact:
                    self._norm.obs_rms.exact_update(raw)
                else:
                    self._norm.obs_rms.merge_partials(s["part"], b.nblk_for(kk), None, kk)
            norm = self._norm.obs_rms
        if b.u8:
            buf._launch_add(ids=ids_t, k=kk, obs=cur, act=act, obs_next_raw=raw, rew=rew,
                            term=term, trunc=trunc, **add_kw)
            cur.copy_(raw)
        else:
            buf._launch_add(ids=ids_t, k=kk, obs=cur, act=act, obs_next=raw, cur_obs=cur,
                            norm=norm, rew=rew, term=term, trunc=trunc, **add_kw)
        torch.logical_or(term, trunc, out=done)
        if b.u8:
            # the reset kernel writes only the finished envs' rows: straight into cur (which
            # now holds the stepped rows), no masked select pass over all rows
            b._reset_raw(ids_t, done, kk, cur, s["part2"])
        else:
            b._reset_raw(ids_t, done, kk, s["reset_raw"][:kk], s["part2"])
            self._finish_obs(s["reset_raw"][:kk], cur, s["part2"], done, kk)
        self._parity ^= 1

    def _graph_key(self, G: int):
        buf, b = self.buffer, self._base
        ptrs = [t.data_ptr() for t in buf._meta.values() if isinstance(t, torch.Tensor)]
        ptrs += [t.data_ptr() for t in buf._dev.values()]
        ptrs += [b.ep_j.data_ptr(), b.ep_t.data_ptr()]
        ptrs += [t.data_ptr() for t in self._scratch.values() if isinstance(t, torch.Tensor)]
        ptrs += [p.data_ptr() for p in self.policy.parameters()]
        if self._norm is not None:
            r = self._norm.obs_rms
            ptrs += [r.mean_t.data_ptr(), r.var_t.data_ptr(), r.count_t.data_ptr(),
                     self._norm.update_obs_rms]
        return (G, self.policy.training, self.exploration_noise, self._fused_act_on,
                self._step_on, (self.exact_pipeline, self.exact_branches, self._xpipe_group())
                if self._xpipe_ok() else 0, tuple(ptrs))

    def _replay_steps(self, no_grad, n_steps: int, written: list) -> int:
        """Run up to n_steps uniform steps as replays of captured HIP graphs of G steps
        (graph_steps, then one shorter even-length graph for the remainder, each captured
        once per shape); returns the number of steps done (the rest, at most one step, is
        left to the eager loop)."""
        Gmax = self.graph_steps
        assert Gmax % 2 == 0, "graph_steps must be even (ping-pong step counters)"
        if n_steps < 2:
            return 0
        buf = self.buffer
        self._flush()
        sc = self._scratch["step_ctr"]
        if self._parity:  # the live counters sit in slot 1: the graph starts from slot 0
            sc[0].copy_(sc[1])
            self._parity = 0
        if getattr(self, "_graphs", None) is None:
            self._graphs = {}
        sc[0, 0].fill_(int(buf._ring.index[0]))
        done = 0
        xpipe = self._xpipe_ok()
        if xpipe:
            self._xpipe_scratch()
        self._xp_keep = []
        while n_steps - done >= 2:
            G = min(Gmax, (n_steps - done) // 2 * 2)
            key = self._graph_key(G)
            graph = self._graphs.get(G)
            if graph is None or graph[0] != key:
                g = torch.cuda.CUDAGraph()
                torch.cuda.synchronize()
                LOG.capture_begin()
                with graph_capture(g):
                    if xpipe:
                        self._xpipe_steps(G, sc)
                    else:
                        for i in range(G):
                            self._device_step(self._scratch["cur"], self.env_num, None, False,
                                              no_grad, dict(rel_dev=sc[i % 2, 0:1],
                                                            rel_next=sc[(i + 1) % 2, 0:1]))
                        self._flush()
                self._graphs[G] = graph = (key, g, LOG.capture_end())
                self._parity = 0
            graph[1].replay()
            LOG.replayed(graph[2])
            for _ in range(G):
                written.append(int(buf._ring.index[0]))
                buf._ring.advance(None)
            done += G
        return done

    def _collect_fused(self, n_step, n_episode, random, no_grad):
        self._alloc_scratch()
        prep = getattr(self.policy, "prepare_fused_act", None)
        self._fused_act_on = bool(not random and not self._noise_active() and
                                  self.use_fused_act and prep is not None and prep())
        self._flush()
        s, b, buf = self._scratch, self._base, self.buffer
        N = self.env_num
        act_shape, act_dtype = self._act_spec()
        buf._alloc_storage(b.obs_shape, b.obs_torch_dtype, act_shape, act_dtype)
        dev = buf.device
        # rows r < kk of the scratch arrays belong to env ready[r] (ready None: env r)
        kk = N if n_step is not None else min(N, n_episode)
        self._step_on = self._fused_step_ok(n_step, kk)
        ready = None
        ids_t = None
        cur = s["cur"] if kk == N else s["cur"][:kk]
        step_count = episode_count = 0
        written = []          # per step: uniform ring position (int) or the ptr array
        ep_stats = []         # (rew, len, idx) arrays of finished episodes, in step order
        eager_steps = 0
        S = buf._ring.size    # rows per sub-buffer: a collect of more steps wraps the ring
        while True:
            if n_step is not None and len(written) >= S:
                # the next step overwrites a row this collect wrote: read the finished
                # episodes' statistics of the steps so far before the ring laps them
                ep_stats.append(self._episode_stats(written))
                written = []
            if (n_step is not None and self.graph_steps and not random and kk == N
                    and kk == buf.buffer_num and buf._ring.uniform_rel() is not None
                    and eager_steps > 0 and not self._noise_active()):
                n_left = min(-(-(n_step - step_count) // N), S - len(written))
                done_steps = self._replay_steps(no_grad, n_left, written)
                step_count += done_steps * N
                if step_count >= n_step:
                    break
                if len(written) >= S:
                    continue
            ids_np = None if ready is None else ready
            uni = buf._ring.uniform_rel() if ids_np is None and kk == buf.buffer_num else None
            if ids_np is None and kk != buf.buffer_num:
                ids_np = np.arange(kk)
            ptr, next_rel = buf._ring.advance(ids_np)
            if uni is not None:
                kw = dict(uniform_rel=uni, uniform_next=int(next_rel[0]))
                written.append(uni)
            else:
                kw = dict(ptr=torch.as_tensor(ptr, device=dev),
                          next_rel=torch.as_tensor(next_rel, device=dev))
                written.append(np.asarray(ptr))
            self._device_step(cur, kk, ids_t, random, no_grad, kw)
            eager_steps += 1
            step_count += kk
            if n_episode:
                done_np = s["done"][:kk].cpu().numpy()
                if done_np.any():
                    env_ind_local = np.flatnonzero(done_np)
                    episode_count += len(env_ind_local)
                    # read now: a later step of this collect may overwrite these rows (the
                    # trainer's test collector holds one row per env, trainer/utils.py:11-33)
                    rows_t = torch.as_tensor(np.asarray(ptr)[env_ind_local], device=dev)
                    ep_stats.append(tuple(buf._dev[k][rows_t].cpu().numpy() for k in
                                          ("stat_rew", "stat_len", "stat_idx")))
                    surplus = kk - (n_episode - episode_count)
                    if surplus > 0:
                        mask = np.ones(kk, dtype=bool)
                        mask[env_ind_local[:surplus]] = False
                        keep = torch.as_tensor(np.flatnonzero(mask), device=dev)
                        cur = cur[keep].contiguous()
                        ready = (np.arange(kk) if ready is None else ready)[mask]
                        ids_t = torch.as_tensor(ready, device=dev)
                        kk = len(ready)
                if episode_count >= n_episode:
                    break
            elif step_count >= n_step:
                break
        self._flush()
        if not n_episode and written:
            ep_stats.append(self._episode_stats(written))
        # the episode statistics in the reference's (step, env) order
        if ep_stats:
            rews, lens, idxs = (np.concatenate([e[i] for e in ep_stats]) for i in range(3))
        else:
            rews, lens, idxs = np.zeros(0), np.zeros(0, np.int64), np.zeros(0, np.int64)
        if not n_episode:
            episode_count = len(rews)
        self.data.obs = s["cur"]
        return step_count, episode_count, rews, lens, idxs

    def _episode_stats(self, written):
        """One read-back of the statistics of the episodes that finished in the steps of
        ``written`` (uniform ring positions or ptr arrays, in step order; none of their rows
        overwritten since): (rew, len, start index) in the reference's (step, env) order."""
        self._flush()
        buf = self.buffer
        d, dev = buf._dev, buf.device
        if all(isinstance(w, int) for w in written):
            rel = torch.as_tensor(np.asarray(written, np.int64), device=dev)
            rows_t = (rel[:, None] + d["offset"][None, :]).reshape(-1)
        else:
            rows_t = torch.as_tensor(np.concatenate(
                [np.asarray(w).reshape(-1) if not isinstance(w, int) else w + buf._offset
                 for w in written]), device=dev)
        rows_t = rows_t[buf._meta.done[rows_t]]
        return tuple(d[k][rows_t].cpu().numpy() for k in ("stat_rew", "stat_len", "stat_idx"))

    def _collect_generic(self, n_step, n_episode, random, render, no_grad, gym_reset_kwargs):
        """The reference loop (collector.py:250-361) for host envs; buffer still on device."""
        self.buffer.obs_chain = False  # host envs: no guarantee on obs / obs_next identity
        if n_step is not None:
            ready_env_ids = np.arange(self.env_num)
        else:
            ready_env_ids = np.arange(min(self.env_num, n_episode))
            self.data = self.data[:min(self.env_num, n_episode)]
        step_count = episode_count = 0
        episode_rews, episode_lens, episode_start_indices = [], [], []
        while True:
            obs = torch.as_tensor(np.asarray(self.data.obs), device=self.buffer._ensure_device())
            act, policy = self._policy_act(obs, self.data.info, random, no_grad,
                                           len(ready_env_ids), ready_env_ids)
            act_np = act.detach().cpu().numpy() if isinstance(act, torch.Tensor) else act
            self.data.update(policy=policy, act=act_np)
            action_remap = self.policy.map_action(act_np)
            obs_next, rew, terminated, truncated, info = self.env.step(action_remap,
                                                                       ready_env_ids)
            to_np = (lambda x: x.cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x))
            obs_next, rew, terminated, truncated = map(to_np, (obs_next, rew, terminated,
                                                               truncated))
            done = np.logical_or(terminated, truncated)
            self.data.update(obs_next=obs_next, rew=rew, terminated=terminated,
                             truncated=truncated, done=done, info=info)
            if self.preprocess_fn:
                self.data.update(self.preprocess_fn(
                    obs_next=self.data.obs_next, rew=self.data.rew, done=self.data.done,
                    info=self.data.info, policy=self.data.policy, env_id=ready_env_ids,
                    act=self.data.act))
            if render:
                self.env.render()
                if render > 0 and not np.isclose(render, 0):
                    time.sleep(render)
            ptr, ep_rew, ep_len, ep_idx = self.buffer.add(self.data, buffer_ids=ready_env_ids)
            step_count += len(ready_env_ids)
            if np.any(done):
                env_ind_local = np.where(done)[0]
                env_ind_global = ready_env_ids[env_ind_local]
                episode_count += len(env_ind_local)
                episode_lens.append(ep_len[env_ind_local])
                episode_rews.append(ep_rew[env_ind_local])
                episode_start_indices.append(ep_idx[env_ind_local])
                gkw = gym_reset_kwargs or {}
                obs_reset, info_r = self.env.reset(env_ind_global, **gkw)
                obs_reset = to_np(obs_reset)
                if self.preprocess_fn:
                    processed = self.preprocess_fn(obs=obs_reset, info=info_r,
                                                   env_id=env_ind_global)
                    obs_reset = processed.get("obs", obs_reset)
                obs_next = np.array(self.data.obs_next, copy=True)
                obs_next[env_ind_local] = obs_reset
                self.data.obs_next = obs_next
                if n_episode:
                    surplus = len(ready_env_ids) - (n_episode - episode_count)
                    if surplus > 0:
                        mask = np.ones_like(ready_env_ids, dtype=bool)
                        mask[env_ind_local[:surplus]] = False
                        ready_env_ids = ready_env_ids[mask]
                        self.data = self.data[mask]
            self.data.obs = self.data.obs_next
            if (n_step and step_count >= n_step) or (n_episode and episode_count >= n_episode):
                break
        if episode_count > 0:
            rews, lens, idxs = map(np.concatenate,
                                   [episode_rews, episode_lens, episode_start_indices])
        else:
            rews, lens, idxs = np.array([]), np.array([], int), np.array([], int)
        return step_count, episode_count, rews, lens, idxs
