"""ORACLE (test infrastructure only) -- CPU restatements of the reference hot path.

Importable ONLY from ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg.  The product (``tianshou-fork_amd/tianshou_amd``) never imports it;
it is the checker the HIP path is compared against.

Pinned against the reference's own outputs: ``tests/golden/*`` were recorded from
/root/reference by ``tools/gen_goldens.py`` and ``tests/test_oracle.py`` checks every
function here against them (bit-exact for index math and the GAE f64 results).

Each function cites the reference code it restates.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    """liboracle.so (plain C, built by oracle/Makefile)."""
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.run(["make", "-C", _HERE], check=True, capture_output=True)
        L = ctypes.CDLL(path)
        for name, vt in (("oracle_gae_f32vals", ctypes.c_void_p),
                         ("oracle_gae_f64vals", ctypes.c_void_p)):
            fn = getattr(L, name)
            fn.restype = None
            fn.argtypes = [vt, vt, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                           ctypes.c_double, ctypes.c_double, ctypes.c_void_p]
        L.oracle_shuffle_apply.restype = None
        L.oracle_shuffle_apply.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
        _LIB = L
    return _LIB


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def shuffle_apply(draws):
    """arange(n) shuffled by the draws of NumPy's legacy shuffle (mtrand.pyx _shuffle_raw:
    for i = n-1 .. 1 swap x[i], x[draws[i]]), sequentially in C."""
    d = np.ascontiguousarray(draws, np.uint32)
    out = np.empty(len(d), np.int64)
    if len(d):
        lib().oracle_shuffle_apply(_ptr(d), len(d), _ptr(out))
    return out


# ---------------------------------------------------------------------------------------
# GAE: tianshou/policy/base.py:337-384 (compute_episodic_return) + :453-497 (_gae_return)
# ---------------------------------------------------------------------------------------
def gae_return(v_s, v_next_masked, rew, end_flag, gamma, gae_lambda):
    """_gae_return restated (base.py:453-497). f32 values -> NEP-50 f32 product path."""
    n = len(rew)
    rew = np.ascontiguousarray(rew, np.float64)
    end = np.ascontiguousarray(end_flag, np.uint8)
    out = np.zeros(n, np.float64)
    if v_s.dtype == np.float32 and v_next_masked.dtype == np.float32:
        lib().oracle_gae_f32vals(_ptr(np.ascontiguousarray(v_s)),
                                 _ptr(np.ascontiguousarray(v_next_masked)), _ptr(rew),
                                 _ptr(end), n, float(gamma), float(gae_lambda), _ptr(out))
    else:
        lib().oracle_gae_f64vals(_ptr(np.ascontiguousarray(v_s, np.float64)),
                                 _ptr(np.ascontiguousarray(v_next_masked, np.float64)),
                                 _ptr(rew), _ptr(end), n, float(gamma), float(gae_lambda),
                                 _ptr(out))
    return out


def compute_episodic_return(rew, terminated, truncated, indices, unfinished, v_s_=None,
                            v_s=None, gamma=0.99, gae_lambda=0.95):
    """BasePolicy.compute_episodic_return restated (base.py:337-384).

    ``terminated`` doubles as the value mask (base.py:317-335: ~buffer.terminated[indices],
    and batch = buffer[indices]).  Returns (returns f64, advantage f64).
    """
    rew = np.asarray(rew)
    terminated = np.asarray(terminated).astype(bool)
    if v_s_ is None:
        assert np.isclose(gae_lambda, 1.0)
        v_s_ = np.zeros_like(rew)
    else:
        v_s_ = np.asarray(v_s_).flatten()
        v_s_ = v_s_ * ~terminated          # dtype kept: f32 stays f32 (NEP 50)
    v_s = np.roll(v_s_, 1) if v_s is None else np.asarray(v_s).flatten()
    end_flag = np.logical_or(terminated, np.asarray(truncated).astype(bool))
    end_flag[np.isin(indices, unfinished)] = True
    if v_s.dtype != v_s_.dtype:
        v_s, v_s_ = v_s.astype(np.float64), v_s_.astype(np.float64)
    adv = gae_return(v_s, v_s_, rew, end_flag, gamma, gae_lambda)
    returns = adv + v_s
    return returns, adv


# ---------------------------------------------------------------------------------------
# VectorReplayBuffer index math: tianshou/data/buffer/vecbuf.py:33-37,
# manager.py:54-192,259-297, base.py:140-214,276-305
# ---------------------------------------------------------------------------------------
class VecBufferIndex:
    """Vectorised restatement of ReplayBufferManager's index bookkeeping (no per-env loop;
    buffer_ids within one add are unique, as in every reference call site)."""

    def __init__(self, total_size, buffer_num):
        assert buffer_num > 0
        self.num = buffer_num
        self.size = int(np.ceil(total_size / buffer_num))        # vecbuf.py:35
        self.maxsize = self.size * buffer_num
        self.offset = np.arange(buffer_num, dtype=np.int64) * self.size
        self.done = np.zeros(self.maxsize, bool)
        self.rew = np.zeros(self.maxsize, np.float64)
        self.ep_rew = np.zeros(buffer_num, np.float64)
        self.ep_len = np.zeros(buffer_num, np.int64)
        self.ep_idx = np.zeros(buffer_num, np.int64)
        self.reset(False)

    def reset(self, keep_statistics=False):                     # manager.py:54-58
        self.index = np.zeros(self.num, np.int64)
        self.sizes = np.zeros(self.num, np.int64)
        self.last_index = self.offset.copy()
        if not keep_statistics:
            self.ep_rew[:] = 0.0
            self.ep_len[:] = 0
            self.ep_idx[:] = 0

    def __len__(self):
        return int(self.sizes.sum())

    def add(self, rew, terminated, truncated, buffer_ids=None):  # manager.py:104-161
        ids = np.arange(self.num) if buffer_ids is None else np.asarray(buffer_ids, np.int64)
        rew = np.asarray(rew)
        done = np.logical_or(terminated, truncated).astype(bool)
        ptr = self.index[ids].copy()                             # base.py:202
        self.sizes[ids] = np.minimum(self.sizes[ids] + 1, self.size)
        self.index[ids] = (ptr + 1) % self.size
        self.ep_rew[ids] += rew
        self.ep_len[ids] += 1
        out_rew = np.where(done, self.ep_rew[ids], self.ep_rew[ids] * 0.0)
        out_len = np.where(done, self.ep_len[ids], 0)
        out_idx = self.ep_idx[ids] + self.offset[ids]
        d = ids[done]
        self.ep_rew[d] = 0.0
        self.ep_len[d] = 0
        self.ep_idx[d] = self.index[d]
        gptr = ptr + self.offset[ids]
        self.last_index[ids] = gptr
        self.done[gptr] = done
        self.rew[gptr] = rew
        return gptr, out_rew, out_len, out_idx

    def sample_indices0(self):                                   # manager.py:177-192
        parts = []
        for b in range(self.num):
            parts.append(np.concatenate([np.arange(self.index[b], self.sizes[b]),
                                         np.arange(self.index[b])]) + self.offset[b])
        return np.concatenate(parts).astype(np.int64)

    def unfinished_index(self):                                  # manager.py:68-74
        out = []
        for b in range(self.num):
            if self.sizes[b]:
                last = (self.index[b] - 1) % self.sizes[b] + self.offset[b]
                if not self.done[last]:
                    out.append(last)
        return np.array(out, np.int64)

    def _seg(self, index):
        index = np.asarray(index, np.int64) % self.maxsize
        b = index // self.size
        start = self.offset[b]
        cur = np.maximum(1, self.sizes[b])
        return index, b, start, cur

    def prev(self, index):                                       # manager.py:259-277
        index, b, start, cur = self._seg(index)
        sub = (index - start - 1) % cur
        end = self.done[sub + start] | (sub + start == self.last_index[b])
        return (sub + end) % cur + start

    def next(self, index):                                       # manager.py:280-297
        index, b, start, cur = self._seg(index)
        end = self.done[index] | (index == self.last_index[b])
        return (index - start + 1 - end) % cur + start


def stack_get(val, index, stack_num, prev):
    """ReplayBuffer.get(index, key, stack_num) restated (buffer/base.py:317-358): the newest
    frame is val[index], older frames step back through prev (episode-aware)."""
    indices = np.asarray(index)
    if stack_num == 1:
        return val[indices]
    stack = []
    for _ in range(stack_num):
        stack = [val[indices]] + stack
        indices = prev(indices)
    return np.stack(stack, axis=indices.ndim)


def avail_indices(ix, stack_num):
    """sample_indices(0) with sample_avail and stack_num > 1 (manager.py:165-171 ->
    base.py:291-303 per sub-buffer): rows whose stack_num-1 predecessors are all in the
    same episode."""
    all_idx = ix.sample_indices0()
    p = all_idx
    for _ in range(stack_num - 2):
        p = ix.prev(p)
    return all_idx[p != ix.prev(p)]


# ---------------------------------------------------------------------------------------
# RunningMeanStd: tianshou/utils/statistics.py:69-114
# ---------------------------------------------------------------------------------------
class RMS:
    def __init__(self, eps=np.finfo(np.float32).eps.item(), clip_max=10.0):
        self.mean, self.var, self.count = 0.0, 1.0, 0
        self.eps, self.clip_max = eps, clip_max

    def update(self, x):
        bm, bv, bc = np.mean(x, axis=0), np.var(x, axis=0), len(x)
        delta = bm - self.mean
        tot = self.count + bc
        new_mean = self.mean + delta * bc / tot
        m2 = self.var * self.count + bv * bc + delta ** 2 * self.count * bc / tot
        self.mean, self.var, self.count = new_mean, m2 / tot, tot

    def norm(self, x):
        y = (x - self.mean) / np.sqrt(self.var + self.eps)
        return np.clip(y, -self.clip_max, self.clip_max) if self.clip_max else y


# ---------------------------------------------------------------------------------------
# Batch.split: tianshou/data/batch.py:896-912
# ---------------------------------------------------------------------------------------
def split_parts(n, size, shuffle=True, merge_last=False):
    if size == -1:
        size = n
    assert 1 <= size
    idx = np.random.permutation(n) if shuffle else np.arange(n)
    merge_last = merge_last and n % size > 0
    parts = []
    for s in range(0, n, size):
        if merge_last and s + size + size >= n:
            parts.append(idx[s:])
            break
        parts.append(idx[s:s + size])
    return parts


# ---------------------------------------------------------------------------------------
# PPO minibatch loss (tianshou/policy/modelfree/ppo.py:106-151), Gaussian
# Independent(Normal(mu, exp(sigma_param)), 1) (utils/models.py:96-97,
# utils/net/continuous.py:229-235).  torch fp32 on CPU = the fp32 reference the fused
# HIP loss kernel is checked against.
# ---------------------------------------------------------------------------------------
def ppo_gaussian_loss_torch(mu, sigma_param, value, act, logp_old, adv, returns, v_s,
                            eps_clip=0.2, dual_clip=None, value_clip=False, norm_adv=True,
                            vf_coef=0.5, ent_coef=0.01, eps=1e-8):
    """Returns (loss, clip_loss, vf_loss, ent_loss, grads{mu, sigma_param, value})."""
    import torch
    from torch.distributions import Independent, Normal
    mu = mu.detach().clone().requires_grad_(True)
    sp = sigma_param.detach().clone().requires_grad_(True)
    value = value.detach().clone().requires_grad_(True)
    shape = [1] * mu.dim()
    shape[1] = -1
    sigma = (sp.view(shape) + torch.zeros_like(mu)).exp()
    dist = Independent(Normal(mu, sigma), 1)
    if norm_adv:
        adv = (adv - adv.mean()) / (adv.std() + eps)
    ratio = (dist.log_prob(act) - logp_old).exp().float()
    ratio = ratio.reshape(ratio.size(0), -1).transpose(0, 1)
    surr1 = ratio * adv
    surr2 = ratio.clamp(1.0 - eps_clip, 1.0 + eps_clip) * adv
    if dual_clip:
        clip1 = torch.min(surr1, surr2)
        clip2 = torch.max(clip1, dual_clip * adv)
        clip_loss = -torch.where(adv < 0, clip2, clip1).mean()
    else:
        clip_loss = -torch.min(surr1, surr2).mean()
    if value_clip:
        v_clip = v_s + (value - v_s).clamp(-eps_clip, eps_clip)
        vf1 = (returns - value).pow(2)
        vf2 = (returns - v_clip).pow(2)
        vf_loss = torch.max(vf1, vf2).mean()
    else:
        vf_loss = (returns - value).pow(2).mean()
    ent_loss = dist.entropy().mean()
    loss = clip_loss + vf_coef * vf_loss - ent_coef * ent_loss
    loss.backward()
    return (loss.detach(), clip_loss.detach(), vf_loss.detach(), ent_loss.detach(),
            dict(mu=mu.grad, sigma_param=sp.grad, value=value.grad))


def ppo_learn_torch(actor, critic, optim, obs, act, logp_old, adv, returns, batch_size,
                    repeat, perm_fn, eps_clip=0.2, vf_coef=0.5, ent_coef=0.01,
                    max_grad_norm=None, norm_adv=True, eps=1e-8):
    """PPOPolicy.learn restated (ppo.py:99-162) for the Gaussian Independent(Normal) actor
    over plain torch modules in fp32 (no dual / value clip, no advantage recomputation):
    ``repeat`` epochs of Batch.split(batch_size, shuffle=True, merge_last=True)
    (batch.py:896-912; ``perm_fn(n)`` = np.random.permutation(n)), per minibatch the
    advantage normalisation, clipped surrogate, value and entropy losses, loss.backward(),
    nn.utils.clip_grad_norm_ over the actor-critic parameters and optim.step().  Tensors live
    on the caller's device; returns the [n_minibatch, 4] (loss, clip, vf, ent) terms."""
    import torch
    from torch.distributions import Independent, Normal
    params = list(actor.parameters()) + list(critic.parameters())
    n = len(adv)
    out = []
    for _ in range(repeat):
        perm = torch.as_tensor(perm_fn(n), device=adv.device)
        bounds = [(s, min(s + batch_size, n)) for s in range(0, n, batch_size)]
        if n % batch_size and len(bounds) > 1:   # merge_last
            bounds = bounds[:-2] + [(bounds[-2][0], n)]
        for s, e in bounds:
            idx = perm[s:e]
            o = obs[idx]
            (mu, sigma), _ = actor(o)
            dist = Independent(Normal(mu, sigma), 1)
            a = adv[idx]
            if norm_adv:
                mean, std = a.mean(), a.std()
                a = (a - mean) / (std + eps)
            ratio = (dist.log_prob(act[idx]) - logp_old[idx]).exp().float()
            ratio = ratio.reshape(ratio.size(0), -1).transpose(0, 1)
            surr1 = ratio * a
            surr2 = ratio.clamp(1.0 - eps_clip, 1.0 + eps_clip) * a
            clip_loss = -torch.min(surr1, surr2).mean()
            value = critic(o).flatten()
            vf_loss = (returns[idx] - value).pow(2).mean()
            ent_loss = dist.entropy().mean()
            loss = clip_loss + vf_coef * vf_loss - ent_coef * ent_loss
            optim.zero_grad()
            loss.backward()
            if max_grad_norm:
                torch.nn.utils.clip_grad_norm_(params, max_norm=max_grad_norm)
            optim.step()
            out.append(torch.stack([loss, clip_loss, vf_loss, ent_loss]).detach())
    return torch.stack(out)


# ---------------------------------------------------------------------------------------
# PPO minibatch loss (ppo.py:106-151) for Categorical policies: Categorical(logits=x)
# (examples/atari/atari_ppo.py:136-137) or Categorical(probs=x) (test/discrete/test_ppo.py:95).
# torch fp32 on CPU = the fp32 reference of the fused tsrl_ppo_cat kernel.
# ---------------------------------------------------------------------------------------
def ppo_categorical_loss_torch(x, value, act, logp_old, adv, returns, v_s, mode,
                               eps_clip=0.2, dual_clip=None, value_clip=False, norm_adv=True,
                               vf_coef=0.5, ent_coef=0.01, eps=1e-8):
    """Returns (loss, clip_loss, vf_loss, ent_loss, grads{x, value})."""
    import torch
    x = x.detach().clone().requires_grad_(True)
    value = value.detach().clone().requires_grad_(True)
    dist = torch.distributions.Categorical(logits=x) if mode == 0 else \
        torch.distributions.Categorical(probs=x, validate_args=False)
    if norm_adv:
        adv = (adv - adv.mean()) / (adv.std() + eps)
    ratio = (dist.log_prob(act) - logp_old).exp().float()
    ratio = ratio.reshape(ratio.size(0), -1).transpose(0, 1)
    surr1 = ratio * adv
    surr2 = ratio.clamp(1.0 - eps_clip, 1.0 + eps_clip) * adv
    if dual_clip:
        clip1 = torch.min(surr1, surr2)
        clip2 = torch.max(clip1, dual_clip * adv)
        clip_loss = -torch.where(adv < 0, clip2, clip1).mean()
    else:
        clip_loss = -torch.min(surr1, surr2).mean()
    if value_clip:
        v_clip = v_s + (value - v_s).clamp(-eps_clip, eps_clip)
        vf_loss = torch.max((returns - value).pow(2), (returns - v_clip).pow(2)).mean()
    else:
        vf_loss = (returns - value).pow(2).mean()
    ent_loss = dist.entropy().mean()
    loss = clip_loss + vf_coef * vf_loss - ent_coef * ent_loss
    loss.backward()
    return (loss.detach(), clip_loss.detach(), vf_loss.detach(), ent_loss.detach(),
            dict(x=x.grad, value=value.grad))


def nstep_return(vb, terminated, indices, target_q, gamma, n_step):
    """compute_nstep_return + _nstep_return (policy/base.py:417-440, 500-524) over a
    VecBufferIndex ``vb`` (done / rew / ring state) and the per-row terminated flags; target_q
    is Q_target at the terminal rows, [bsz] or [bsz, X].  Returns (returns [bsz, X] in the
    target dtype, terminal indices)."""
    indices = np.asarray(indices, np.int64)
    bsz = len(indices)
    chain = [indices % vb.maxsize]
    for _ in range(n_step - 1):
        chain.append(vb.next(chain[-1]))
    chain = np.stack(chain)
    terminal = chain[-1]
    tq = np.asarray(target_q).reshape(bsz, -1)
    out_dtype = tq.dtype
    tq = tq * (~np.asarray(terminated, bool)[terminal]).reshape(-1, 1)
    end_flag = vb.done.copy()
    end_flag[vb.unfinished_index()] = True
    gamma_buffer = np.ones(n_step + 1)
    for i in range(1, n_step + 1):
        gamma_buffer[i] = gamma_buffer[i - 1] * gamma
    returns = np.zeros(tq.shape)
    gammas = np.full(bsz, n_step)
    for n in range(n_step - 1, -1, -1):
        now = chain[n]
        gammas[end_flag[now] > 0] = n + 1
        returns[end_flag[now] > 0] = 0.0
        returns = vb.rew[now].reshape(bsz, 1) + gamma * returns
    return (tq * gamma_buffer[gammas].reshape(bsz, 1) + returns).astype(out_dtype), terminal


class SegTree:
    """SegmentTree (data/utils/segtree.py:7-137): f64 binary-heap sum tree."""

    def __init__(self, size):
        bound = 1
        while bound < size:
            bound *= 2
        self.size, self.bound = size, bound
        self.value = np.zeros(2 * bound)

    def set(self, index, value):                                # :98-104
        index = np.asarray(index, np.int64) + self.bound
        self.value[index] = value
        while index[0] > 1:
            index = index // 2
            self.value[index] = self.value[index * 2] + self.value[index * 2 + 1]

    def reduce(self, start=0, end=None):                        # :56-64, 107-119
        if start == 0 and end is None:
            return self.value[1]
        if end is None:
            end = self.size
        if end < 0:
            end += self.size
        start, end = start + self.bound - 1, end + self.bound
        result = 0.0
        while end - start > 1:
            if start % 2 == 0:
                result += self.value[start + 1]
            start //= 2
            if end % 2 == 1:
                result += self.value[end - 1]
            end //= 2
        return result

    def prefix_idx(self, value):                                # :122-137
        value = np.array(value, copy=True)
        index = np.ones(value.shape, dtype=np.int64)
        while index[0] < self.bound:
            index *= 2
            lsons = self.value[index]
            direct = lsons < value
            value -= lsons * direct
            index += direct
        return index - self.bound
