"""Padded observation storage: wide f32 observation rows are kept
with a 128-byte pitch (VectorReplayBuffer._alloc_storage, 376 -> 384 floats), exposed as
[m, D] views.  Every read path of the buffer must give the same bytes as an unpadded twin
buffer fed the same trace (PAD_MIN raised so it stores rows packed) and as torch's own
indexing of the storage view: partial samples, a wrapped ring, sample(0) with
ignore_obs_next, get(..., stack_num), stack_num > 1 buffers (save_only_last_obs too), and the
non-fused / fused PPO learn paths that gather minibatch rows from it.  Index and byte work:
bit-exact (reference semantics: buffer/base.py:317-389, manager.py:104-192)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    return torch.device("cuda", 0)


def _twins(dev, total, num, **kw):
    from tianshou_amd.data import VectorReplayBuffer
    padded = VectorReplayBuffer(total, num, device=dev, **kw)
    packed = VectorReplayBuffer(total, num, device=dev, **kw)
    packed.PAD_MIN = 1 << 30
    return padded, packed


def _trace(bufs, rng, steps, num, obs_shape, A, p_term=0.08):
    from tianshou_amd.data import Batch
    for _ in range(steps):
        ids = np.sort(rng.choice(num, size=int(rng.integers(1, num + 1)), replace=False))
        k = len(ids)
        term = rng.random(k) < p_term
        trunc = (rng.random(k) < 0.03) & ~term
        b = Batch(obs=rng.standard_normal((k,) + obs_shape).astype(np.float32),
                  act=rng.standard_normal((k, A)).astype(np.float32),
                  rew=rng.standard_normal(k), terminated=term, truncated=trunc,
                  obs_next=rng.standard_normal((k,) + obs_shape).astype(np.float32),
                  info=Batch(env_id=ids))
        for buf in bufs:
            buf.add(b, buffer_ids=ids)


def _eq(a, b):
    return torch.equal(a.cpu(), b.cpu()) if isinstance(a, torch.Tensor) else \
        np.array_equal(np.asarray(a), np.asarray(b))


@pytest.mark.parametrize("ignore_obs_next", [False, True])
def test_padded_rows_read_paths_match_packed(dev, ignore_obs_next):
    D, A, num, size = 376, 17, 6, 16
    pad, pack = _twins(dev, num * size, num, ignore_obs_next=ignore_obs_next)
    rng = np.random.default_rng(11)
    _trace((pad, pack), rng, 70, num, (D,), A)  # > size adds per env: the ring wraps
    assert pad.obs.stride(0) == 384 and pad.obs.shape[1] == D
    assert pack.obs.stride(0) == D and pack.obs.is_contiguous()
    assert _eq(pad.obs, pack.obs)
    # partial sample (random rows, repeats) and wrapped-ring sample(0)
    q = rng.integers(0, pad.maxsize, 257)
    for idx in (q, pad.sample_indices(0), np.array([], np.int64)):
        a, b = pad[idx], pack[idx]
        want = pack.obs[torch.as_tensor(idx, device=dev, dtype=torch.int64)]
        assert _eq(a.obs, want) and _eq(b.obs, want)
        assert _eq(a.obs_next, b.obs_next)
        assert _eq(a.act, b.act) and _eq(a.rew, b.rew)
    # get(): plain and stacked through the prev chain
    assert _eq(pad.get(q, "obs"), pack.get(q, "obs"))
    sp, sk = pad.get(q, "obs", stack_num=4), pack.get(q, "obs", stack_num=4)
    assert sp.shape == (len(q), 4, D) and _eq(sp, sk)
    prev = q.copy()
    for col in range(3, -1, -1):
        assert _eq(sp[:, col], pack.obs[torch.as_tensor(prev, device=dev)])
        prev = pack.prev(prev)
    if not ignore_obs_next:
        assert _eq(pad.get(q, "obs_next", stack_num=3), pack.get(q, "obs_next", stack_num=3))


@pytest.mark.parametrize("last_only", [False, True])
def test_padded_rows_stack_buffer_matches_packed(dev, last_only):
    """stack_num = 4 buffers of wide f32 rows (D = 120 -> a 128-float pitch), with and without
    save_only_last_obs (the stored row is then obs[:, -1])."""
    D, A, num, size, S = 120, 3, 5, 12, 4
    pad, pack = _twins(dev, num * size, num, stack_num=S, save_only_last_obs=last_only)
    rng = np.random.default_rng(12)
    shape = (S, D) if last_only else (D,)
    _trace((pad, pack), rng, 50, num, shape, A)
    assert pad.obs.stride(0) == 128
    q = rng.integers(0, pad.maxsize, 100)
    for idx in (q, pad.sample_indices(0)):
        a, b = pad[idx], pack[idx]
        assert a.obs.shape == b.obs.shape and _eq(a.obs, b.obs)
        assert _eq(a.obs_next, b.obs_next)
        assert _eq(a.info.env_id, b.info.env_id)


@pytest.mark.parametrize("fused_mlp", [False, True])
def test_padded_rows_ppo_learn_matches_packed(dev, fused_mlp):
    """PPO update from a padded buffer = the same update from the packed twin, bit for bit
    (the non-fused minibatch gathers X rows with gather_rows, ppo.py:306; the fused one reads
    the pitched view in place)."""
    from tianshou_amd.policy import PPOPolicy
    from tianshou_amd.utils.models import fixed_std_normal, get_actor_critic, init_and_get_optim
    from tianshou_amd.env import SyntheticVectorEnv
    D, A, num, size = 376, 17, 8, 64
    pad, pack = _twins(dev, num * size, num)
    rng = np.random.default_rng(13)
    _trace((pad, pack), rng, size, num, (D,), A, p_term=0.02)
    out, params = [], []
    for buf in (pad, pack):
        torch.manual_seed(0)
        np.random.seed(0)
        actor, critic = get_actor_critic((D,), (64, 64), (A,), dev)
        optim = init_and_get_optim(actor, critic, 3e-4)
        pol = PPOPolicy(actor, critic, optim, fixed_std_normal,
                        action_space=SyntheticVectorEnv(1, (D,), A, device=dev).action_space,
                        max_grad_norm=0.5, reward_normalization=True,
                        fused_mlp=fused_mlp).to(dev)
        res = pol.update(0, buf, batch_size=128, repeat=2)
        out.append(res)
        params.append(torch.cat([p.detach().flatten() for p in pol.parameters()]).cpu())
    for key in out[0]:
        assert np.array_equal(np.asarray(out[0][key]), np.asarray(out[1][key])), key
    assert torch.equal(params[0], params[1])
