"""Frame-stack storage of the device VectorReplayBuffer against the
reference (tests/golden/stack.npz, recorded by tools/gen_goldens.py gen_stack) and the
oracle restatement (oracle/ref.py stack_get / avail_indices) at larger sizes.  Everything
here is index / byte work: bit-exact."""
import os

import numpy as np
import pytest
import torch

from oracle import ref

from .test_oracle import STACK_CASES, replay_stack_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    return torch.device("cuda", 0)


@pytest.mark.parametrize("name,stack_num,last_only,ign_next,avail", STACK_CASES)
def test_stack_buffer_matches_reference(golden_dir, dev, name, stack_num, last_only, ign_next,
                                        avail):
    from tianshou_amd.data import Batch, VectorReplayBuffer
    z = np.load(os.path.join(golden_dir, "stack.npz"))
    p = name + "_"
    buf = VectorReplayBuffer(5 * 8, 5, stack_num=stack_num, save_only_last_obs=last_only,
                             ignore_obs_next=ign_next, sample_avail=avail, device=dev)
    o = 0
    for step, k in enumerate(z[p + "sizes"]):
        sl = slice(o, o + k)
        o += k
        ids = z[p + "ids"][sl]
        buf.add(Batch(obs=z[p + "in_obs"][sl], act=ids, rew=z[p + "in_rew"][sl],
                      terminated=z[p + "in_term"][sl], truncated=z[p + "in_trunc"][sl],
                      obs_next=z[p + "in_obs_next"][sl], info=Batch(env_id=ids + 100)),
                buffer_ids=ids)
        if step == 40:
            buf.reset(keep_statistics=True)
    assert np.array_equal(buf.obs.cpu().numpy(), z[p + "stored_obs"])
    if not ign_next:
        assert np.array_equal(buf.obs_next.cpu().numpy(), z[p + "stored_obs_next"])
    else:
        assert "obs_next" not in buf._meta.keys()
    assert np.array_equal(buf.sample_indices(0), z[p + "sample0"])
    q = z[p + "q_idx"]
    b = buf[q]
    assert np.array_equal(b.obs.cpu().numpy(), z[p + "q_obs"])
    assert np.array_equal(b.obs_next.cpu().numpy(), z[p + "q_obs_next"])
    assert np.array_equal(b.info.env_id.cpu().numpy(), z[p + "q_env_id"])
    assert np.array_equal(b.act.cpu().numpy(), z[p + "q_act"])
    allidx = np.arange(buf.maxsize)
    assert np.array_equal(buf.prev(allidx), z[p + "prev"])
    assert np.array_equal(buf.next(allidx), z[p + "next"])
    it = torch.as_tensor(allidx, device=dev)
    assert np.array_equal(buf._step_dev(it, 1).cpu().numpy(), z[p + "prev"])
    assert np.array_equal(buf._step_dev(it, -1).cpu().numpy(), z[p + "next"])
    assert np.array_equal(buf.get(q, "obs").cpu().numpy(), z[p + "q_obs"])
    if avail:
        np.random.seed(3)
        assert np.array_equal(buf.sample_indices(7), z[p + "sample7"])
    with pytest.raises(IndexError):
        buf[np.array([buf.maxsize * 2])]


def test_stack_gather_large_vs_oracle(dev):
    """Atari-sized frames (84x84 u8), 64 envs with ragged lengths, random done flags and a
    wrapped ring: tsrl_stack_gather and tsrl_ring_step_index vs the NumPy restatement."""
    from tianshou_amd import _C
    rng = np.random.default_rng(5)
    num, size, S = 64, 96, 4
    ix = ref.VecBufferIndex(num * size, num)
    for step in range(150):
        ids = np.sort(rng.choice(num, size=int(rng.integers(1, num + 1)), replace=False))
        term = rng.random(len(ids)) < 0.03
        trunc = (rng.random(len(ids)) < 0.02) & ~term
        ix.add(np.zeros(len(ids)), term, trunc, ids)
    frames = rng.integers(0, 256, (ix.maxsize, 84, 84), dtype=np.uint8)
    q = np.concatenate([ix.sample_indices0(), rng.integers(0, ix.maxsize, 1000)])
    want = ref.stack_get(frames, q, S, ix.prev)
    d = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
    src, done, last, lens, qt = d(frames), d(ix.done.astype(np.uint8)), d(ix.last_index), \
        d(ix.sizes), d(q.astype(np.int64))
    out = torch.empty((len(q), S, 84, 84), dtype=torch.uint8, device=dev)
    chain = torch.empty((len(q), S), dtype=torch.int64, device=dev)
    s = _C.stream_ptr(dev)
    L = _C.lib()
    _C.check(L.tsrl_stack_gather(_C.ptr(src), 84 * 84, _C.ptr(qt), len(q), S, _C.ptr(done),
                                 _C.ptr(last), _C.ptr(lens), size, num, _C.ptr(out),
                                 _C.ptr(chain), s), "tsrl_stack_gather")
    assert np.array_equal(out.cpu().numpy(), want)
    pc = q.copy()
    for col in range(S - 1, -1, -1):
        assert np.array_equal(chain[:, col].cpu().numpy(), pc)
        pc = ix.prev(pc)
    for steps in (3, 1, 0, -1, -2):
        o = torch.empty_like(qt)
        _C.check(L.tsrl_ring_step_index(_C.ptr(qt), len(q), _C.ptr(done), _C.ptr(last),
                                        _C.ptr(lens), size, num, steps, _C.ptr(o), s),
                 "tsrl_ring_step_index")
        w = q % ix.maxsize
        for _ in range(max(steps, 0)):
            w = ix.prev(w)
        for _ in range(max(-steps, 0)):
            w = ix.next(w)
        assert np.array_equal(o.cpu().numpy(), w), steps
