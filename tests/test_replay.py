"""Off-policy neighbours of the on-policy path vs the reference's own
outputs (tests/golden/replay.npz, tools/gen_goldens.py gen_replay):

* SegmentTree (data/utils/segtree.py:7-137): batch updates with duplicate indices, reduce over
  ranges, prefix-sum queries in f64 and f32 -- bit-exact (the same f64 sums in the same order);
* compute_nstep_return / _nstep_return (policy/base.py:386-440, 500-524) on the reference's
  test buffers (test_returns.py:170-296) and on a ragged 6-env VectorReplayBuffer with random
  flags, n in {1, 3, 5, 12}, 1 / 3 target columns, f32 and f64 targets -- bit-exact;
* PrioritizedReplayBuffer / PrioritizedVectorReplayBuffer (buffer/prio.py:9-105): the
  priority tree after adds, 6 rounds of sample(16) (same np.random stream) -> importance
  weights -> update_weight(f32 TD errors).

CPU tests pin the oracle (oracle/ref.py SegTree, nstep_return) to the goldens; GPU tests run
the HIP kernels (csrc/replay.hip) through the product classes."""
import os

import numpy as np
import pytest
import torch

from oracle import ref
from tests.conftest import GOLDEN

SEG_SIZES = (1, 8, 10, 1000, 16384)


@pytest.fixture(scope="module")
def z():
    return np.load(os.path.join(GOLDEN, "replay.npz"))


def _updates(z, p):
    o = 0
    for k in z[p + "upd_len"]:
        yield z[p + "upd_idx"][o:o + k], z[p + "upd_val"][o:o + k]
        o += k


def _replay_vec_adds(z, vb_add):
    o = 0
    for k in z["nsv_add_len"]:
        sl = slice(o, o + k)
        vb_add(z["nsv_add_ids"][sl], z["nsv_add_rew"][sl], z["nsv_add_term"][sl],
               z["nsv_add_trunc"][sl])
        o += k


# -- oracle pinned to the reference (CPU) ---------------------------------------------------
@pytest.mark.parametrize("size", SEG_SIZES)
def test_segtree_oracle_matches_reference(z, size):
    p = f"seg{size}_"
    t = ref.SegTree(size)
    for idx, val in _updates(z, p):
        t.set(idx, val)
    np.testing.assert_array_equal(t.value, z[p + "tree"])
    red = [t.reduce(int(a), int(b)) for a, b in zip(z[p + "red_start"], z[p + "red_end"])]
    np.testing.assert_array_equal(red, z[p + "red"])
    np.testing.assert_array_equal(t.prefix_idx(z[p + "q64"]), z[p + "i64"])
    np.testing.assert_array_equal(t.prefix_idx(z[p + "q32"]), z[p + "i32"])


def test_nstep_oracle_matches_reference(z):
    E, S = 6, 40
    vb = ref.VecBufferIndex(E * S, E)
    term = np.zeros(vb.maxsize, bool)

    def add(ids, rew, te, tr):
        ptr, *_ = vb.add(rew, te, tr, ids)
        term[ptr] = te
    _replay_vec_adds(z, add)
    np.testing.assert_array_equal(vb.sizes, z["nsv_lengths"])
    np.testing.assert_array_equal(vb.last_index, z["nsv_last_index"])
    idx = z["nsv_indices"]
    for n in (1, 3, 5, 12):
        for tag, tab in (("x1", z["nsv_table"][:, 0]), ("x3", z["nsv_table"]),
                         ("f64", z["nsv_table64"])):
            chain_end = idx % vb.maxsize
            for _ in range(n - 1):
                chain_end = vb.next(chain_end)
            got, terminal = ref.nstep_return(vb, term, idx, tab[chain_end], 0.97, n)
            np.testing.assert_array_equal(terminal, chain_end)
            np.testing.assert_array_equal(got, z[f"nsv_n{n}_{tag}"], err_msg=f"n={n} {tag}")


# -- device kernels through the product classes (GPU) -----------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("size", SEG_SIZES)
def test_segtree_device_matches_reference(z, size):
    from tianshou_amd.data import SegmentTree
    p = f"seg{size}_"
    t = SegmentTree(size, device="cuda")
    assert len(t) == size
    for idx, val in _updates(z, p):
        t[idx] = val
    np.testing.assert_array_equal(t._value.cpu().numpy(), z[p + "tree"])
    red = [t.reduce(int(a), int(b)) for a, b in zip(z[p + "red_start"], z[p + "red_end"])]
    np.testing.assert_array_equal(red, z[p + "red"])
    assert t.reduce() == float(z[p + "root"])
    np.testing.assert_array_equal(t.get_prefix_sum_idx(z[p + "q64"].copy()), z[p + "i64"])
    np.testing.assert_array_equal(t.get_prefix_sum_idx(z[p + "q32"].copy()), z[p + "i32"])
    if size == 8:
        with pytest.raises(IndexError):
            t[size]


@pytest.mark.gpu
def test_segtree_device_edge_cases(z):
    from tianshou_amd.data import SegmentTree
    t = SegmentTree(10, device="cuda")
    t[np.arange(3)] = np.array([0.1, 0, 0.1])
    np.testing.assert_array_equal(
        t.get_prefix_sum_idx(np.array([0, .1, .1 + 1e-6, .2 - 1e-6])), z["seg_corner_i"])
    with pytest.raises(AssertionError):
        t.get_prefix_sum_idx(.2)
    assert t.get_prefix_sum_idx(0.05) == 0
    # empty / inverted ranges sum nothing, as the reference's loop
    assert t.reduce(3, 3) == 0.0 and t.reduce(5, 2) == 0.0


@pytest.mark.gpu
def test_segtree_device_large_vs_oracle():
    """2^20 + 3 leaves, 4096-index updates with duplicates, 100k prefix queries: bit-exact vs
    the oracle restatement."""
    from tianshou_amd.data import SegmentTree
    rng = np.random.default_rng(5)
    size = (1 << 20) + 3
    t, o = SegmentTree(size, device="cuda"), ref.SegTree(size)
    for _ in range(4):
        idx = rng.integers(0, size, 4096)
        val = rng.random(4096)
        t[idx] = val
        o.set(idx, val)
    full = np.arange(size)
    val = rng.random(size)
    t[full] = val
    o.set(full, val)
    np.testing.assert_array_equal(t._value.cpu().numpy(), o.value)
    q = rng.random(100000) * o.reduce()
    np.testing.assert_array_equal(t.get_prefix_sum_idx(q.copy()), o.prefix_idx(q))
    for a, b in ((0, size), (17, size - 5), (size // 2, size // 2 + 1)):
        assert t.reduce(a, b) == o.reduce(a, b)


def _test_q_fn(buffer, indices):  # test/base/test_returns.py:137-140
    indices = buffer.next(indices)
    return -buffer.rew[torch.as_tensor(indices, device=buffer.device)].to(torch.float32)


@pytest.mark.gpu
@pytest.mark.parametrize("tl", [0, 1])
def test_nstep_reference_test_buffers(z, tl):
    from tianshou_amd.data import Batch, ReplayBuffer
    from tianshou_amd.policy import BasePolicy
    buf = ReplayBuffer(10, device="cuda")
    for i in range(12):
        if tl:
            buf.add(Batch(obs=0, act=0, rew=i + 1, terminated=i % 4 == 3 and i != 3,
                          truncated=i == 3, info={"TimeLimit.truncated": i == 3}))
        else:
            buf.add(Batch(obs=0, act=0, rew=i + 1, terminated=i % 4 == 3, truncated=False))
    batch, indices = buf.sample(0)
    np.testing.assert_array_equal(indices, z[f"ns_tl{tl}_indices"])
    for n in (1, 2, 10):
        r = BasePolicy.compute_nstep_return(batch, buf, indices, _test_q_fn, gamma=.1, n_step=n)
        np.testing.assert_array_equal(r.returns.cpu().numpy(), z[f"ns_tl{tl}_n{n}"])


@pytest.mark.gpu
def test_nstep_vector_buffer_matches_reference(z):
    from tianshou_amd.data import Batch, VectorReplayBuffer
    from tianshou_amd.policy import BasePolicy
    E, S = 6, 40
    vb = VectorReplayBuffer(E * S, E, device="cuda")

    def add(ids, rew, te, tr):
        k = len(ids)
        vb.add(Batch(obs=np.zeros((k, 2), np.float32), act=np.zeros(k, np.int64), rew=rew,
                     terminated=te, truncated=tr, obs_next=np.zeros((k, 2), np.float32)),
               buffer_ids=ids)
    _replay_vec_adds(z, add)
    np.testing.assert_array_equal(vb._lengths, z["nsv_lengths"])
    np.testing.assert_array_equal(vb.last_index, z["nsv_last_index"])
    idx = z["nsv_indices"]
    for n in (1, 3, 5, 12):
        for tag, tab in (("x1", z["nsv_table"][:, 0].copy()), ("x3", z["nsv_table"]),
                         ("f64", z["nsv_table64"])):
            def fn(buffer, indices, tab=tab):
                return torch.as_tensor(tab[np.asarray(indices)])
            r = BasePolicy.compute_nstep_return(Batch(), vb, idx, fn, gamma=0.97, n_step=n)
            want = z[f"nsv_n{n}_{tag}"]
            assert r.returns.dtype == (torch.float64 if tag == "f64" else torch.float32)
            np.testing.assert_array_equal(r.returns.cpu().numpy(), want, err_msg=f"n={n} {tag}")


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["vec", "single"])
@pytest.mark.parametrize("alpha", [1.0, 0.6])
def test_prioritized_buffer_matches_reference(z, kind, alpha):
    from tianshou_amd.data import Batch, PrioritizedReplayBuffer, PrioritizedVectorReplayBuffer
    p = f"per_{kind}_a{int(alpha * 10)}_"
    pb = PrioritizedVectorReplayBuffer(60, buffer_num=3, alpha=alpha, beta=0.4, device="cuda") \
        if kind == "vec" else PrioritizedReplayBuffer(20, alpha=alpha, beta=0.4, device="cuda")
    nenv = 3 if kind == "vec" else 1
    for t in range(z[p + "obs"].shape[0]):
        obs = z[p + "obs"][t]
        pb.add(Batch(obs=obs, act=np.zeros(nenv, np.int64), rew=z[p + "rew"][t],
                     terminated=z[p + "term"][t], truncated=np.zeros(nenv, bool), obs_next=obs),
               buffer_ids=list(range(nenv)))
    np.testing.assert_array_equal(pb.weight._value.cpu().numpy(), z[p + "tree0"])
    np.random.seed(12)
    for rnd in range(6):
        batch, idx = pb.sample(16)
        # alpha = 1: the priorities are the TD magnitudes themselves, the tree is bit-exact
        # and so is every sampled index; alpha = 0.6: |td|^0.6 in f32 on the GPU vs NumPy's
        # f32 power can differ by an ulp, which moves a sum by ~1e-7 relative
        np.testing.assert_array_equal(idx, z[p + "sidx"][rnd])
        np.testing.assert_allclose(batch.weight.cpu().numpy(), z[p + "sw"][rnd], rtol=1e-6)
        pb.update_weight(idx, torch.as_tensor(z[p + "td"][rnd], device="cuda"))
        tree = pb.weight._value.cpu().numpy()
        if alpha == 1.0:
            np.testing.assert_array_equal(tree, z[p + "trees"][rnd])
        else:
            np.testing.assert_allclose(tree, z[p + "trees"][rnd], rtol=1e-6)
    np.testing.assert_allclose([pb._max_prio, pb._min_prio], z[p + "prio"], rtol=1e-7)


@pytest.mark.gpu
def test_prioritized_buffer_reference_semantics():
    """test_buffer.py:256-302 restated: weights after update_weight, init weight 1, and
    max/min priority bookkeeping on the vector buffer."""
    from tianshou_amd.data import Batch, PrioritizedVectorReplayBuffer
    buf2 = PrioritizedVectorReplayBuffer(15, buffer_num=3, alpha=0.5, beta=0.5, device="cuda")
    for i in range(25):
        b = Batch(obs=np.full((3, 1), i, np.float32), act=np.ones(3, np.int64),
                  rew=np.zeros(3), terminated=np.array([i % 7 == 6] * 3),
                  truncated=np.zeros(3, bool), obs_next=np.full((3, 1), i + 1, np.float32))
        buf2.add(b, buffer_ids=[0, 1, 2])
        assert len(buf2) == min(15, 3 * (i + 1))
    assert np.allclose(buf2[np.arange(buf2.maxsize)].weight.cpu().numpy(), 1)
    np.random.seed(0)
    batch, indices = buf2.sample(10)
    buf2.update_weight(indices, batch.weight * 0)
    weight = buf2[np.arange(buf2.maxsize)].weight.cpu().numpy()
    mask = np.isin(np.arange(buf2.maxsize), indices)
    assert np.all(weight[mask] == weight[mask][0])
    assert np.all(weight[~mask] == weight[~mask][0])
    assert weight[~mask][0] < weight[mask][0] and weight[mask][0] <= 1
