"""Device np.random.permutation (utils/np_perm.py): bit-exact against NumPy's legacy
RandomState (Batch.split's shuffle, tianshou/data/batch.py:896-912), global state advanced
identically, prefetched draws used only when the state still matches."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def dev():
    return torch.device("cuda", 0)


@pytest.mark.parametrize("n", [1, 2, 3, 5, 100, 4097, 65537, 262144, 4096 * 2048])
def test_device_permutation_matches_numpy(dev, n):
    from tianshou_amd.utils.np_perm import LegacyPermutation
    perm = LegacyPermutation()
    for seed in (0, 3):
        np.random.seed(seed)
        np.random.rand(seed * 101)
        st = np.random.get_state()
        got = perm(n, dev).cpu().numpy()
        st_got = np.random.get_state()
        np.random.set_state(st)
        want = np.random.permutation(n)
        st_want = np.random.get_state()
        np.testing.assert_array_equal(got, want)
        assert st_got[2] == st_want[2] and np.array_equal(st_got[1], st_want[1])


def test_prefetch_stream_and_invalidation(dev):
    from tianshou_amd.utils.np_perm import LegacyPermutation
    perm = LegacyPermutation()
    n = 1 << 20
    np.random.seed(11)
    st = np.random.get_state()
    want = [np.random.permutation(n) for _ in range(5)]
    st_end = np.random.get_state()
    np.random.set_state(st)
    perm.prefetch(n, 3)
    got = [perm(n, dev).cpu().numpy() for _ in range(5)]  # 3 prefetched + 2 synchronous
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)
    assert np.array_equal(np.random.get_state()[1], st_end[1])
    # someone else consumes the global stream after the prefetch: the draws are discarded
    np.random.seed(12)
    perm.prefetch(n, 2)
    np.random.rand(3)
    st = np.random.get_state()
    w = np.random.permutation(n)
    np.random.set_state(st)
    np.testing.assert_array_equal(perm(n, dev).cpu().numpy(), w)
    # a different size than prefetched
    np.random.seed(13)
    perm.prefetch(n, 2)
    st = np.random.get_state()
    w = np.random.permutation(n - 7)
    np.random.set_state(st)
    np.testing.assert_array_equal(perm(n - 7, dev).cpu().numpy(), w)


def test_shuffle_apply_arbitrary_draws(dev):
    """Any valid draw sequence (not only MT19937's) resolves to the sequential swaps."""
    from oracle import ref
    from tianshou_amd import _C
    rng = np.random.default_rng(5)
    for n in (2, 7, 1000, 300001):
        for kind in ("uniform", "zeros", "self", "low"):
            i = np.arange(n, dtype=np.int64)
            if kind == "uniform":
                d = (rng.random(n) * (i + 1)).astype(np.int64)
            elif kind == "zeros":
                d = np.zeros(n, np.int64)
            elif kind == "self":
                d = i.copy()
            else:
                d = np.minimum(i, rng.integers(0, 3, n))
            d[0] = 0
            d = d.astype(np.uint32)
            L = _C.lib()
            wsb = int(L.tsrl_shuffle_apply_workspace_bytes(n))
            ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
            dd = torch.as_tensor(d.view(np.int32), device=dev)
            out = torch.empty(n, dtype=torch.int64, device=dev)
            _C.check(L.tsrl_shuffle_apply(_C.ptr(dd), n, _C.ptr(out), _C.ptr(ws), wsb,
                                          _C.stream_ptr(dev)), "tsrl_shuffle_apply")
            np.testing.assert_array_equal(out.cpu().numpy(), ref.shuffle_apply(d), err_msg=kind)
