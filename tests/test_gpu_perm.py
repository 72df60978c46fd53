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


def test_device_permutation_global_size_successive(dev):
    """The 8-rank global permutation size (8 x 4096 x 2048 rows): threaded host draws
    (csrc/np_perm_mt.cpp) + device resolution equal NumPy over two successive calls."""
    from tianshou_amd.utils.np_perm import LegacyPermutation
    perm = LegacyPermutation()
    n = 8 * 4096 * 2048
    np.random.seed(21)
    st = np.random.get_state()
    got = [perm(n, dev).cpu().numpy() for _ in range(2)]
    st_got = np.random.get_state()
    np.random.set_state(st)
    for g in got:
        np.testing.assert_array_equal(g, np.random.permutation(n))
    st_want = np.random.get_state()
    assert st_got[2] == st_want[2] and np.array_equal(st_got[1], st_want[1])


class _FakeDP:
    """The rank view _issue_plan reads (world, rank, all_gather_cat of one rank's tensor)."""
    active, capturable = True, False

    def __init__(self, world, rank):
        self.world, self.rank = world, rank

    def all_gather_cat(self, t, kind=None):
        return t.repeat(self.world)


@pytest.mark.parametrize("world,rank", [(1, 0), (8, 3)])
def test_plan_pipeline_matches_sequential_split(dev, world, rank):
    """PPOPolicy's pipelined minibatch plans (side-stream permutation, one repeat ahead,
    sync-free share compaction) equal the reference Batch.split over the global batch
    (batch.py:896-912) restricted to this rank's rows, for every repeat, with the global
    RandomState advanced as by ``repeat`` sequential np.random.permutation calls."""
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__)))
    import dist_worker as w
    policy = w.build_policy(23, 5, dev)
    if world > 1:
        policy.dp = _FakeDP(world, rank)
    n, bs, repeat = (1 << 20) + 12345, 1 << 15, 4
    N, B = n * world, bs * world
    np.random.seed(5)
    st = np.random.get_state()
    policy._np_perm.prefetch(N, 2)  # two prefetched, two computed on demand
    policy._np_perm_used = False
    plans = policy._plan_pipeline(n, dev, bs, repeat, True)
    got = [plans(k) for k in range(repeat)]
    torch.cuda.synchronize()
    st_got = np.random.get_state()
    np.random.set_state(st)
    lo = rank * n
    for idx, chunks in got:
        perm = np.random.permutation(N)
        starts = list(range(0, N, B))
        if N - starts[-1] < B and len(starts) > 1:
            starts.pop()  # merge_last
        ends = starts[1:] + [N]
        want_chunks, o = [], 0
        want_idx = []
        for s, e in zip(starts, ends):
            part = perm[s:e]
            mine = part[(part >= lo) & (part < lo + n)] - lo
            want_idx.append(mine)
            want_chunks.append((o, o + len(mine), e - s))
            o += len(mine)
        np.testing.assert_array_equal(idx.cpu().numpy(), np.concatenate(want_idx))
        assert [tuple(c) for c in chunks] == want_chunks
    st_want = np.random.get_state()
    assert st_got[2] == st_want[2] and np.array_equal(st_got[1], st_want[1])
