"""np.random.permutation of the global legacy RandomState (Batch.split's shuffle,
tianshou/data/batch.py:896-912) reproduced by tsrl_np_shuffle_draws (host MT19937 + masked
rejection) and tsrl_shuffle_apply (device resolution of the swap sequence).

CPU: the host draws, applied by the sequential C checker (oracle.ref.shuffle_apply), equal
NumPy's own permutation, and the advanced (key, pos) equals NumPy's state afterwards, across
seeds, positions inside the 624-word block, successive calls and sizes up to the headline's
8 388 608.  GPU: the device resolution equals NumPy bit for bit (tests/test_gpu_perm.py)."""
import ctypes

import numpy as np
import pytest

from oracle import ref


def _draws(n, st):
    from tianshou_amd import _C
    key = np.ascontiguousarray(st[1], dtype=np.uint32).copy()
    pos = ctypes.c_int32(int(st[2]))
    d = np.empty(max(n, 1), np.uint32)
    rc = _C.lib().tsrl_np_shuffle_draws(key.ctypes.data, ctypes.addressof(pos), n,
                                        d.ctypes.data)
    assert rc == 0
    return d[:n], key, pos.value


@pytest.mark.parametrize("seed", [0, 1, 12345])
def test_draws_match_numpy_small_sizes(seed):
    np.random.seed(seed)
    np.random.rand(seed % 600)  # start inside the 624-word block
    for n in [0, 1, 2, 3, 4, 5, 8, 9, 17, 100, 1023, 1024, 1025, 65537]:
        st = np.random.get_state()
        d, key, pos = _draws(n, st)
        want = np.random.permutation(n)
        st2 = np.random.get_state()
        np.testing.assert_array_equal(ref.shuffle_apply(d), want)
        np.testing.assert_array_equal(st2[1], key)
        assert st2[2] == pos
        assert (d[1:] <= np.arange(1, n)).all()


@pytest.mark.parametrize("seed", [0, 7])
def test_draws_match_numpy_headline_size_successive(seed):
    """Four successive permutations of the 4096 x 2048 headline batch (one PPO update)."""
    np.random.seed(seed)
    n = 4096 * 2048
    for _ in range(4):
        st = np.random.get_state()
        d, key, pos = _draws(n, st)
        want = np.random.permutation(n)
        st2 = np.random.get_state()
        assert st2[2] == pos and np.array_equal(st2[1], key)
        np.testing.assert_array_equal(ref.shuffle_apply(d), want)


def test_draws_reject_bad_arguments():
    from tianshou_amd import _C
    key = np.zeros(624, np.uint32)
    pos = ctypes.c_int32(700)
    d = np.empty(4, np.uint32)
    assert _C.lib().tsrl_np_shuffle_draws(key.ctypes.data, ctypes.addressof(pos), 4,
                                          d.ctypes.data) != 0
    assert b"pos" in _C.lib().tsrl_last_error()


@pytest.mark.parametrize("threads", [1, 4])
def test_threaded_draws_equal_sequential(threads):
    """tsrl_np_shuffle_draws_mt (MT19937 jump-ahead + chunk-parallel masked rejection) gives
    exactly the sequential loop's draws and final RandomState, over successive calls at sizes
    above its 2^21 threshold (the sequential loop is pinned to np.random.permutation above)."""
    import ctypes

    from tianshou_amd import _C
    L = _C.lib()
    rng = np.random.RandomState(2024)
    for n in (1 << 21, 3_000_017, 12_582_912):
        st = rng.get_state()
        out = []
        for fn, extra in ((L.tsrl_np_shuffle_draws, ()), (L.tsrl_np_shuffle_draws_mt, (threads,))):
            k = np.ascontiguousarray(st[1], dtype=np.uint32).copy()
            p = ctypes.c_int32(int(st[2]))
            d = np.empty(n, np.uint32)
            _C.check(fn(k.ctypes.data, ctypes.addressof(p), n, d.ctypes.data, *extra))
            out.append((k, p.value, d))
        assert np.array_equal(out[0][2], out[1][2]), n
        assert np.array_equal(out[0][0], out[1][0]) and out[0][1] == out[1][1], n
        rng.set_state(("MT19937", out[0][0], out[0][1], 0, 0.0))
