"""Buffer persistence without h5py: ReplayBuffer.from_data + set_batch
(tianshou/data/buffer/base.py:109-146) followed by single adds, ReplayBufferManager.set_batch
(manager.py:64-66) in the middle of a ragged VectorReplayBuffer trace, and a pickle round
trip of a device buffer (base.py:81-87), against the reference (tests/golden/persist.npz,
tools/gen_goldens.py gen_persist).  Index math and stored payloads bit-exact.  (save_hdf5 /
load_hdf5 need h5py, which is not installed.)"""
import json
import os
import pickle

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

KEYS = ("obs", "act", "rew", "terminated", "truncated", "obs_next")


def _check(z, p, buf):
    for k in KEYS + ("done",):
        got = getattr(buf, k).cpu().numpy()
        assert np.array_equal(got.astype(z[p + k].dtype), z[p + k]), (p, k)
    n = buf.maxsize
    assert np.array_equal(buf.sample_indices(0), z[p + "sample0"]), p
    assert np.array_equal(buf.unfinished_index(), z[p + "unfinished"]), p
    assert np.array_equal(buf.prev(np.arange(n)), z[p + "prev"]), p
    assert np.array_equal(buf.next(np.arange(n)), z[p + "next"]), p
    assert np.array_equal(buf.last_index, z[p + "last_index"]), p
    assert len(buf) == int(z[p + "len"]), p


def test_from_data_set_batch_and_adds(golden_dir):
    from tianshou_amd.data import Batch, ReplayBuffer
    z = np.load(os.path.join(golden_dir, "persist.npz"))
    g = lambda k: z["fd_in_" + k]  # noqa: E731
    buf = ReplayBuffer.from_data(g("obs"), g("act"), g("rew"), g("terminated"),
                                 g("truncated"), g("done"), g("obs_next"))
    _check(z, "fd0_", buf)
    for i in range(len(z["fd_add_ptr"])):
        one = Batch(**{k: z["fd_add_" + k][i] for k in KEYS})
        ptr, ep_rew, ep_len, ep_idx = buf.add(one)
        assert ptr[0] == z["fd_add_ptr"][i]
        np.testing.assert_array_equal([ep_rew[0], ep_len[0], ep_idx[0]], z["fd_add_ep"][i])
    _check(z, "fd1_", buf)


def test_manager_set_batch_mid_trace_and_pickle(golden_dir):
    from tianshou_amd.data import Batch, VectorReplayBuffer
    z = np.load(os.path.join(golden_dir, "persist.npz"))
    buf = VectorReplayBuffer(24, 3, device=torch.device("cuda", 0))
    for i, ids in enumerate(json.loads(str(z["mg_ids"]))):
        buf.add(Batch(**{k: z[f"mg_add{i}_" + k] for k in KEYS}), buffer_ids=ids)
    _check(z, "mg0_", buf)
    buf.set_batch(Batch(**{k: z["mg_set_" + k] for k in KEYS + ("done",)}))
    _check(z, "mg1_", buf)
    # pickle round trip (storage via host arrays, back into HBM)
    buf = pickle.loads(pickle.dumps(buf))
    assert buf.obs.is_cuda
    _check(z, "mg1_", buf)
    for i, ids in enumerate(json.loads(str(z["mg_ids2"]))):
        ret = buf.add(Batch(**{k: z[f"mg_more{i}_" + k] for k in KEYS}), buffer_ids=ids)
        np.testing.assert_array_equal(np.stack([np.asarray(r, np.float64) for r in ret]),
                                      z[f"mg_more{i}_ret"])
    _check(z, "mg2_", buf)
