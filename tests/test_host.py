"""CPU-only checks of the host side: the C-ABI library loads and exports every symbol the
header declares, the host ring arithmetic reproduces the reference buffer traces bit-exactly,
minibatch splitting follows Batch.split, and the Batch container behaves."""
import json
import os
import re

import numpy as np
import pytest

from tests.conftest import ROOT


def _header_symbols():
    with open(os.path.join(ROOT, "include", "tsrl.h")) as f:
        txt = f.read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(tsrl_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    import ctypes
    from tianshou_amd import _C
    syms = _header_symbols()
    assert len(syms) >= 20
    lib = ctypes.CDLL(_C.LIB_PATH)
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) == set(_C.EXPORTED), set(syms) ^ set(_C.EXPORTED)
    assert _C.lib().tsrl_version().startswith(b"tsrl")


def test_ctypes_struct_layout_matches_header(tmp_path):
    """AddArgs / PPOParams / CollectArgs mirror the C structs (sizes via a compiled probe)."""
    import ctypes
    import subprocess
    from tianshou_amd import _C
    src = tmp_path / "probe.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "tsrl.h"\n'
                   'int main(){printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\\n", '
                   'sizeof(tsrl_add_args), '
                   'sizeof(tsrl_ppo_params), offsetof(tsrl_add_args, stat_idx), '
                   'offsetof(tsrl_ppo_params, norm_adv), sizeof(tsrl_collect_args), '
                   'offsetof(tsrl_collect_args, sample), offsetof(tsrl_collect_args, no_moments), '
                   'offsetof(tsrl_collect_args, rms_step), offsetof(tsrl_collect_args, xpipe), '
                   'offsetof(tsrl_collect_args, spec_done));}')
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    assert int(out[0]) == ctypes.sizeof(_C.AddArgs)
    assert int(out[1]) == ctypes.sizeof(_C.PPOParams)
    assert int(out[2]) == _C.AddArgs.stat_idx.offset
    assert int(out[3]) == _C.PPOParams.norm_adv.offset
    assert int(out[4]) == ctypes.sizeof(_C.CollectArgs)
    assert int(out[5]) == _C.CollectArgs.sample.offset
    assert int(out[6]) == _C.CollectArgs.no_moments.offset
    assert int(out[7]) == _C.CollectArgs.rms_step.offset
    assert int(out[8]) == _C.CollectArgs.xpipe.offset
    assert int(out[9]) == _C.CollectArgs.spec_done.offset


@pytest.mark.parametrize("name", ["manager", "ragged"])
def test_ring_index_matches_reference(golden_dir, name):
    from tianshou_amd.data.buffer import RingIndex
    with open(os.path.join(golden_dir, "buffer_traces.json")) as f:
        tr = json.load(f)[name]
    size = int(np.ceil(tr["total"] / tr["num"]))
    ring = RingIndex(size, tr["num"])
    for step in tr["trace"]:
        if step["op"] == "add":
            ptr, _ = ring.advance(np.asarray(step["ids"], np.int64))
            assert ptr.tolist() == step["ptr"]
        else:
            ring.reset()
        st = step["state"]
        assert ring.sample0().tolist() == st["sample0"]
        assert ring.last_index.tolist() == st["last_index"]
        assert ring.lengths.tolist() == st["lengths"]


def test_ring_uniform_fast_paths():
    from tianshou_amd.data.buffer import RingIndex
    ring = RingIndex(16, 8)
    for t in range(16):
        assert ring.uniform_rel() == t
        ptr, nxt = ring.advance(None)
        assert ptr.tolist() == (np.arange(8) * 16 + t).tolist()
    assert ring.is_identity()
    assert ring.sample0().tolist() == list(range(128))
    assert ring.chunk_layout()[0] == 16
    ring.advance(np.array([3]))
    assert ring.uniform_rel() is None and not ring.is_identity()


def test_split_bounds_and_indices(golden_dir):
    from tianshou_amd.data.batch import split_indices
    from tianshou_amd.policy.ppo import split_bounds
    with open(os.path.join(golden_dir, "split.json")) as f:
        g = json.load(f)
    for c in g["cases"]:
        if c["seed"] is not None:
            np.random.seed(c["seed"])
        parts = split_indices(c["n"], c["size"], c["shuffle"], c["merge_last"])
        assert [p.tolist() for p in parts] == c["parts"]
        if c["merge_last"]:
            b = split_bounds(c["n"], c["size"], True)
            assert [e - s for s, e in b] == [len(p) for p in c["parts"]]


def test_batch_container():
    from tianshou_amd.data import Batch
    b = Batch(obs=np.arange(10).reshape(5, 2), rew=np.arange(5.0), info={"env_id": np.arange(5)})
    assert len(b) == 5
    s = b[np.array([4, 0])]
    assert s.obs.tolist() == [[8, 9], [0, 1]] and s.info.env_id.tolist() == [4, 0]
    b[np.array([1])] = Batch(rew=np.array([7.0]))
    assert b.rew[1] == 7.0
    parts = list(b.split(2, shuffle=False, merge_last=True))
    assert [len(p) for p in parts] == [2, 3]
    with pytest.raises(AssertionError):
        list(b.split(0))


def test_product_refuses_cpu_tensors():
    """No CPU fallback: kernels only take HIP device tensors."""
    import torch
    from tianshou_amd import _C
    with pytest.raises(_C.TsrlError):
        _C.ptr(torch.zeros(3))


def test_device_stats_construct_without_gpu_use():
    """Host-side state of the device statistics objects (constructed on CPU tensors; no
    kernel is launched)."""
    from tianshou_amd.utils.statistics import DeviceRunningMeanStd, DeviceScalarRMS
    r = DeviceRunningMeanStd(4, "cpu")
    assert r.dp is None and r.count == 0 and r.mean.tolist() == [0.0] * 4
    r.sync_with("dp")
    assert r.dp == "dp"
    s = DeviceScalarRMS("cpu")
    assert (s.mean, s.var, s.count) == (0.0, 1.0, 0)


@pytest.mark.parametrize("n,bs", [(1024, 128), (1000, 128), (1000, 300), (7, 10)])
def test_sorted_minibatch_permutation_same_sets(n, bs):
    """PPOPolicy.sort_minibatch: each minibatch holds the same rows as Batch.split over the
    reference's np.random.permutation stream, visited in ascending order."""
    import types
    import torch
    from tianshou_amd.policy.ppo import PPOPolicy, split_bounds
    # host logic only: the device permutation itself is tests/test_gpu_perm.py
    fake = types.SimpleNamespace(perm_device=False, sort_minibatch=True,
                                 _np_perm=lambda k, d: torch.as_tensor(np.random.permutation(k)))
    np.random.seed(5)
    got = PPOPolicy._permutation(fake, n, torch.device("cpu"), bs).numpy()
    np.random.seed(5)
    want = np.random.permutation(n)
    for s, e in split_bounds(n, bs, merge_last=True):
        np.testing.assert_array_equal(got[s:e], np.sort(want[s:e]))


@pytest.mark.parametrize("n,bs", [(1024, 128), (1000, 128), (1000, 300), (7, 10)])
def test_sorted_minibatch_device_labels(n, bs):
    """Device path of sort_minibatch: the returned order is a permutation whose Batch.split
    chunks are ascending and have the split sizes."""
    import types
    import torch
    from tianshou_amd.policy.ppo import PPOPolicy, split_bounds
    fake = types.SimpleNamespace(perm_device=True, sort_minibatch=True)
    torch.manual_seed(0)
    got = PPOPolicy._permutation(fake, n, torch.device("cpu"), bs).numpy()
    np.testing.assert_array_equal(np.sort(got), np.arange(n))
    for s, e in split_bounds(n, bs, merge_last=True):
        assert np.all(np.diff(got[s:e]) > 0)


def test_exact_group_clamped_to_library_bound():
    """the pipelined exact obs_rms carries at most tsrl_rms_exact_stats_max_steps()
    steps per statistics launch (rms.hip XSTEPS) and at most exact_pipeline - 1 (the group's
    last rows must exist before its first step is merged); Collector._xpipe_group clamps to
    both (no GPU call: the bound is a host-side constant of the library)."""
    import types
    from tianshou_amd import _C
    from tianshou_amd.data.collector import Collector
    cap = int(_C.lib().tsrl_rms_exact_stats_max_steps())
    assert cap >= 2
    grp = lambda g, d: Collector._xpipe_group(types.SimpleNamespace(  # noqa: E731
        exact_group=g, exact_pipeline=d))
    assert grp(2, 5) == 2
    assert grp(cap + 3, cap + 10) == cap
    assert grp(6, 3) == 2
    assert grp(4, 1) == 1
