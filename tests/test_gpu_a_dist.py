"""Data-parallel (env-sharded) PPO update with 2 and 4 ranks on one MI355X over gloo: one global
minibatch split across ranks must give the single-process full-batch update (up to
summation order) -- one minibatch, and several global minibatches of the reference's
Batch.split over the global batch (every rank draws the same permutation) -- and the default
global obs_rms must leave every rank with the statistics of ONE VectorEnvNormObs over all
env shards (checked against the NumPy env and a host RunningMeanStd).

Runs first among the GPU tests (file name), and both rank groups (6 processes) are started
together by a module fixture before any test body touches the GPU, so that this pytest
process has not initialised HIP when it starts the rank processes."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def rank_runs(tmp_path_factory):
    """Both rank groups (2 and 4 ranks, gloo) run concurrently, before the parent process
    initialises HIP; returns {world: output directory}."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    dirs, procs = {}, []
    for world in (2, 4):
        port = str(_free_port())
        d = tmp_path_factory.mktemp(f"dp{world}")
        dirs[world] = d
        procs += [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "dist_worker.py"),
                                    str(r), str(world), port, str(d)], env=env)
                  for r in range(world)]
    # BASELINE config 4's per-rank shape, 2 ranks (dist_c4_worker.py)
    port = str(_free_port())
    d = tmp_path_factory.mktemp("c4")
    dirs["c4"] = d
    procs += [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "dist_c4_worker.py"),
                                str(r), "2", port, str(d)], env=env) for r in range(2)]
    # unequal env shards (48 + 80 envs), fused collect step, global split (dist_unequal_worker)
    port = str(_free_port())
    d = tmp_path_factory.mktemp("uneq")
    dirs["uneq"] = d
    procs += [subprocess.Popen([sys.executable,
                                os.path.join(ROOT, "tests", "dist_unequal_worker.py"),
                                str(r), "2", port, str(d)], env=env) for r in range(2)]
    rcs = [p.wait(timeout=600) for p in procs]
    assert rcs == [0] * len(procs), rcs
    return dirs


@pytest.mark.parametrize("world", [2, 4])
def test_rank_update_matches_single_process(rank_runs, world):
    outs = [torch.load(rank_runs[world] / f"rank{r}.pt", weights_only=True)
            for r in range(world)]
    r0 = outs[0]
    for r1 in outs[1:]:
        # identical parameters on every rank
        for k in r0["sd"]:
            assert torch.equal(r0["sd"][k], r1["sd"][k]), k
        np.testing.assert_allclose(r0["loss"].numpy(), r1["loss"].numpy(), rtol=1e-6)
        # global obs_rms identical on every rank, counting every shard's rows
        assert torch.equal(r0["rms_mean"], r1["rms_mean"])
        assert torch.equal(r0["rms_var"], r1["rms_var"])
        assert int(r0["rms_count"]) == int(r1["rms_count"]) > 0
        for k in r0["sd2"]:
            assert torch.equal(r0["sd2"][k], r1["sd2"][k]), k
        torch.testing.assert_close(r0["loss2"], r1["loss2"], rtol=1e-6, atol=0)
    # single-process reference: the whole batch as one minibatch
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import dist_worker as w
    dev = torch.device("cuda", 0)
    data = w.make_data(4096, 23, 5, dev)
    policy = w.build_policy(23, 5, dev)
    from tianshou_amd.data import Batch
    np.random.seed(0)
    res = policy.learn(Batch(**data), batch_size=4096, repeat=1)
    np.testing.assert_allclose(r0["loss"].numpy(), res["loss"], rtol=1e-4, atol=1e-6)
    sd = policy.state_dict()
    # one Adam step moves a weight by up to lr = 3e-4 whatever its gradient's size, so a
    # near-zero gradient summed in another order can move it differently: atol = lr / 3
    for k, v in r0["sd"].items():
        np.testing.assert_allclose(v.numpy(), sd[k].cpu().numpy(), rtol=1e-4, atol=1e-4)
    # global minibatches of 256 x world rows (rank shares of varying size), 2 repeats
    policy2 = w.build_policy(23, 5, dev)
    np.random.seed(0)
    res2 = policy2.learn(Batch(**data), batch_size=256 * world, repeat=2)
    want = np.array([res2[k] for k in ("loss", "loss/clip", "loss/vf", "loss/ent")])
    assert want.shape == tuple(r0["loss2"].shape) == (4, 2 * 4096 // (256 * world))
    np.testing.assert_allclose(r0["loss2"].numpy(), want, rtol=1e-4, atol=1e-5)
    sd2 = policy2.state_dict()
    for k, v in r0["sd2"].items():
        np.testing.assert_allclose(v.numpy(), sd2[k].cpu().numpy(), rtol=1e-4, atol=1e-4)
    # obs_rms of one VectorEnvNormObs over both shards: NumPy env (rank r = seed r, E envs)
    # and a RunningMeanStd with f64 batch moments stored as f32 (the device recipe)
    from oracle.synth_env import SynthVecEnvNP
    E, T, D = 32, 24, 23
    envs = [SynthVecEnvNP(E, (D,), 5, 9, seed=r) for r in range(world)]
    mean, var, count = np.zeros(D, np.float32), np.ones(D, np.float32), 0.0

    def upd(x):
        nonlocal mean, var, count
        if len(x) == 0:
            return
        x = x.astype(np.float64)
        bm, bv, bc = x.mean(0), x.var(0), float(len(x))
        delta = bm - mean
        tot = count + bc
        nm = mean + delta * bc / tot
        m2 = var * count + bv * bc + delta ** 2 * count * bc / tot
        mean, var, count = nm.astype(np.float32), (m2 / tot).astype(np.float32), tot

    upd(np.concatenate([e.reset() for e in envs]))
    for _ in range(T):
        outs = [e.step() for e in envs]
        upd(np.concatenate([o[0] for o in outs]))
        resets = []
        for e, o in zip(envs, outs):
            ids = np.flatnonzero(o[2] | o[3])
            if len(ids):
                resets.append(e.reset(ids))
        upd(np.concatenate(resets) if resets else np.zeros((0, D), np.float32))
    assert int(r0["rms_count"]) == int(count)
    np.testing.assert_allclose(r0["rms_mean"].numpy(), mean, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(r0["rms_var"].numpy(), var, rtol=1e-5, atol=1e-6)


def test_config4_shape_dp_update(rank_runs):
    """2 ranks x 512 envs x 2048 steps x D = 376 (config 4's per-rank shape): global obs_rms
    collect + one update with the global-batch split equals the single process over the
    union of both ranks' envs (dist_c4_worker.py)."""
    r = torch.load(rank_runs["c4"] / "c4.pt", weights_only=True)
    assert r["rms_count"] >= 2 * 512 * 2049  # both shards' reset + step rows (+ auto-resets)
    assert r["loss"].shape == r["loss_ref"].shape == (4, 32)
    np.testing.assert_allclose(r["loss"].numpy(), r["loss_ref"].numpy(), rtol=1e-4, atol=1e-6)
    for k, v in r["sd"].items():
        # one Adam step moves a weight by up to lr = 3e-4: atol = lr / 3
        np.testing.assert_allclose(v.numpy(), r["sd_ref"][k].numpy(), rtol=1e-4, atol=1e-4,
                                   err_msg=k)


def test_unequal_env_shards(rank_runs):
    """Data parallelism over unequal env shards (48 and 80 envs, D = 376, the fused collect
    step; dist_unequal_worker.py): every rank holds the obs_rms of ONE VectorEnvNormObs over
    all 128 envs (count exact, mean / var vs a host RunningMeanStd over the NumPy env at the
    device recipe's tolerance), and one update with the global-batch split equals the single
    process over the union (venv_wrappers.py:93-99, batch.py:896-912)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import dist_unequal_worker as w
    r = torch.load(rank_runs["uneq"] / "uneq.pt", weights_only=True)
    assert torch.equal(r["rms_mean"], r["rms_mean1"]) and torch.equal(r["rms_var"], r["rms_var1"])
    from oracle.synth_env import SynthVecEnvNP
    envs = [SynthVecEnvNP(E, (w.D,), w.A, w.L, seed=k) for k, E in enumerate(w.SHARDS)]
    mean, var, count = np.zeros(w.D), np.ones(w.D), 0.0

    def upd(x):
        nonlocal mean, var, count
        if len(x) == 0:
            return
        x = x.astype(np.float64)
        bm, bv, bc = x.mean(0), x.var(0), float(len(x))
        delta = bm - mean
        tot = count + bc
        mean, var = mean + delta * bc / tot, \
            (var * count + bv * bc + delta ** 2 * count * bc / tot) / tot
        count = tot

    upd(np.concatenate([e.reset() for e in envs]))
    for _ in range(w.T):
        outs = [e.step() for e in envs]
        upd(np.concatenate([o[0] for o in outs]))
        resets = [e.reset(np.flatnonzero(o[2] | o[3])) for e, o in zip(envs, outs)
                  if (o[2] | o[3]).any()]
        upd(np.concatenate(resets) if resets else np.zeros((0, w.D), np.float32))
    assert int(r["rms_count"]) == int(count)
    np.testing.assert_allclose(r["rms_mean"].numpy(), mean, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(r["rms_var"].numpy(), var, rtol=1e-5, atol=1e-6)
    assert r["loss"].shape == r["loss_ref"].shape == (4, sum(w.SHARDS) * w.T // (2 * w.BS))
    print("unequal shards: losses (dp, single)\n", r["loss"].numpy(), "\n", r["loss_ref"].numpy())
    for k, v in r["pf"].items():
        ref = r["pf_ref"][k]
        err = (v - ref).abs().max().item()
        print(f"process_fn {k}: max |dp - single| {err:.3g} (max |single| {ref.abs().max():.3g})")
        bad = np.flatnonzero(~np.isclose(v.numpy(), ref.numpy(), rtol=1e-4, atol=1e-5))
        if len(bad):
            n0 = w.SHARDS[0] * w.T
            print(f"  mismatched rows: {int((bad < n0).sum())} of rank 0's {n0}, "
                  f"{int((bad >= n0).sum())} of rank 1's; first {bad[:12].tolist()}, "
                  f"step-in-env {(bad[:12] % w.T).tolist()}")
            print("  dp    ", v.numpy()[bad[:8]], "\n  single", ref.numpy()[bad[:8]])
        np.testing.assert_allclose(v.numpy(), ref.numpy(), rtol=1e-4, atol=1e-5, err_msg=k)
    # per-minibatch loss terms of 512-row global minibatches (the tolerance of the 2/4-rank
    # test's 256 x world minibatches)
    np.testing.assert_allclose(r["loss"].numpy(), r["loss_ref"].numpy(), rtol=1e-4, atol=1e-5)
    for k, v in r["sd"].items():
        # one Adam step moves a weight by up to lr = 3e-4: atol = lr / 3
        np.testing.assert_allclose(v.numpy(), r["sd_ref"][k].numpy(), rtol=1e-4, atol=1e-4,
                                   err_msg=k)
