"""GAE parity on the GPU: tsrl_gae vs the reference goldens and the C oracle.

Tolerance: f32 outputs allclose(rtol=1e-5, atol=1e-6*max|ref|) -- a pure rtol
is ill-posed at near-zero advantages; the bit-exact fraction is
reported and required to be high.  f64 outputs (the general path's carries re-associate only
at 8-element thread boundaries) must agree to ~1e-12 relative.
"""
import os

import numpy as np
import pytest
import torch

from oracle import ref

pytestmark = pytest.mark.gpu


def _tol(got, want, rtol=1e-5):
    want = np.asarray(want, np.float64)
    np.testing.assert_allclose(np.asarray(got, np.float64), want, rtol=rtol,
                               atol=1e-6 * max(np.abs(want).max(), 1e-30))


def _bitexact_frac(got32, want64):
    return float(np.mean(np.asarray(got32, np.float32) == np.asarray(want64).astype(np.float32)))


@pytest.fixture(scope="module")
def dev():
    return torch.device("cuda", 0)


def test_known_answers_device(golden_dir, dev):
    """test/base/test_returns.py:22-112 through BasePolicy.compute_episodic_return."""
    from tianshou_amd.data import Batch, ReplayBuffer
    from tianshou_amd.policy import BasePolicy
    z = np.load(os.path.join(golden_dir, "returns_known.npz"))
    for c in range(int(z["ncases"])):
        p = f"c{c}_"
        buf = ReplayBuffer(20, device=dev)
        n = len(z[p + "rew"])
        for i in range(n):
            buf.add(Batch(obs=1, act=1, rew=z[p + "rew"][i], terminated=z[p + "term"][i],
                          truncated=z[p + "trunc"][i]))
        idx = buf.sample_indices(0)
        assert idx.tolist() == z[p + "indices"].tolist()
        assert buf.unfinished_index().tolist() == z[p + "unfinished"].tolist()
        batch = Batch(rew=z[p + "rew"], terminated=z[p + "term"], truncated=z[p + "trunc"])
        v = z[p + "v_next"] if bool(z[p + "has_v"]) else None
        ret, adv = BasePolicy.compute_episodic_return(batch, buf, idx, v, None,
                                                      float(z[p + "gamma"]), float(z[p + "lam"]))
        np.testing.assert_allclose(ret, z[p + "returns"], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(adv, z[p + "adv"], rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("tag", ["full", "wrap", "part"])
@pytest.mark.parametrize("scaled", [False, True])
def test_gae_random_golden_general_path(golden_dir, dev, tag, scaled):
    """Reference outputs on VectorReplayBuffer.sample(0) layouts (full / wrapped / partial)
    through the general (any index order) path with the unfinished mask."""
    from tianshou_amd.policy.base import gae_device
    z = np.load(os.path.join(golden_dir, "gae_random.npz"))
    p = tag + "_"
    extra = np.isin(z[p + "indices"], z[p + "unfinished"]).astype(np.uint8)
    t = lambda a, dt=None: torch.as_tensor(np.ascontiguousarray(a), device=dev, dtype=dt)
    scale = t(np.array([z[p + "scale"]]), torch.float64) if scaled else None
    adv32, ret32, adv64, ret64 = gae_device(
        t(z[p + "v_s"]), t(z[p + "v_s_"]), t(z[p + "rew"]), t(z[p + "term"]),
        t(z[p + "trunc"]), 0.99, 0.95, 0, t(extra), scale, want_f64=True)
    want_adv = z[p + ("adv_scaled" if scaled else "adv")]
    want_ret = z[p + ("returns_scaled" if scaled else "returns")]
    np.testing.assert_allclose(adv64.cpu().numpy(), want_adv, rtol=1e-11, atol=1e-11)
    np.testing.assert_allclose(ret64.cpu().numpy(), want_ret, rtol=1e-11, atol=1e-11)
    _tol(adv32.cpu().numpy(), want_adv)
    want_r32 = want_ret / float(z[p + "scale"]) if scaled else want_ret
    _tol(ret32.cpu().numpy(), want_r32)
    assert _bitexact_frac(adv32.cpu().numpy(), want_adv) > 0.999


def test_gae_full_golden_fast_path(golden_dir, dev):
    """The one-pass row path (row_len = per-env chunk) on the full on-policy layout."""
    from tianshou_amd.policy.base import gae_device
    z = np.load(os.path.join(golden_dir, "gae_random.npz"))
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)
    T = int(z["full_steps"])
    adv32, ret32, adv64, ret64 = gae_device(
        t(z["full_v_s"]), t(z["full_v_s_"]), t(z["full_rew"]), t(z["full_term"]),
        t(z["full_trunc"]), 0.99, 0.95, T, None, None, want_f64=True)
    np.testing.assert_allclose(adv64.cpu().numpy(), z["full_adv"], rtol=1e-11, atol=1e-11)
    _tol(adv32.cpu().numpy(), z["full_adv"])
    _tol(ret32.cpu().numpy(), z["full_returns"])
    assert _bitexact_frac(adv32.cpu().numpy(), z["full_adv"]) > 0.999


@pytest.mark.parametrize("envs,steps", [(4096, 2048), (512, 128), (3, 5000), (7, 1000),
                                        (80, 32), (48, 32)])
def test_gae_full_size_vs_c_oracle(dev, envs, steps):
    """BASELINE sizes (4096x2048 = 8.4M transitions) against the C oracle, both paths."""
    from tianshou_amd.policy.base import gae_device
    g = torch.Generator(device=dev).manual_seed(envs * 7 + steps)
    n = envs * steps
    v_s = torch.randn(n, device=dev, generator=g)
    v_n = torch.randn(n, device=dev, generator=g)
    rew = torch.rand(n, device=dev, generator=g, dtype=torch.float64)
    u = torch.rand(n, device=dev, generator=g)
    term = u < 0.001
    trunc = (u > 0.999) & ~term
    # host oracle: unfinished = every env's last row
    idx = np.arange(n)
    unfinished = np.arange(steps - 1, n, steps)
    ret_o, adv_o = ref.compute_episodic_return(rew.cpu().numpy(), term.cpu().numpy(),
                                               trunc.cpu().numpy(), idx, unfinished,
                                               v_n.cpu().numpy(), v_s.cpu().numpy(), 0.99, 0.95)
    for row_len, extra in ((steps, None), (0, None)):
        if row_len == 0:
            m = np.zeros(n, np.uint8)
            m[unfinished] = 1
            extra = torch.as_tensor(m, device=dev)
        adv32, ret32, adv64, _ = gae_device(v_s, v_n, rew, term, trunc, 0.99, 0.95, row_len,
                                            extra, None, want_f64=True)
        a64 = adv64.cpu().numpy()
        np.testing.assert_allclose(a64, adv_o, rtol=1e-10, atol=1e-10 * np.abs(adv_o).max())
        _tol(adv32.cpu().numpy(), adv_o)
        _tol(ret32.cpu().numpy(), ret_o)
        assert _bitexact_frac(adv32.cpu().numpy(), adv_o) > 0.999


def test_gae_edge_cases(dev):
    """Empty input, one element, all-done, no-done (one long segment: general path must carry
    across every tile), misaligned views (scalar load path)."""
    from tianshou_amd.policy.base import gae_device
    z = torch.zeros(0, device=dev)
    out = gae_device(z, z, z.double(), z.bool(), z.bool(), 0.99, 0.95, 0)
    assert out[0].numel() == 0
    for n, p_end in ((1, 0.0), (10000, 1.0), (100003, 0.0), (70001, 0.01)):
        v_s = torch.randn(n + 1, device=dev)[1:]  # misaligned views
        v_n = torch.randn(n + 1, device=dev)[1:]
        rew = torch.rand(n + 1, device=dev, dtype=torch.float64)[1:]
        term = (torch.rand(n, device=dev) < p_end)
        trunc = torch.zeros(n, dtype=torch.bool, device=dev)
        ret_o, adv_o = ref.compute_episodic_return(
            rew.cpu().numpy(), term.cpu().numpy(), trunc.cpu().numpy(), np.arange(n),
            np.array([n - 1]), v_n.cpu().numpy(), v_s.cpu().numpy(), 0.99, 0.95)
        m = np.zeros(n, np.uint8)
        m[n - 1] = 1
        adv32, ret32, adv64, _ = gae_device(v_s.contiguous(), v_n.contiguous(),
                                            rew.contiguous(), term, trunc, 0.99, 0.95, 0,
                                            torch.as_tensor(m, device=dev), want_f64=True)
        np.testing.assert_allclose(adv64.cpu().numpy(), adv_o, rtol=1e-9,
                                   atol=1e-9 * max(1.0, np.abs(adv_o).max()))
        _tol(ret32.cpu().numpy(), ret_o)


def test_ret_rms_update(dev):
    """rew_norm: ret_rms folded from the GAE kernel's per-block Welford partials equals
    RunningMeanStd.update on the unnormalised f64 returns (statistics.py:93-114)."""
    from tianshou_amd.policy.base import gae_device
    from tianshou_amd.utils.statistics import DeviceScalarRMS
    from tianshou_amd import _C
    n, T = 64 * 300, 300
    g = torch.Generator(device=dev).manual_seed(3)
    v_s = torch.randn(n, device=dev, generator=g)
    v_n = torch.randn(n, device=dev, generator=g)
    rew = torch.rand(n, device=dev, generator=g, dtype=torch.float64)
    term = torch.zeros(n, dtype=torch.bool, device=dev)
    rms = DeviceScalarRMS(dev)
    host = ref.RMS()
    for it in range(3):
        scale = (rms.state[1:2] + 1e-8).sqrt()
        nparts = int(_C.lib().tsrl_gae_num_partials(n, T))
        parts = torch.empty(nparts * 3, dtype=torch.float64, device=dev)
        _, ret32, _, ret64 = gae_device(v_s, v_n, rew, term, term, 0.99, 0.95, T, None, scale,
                                        want_f64=True, ret_partials=parts)
        s_host = np.sqrt(host.var + 1e-8)
        ret_o, _ = ref.compute_episodic_return(
            rew.cpu().numpy(), term.cpu().numpy(), term.cpu().numpy(), np.arange(n),
            np.arange(T - 1, n, T), v_n.cpu().numpy() * s_host, v_s.cpu().numpy() * s_host,
            0.99, 0.95)
        np.testing.assert_allclose(ret64.cpu().numpy(), ret_o, rtol=1e-10)
        _tol(ret32.cpu().numpy(), ret_o / s_host)
        rms.update_from_partials(parts, nparts)
        host.update(ret_o)
        np.testing.assert_allclose(rms.mean, host.mean, rtol=1e-10)
        np.testing.assert_allclose(rms.var, host.var, rtol=1e-10)
        assert rms.count == host.count


@pytest.mark.parametrize("envs,steps", [(4096, 2048), (64, 4096), (256, 128), (96, 512),
                                        (80, 32), (48, 32), (600, 2048), (3, 6144)])
@pytest.mark.parametrize("scaled", [False, True])
def test_gae_staged_rows_kernel(dev, envs, steps, scaled, monkeypatch):
    """The LDS-staged row kernel (f32 outputs only, rows a multiple of the 2048-transition
    tile -- the layout process_fn hands over) gives the same bits as the per-thread-load row
    kernel (adv, ret, ret_rms partials) and matches the C oracle."""
    from tianshou_amd.policy.base import gae_device
    from tianshou_amd import _C
    g = torch.Generator(device=dev).manual_seed(envs + 11 * steps)
    n = envs * steps
    v_s = torch.randn(n, device=dev, generator=g)
    v_n = torch.randn(n, device=dev, generator=g)
    rew = torch.rand(n, device=dev, generator=g, dtype=torch.float64)
    u = torch.rand(n, device=dev, generator=g)
    term = u < 0.002
    trunc = (u > 0.998) & ~term
    scale = torch.tensor([1.37], dtype=torch.float64, device=dev) if scaled else None
    nparts = int(_C.lib().tsrl_gae_num_partials(n, steps))
    outs = []
    for mode in ("staged", "unstaged"):
        if mode == "unstaged":
            monkeypatch.setenv("TSRL_GAE_UNSTAGED", "1")
        parts = torch.full((nparts * 3,), -1.0, dtype=torch.float64, device=dev) if scaled \
            else None
        adv32, ret32, _, _ = gae_device(v_s, v_n, rew, term, trunc, 0.99, 0.95, steps, None,
                                        scale, ret_partials=parts)
        outs.append((adv32.cpu().numpy(), ret32.cpu().numpy(),
                     None if parts is None else parts.cpu().numpy()))
    monkeypatch.delenv("TSRL_GAE_UNSTAGED")
    a0, r0, p0 = outs[0]
    for a1, r1, p1 in outs[1:]:
        np.testing.assert_array_equal(a0, a1)
        np.testing.assert_array_equal(r0, r1)
        if scaled:
            np.testing.assert_array_equal(p0, p1)
    s = 1.37 if scaled else 1.0
    ret_o, adv_o = ref.compute_episodic_return(
        rew.cpu().numpy(), term.cpu().numpy(), trunc.cpu().numpy(), np.arange(n),
        np.arange(steps - 1, n, steps), v_n.cpu().numpy().astype(np.float64) * s
        if scaled else v_n.cpu().numpy(), v_s.cpu().numpy().astype(np.float64) * s
        if scaled else v_s.cpu().numpy(), 0.99, 0.95)
    _tol(a0, adv_o)
    _tol(r0, ret_o / s)


@pytest.mark.parametrize("envs,steps", [(700, 2048), (5, 4096), (256, 512)])
def test_gae_row_kernels_end_extra(dev, envs, steps, monkeypatch):
    """The extra end flags (process_fn's unfinished-episode mask) through the staged and the
    per-thread-load row kernels: the same bits (adv, ret, partials)."""
    from tianshou_amd.policy.base import gae_device
    from tianshou_amd import _C
    g = torch.Generator(device=dev).manual_seed(7 * envs + steps)
    n = envs * steps
    v_s = torch.randn(n, device=dev, generator=g)
    v_n = torch.randn(n, device=dev, generator=g)
    rew = torch.rand(n, device=dev, generator=g, dtype=torch.float64)
    u = torch.rand(n, device=dev, generator=g)
    term = u < 0.003
    trunc = (u > 0.997) & ~term
    extra = ((u > 0.5) & (u < 0.503)).to(torch.uint8)
    scale = torch.tensor([0.71], dtype=torch.float64, device=dev)
    nparts = int(_C.lib().tsrl_gae_num_partials(n, steps))
    outs = []
    for mode in ("staged", "unstaged"):
        if mode == "unstaged":
            monkeypatch.setenv("TSRL_GAE_UNSTAGED", "1")
        parts = torch.full((nparts * 3,), -1.0, dtype=torch.float64, device=dev)
        adv32, ret32, _, _ = gae_device(v_s, v_n, rew, term, trunc, 0.99, 0.95, steps, extra,
                                        scale, ret_partials=parts)
        outs.append((adv32.cpu().numpy(), ret32.cpu().numpy(), parts.cpu().numpy()))
    monkeypatch.delenv("TSRL_GAE_UNSTAGED")
    for o in outs[1:]:
        for x, y in zip(outs[0], o):
            np.testing.assert_array_equal(x, y)


def test_gae_time_next_kernel_events(dev):
    """tsrl_gae_time_next (bench.py's roofline timer): the next row-path launch records its
    kernel's start / stop into the two HIP events (hipExtLaunchKernel) -- outputs unchanged,
    a positive duration -- and the setting is consumed by that one launch."""
    from tianshou_amd.policy.base import gae_device
    from tianshou_amd import _C
    envs, steps = 1024, 2048
    g = torch.Generator(device=dev).manual_seed(5)
    n = envs * steps
    v_s = torch.randn(n, device=dev, generator=g)
    v_n = torch.randn(n, device=dev, generator=g)
    rew = torch.rand(n, device=dev, generator=g, dtype=torch.float64)
    u = torch.rand(n, device=dev, generator=g)
    term, trunc = u < 0.002, u > 0.998
    plain = gae_device(v_s, v_n, rew, term, trunc, 0.99, 0.95, steps)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    b.record()
    assert _C.lib().tsrl_gae_time_next(a.cuda_event, b.cuda_event) == 0
    timed = gae_device(v_s, v_n, rew, term, trunc, 0.99, 0.95, steps)
    again = gae_device(v_s, v_n, rew, term, trunc, 0.99, 0.95, steps)  # no events: consumed
    torch.cuda.synchronize()
    ms = a.elapsed_time(b)
    assert 0.0 < ms < 50.0, ms
    for x, y, z in zip(plain[:2], timed[:2], again[:2]):
        assert torch.equal(x, y) and torch.equal(x, z)
    assert _C.lib().tsrl_gae_time_next(a.cuda_event, None) != 0  # both or neither
