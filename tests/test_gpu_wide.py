"""The headline path's obs_rms at the PRODUCTION row count against the reference's arithmetic
(VERDICT r04 item 1).  The reference normalises observations with RunningMeanStd updated per
vector step by NumPy's axis-0 f32 mean / var over every env's row (statistics.py:99-114,
venv_wrappers.py:93-99); its rounding grows with the row count, so the 16-env goldens of
test_gpu_rollout.py do not pin the 4096-env headline.  tools/gen_goldens.py gen_collector_wide
records the reference Collector + VectorEnvNormObs + process_fn at 4096 envs x D = 376 x 8
steps (obs_rms after every step, process_fn's v_s / returns / adv, ret_rms); gen_rms_wide one
[4096, 376] update pair.

Tolerances: exact_obs_rms=True must reproduce the reference statistic bit for bit at every
step; returns / adv (and V) within north_star's rtol 1e-5, atol 1e-6 * max|ref|, in BOTH
modes -- the default (exact int64 moments, f64 merge) is more accurate than NumPy's f32 sums,
and this test measures whether that difference stays inside the budget at 4096 rows.  The
default mode's obs_rms error against the reference is printed (ratio to rtol 1e-5)."""
import os

import numpy as np
import pytest
import torch

from oracle import synth_env

from .test_gpu_rollout import _check_stats, _collector_setup, _pf_errors

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    return torch.device("cuda", 0)


def _ratio(got, want, rtol=1e-5, atol=1e-7):
    """max |got - want| / (rtol |want| + atol): <= 1 passes assert_allclose(rtol, atol)."""
    got, want = np.asarray(got, np.float64), np.asarray(want, np.float64)
    return float((np.abs(got - want) / (rtol * np.abs(want) + atol)).max())


@pytest.mark.parametrize("exact", [False, True])
def test_rms_update_production_rows(golden_dir, dev, exact):
    """Two RunningMeanStd updates of [4096, 376] env rows on the device: the exact kernel
    (tsrl_rms_exact_update) equals the reference bitwise; the default f64-moment update
    within rtol 1e-5 of the reference's f32 statistic (mean, var)."""
    from tianshou_amd.utils.statistics import DeviceRunningMeanStd
    z = np.load(os.path.join(golden_dir, "rms_wide.npz"))
    E, D = int(z["E"]), int(z["D"])
    r = DeviceRunningMeanStd(D, dev, exact=exact)
    for i in range(2):
        k = synth_env.key(0, np.arange(E), np.zeros(E, np.int64), np.full(E, int(z[f"t{i}"])))
        r.update(torch.as_tensor(synth_env.box_obs(k, D), device=dev))
        assert r.count == int(z[f"count{i}"])
        if exact:
            assert np.array_equal(r.mean, z[f"mean{i}"]), i
            assert np.array_equal(r.var, z[f"var{i}"]), i
        else:
            rm, rv = _ratio(r.mean, z[f"mean{i}"]), _ratio(r.var, z[f"var{i}"])
            print(f"update {i}: default obs_rms vs reference, max err / (rtol 1e-5, atol 1e-7): "
                  f"mean {rm:.3g}, var {rv:.3g}")
            np.testing.assert_allclose(r.mean, z[f"mean{i}"], rtol=1e-5, atol=1e-7)
            np.testing.assert_allclose(r.var, z[f"var{i}"], rtol=1e-5)


@pytest.mark.parametrize("exact", [False, True])
def test_headline_width_production_rows_matches_reference(golden_dir, dev, exact):
    """4096 envs x D = 376 through the fused one-launch collect step, one vector step per
    collect (obs_rms read after each), then sample(0) -> fused process_fn, against the
    reference run of gen_collector_wide."""
    from tianshou_amd.data import Collector, VectorReplayBuffer
    from tianshou_amd.env import SyntheticVectorEnv, VectorEnvNormObs
    z = np.load(os.path.join(golden_dir, "collector_wide.npz"))
    _, policy, _, _, (E, D, A, L, T) = _collector_setup(z, dev)
    env = VectorEnvNormObs(SyntheticVectorEnv(E, (D,), A, ep_len=L, device=dev),
                           exact_obs_rms=exact)
    buf = VectorReplayBuffer(E * T, E, device=dev)
    c = Collector(policy, env, buf)
    worst = {"mean": 0.0, "var": 0.0}

    def check(t):
        rms = env.get_obs_rms()
        assert rms.count == int(z[f"rms{t}_count"]), t
        if exact:
            assert np.array_equal(rms.mean, z[f"rms{t}_mean"]), t
            assert np.array_equal(rms.var, z[f"rms{t}_var"]), t
        else:
            worst["mean"] = max(worst["mean"], _ratio(rms.mean, z[f"rms{t}_mean"]))
            worst["var"] = max(worst["var"], _ratio(rms.var, z[f"rms{t}_var"]))

    check(0)
    for t in range(T):
        res = c.collect(n_step=E)
        assert c._step_on, "the fused one-launch step did not run"
        _check_stats(z, f"s{t}_", res)
        check(t + 1)
    if not exact:
        print(f"default obs_rms vs reference over {T + 1} states, max err / (rtol 1e-5, atol "
              f"1e-7): "
              f"mean {worst['mean']:.3g}, var {worst['var']:.3g}")
    assert np.array_equal(buf._meta.rew.cpu().numpy(), z["c1_rew"])
    batch, idx = buf.sample(0)
    assert idx.tolist() == z["c1_indices"].tolist()
    batch = policy.process_fn(batch, buf, idx)
    errs = _pf_errors(batch, z, ("v_s", "returns", "adv"))
    for k, (ea, er, ratio) in errs.items():
        print(f"4096 envs exact={exact} {k}: max abs err {ea:.3g}, max rel err {er:.3g}, "
              f"max err / (rtol 1e-5 + atol 1e-6 max) {ratio:.3g}")
    for k in ("v_s", "returns", "adv"):
        want = z["pf_" + k]
        np.testing.assert_allclose(batch[k].detach().cpu().numpy(), want, rtol=1e-5,
                                   atol=1e-6 * np.abs(want).max(), err_msg=k)
    assert policy.ret_rms.mean == pytest.approx(float(z["pf_ret_rms_mean"]), rel=1e-5)
    assert policy.ret_rms.var == pytest.approx(float(z["pf_ret_rms_var"]), rel=1e-5)
    assert policy.ret_rms.count == int(z["pf_ret_rms_count"])
