"""One-launch collect step (csrc/collect.hip, tsrl_collect_box_step) vs the four-launch step it
replaces (tsrl_gauss_policy_act_rng -> tsrl_synth_box_step_reset -> tsrl_rms_merge2 ->
tsrl_buffer_add), both inside Collector.collect (collector.py:258-361) with the same seeds.

The synthetic env ignores actions, so rewards, flags, env ids and episode statistics must be
bit-identical; observations pass through obs_rms, whose column sums the fused step folds in a
different (fixed) order, so normalised rows and statistics agree to f32 rounding (rtol 1e-6);
actions use the same noise stream and differ only by the actor's f32 summation order
(rtol / atol 1e-5, as the fused-act tests)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    return torch.device("cuda", 0)


def _run(dev, fused, E, D, A, L, T, graph_steps, collects=2, bound="clip", det=False,
         act_coef=0.0):
    from tianshou_amd.data import Collector, VectorReplayBuffer
    from tianshou_amd.env import Box, SyntheticVectorEnv, VectorEnvNormObs
    from tianshou_amd.policy import PPOPolicy
    from tianshou_amd.utils.models import fixed_std_normal, get_actor_critic, init_and_get_optim
    torch.manual_seed(0)
    actor, critic = get_actor_critic((D,), (64, 64), (A,), dev)
    optim = init_and_get_optim(actor.to(dev), critic.to(dev), 3e-4)
    with torch.no_grad():
        for p in actor.parameters():
            p.add_(0.05 * torch.randn_like(p))
    pol = PPOPolicy(actor, critic, optim, fixed_std_normal,
                    action_space=Box(-2.0, 3.0, (A,)), action_bound_method=bound,
                    deterministic_eval=det).to(dev)
    if det:
        pol.eval()
    env = VectorEnvNormObs(SyntheticVectorEnv(E, (D,), A, ep_len=L, seed=5, device=dev,
                                              act_coef=act_coef))
    buf = VectorReplayBuffer(E * T * collects, E, device=dev)
    c = Collector(pol, env, buf)
    c.use_fused_step = fused
    c.graph_steps = graph_steps
    torch.manual_seed(1)
    res = []
    for _ in range(collects):
        res.append(c.collect(n_step=E * T))
        assert c._step_on == fused
    assert c._pending is None
    m = buf._meta
    out = {k: getattr(m, k).detach().cpu().clone() for k in
           ("obs", "obs_next", "act", "rew", "terminated", "truncated", "done")}
    out["env_id"] = m.info.env_id.cpu().clone()
    rms = env.obs_rms
    out["rms"] = (rms.mean_t.cpu().clone(), rms.var_t.cpu().clone(), rms.count)
    out["cur"] = c.data.obs.cpu().clone()
    d = buf._dev
    out["stats"] = [d[k].cpu().clone() for k in ("stat_rew", "stat_len", "stat_idx", "ep_rew",
                                                 "ep_len", "ep_idx")]
    return out, res


@pytest.mark.parametrize("E,D,A,L,T,G", [
    (64, 24, 5, 13, 40, 8),        # one group, graph-replayed steps
    (100, 376, 17, 7, 12, 4),      # partial 16-row tile, 7 workgroups
    (600, 376, 17, 9, 10, 0),      # 3 groups (last partial), eager steps only
    (4096, 376, 17, 30, 20, 16),   # the headline shape: 256 workgroups, 16 groups
    (512, 17, 6, 25, 24, 8),       # config 2's width (D % 4 != 0: scalar row paths)
    (77, 5, 2, 6, 14, 4),          # D = 5, partial tile
])
def test_fused_step_matches_four_launch_step(dev, E, D, A, L, T, G):
    a, ra = _run(dev, True, E, D, A, L, T, G)
    b, rb = _run(dev, False, E, D, A, L, T, G)
    for k in ("rew", "terminated", "truncated", "done", "env_id"):
        assert torch.equal(a[k], b[k]), k
    for x, y in zip(a["stats"], b["stats"]):
        assert torch.equal(x, y)
    for x, y in zip(ra, rb):
        assert x["n/ep"] == y["n/ep"] and x["n/st"] == y["n/st"]
        assert np.array_equal(x["rews"], y["rews"]) and np.array_equal(x["lens"], y["lens"])
        assert np.array_equal(x["idxs"], y["idxs"])
    assert a["rms"][2] == b["rms"][2]
    np.testing.assert_allclose(a["rms"][0].numpy(), b["rms"][0].numpy(), rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(a["rms"][1].numpy(), b["rms"][1].numpy(), rtol=1e-6, atol=1e-7)
    for k in ("obs", "obs_next", "cur"):
        np.testing.assert_allclose(a[k].numpy(), b[k].numpy(), rtol=1e-6, atol=1e-6, err_msg=k)
    np.testing.assert_allclose(a["act"].numpy(), b["act"].numpy(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("E,D,A,L,T,G", [
    (64, 24, 5, 13, 40, 8),
    (100, 376, 17, 7, 12, 4),
    (512, 17, 6, 25, 24, 8),
    (4096, 376, 17, 30, 20, 16),
])
def test_fused_step_action_coupled_env(dev, E, D, A, L, T, G):
    """The general fused step: an env whose transition reads the action (SyntheticVectorEnv
    act_coef: obs = box + 0.05 * a[d mod A], not 2^-23-quantised) runs its env phase AFTER the
    actor in the same launch and sums obs_rms moments in f64 (atomic f64 adds) -- against the
    four-launch step (torch-free fused act -> coupled step+reset kernel -> f64 partials merge ->
    add) with the same noise stream.  Rewards / flags / episode statistics bit-identical;
    actions differ by the actors' f32 summation order (rtol 1e-5) and feed the observations,
    so obs / statistics agree at rtol 1e-5."""
    a, ra = _run(dev, True, E, D, A, L, T, G, act_coef=0.05)
    b, rb = _run(dev, False, E, D, A, L, T, G, act_coef=0.05)
    for k in ("rew", "terminated", "truncated", "done", "env_id"):
        assert torch.equal(a[k], b[k]), k
    for x, y in zip(a["stats"], b["stats"]):
        assert torch.equal(x, y)
    for x, y in zip(ra, rb):
        assert x["n/ep"] == y["n/ep"] and np.array_equal(x["lens"], y["lens"])
        assert np.array_equal(x["rews"], y["rews"])
    assert a["rms"][2] == b["rms"][2]
    np.testing.assert_allclose(a["rms"][0].numpy(), b["rms"][0].numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(a["rms"][1].numpy(), b["rms"][1].numpy(), rtol=1e-5, atol=1e-6)
    for k in ("obs", "obs_next", "cur"):
        np.testing.assert_allclose(a[k].numpy(), b[k].numpy(), rtol=1e-5, atol=1e-5, err_msg=k)
    np.testing.assert_allclose(a["act"].numpy(), b["act"].numpy(), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("bound,det", [("tanh", False), (None, True)])
def test_fused_step_bounds_and_deterministic_eval(dev, bound, det):
    a, _ = _run(dev, True, 48, 32, 6, 11, 16, 8, collects=1, bound=bound, det=det)
    b, _ = _run(dev, False, 48, 32, 6, 11, 16, 8, collects=1, bound=bound, det=det)
    for k in ("rew", "terminated", "truncated", "env_id"):
        assert torch.equal(a[k], b[k]), k
    np.testing.assert_allclose(a["obs"].numpy(), b["obs"].numpy(), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(a["act"].numpy(), b["act"].numpy(), rtol=1e-5, atol=1e-5)


def test_fused_step_rejects_mismatched_pending_add(dev):
    """The C ABI refuses a pending add that does not cover the launch's rows."""
    from tianshou_amd import _C
    c = _C.CollectArgs()
    c.k, c.dim = 16, 8
    c.add.k = 8
    rc = _C.lib().tsrl_collect_box_step(c, _C.stream_ptr(dev))
    assert rc != 0


@pytest.mark.parametrize("fused", [True, False])
def test_collect_longer_than_ring_keeps_every_episode(dev, fused):
    """An n_step collect of more steps than the buffer holds per env (the ring laps rows this
    collect wrote): the returned episode statistics are still every finished episode's, in
    (step, env) order -- the same rews / lens as a collect into a buffer that never wraps
    (collector.py:330-342 reads ep_rew / ep_len from buffer.add at every step)."""
    from tianshou_amd.data import Collector, VectorReplayBuffer
    from tianshou_amd.env import Box, SyntheticVectorEnv, VectorEnvNormObs
    from tianshou_amd.policy import PPOPolicy
    from tianshou_amd.utils.models import fixed_std_normal, get_actor_critic, init_and_get_optim
    E, D, A, L, T = 16, 8, 3, 3, 37
    out = []
    for per_env in (4, T):
        torch.manual_seed(0)
        actor, critic = get_actor_critic((D,), (64, 64), (A,), dev)
        optim = init_and_get_optim(actor.to(dev), critic.to(dev), 3e-4)
        pol = PPOPolicy(actor, critic, optim, fixed_std_normal,
                        action_space=Box(-1.0, 1.0, (A,))).to(dev)
        env = VectorEnvNormObs(SyntheticVectorEnv(E, (D,), A, ep_len=L, seed=2, device=dev))
        c = Collector(pol, env, VectorReplayBuffer(E * per_env, E, device=dev))
        c.use_fused_step = fused
        c.graph_steps = 4
        res = c.collect(n_step=E * T)
        out.append(res)
    a, b = out
    assert a["n/st"] == b["n/st"] == E * T
    assert a["n/ep"] == b["n/ep"] > 0
    assert np.array_equal(a["rews"], b["rews"]) and np.array_equal(a["lens"], b["lens"])
