"""Fused collector policy step (csrc/policy.hip) vs the torch formulation of
pg.py:133-171 + base.py:183-215 (actor forward, randn * sigma + mu, clip/tanh, scaling).
Tolerance rtol/atol 1e-5 (f32 GEMM summation order differs from hipBLASLt's)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    return torch.device("cuda", 0)


def _actor(D, A, dev, seed):
    from tianshou_amd.utils.models import get_actor_critic, init_actor_critic
    torch.manual_seed(seed)
    actor, critic = get_actor_critic((D,), (64, 64), (A,), dev)
    actor, critic = actor.to(dev), critic.to(dev)
    init_actor_critic(actor, critic)
    with torch.no_grad():
        for p in actor.parameters():
            p.add_(0.05 * torch.randn_like(p))
    return actor


@pytest.mark.parametrize("D,A,n,bound,scale,sample", [
    (376, 17, 4096, "clip", True, True),
    (24, 5, 100, "tanh", True, True),
    (8, 1, 33, None, False, True),
    (376, 17, 1000, "clip", False, False),
])
def test_gauss_policy_act_matches_torch(dev, D, A, n, bound, scale, sample):
    from tianshou_amd import _C
    from tianshou_amd.policy.fused_act import _BOUND, FusedGaussAct, match_actor
    actor = _actor(D, A, dev, D + A)
    layers = match_actor(actor)
    assert layers is not None
    fa = FusedGaussAct(layers)
    fa.pack()
    g = torch.Generator().manual_seed(n)
    obs = torch.randn(n, D, generator=g).to(dev)
    eps = torch.randn(n, A, generator=g).to(dev)
    low = (-1.0 - torch.rand(A, generator=g)).to(dev)
    high = (1.0 + 2 * torch.rand(A, generator=g)).to(dev)
    act = torch.empty(n, A, device=dev)
    remap = torch.empty(n, A, device=dev)
    L = _C.lib()
    _C.check(L.tsrl_gauss_policy_act(
        _C.ptr(obs), D, n, D, _C.ptr(fa.packed), _C.ptr(layers["w1"].bias.detach()),
        _C.ptr(layers["w2"].weight.detach()), _C.ptr(layers["w2"].bias.detach()),
        _C.ptr(layers["w3"].weight.detach()), _C.ptr(layers["w3"].bias.detach()),
        _C.ptr(layers["sigma"].detach()), A, _C.ptr(eps) if sample else None, _BOUND[bound],
        _C.ptr(low) if scale else None, _C.ptr(high) if scale else None, _C.ptr(act),
        _C.ptr(remap), _C.stream_ptr(dev)))
    with torch.no_grad():
        mu = actor.forward_mu(obs)
        sigma = actor.sigma_param.view(1, -1).exp().expand_as(mu)
        want = eps.mul(sigma).add(mu) if sample else mu
        y = want
        if bound == "clip":
            y = y.clamp(-1.0, 1.0)
        elif bound == "tanh":
            y = torch.tanh(y)
        if scale:
            y = low + (high - low) * (y + 1.0) / 2.0
    torch.cuda.synchronize()
    np.testing.assert_allclose(act.cpu().numpy(), want.cpu().numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(remap.cpu().numpy(), y.cpu().numpy(), rtol=1e-5, atol=1e-5)


def test_collector_fused_act_matches_torch_path(dev):
    """Same seeds, fused vs torch policy step inside the (graph-replayed) collector: the
    env stream is action-independent, so obs/rew/flags must be identical and the stored
    actions equal up to the GEMM order."""
    from tianshou_amd.data import Collector, VectorReplayBuffer
    from tianshou_amd.env import Box, SyntheticVectorEnv, VectorEnvNormObs
    from tianshou_amd.policy import PPOPolicy
    from tianshou_amd.utils.models import fixed_std_normal, get_actor_critic, init_and_get_optim
    E, D, A, T = 64, 24, 5, 40
    out = []
    for fused in (True, False):
        torch.manual_seed(0)
        actor, critic = get_actor_critic((D,), (64, 64), (A,), dev)
        optim = init_and_get_optim(actor.to(dev), critic.to(dev), 3e-4)
        pol = PPOPolicy(actor, critic, optim, fixed_std_normal,
                        action_space=Box(-1.0, 1.0, (A,))).to(dev)
        pol.fused_act_rng = "torch"  # the torch path's noise stream, for an exact comparison
        env = VectorEnvNormObs(SyntheticVectorEnv(E, (D,), A, ep_len=13, seed=3, device=dev))
        buf = VectorReplayBuffer(E * T, E, device=dev)
        c = Collector(pol, env, buf)
        c.use_fused_act = fused
        c.graph_steps = 8  # T = 40: replayed from a captured HIP graph after the first step
        torch.manual_seed(1)
        c.collect(n_step=E * T)
        assert c._fused_act_on == fused
        m = buf._meta
        out.append({k: getattr(m, k).detach().cpu().clone() for k in
                     ("obs", "obs_next", "act", "rew", "terminated", "truncated")})
    for k in ("obs", "obs_next", "rew", "terminated", "truncated"):
        assert torch.equal(out[0][k], out[1][k]), k
    np.testing.assert_allclose(out[0]["act"].numpy(), out[1]["act"].numpy(), rtol=1e-5,
                               atol=1e-5)


def test_device_rng_noise_is_standard_normal(dev):
    """tsrl_gauss_policy_act_rng: zero weights make mu = b3 = 0 and sigma = 1, so the actions
    are the raw noise: mean ~ 0, std ~ 1, fresh per call, reproducible per seed."""
    from tianshou_amd import _C
    from tianshou_amd.policy.fused_act import FusedGaussAct, match_actor
    D, A, n = 8, 6, 8192
    actor = _actor(D, A, dev, 1)
    with torch.no_grad():
        for p in actor.parameters():
            p.zero_()
    fa = FusedGaussAct(match_actor(actor))
    obs = torch.randn(n, D, device=dev)
    outs = []
    for rep in range(2):
        torch.manual_seed(123)
        fa.pack()
        for _ in range(2):
            act = torch.empty(n, A, device=dev)
            remap = torch.empty(n, A, device=dev)
            fa(obs, act, remap, True, None, None)
            outs.append(act.cpu())
    x = torch.cat(outs[:2]).double()
    assert abs(x.mean().item()) < 0.02 and abs(x.std().item() - 1.0) < 0.02
    assert abs(((x - x.mean()) ** 3).mean().item()) < 0.05        # symmetric
    assert abs(((x - x.mean()) ** 4).mean().item() - 3.0) < 0.15  # normal kurtosis
    assert not torch.equal(outs[0], outs[1])      # counter advances per call
    assert torch.equal(outs[0], outs[2]) and torch.equal(outs[1], outs[3])  # seeded
