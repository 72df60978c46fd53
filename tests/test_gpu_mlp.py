"""Fused actor/critic MLP kernels (csrc/mlp.hip) vs PyTorch.

* tsrl_mlp_l1_fwd vs torch fp32 (both output layouts), rtol 1e-5 / atol 1e-5.
* One whole PPO minibatch (forward, loss, backward of both nets) vs a float64 CPU autograd
  restatement of ppo.py:121-142 on the same weights: the fused f32 gradients must be as
  accurate as torch's own f32 GPU autograd of the same graph (relative L2 error within 4x
  of torch's, or below 2e-6), loss terms rtol 1e-5.
* PPOPolicy.learn with and without the fused MLP: same losses (rtol 1e-4) and parameters
  (atol 2e-3 after Adam, which turns noise-level gradient differences into lr-sized steps).
"""
import copy

import numpy as np
import pytest
import torch
from torch.distributions import Independent, Normal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    return torch.device("cuda", 0)


def _rho(r):
    return (r & 3) + 8 * (r >> 2)


def frag_to_rows(frag, n, nt=4):
    """MFMA-fragment layout ([row tile][feature tile][q][lane][4], x6.h frag_off4: lane l's
    16 values as four float4 pieces) -> [n, 32*nt]."""
    ntile = (n + 31) // 32
    f = frag[:ntile * nt * 64 * 16].view(ntile, nt, 4, 64, 4).permute(0, 1, 3, 2, 4)
    f = f.reshape(ntile, nt, 64, 16).cpu()
    out = torch.empty(ntile * 32, nt * 32)
    lane = torch.arange(64)
    for r in range(16):
        feat = _rho(r) + 4 * (lane >> 5)
        rows = lane & 31
        for ft in range(nt):
            out[(torch.arange(ntile)[:, None] * 32 + rows[None, :]).reshape(-1),
                (32 * ft + feat).repeat(ntile)] = f[:, ft, :, r].reshape(-1)
    return out[:n]


def _nets(D, A, dev, seed):
    from tianshou_amd.utils.models import get_actor_critic, init_actor_critic
    torch.manual_seed(seed)
    actor, critic = get_actor_critic((D,), (64, 64), (A,), dev)
    actor, critic = actor.to(dev), critic.to(dev)
    init_actor_critic(actor, critic)
    with torch.no_grad():
        for p in list(actor.parameters()) + list(critic.parameters()):
            p.add_(0.02 * torch.randn_like(p))
    return actor, critic


@pytest.mark.parametrize("D,n", [(376, 1000), (24, 4096), (8, 33), (128, 128), (376, 262144)])
def test_l1_fwd_x6_f32_accuracy(dev, D, n):
    """tsrl_mlp_l1_fwd_x6 (exact 3-way bf16 split, six bf16 products, f32 accumulation) is an
    f32 GEMM: against an fp64 product of the same f32 operands its error must be within 2x of
    the error of torch's own f32 GEMM (hipBLASLt, f32-input MFMA) and of the f32-input MFMA
    kernel, elementwise bounded by 1e-6 * sum|w x| + 1e-7, and the outputs (both layouts,
    tanh) must match torch fp32 at rtol 1e-5 / atol 1e-5 like the f32 kernel's."""
    from tianshou_amd import _C
    g = torch.Generator().manual_seed(D + n + 1)
    N = n + 50
    X = (torch.randn(N, D, generator=g) * 2).to(dev)
    idx = torch.randperm(N, generator=g)[:n].to(dev)
    Wa, Wc = torch.randn(64, D, generator=g).to(dev) * 0.1, torch.randn(64, D, generator=g).to(dev) * 0.1
    ba, bc = torch.randn(64, generator=g).to(dev), torch.randn(64, generator=g).to(dev)
    L = _C.lib()
    s = _C.stream_ptr(dev)
    ws = torch.empty((int(L.tsrl_mlp_split_bytes(D)) + 3) // 4, device=dev)
    _C.check(L.tsrl_mlp_split_w(_C.ptr(Wa), _C.ptr(Wc), D, _C.ptr(ws), s))
    W = torch.cat([Wa, Wc])
    Xi = X[idx]
    lin = torch.empty(n, 128, device=dev)
    _C.check(L.tsrl_mlp_l1_fwd_x6(_C.ptr(X), D, _C.ptr(idx), n, D, _C.ptr(ws), _C.ptr(ba),
                                  _C.ptr(bc), 0, _C.ptr(lin), 0, s))
    lin32 = torch.empty(n, 128, device=dev)
    _C.check(L.tsrl_mlp_l1_fwd(_C.ptr(X), D, _C.ptr(idx), n, D, _C.ptr(Wa), _C.ptr(ba),
                               _C.ptr(Wc), _C.ptr(bc), 0, _C.ptr(lin32), 0, s))
    b = torch.cat([ba, bc])
    ref64 = Xi.double() @ W.double().T + b.double()
    torch_f32 = Xi @ W.T + b
    mag = Xi.double().abs() @ W.double().abs().T + b.double().abs()
    err = (lin.double() - ref64).abs()
    err_t = (torch_f32.double() - ref64).abs()
    err_k = (lin32.double() - ref64).abs()
    assert float((err - (1e-6 * mag + 1e-7)).max()) <= 0.0
    assert float(err.pow(2).mean().sqrt()) <= 2.0 * max(float(err_t.pow(2).mean().sqrt()),
                                                       float(err_k.pow(2).mean().sqrt()))
    want = torch.tanh(torch_f32)
    rows = torch.empty(n, 128, device=dev)
    _C.check(L.tsrl_mlp_l1_fwd_x6(_C.ptr(X), D, _C.ptr(idx), n, D, _C.ptr(ws), _C.ptr(ba),
                                  _C.ptr(bc), 1, _C.ptr(rows), 0, s))
    frag = torch.empty(int(L.tsrl_mlp_frag_floats(n)), device=dev)
    _C.check(L.tsrl_mlp_l1_fwd_x6(_C.ptr(X), D, _C.ptr(idx), n, D, _C.ptr(ws), _C.ptr(ba),
                                  _C.ptr(bc), 1, _C.ptr(frag), 1, s))
    torch.cuda.synchronize()
    np.testing.assert_allclose(rows.cpu(), want.cpu(), rtol=1e-5, atol=1e-5)
    if n <= 4096:
        np.testing.assert_allclose(frag_to_rows(frag, n), want.cpu(), rtol=1e-5, atol=1e-5)


def frag_to_rows_dev(frag, n, nt=4):
    """frag_to_rows on the device (for large n)."""
    ntile = (n + 31) // 32
    f = frag[:ntile * nt * 64 * 16].view(ntile, nt, 4, 64, 4).permute(0, 1, 3, 2, 4)
    f = f.reshape(ntile, nt, 64, 16)
    lane = torch.arange(64, device=frag.device)
    r = torch.arange(16, device=frag.device)
    feat = (r[None, :] & 3) + 8 * (r[None, :] >> 2) + 4 * (lane[:, None] >> 5)  # [64, 16]
    rows = (lane & 31)[:, None].expand(64, 16)
    out = torch.empty(ntile, 32, nt * 32, device=frag.device)
    for ft in range(nt):
        out[:, rows, 32 * ft + feat] = f[:, ft]
    return out.view(-1, nt * 32)[:n]


@pytest.mark.parametrize("D,n,use_idx", [(376, 262144 + 77, True), (376, 1000, True),
                                         (17, 5000, True), (8, 33, False), (128, 256, True),
                                         (376, 4 * 256 * 9 + 300, False), (24, 1, True)])
def test_l1_ring_kernel_bitwise_equals_staged_kernel(dev, D, n, use_idx):
    """The LDS-DMA pipelined layer-1 kernel (fragment output, l1_ring_kernel) accumulates
    exactly as the register-staged kernel (row-major output, l1_fwd_x6_kernel): same
    k-steps, same six-product order per accumulator -> bit-identical results, for partial
    tiles, partial workgroups, padded rows (ldx > D) and both index modes."""
    from tianshou_amd import _C
    g = torch.Generator(device=dev).manual_seed(D * 7 + n)
    ldx = (D + 3) // 4 * 4
    N = n + 300
    X = torch.zeros(N, ldx, device=dev)
    X[:, :D] = torch.randn(N, D, device=dev, generator=g) * 2
    idx = torch.randperm(N, device=dev, generator=g)[:n] if use_idx else None
    Wa = torch.randn(64, D, device=dev, generator=g) * 0.1
    Wc = torch.randn(64, D, device=dev, generator=g) * 0.1
    ba, bc = torch.randn(64, device=dev, generator=g), torch.randn(64, device=dev, generator=g)
    L = _C.lib()
    s = _C.stream_ptr(dev)
    ws = torch.empty((int(L.tsrl_mlp_split_bytes(D)) + 3) // 4, device=dev)
    _C.check(L.tsrl_mlp_split_w(_C.ptr(Wa), _C.ptr(Wc), D, _C.ptr(ws), s))
    for act in (1, 0):
        rows = torch.empty(n, 128, device=dev)
        _C.check(L.tsrl_mlp_l1_fwd_x6(_C.ptr(X), ldx, _C.ptr(idx), n, D, _C.ptr(ws), _C.ptr(ba),
                                      _C.ptr(bc), act, _C.ptr(rows), 0, s))
        frag = torch.full((int(L.tsrl_mlp_frag_floats(n)) + 4096,), 7.0, device=dev)
        _C.check(L.tsrl_mlp_l1_fwd_x6(_C.ptr(X), ldx, _C.ptr(idx), n, D, _C.ptr(ws), _C.ptr(ba),
                                      _C.ptr(bc), act, _C.ptr(frag), 1, s))
        got = frag_to_rows_dev(frag, n)
        assert torch.equal(got.view(torch.int32), rows.view(torch.int32)), act
        # nothing written past tsrl_mlp_frag_floats(n)
        assert bool((frag[int(L.tsrl_mlp_frag_floats(n)):] == 7.0).all())


@pytest.mark.parametrize("D,n", [(376, 1000), (24, 4096), (8, 33), (128, 128)])
def test_l1_fwd_matches_torch(dev, D, n):
    from tianshou_amd import _C
    g = torch.Generator().manual_seed(D + n)
    N = n + 50
    X = torch.randn(N, D, generator=g).to(dev)
    idx = torch.randperm(N, generator=g)[:n].to(dev)
    Wa, Wc = torch.randn(64, D, generator=g).to(dev) * 0.1, torch.randn(64, D, generator=g).to(dev) * 0.1
    ba, bc = torch.randn(64, generator=g).to(dev), torch.randn(64, generator=g).to(dev)
    L = _C.lib()
    s = _C.stream_ptr(dev)
    want = torch.tanh(X[idx] @ torch.cat([Wa, Wc]).T + torch.cat([ba, bc]))
    rows = torch.empty(n, 128, device=dev)
    _C.check(L.tsrl_mlp_l1_fwd(_C.ptr(X), D, _C.ptr(idx), n, D, _C.ptr(Wa), _C.ptr(ba),
                               _C.ptr(Wc), _C.ptr(bc), 1, _C.ptr(rows), 0, s))
    frag = torch.empty(int(L.tsrl_mlp_frag_floats(n)), device=dev)
    _C.check(L.tsrl_mlp_l1_fwd(_C.ptr(X), D, _C.ptr(idx), n, D, _C.ptr(Wa), _C.ptr(ba),
                               _C.ptr(Wc), _C.ptr(bc), 1, _C.ptr(frag), 1, s))
    lin = torch.empty(n, 128, device=dev)
    _C.check(L.tsrl_mlp_l1_fwd(_C.ptr(X), D, None, n, D, _C.ptr(Wa), _C.ptr(ba),
                               _C.ptr(Wc), _C.ptr(bc), 0, _C.ptr(lin), 0, s))
    torch.cuda.synchronize()
    np.testing.assert_allclose(rows.cpu(), want.cpu(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(frag_to_rows(frag, n), want.cpu(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(lin.cpu(), (X[:n] @ torch.cat([Wa, Wc]).T +
                                           torch.cat([ba, bc])).cpu(), rtol=1e-5, atol=1e-5)


def _ref_minibatch(W, obs, act, logp_old, adv, ret, v_s, kw, dtype, device):
    """ppo.py:121-142 on the functional form of get_actor_critic's networks."""
    P = {k: v.detach().to(device, dtype).clone().requires_grad_(True) for k, v in W.items()}
    x = obs.to(device, dtype)
    c = lambda t: t.to(device, dtype)  # noqa: E731
    ha = torch.tanh(torch.tanh(x @ P["w1a"].T + P["b1a"]) @ P["w2a"].T + P["b2a"])
    mu = ha @ P["w3a"].T + P["b3a"]
    hc = torch.tanh(torch.tanh(x @ P["w1c"].T + P["b1c"]) @ P["w2c"].T + P["b2c"])
    value = (hc @ P["w3c"].T + P["b3c"]).flatten()
    sigma = (P["sigma"].view(1, -1) + torch.zeros_like(mu)).exp()
    dist = Independent(Normal(mu, sigma), 1)
    adv = c(adv)
    if kw.get("norm_adv", True):
        adv = (adv - adv.mean()) / (adv.std() + 1e-8)
    eps_clip = kw.get("eps_clip", 0.2)
    ratio = (dist.log_prob(c(act)) - c(logp_old)).exp()
    surr1 = ratio * adv
    surr2 = ratio.clamp(1.0 - eps_clip, 1.0 + eps_clip) * adv
    if kw.get("dual_clip"):
        clip1 = torch.min(surr1, surr2)
        clip2 = torch.max(clip1, kw["dual_clip"] * adv)
        clip_loss = -torch.where(adv < 0, clip2, clip1).mean()
    else:
        clip_loss = -torch.min(surr1, surr2).mean()
    ret, v_s = c(ret), c(v_s)
    if kw.get("value_clip"):
        v_clip = v_s + (value - v_s).clamp(-eps_clip, eps_clip)
        vf_loss = torch.max((ret - value).pow(2), (ret - v_clip).pow(2)).mean()
    else:
        vf_loss = (ret - value).pow(2).mean()
    ent = dist.entropy().mean()
    loss = clip_loss + kw.get("vf_coef", 0.25) * vf_loss - kw.get("ent_coef", 0.01) * ent
    loss.backward()
    terms = torch.stack([loss, clip_loss, vf_loss, ent]).detach().cpu().double()
    return terms, {k: v.grad.detach().cpu().double() for k, v in P.items()}


CASES = [
    (376, 17, 4096, {}),
    (24, 5, 1000, dict(dual_clip=3.0)),
    (8, 1, 257, dict(value_clip=True)),
    (376, 17, 2048, dict(norm_adv=False, ent_coef=0.0)),
    (64, 32, 4096, dict(dual_clip=5.0, value_clip=True, eps_clip=0.1, ent_coef=0.05)),
    # a partial last 32-row chunk of the dW1 split, the db1 ones column in the third 128-column tile
    (300, 7, 1000, dict(value_clip=True)),
    (380, 3, 777, {}),
    # the production shape of the headline bench (config 3: D 376, A 17, 262144-row minibatch)
    (376, 17, 262144, {}),
    (376, 17, 262144, dict(dual_clip=3.0, value_clip=True)),
]


@pytest.mark.parametrize("D,A,B,kw", CASES)
def test_fused_minibatch_matches_autograd(dev, D, A, B, kw):
    from tianshou_amd import _C
    from tianshou_amd.dist import DataParallel
    from tianshou_amd.policy import fused_mlp
    from tianshou_amd.utils.net import ActorCritic
    actor, critic = _nets(D, A, dev, D + A + B)
    layers = fused_mlp.match(actor, critic)
    assert layers is not None
    fm = fused_mlp.FusedActorCritic(layers, ActorCritic(actor, critic).parameters())
    g = torch.Generator().manual_seed(B)
    n = B + 101
    obs = torch.randn(n, D, generator=g).to(dev)
    act = torch.randn(n, A, generator=g).to(dev)
    adv = (torch.randn(n, generator=g) * 2 + 0.3).to(dev)
    ret = torch.randn(n, generator=g).to(dev)
    v_s = (ret.cpu() + torch.randn(n, generator=g) * 0.3).to(dev)
    idx = torch.randperm(n, generator=g)[:B].to(dev)
    with torch.no_grad():
        mu = actor.forward_mu(obs)
        lp = Independent(Normal(mu, actor.sigma_param.view(1, -1).exp().expand_as(mu)),
                         1).log_prob(act)
        logp_old = (lp + 0.2 * torch.randn(n, generator=g).to(dev)).contiguous()
    W = {"w1a": layers["w1a"].weight, "b1a": layers["w1a"].bias,
         "w2a": layers["w2a"].weight, "b2a": layers["w2a"].bias,
         "w3a": layers["w3a"].weight, "b3a": layers["w3a"].bias,
         "w1c": layers["w1c"].weight, "b1c": layers["w1c"].bias,
         "w2c": layers["w2c"].weight, "b2c": layers["w2c"].bias,
         "w3c": layers["w3c"].weight, "b3c": layers["w3c"].bias,
         "sigma": layers["sigma"]}
    p = _C.PPOParams()
    p.eps_clip = kw.get("eps_clip", 0.2)
    p.dual_clip = kw.get("dual_clip") or 0.0
    p.vf_coef = kw.get("vf_coef", 0.25)
    p.ent_coef = kw.get("ent_coef", 0.01)
    p.adv_eps = 1e-8
    p.b_global = float(B)
    p.value_clip = int(bool(kw.get("value_clip")))
    p.norm_adv = int(kw.get("norm_adv", True))
    terms = fm.minibatch(obs, idx, B, act, logp_old, adv, ret, v_s, p, DataParallel())
    torch.cuda.synchronize()
    got = {k: v.grad.detach().cpu().double() for k, v in W.items()}
    mb = [t[idx] for t in (obs, act, logp_old, adv, ret, v_s)]
    # fp64 autograd on the GPU for the production-size cases (CPU fp64 is minutes there)
    t64, g64 = _ref_minibatch(W, *mb, kw, torch.float64, dev if B > 65536 else "cpu")
    t32, g32 = _ref_minibatch(W, *mb, kw, torch.float32, dev)
    np.testing.assert_allclose(terms.cpu().double().numpy(), t64.numpy(), rtol=1e-5, atol=1e-6)
    for k in W:
        ref = g64[k]
        den = ref.norm().item() + 1e-30
        e_fused = (got[k] - ref).norm().item() / den
        e_torch = (g32[k] - ref).norm().item() / den
        print(f"B={B} {k}: rel L2 err fused {e_fused:.3g}, torch f32 {e_torch:.3g}")
        assert e_fused <= max(4 * e_torch, 2e-6), (k, e_fused, e_torch)


@pytest.mark.parametrize("B", [262144 + 45, 1000, 16384, 16385])
def test_tail_reduction_on_side_stream_is_bitwise_single_stream(dev, monkeypatch, B):
    """The tail's reduction on a second stream beside dW1 (TSRL_TAIL_OVERLAP, the default) --
    and, up to TAIL_SPLIT_ROWS rows, the critic's tail kernel on that stream beside the
    actor's -- gives the same bits as the one-stream sequence: same kernels, only the streams
    differ.  A third run writes the loss terms into a caller's buffer (terms_out, the
    captured epochs' rows): same values, in place."""
    from tianshou_amd import _C
    from tianshou_amd.dist import DataParallel
    from tianshou_amd.policy import fused_mlp
    from tianshou_amd.utils.net import ActorCritic
    D, A = 376, 17
    actor, critic = _nets(D, A, dev, 7)
    layers = fused_mlp.match(actor, critic)
    fm = fused_mlp.FusedActorCritic(layers, ActorCritic(actor, critic).parameters())
    g = torch.Generator().manual_seed(3)
    n = B + 300
    obs = torch.randn(n, D, generator=g).to(dev)
    act = torch.randn(n, A, generator=g).to(dev)
    adv = torch.randn(n, generator=g).to(dev)
    ret = torch.randn(n, generator=g).to(dev)
    v_s = torch.randn(n, generator=g).to(dev)
    logp_old = (0.3 * torch.randn(n, generator=g) - 24.0).to(dev)  # ratio near 1
    idx = torch.randperm(n, generator=g)[:B].to(dev)
    p = _C.PPOParams()
    p.eps_clip, p.dual_clip, p.vf_coef, p.ent_coef, p.adv_eps = 0.2, 3.0, 0.25, 0.01, 1e-8
    p.b_global, p.value_clip, p.norm_adv = float(B), 1, 1
    params = list(ActorCritic(actor, critic).parameters())
    out = []
    for overlap in (True, False):
        monkeypatch.setattr(fused_mlp, "TAIL_OVERLAP", overlap)
        terms = fm.minibatch(obs, idx, B, act, logp_old, adv, ret, v_s, p, DataParallel())
        torch.cuda.synchronize()
        out.append((terms.cpu().clone(),
                    [q.grad.detach().cpu().clone() for q in params if q.grad is not None]))
    monkeypatch.setattr(fused_mlp, "TAIL_OVERLAP", True)
    buf = torch.full((2, 4), -7.0, device=dev)
    terms = fm.minibatch(obs, idx, B, act, logp_old, adv, ret, v_s, p, DataParallel(),
                         terms_out=buf[1])
    torch.cuda.synchronize()
    assert terms.data_ptr() == buf[1].data_ptr()
    out.append((buf[1].cpu().clone(),
                [q.grad.detach().cpu().clone() for q in params if q.grad is not None]))
    assert torch.equal(buf[0].cpu(), torch.full((4,), -7.0))
    for o in out[1:]:
        assert torch.equal(out[0][0], o[0])
        assert len(out[0][1]) == len(o[1]) >= 13  # both nets' Linear weights/biases + log-std
        for a, b in zip(out[0][1], o[1]):
            assert torch.equal(a, b)


@pytest.mark.parametrize("value_clip", [False, True])
def test_learn_fused_mlp_vs_layers(dev, value_clip):
    from tianshou_amd.data import Batch
    from tianshou_amd.env import Box
    from tianshou_amd.policy import PPOPolicy
    from tianshou_amd.utils.models import fixed_std_normal
    D, A, n = 40, 6, 3000
    base_a, base_c = _nets(D, A, dev, 5)
    res, states = [], []
    for fused in (True, False):
        actor, critic = copy.deepcopy(base_a), copy.deepcopy(base_c)
        params = list(actor.parameters()) + [p for p in critic.parameters()
                                             if all(p is not q for q in actor.parameters())]
        optim = torch.optim.Adam(params, lr=3e-4)
        pol = PPOPolicy(actor, critic, optim, fixed_std_normal, action_space=Box(-1.0, 1.0, (A,)),
                        max_grad_norm=0.5, vf_coef=0.25, ent_coef=0.01, value_clip=value_clip,
                        fused_mlp=fused)
        assert (pol._mlp is not None) == fused
        g = torch.Generator().manual_seed(1)
        data = dict(obs=torch.randn(n, D, generator=g), act=torch.randn(n, A, generator=g),
                    logp_old=torch.randn(n, generator=g) * 0.2 - A * 1.2,
                    adv=torch.randn(n, generator=g), returns=torch.randn(n, generator=g))
        data["v_s"] = data["returns"] + 0.3 * torch.randn(n, generator=g)
        batch = Batch(**{k: v.to(dev) for k, v in data.items()})
        np.random.seed(3)
        res.append(pol.learn(batch, batch_size=512, repeat=2))
        states.append({k: v.detach().cpu() for k, v in pol.state_dict().items()})
    for k in res[0]:
        np.testing.assert_allclose(res[0][k], res[1][k], rtol=1e-4, atol=1e-5, err_msg=k)
    for k in states[0]:
        np.testing.assert_allclose(states[0][k].numpy(), states[1][k].numpy(), rtol=1e-3,
                                   atol=2e-3, err_msg=k)


def test_process_fn_fused_eval_matches_torch_layers(dev):
    """PPOPolicy.process_fn with the fused evaluation (layer-1 kernel + eval kernel, V(s')
    reused from V(s) along the Collector's obs chain) vs the torch layers on the same
    collected buffer: v_s, returns, adv, logp_old within rtol 1e-5 / atol 1e-5."""
    import copy
    from tianshou_amd.data import Collector, VectorReplayBuffer
    from tianshou_amd.env import Box, SyntheticVectorEnv, VectorEnvNormObs
    from tianshou_amd.policy import PPOPolicy
    from tianshou_amd.utils.models import fixed_std_normal
    E, D, A, T = 64, 40, 6, 50
    base_a, base_c = _nets(D, A, dev, 11)
    out = []
    for fused in (True, False):
        actor, critic = copy.deepcopy(base_a), copy.deepcopy(base_c)
        optim = torch.optim.Adam(list(actor.parameters()) + list(critic.parameters()), lr=1e-4)
        pol = PPOPolicy(actor, critic, optim, fixed_std_normal, action_space=Box(-1.0, 1.0, (A,)),
                        reward_normalization=True, fused_mlp=fused)
        assert (pol._mlp is not None) == fused
        env = VectorEnvNormObs(SyntheticVectorEnv(E, (D,), A, ep_len=17, seed=2, device=dev))
        buf = VectorReplayBuffer(E * T, E, device=dev)
        torch.manual_seed(4)
        Collector(pol, env, buf).collect(n_step=E * T)
        assert buf.obs_chain
        batch, idx = buf.sample(0)
        batch = pol.process_fn(batch, buf, idx)
        out.append({k: batch[k].detach().cpu() for k in ("v_s", "returns", "adv", "logp_old")})
    for k in out[0]:
        np.testing.assert_allclose(out[0][k].numpy(), out[1][k].numpy(), rtol=1e-5, atol=1e-5,
                                   err_msg=k)


def test_process_fn_fused_eval_headline_width_matches_torch_layers(dev):
    """The same comparison at the headline width and a production-size row count: D = 376,
    A = 17, 4096 envs x 512 steps = 2 097 152 rows (one full 2M-row evaluation chunk).  One
    rollout is collected; process_fn runs on it with the fused evaluation and with the torch
    layers (same weights, each policy with a fresh ret_rms): v_s, returns, adv, logp_old within
    rtol 1e-5 / atol 1e-5 (advantages also atol 1e-6 * max); the measured errors are printed."""
    import copy
    from tianshou_amd.data import Collector, VectorReplayBuffer
    from tianshou_amd.env import Box, SyntheticVectorEnv, VectorEnvNormObs
    from tianshou_amd.policy import PPOPolicy
    from tianshou_amd.utils.models import fixed_std_normal
    E, D, A, T = 4096, 376, 17, 512
    base_a, base_c = _nets(D, A, dev, 13)
    pols = []
    for fused in (True, False):
        actor, critic = copy.deepcopy(base_a), copy.deepcopy(base_c)
        optim = torch.optim.Adam(list(actor.parameters()) + list(critic.parameters()), lr=1e-4)
        pol = PPOPolicy(actor, critic, optim, fixed_std_normal, action_space=Box(-1.0, 1.0, (A,)),
                        reward_normalization=True, fused_mlp=fused)
        assert (pol._mlp is not None) == fused
        pols.append(pol)
    env = VectorEnvNormObs(SyntheticVectorEnv(E, (D,), A, ep_len=300, seed=3, device=dev))
    buf = VectorReplayBuffer(E * T, E, device=dev)
    torch.manual_seed(4)
    Collector(pols[0], env, buf).collect(n_step=E * T)
    assert buf.obs_chain
    out = []
    for pol in pols:
        batch, idx = buf.sample(0)
        assert len(idx) == E * T
        batch = pol.process_fn(batch, buf, idx)
        out.append({k: batch[k].detach() for k in ("v_s", "returns", "adv", "logp_old")})
        del batch
    for k in out[0]:
        a, b = out[0][k].double(), out[1][k].double()
        err = (a - b).abs()
        print(f"{k}: max abs err {float(err.max()):.3g}, max rel err "
              f"{float((err / b.abs().clamp_min(1e-30)).max()):.3g}")
        atol = max(1e-5, 1e-6 * float(b.abs().max())) if k == "adv" else 1e-5
        assert bool((err <= 1e-5 * b.abs() + atol).all()), k


def test_learn_graph_replay_matches_eager(dev):
    """Epochs replayed from the captured HIP graph give exactly the eager fused result (same
    kernels in the same order): losses and parameters bit-identical over 3 updates."""
    from tianshou_amd.data import Batch
    from tianshou_amd.env import Box
    from tianshou_amd.policy import PPOPolicy
    from tianshou_amd.utils.models import fixed_std_normal
    D, A, n = 40, 6, 3000
    base_a, base_c = _nets(D, A, dev, 21)
    res, states = [], []
    for graph in (True, False):
        actor, critic = copy.deepcopy(base_a), copy.deepcopy(base_c)
        params = list(actor.parameters()) + [p for p in critic.parameters()
                                             if all(p is not q for q in actor.parameters())]
        optim = torch.optim.Adam(params, lr=3e-4, fused=True, capturable=True)
        pol = PPOPolicy(actor, critic, optim, fixed_std_normal, action_space=Box(-1.0, 1.0, (A,)),
                        max_grad_norm=0.5, vf_coef=0.25, ent_coef=0.01, perm_device=True)
        pol.graph_learn = graph
        g = torch.Generator().manual_seed(1)
        data = dict(obs=torch.randn(n, D, generator=g), act=torch.randn(n, A, generator=g),
                    logp_old=torch.randn(n, generator=g) * 0.2 - A * 1.2,
                    adv=torch.randn(n, generator=g), returns=torch.randn(n, generator=g))
        data["v_s"] = data["returns"] + 0.3 * torch.randn(n, generator=g)
        batch = Batch(**{k: v.to(dev) for k, v in data.items()})
        torch.manual_seed(3)
        out = [pol.learn(batch, batch_size=512, repeat=2) for _ in range(3)]
        assert (pol._learn_graph is not None) == graph
        res.append(out)
        states.append({k: v.detach().cpu() for k, v in pol.state_dict().items()})
    for a, b in zip(res[0], res[1]):
        for k in a:
            assert a[k] == b[k], k
    for k in states[0]:
        assert torch.equal(states[0][k], states[1][k]), k


@pytest.mark.parametrize("D,n,with_act,gathered", [
    (376, 2 * 262144 + 77, True, False), (376, 5000, False, False), (376, 3001, True, True),
    (17, 1000, True, False), (40, 257, True, True)])
def test_fused_eval_bit_identical_to_two_kernel_eval(dev, D, n, with_act, gathered):
    """tsrl_ppo_eval_fused (layer 1 and process_fn's evaluation in one launch, H1 kept in
    registers) against tsrl_mlp_l1_fwd_x6 + tsrl_ppo_eval on the same rows: values and
    log-probs bit for bit (same products in the same order), ragged row counts, contiguous
    and gathered rows, with and without the stored actions."""
    import tianshou_amd.policy.fused_mlp as fm
    from tianshou_amd.policy import PPOPolicy
    from tianshou_amd.env import Box
    from tianshou_amd.utils.models import fixed_std_normal
    A = 6
    actor, critic = _nets(D, A, dev, 21)
    optim = torch.optim.Adam(list(actor.parameters()) + list(critic.parameters()), lr=1e-4)
    pol = PPOPolicy(actor, critic, optim, fixed_std_normal, action_space=Box(-1.0, 1.0, (A,)),
                    fused_mlp=True)
    mlp = pol._mlp
    assert mlp is not None
    g = torch.Generator(device=dev).manual_seed(n)
    rows = n + 123 if gathered else n
    obs = torch.randn(rows, D, device=dev, generator=g)
    act = torch.randn(n, A, device=dev, generator=g) if with_act else None
    idx = torch.randperm(rows, device=dev, generator=g)[:n] if gathered else None
    prev = fm.EVAL_FUSED
    try:
        fm.EVAL_FUSED = True
        v1, l1 = mlp.evaluate(obs, act, idx)
        fm.EVAL_FUSED = False
        v2, l2 = mlp.evaluate(obs, act, idx)
    finally:
        fm.EVAL_FUSED = prev
    torch.cuda.synchronize()
    assert torch.isfinite(v1).all()
    assert torch.equal(v1, v2), float((v1 - v2).abs().max())
    if with_act:
        assert torch.isfinite(l1).all()
        assert torch.equal(l1, l2), float((l1 - l2).abs().max())
    else:
        assert l1 is None and l2 is None
