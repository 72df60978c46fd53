"""Fused PPO loss kernel vs the torch fp32 restatement (oracle/ref.py), and PPOPolicy.learn
vs the reference's recorded losses/parameters (tests/golden/ppo_learn.npz).

Tolerances: loss terms rtol 1e-5; gradients rtol 1e-4 / atol 1e-6 (f32 reductions in a
different order than torch's); parameters after Adam steps rtol 1e-3 (GEMMs on the GPU
vs the reference's CPU torch)."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    return torch.device("cuda", 0)


CASES = [
    dict(),
    dict(dual_clip=3.0),
    dict(value_clip=True),
    dict(norm_adv=False, ent_coef=0.0),
    dict(dual_clip=5.0, value_clip=True, ent_coef=0.05, eps_clip=0.1),
]


@pytest.mark.parametrize("kw", CASES)
@pytest.mark.parametrize("B,A", [(4096, 17), (1000, 6), (257, 1)])
def test_fused_loss_vs_torch(dev, kw, B, A):
    from tianshou_amd import _C
    from tianshou_amd.policy.ppo import _GaussPPOLoss
    from tianshou_amd.dist import DataParallel
    g = torch.Generator().manual_seed(B + A)
    n = B + 37
    mu = torch.randn(B, A, generator=g)
    sp = torch.randn(A, 1, generator=g) * 0.3 - 0.5
    value = torch.randn(B, generator=g)
    act = torch.randn(n, A, generator=g)
    logp_old = torch.randn(n, generator=g) * 0.3 - A
    adv = torch.randn(n, generator=g) * 2 + 0.3
    ret = torch.randn(n, generator=g)
    v_s = ret + torch.randn(n, generator=g) * 0.3
    idx = torch.randperm(n, generator=g)[:B]
    # make logp_old close to the current logp so the ratio straddles the clip range
    from torch.distributions import Independent, Normal
    with torch.no_grad():
        lp = Independent(Normal(mu, sp.view(1, -1).exp().expand_as(mu)), 1).log_prob(act[idx])
        logp_old[idx] = lp + torch.randn(B, generator=g) * 0.2
    eps_clip = kw.get("eps_clip", 0.2)
    want = ref.ppo_gaussian_loss_torch(
        mu, sp.flatten(), value, act[idx], logp_old[idx], adv[idx], ret[idx], v_s[idx],
        eps_clip=eps_clip, dual_clip=kw.get("dual_clip"), value_clip=kw.get("value_clip", False),
        norm_adv=kw.get("norm_adv", True), vf_coef=0.25, ent_coef=kw.get("ent_coef", 0.01))
    p = _C.PPOParams()
    p.eps_clip, p.dual_clip = eps_clip, kw.get("dual_clip") or 0.0
    p.vf_coef, p.ent_coef, p.adv_eps, p.b_global = 0.25, kw.get("ent_coef", 0.01), 1e-8, B
    p.value_clip, p.norm_adv = int(kw.get("value_clip", False)), int(kw.get("norm_adv", True))
    d = lambda t: t.to(dev).contiguous()
    mu_d = d(mu).requires_grad_(True)
    sp_d = d(sp).requires_grad_(True)
    v_d = d(value).requires_grad_(True)
    loss, terms = _GaussPPOLoss.apply(mu_d, sp_d, v_d, (d(act), d(logp_old), d(adv), d(ret),
                                                         d(v_s), d(idx), p, DataParallel()))
    loss.backward()
    t = terms.cpu().numpy()
    np.testing.assert_allclose(t[1], float(want[1]), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(t[2], float(want[2]), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(t[3], float(want[3]), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(float(loss), float(want[0]), rtol=1e-5, atol=1e-6)
    gw = want[4]
    np.testing.assert_allclose(mu_d.grad.cpu().numpy(), gw["mu"].numpy(), rtol=1e-4,
                               atol=1e-6 * float(gw["mu"].abs().max()) + 1e-9)
    np.testing.assert_allclose(v_d.grad.cpu().numpy(), gw["value"].numpy(), rtol=1e-4,
                               atol=1e-6 * float(gw["value"].abs().max()) + 1e-9)
    np.testing.assert_allclose(sp_d.grad.cpu().numpy().flatten(), gw["sigma_param"].numpy(),
                               rtol=1e-4, atol=1e-6 * float(gw["sigma_param"].abs().max()) + 1e-9)


@pytest.mark.parametrize("tag", ["base", "multi", "clips", "nonorm"])
def test_learn_matches_reference(golden_dir, dev, tag):
    """PPOPolicy.learn on the reference's fixed weights and batch with the same
    np.random.seed (identical minibatch order): losses and post-Adam parameters."""
    from tianshou_amd.data import Batch
    from tianshou_amd.env import Box
    from tianshou_amd.policy import PPOPolicy
    from tianshou_amd.utils.models import fixed_std_normal, get_actor_critic, init_and_get_optim
    z = np.load(os.path.join(golden_dir, "ppo_learn.npz"))
    p = tag + "_"
    cfg = json.loads(str(z[p + "cfg"]))
    actor, critic = get_actor_critic((17,), (64, 64), (6,), dev)
    optim = init_and_get_optim(actor, critic, 3e-4)
    kw = dict(discount_factor=0.99, gae_lambda=0.95, max_grad_norm=0.5, vf_coef=0.25,
              ent_coef=0.0, reward_normalization=False, advantage_normalization=True,
              eps_clip=0.2, value_clip=False, dual_clip=None)
    kw.update({k: v for k, v in cfg.items() if k not in ("n", "batch_size", "repeat")})
    policy = PPOPolicy(actor, critic, optim, fixed_std_normal,
                       action_space=Box(-1.0, 1.0, (6,)), **kw).to(dev)
    assert policy._fused
    policy.load_state_dict({k[len(p + "init_"):]: torch.as_tensor(z[k]) for k in z.files
                            if k.startswith(p + "init_")})
    t = lambda k: torch.as_tensor(z[p + k], device=dev)
    batch = Batch(obs=t("obs"), act=t("act"), logp_old=t("logp_old"), adv=t("adv"),
                  returns=t("returns"), v_s=t("v_s"))
    np.random.seed(21)
    res = policy.learn(batch, batch_size=cfg["batch_size"], repeat=cfg["repeat"])
    def report(tag, g, w):
        g, w = np.asarray(g, np.float64), np.asarray(w, np.float64)
        e = np.abs(g - w)
        print(f"{p}{tag}: max abs err {e.max():.3g}, max rel err "
              f"{(e / np.maximum(np.abs(w), 1e-30)).max():.3g}")
    for k in ("loss", "loss/clip", "loss/vf", "loss/ent"):
        report(k, res[k], z[p + k.replace("/", "_")])
        # measured (round 3): <= 1.3e-5 rel on the clip term (|clip| ~ 0.02), <= 1e-6 abs
        np.testing.assert_allclose(res[k], z[p + k.replace("/", "_")], rtol=2e-5, atol=1e-6)
    if cfg["repeat"] == 1 and cfg["n"] == cfg["batch_size"]:
        for name, prm in policy.named_parameters():
            key = p + "grad_" + name
            if key in z.files:
                report("grad " + name, prm.grad.cpu().numpy(), z[key])
                np.testing.assert_allclose(prm.grad.cpu().numpy(), z[key], rtol=1e-4,
                                           atol=1e-6)
    sd = policy.state_dict()
    for k in z.files:
        if k.startswith(p + "final_actor.") or k.startswith(p + "final_critic."):
            report(k, sd[k[len(p + "final_"):]].cpu().numpy(), z[k])
            # measured (round 3): <= 5.7e-7 abs after the Adam steps (parameters ~0.1)
            np.testing.assert_allclose(sd[k[len(p + "final_"):]].cpu().numpy(), z[k],
                                       rtol=1e-5, atol=2e-6)
