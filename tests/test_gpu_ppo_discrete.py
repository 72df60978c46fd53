"""Categorical PPO (discrete actions): the fused tsrl_ppo_cat kernel vs the torch fp32
restatement (oracle/ref.py ppo_categorical_loss_torch), and PPOPolicy.learn /
Categorical log-probs vs the reference's recorded values (tests/golden/ppo_discrete.npz,
tools/gen_goldens.py gen_ppo_discrete).

Tolerances: loss terms rtol 1e-5; gradients rtol 1e-4 / atol 1e-6 * max|grad| (f32
reductions in another order than torch's); log-probs rtol 1e-5; learn() losses rtol 1e-4
and parameters after Adam rtol 1e-3 (GPU GEMMs vs the reference's CPU torch)."""
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


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("kw", CASES)
@pytest.mark.parametrize("B,A", [(4096, 6), (1000, 2), (257, 18)])
def test_cat_loss_vs_torch(dev, mode, kw, B, A):
    from tianshou_amd import _C
    from tianshou_amd.dist import DataParallel
    from tianshou_amd.policy.ppo import _CatPPOLoss
    g = torch.Generator().manual_seed(B * 3 + A + mode)
    n = B + 41
    z = torch.randn(B, A, generator=g) * 1.5
    x = z if mode == 0 else torch.softmax(z, -1)
    if mode == 1:  # a few rows with a saturated probability (clamp path of probs_to_logits)
        x[:3] = torch.nn.functional.one_hot(torch.arange(3) % A, A).float()
    value = torch.randn(B, generator=g)
    act = torch.randint(0, A, (n,), generator=g)
    logp_old = torch.randn(n, generator=g)
    adv = torch.randn(n, generator=g) * 2 + 0.3
    ret = torch.randn(n, generator=g)
    v_s = ret + torch.randn(n, generator=g) * 0.3
    idx = torch.randperm(n, generator=g)[:B]
    dist = torch.distributions.Categorical(logits=x) if mode == 0 else \
        torch.distributions.Categorical(probs=x)
    with torch.no_grad():
        logp_old[idx] = dist.log_prob(act[idx]) + torch.randn(B, generator=g) * 0.2
    eps_clip = kw.get("eps_clip", 0.2)
    want = ref.ppo_categorical_loss_torch(
        x, value, act[idx], logp_old[idx], adv[idx], ret[idx], v_s[idx], mode,
        eps_clip=eps_clip, dual_clip=kw.get("dual_clip"), value_clip=kw.get("value_clip", False),
        norm_adv=kw.get("norm_adv", True), vf_coef=0.25, ent_coef=kw.get("ent_coef", 0.01))
    p = _C.PPOParams()
    p.eps_clip, p.dual_clip = eps_clip, kw.get("dual_clip") or 0.0
    p.vf_coef, p.ent_coef, p.adv_eps, p.b_global = 0.25, kw.get("ent_coef", 0.01), 1e-8, B
    p.value_clip, p.norm_adv = int(kw.get("value_clip", False)), int(kw.get("norm_adv", True))
    d = lambda t: t.to(dev).contiguous()  # noqa: E731
    x_d = d(x).requires_grad_(True)
    v_d = d(value).requires_grad_(True)
    loss, terms = _CatPPOLoss.apply(x_d, v_d, (d(act), d(logp_old), d(adv), d(ret), d(v_s),
                                               d(idx), p, DataParallel(), mode))
    loss.backward()
    t = terms.cpu().numpy()
    for i in range(1, 4):
        np.testing.assert_allclose(t[i], float(want[i]), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(float(loss), float(want[0]), rtol=1e-5, atol=1e-6)
    gw = want[4]
    np.testing.assert_allclose(x_d.grad.cpu().numpy(), gw["x"].numpy(), rtol=1e-4,
                               atol=1e-6 * float(gw["x"].abs().max()) + 1e-9)
    np.testing.assert_allclose(v_d.grad.cpu().numpy(), gw["value"].numpy(), rtol=1e-4,
                               atol=1e-6 * float(gw["value"].abs().max()) + 1e-9)
    from tianshou_amd.policy.ppo import cat_logp
    lp = cat_logp(d(x), d(act[idx]), mode).cpu()
    np.testing.assert_allclose(lp.numpy(), dist.log_prob(act[idx]).numpy(), rtol=1e-5,
                               atol=1e-6)



def test_cat_loss_seed_paths(dev):
    """_CatPPOLoss's backward under the learn path's constant unit seed (the kernel's
    gradients handed over as they are, round 6) equals loss.backward()'s (x * 1.0 is x, bit
    for bit), and any other seed still scales them (2.5 * loss)."""
    from tianshou_amd import _C
    from tianshou_amd.dist import DataParallel
    from tianshou_amd.policy.ppo import _CatPPOLoss, _unit_seed
    g = torch.Generator().manual_seed(11)
    B, A, n = 96, 6, 137
    x = torch.randn(B, A, generator=g)
    value = torch.randn(B, generator=g)
    act = torch.randint(0, A, (n,), generator=g)
    logp_old, adv, ret = (torch.randn(n, generator=g) for _ in range(3))
    v_s = ret + 0.3 * torch.randn(n, generator=g)
    idx = torch.randperm(n, generator=g)[:B]
    p = _C.PPOParams()
    p.eps_clip, p.dual_clip, p.vf_coef, p.ent_coef, p.adv_eps, p.b_global = \
        0.2, 0.0, 0.25, 0.01, 1e-8, B
    p.value_clip, p.norm_adv = 1, 1
    d = lambda t: t.to(dev).contiguous()  # noqa: E731
    args = (d(act), d(logp_old), d(adv), d(ret), d(v_s), d(idx), p, DataParallel(), 0)
    grads = []
    for seed in ("ones", "unit", 2.5):
        x_d, v_d = d(x).requires_grad_(True), d(value).requires_grad_(True)
        loss, _ = _CatPPOLoss.apply(x_d, v_d, args)
        if seed == "ones":
            loss.backward()
        elif seed == "unit":
            loss.backward(_unit_seed(loss.device))
        else:
            (loss * seed).backward()
        grads.append((x_d.grad.clone(), v_d.grad.clone()))
    assert torch.equal(grads[0][0], grads[1][0]) and torch.equal(grads[0][1], grads[1][1])
    torch.testing.assert_close(grads[2][0], 2.5 * grads[0][0], rtol=1e-6, atol=0)
    torch.testing.assert_close(grads[2][1], 2.5 * grads[0][1], rtol=1e-6, atol=0)

def _discrete_policy(z, tag, dev):
    from tianshou_amd.env import Discrete
    from tianshou_amd.policy import PPOPolicy
    from tianshou_amd.utils.net import ActorCritic, DiscreteActor, DiscreteCritic, Net
    cfg = json.loads(str(z[tag + "_cfg"]))
    net = Net(cfg["obs"], hidden_sizes=(64, 64), device=dev)
    actor = DiscreteActor(net, cfg["act"], softmax_output=cfg["softmax"], device=dev).to(dev)
    critic = DiscreteCritic(Net(cfg["obs"], hidden_sizes=(64, 64), device=dev),
                            device=dev).to(dev)
    optim = torch.optim.Adam(ActorCritic(actor, critic).parameters(), lr=1e-3)
    dist = torch.distributions.Categorical if cfg["softmax"] else \
        (lambda q: torch.distributions.Categorical(logits=q))
    kw = dict(discount_factor=0.99, gae_lambda=0.95, max_grad_norm=0.5, vf_coef=0.5,
              eps_clip=0.2, advantage_normalization=True, action_scaling=False)
    kw.update({k: v for k, v in cfg.items()
               if k not in ("n", "batch_size", "repeat", "obs", "act", "softmax")})
    policy = PPOPolicy(actor, critic, optim, dist, action_space=Discrete(cfg["act"]),
                       **kw).to(dev)
    policy.load_state_dict({k[len(tag + "_init_"):]: torch.as_tensor(z[k]) for k in z.files
                            if k.startswith(tag + "_init_")})
    return policy, cfg


@pytest.mark.parametrize("tag", ["probs", "logits", "logits_multi"])
def test_learn_discrete_matches_reference(golden_dir, dev, tag):
    """PPOPolicy.learn (Categorical, fused loss) on the reference's fixed weights and batch
    with the same np.random.seed (identical minibatch order)."""
    from tianshou_amd.data import Batch
    z = np.load(os.path.join(golden_dir, "ppo_discrete.npz"))
    policy, cfg = _discrete_policy(z, tag, dev)
    assert policy._cat == (1 if cfg["softmax"] else 0)
    p = tag + "_"
    t = lambda k: torch.as_tensor(z[p + k], device=dev)  # noqa: E731
    lp = policy._logp_cat(t("obs"), t("act"))
    np.testing.assert_allclose(lp.cpu().numpy(), z[p + "logp_fresh"], rtol=1e-5, atol=1e-6)
    batch = Batch(obs=t("obs"), act=t("act"), logp_old=t("logp_old"), adv=t("adv"),
                  returns=t("returns"), v_s=t("v_s"))
    np.random.seed(21)
    res = policy.learn(batch, batch_size=cfg["batch_size"], repeat=cfg["repeat"])
    for k in ("loss", "loss/clip", "loss/vf", "loss/ent"):
        np.testing.assert_allclose(res[k], z[p + k.replace("/", "_")], rtol=1e-4, atol=1e-5)
    sd = policy.state_dict()
    for k in z.files:
        if k.startswith(p + "final_actor.") or k.startswith(p + "final_critic."):
            # measured (round 3): <= 2.1e-7 abs after the Adam steps (round 2: 1e-3 / 1e-5)
            np.testing.assert_allclose(sd[k[len(p + "final_"):]].cpu().numpy(), z[k],
                                       rtol=1e-5, atol=1e-6)
