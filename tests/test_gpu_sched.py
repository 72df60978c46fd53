"""BasePolicy.update with an lr_scheduler (base.py:288-315, get_linear_lr_schedular of
utils/lr_scheduler.py:47-56 -- the fork's lr_decay default) and recompute_advantage
(ppo.py:104-105) over three updates of one filled VectorReplayBuffer, against the reference
(tests/golden/ppo_sched.npz, tools/gen_goldens.py gen_sched).  The "graph" variant's
32-row minibatches replay captured learn graphs: the schedule's learning rate reaches the
fused Adam through a device word, so the graph is captured once, not once per update.

Tolerances: losses rtol 1e-4 (atol 1e-5), lr exact, ret_rms rel 1e-5, parameters after
27 Adam steps rtol 1e-3 (GPU vs CPU GEMMs, as test_gpu_ppo.py)."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tag", ["recompute", "graph", "graph_torch_adam"])
def test_scheduled_updates_match_reference(golden_dir, tag):
    """graph_torch_adam: the "graph" golden with the flat Adam pass off, so torch's capturable
    fused Adam runs inside the captured learn graph with its float lr baked in: each schedule
    step must re-capture (the lr is part of the graph key), or later updates would replay the
    first update's lr."""
    torch_adam = tag == "graph_torch_adam"
    tag = "graph" if torch_adam else tag
    from tianshou_amd.data import Batch, VectorReplayBuffer
    from tianshou_amd.env import Box
    from tianshou_amd.policy import PPOPolicy
    from tianshou_amd.utils.lr_scheduler import get_linear_lr_schedular
    from tianshou_amd.utils.models import fixed_std_normal, get_actor_critic, init_and_get_optim
    dev = torch.device("cuda", 0)
    z = np.load(os.path.join(golden_dir, "ppo_sched.npz"))
    p = tag + "_"
    cfg = json.loads(str(z[p + "cfg"]))
    E, T, D, A, bs = cfg["E"], cfg["T"], cfg["D"], cfg["A"], cfg["bs"]
    actor, critic = get_actor_critic((D,), (64, 64), (A,), dev)
    if torch_adam:  # on the device first: init_and_get_optim then builds a capturable Adam
        actor, critic = actor.to(dev), critic.to(dev)
    optim = init_and_get_optim(actor, critic, 3e-4)
    if torch_adam:
        assert optim.defaults["capturable"]
    policy = PPOPolicy(actor, critic, optim, fixed_std_normal, action_space=Box(-1.0, 1.0, (A,)),
                       discount_factor=0.99, gae_lambda=0.95, max_grad_norm=0.5, vf_coef=0.25,
                       ent_coef=0.01, reward_normalization=True, advantage_normalization=True,
                       recompute_advantage=cfg["recompute"], eps_clip=0.2).to(dev)
    assert policy._fused and policy._mlp is not None
    policy.fused_adam = not torch_adam
    policy.load_state_dict({k[len(p + "init_"):]: torch.as_tensor(z[k]) for k in z.files
                            if k.startswith(p + "init_")})
    policy.lr_scheduler = get_linear_lr_schedular(optim, step_per_epoch=3000,
                                                  step_per_collect=1000, epochs=2)
    buf = VectorReplayBuffer(E * T, E, device=dev)
    g = lambda k: z[p + "buf_" + k]  # noqa: E731
    for t in range(T):
        rows = np.arange(E) * T + t
        buf.add(Batch(obs=g("obs")[rows], act=g("act")[rows], rew=g("rew")[rows],
                      terminated=g("terminated")[rows], truncated=g("truncated")[rows],
                      obs_next=g("obs_next")[rows]), buffer_ids=np.arange(E))
    assert np.array_equal(buf._meta.done.cpu().numpy(), g("done"))
    np.random.seed(8)
    graphs = []
    for u in range(3):
        res = policy.update(0, buf, batch_size=bs, repeat=3)
        for k in ("loss", "loss/clip", "loss/vf", "loss/ent"):
            np.testing.assert_allclose(res[k], z[p + f"u{u}_" + k.replace("/", "_")],
                                       rtol=1e-4, atol=1e-5, err_msg=f"update {u} {k}")
        assert optim.param_groups[0]["lr"] == float(z[p + f"u{u}_lr"])
        rr = z[p + f"u{u}_ret_rms"]
        assert policy.ret_rms.mean == pytest.approx(rr[0], rel=1e-5)
        assert policy.ret_rms.var == pytest.approx(rr[1], rel=1e-5)
        assert policy.ret_rms.count == int(rr[2])
        graphs.append(policy._learn_graph["graph"] if policy._learn_graph else None)
    if torch_adam:
        # update 0 runs eagerly (no Adam state yet); the lr changes every update
        assert graphs[1] is not None and graphs[2] is not None and graphs[1] is not graphs[2]
        assert not policy._mlp.adam_bound(optim)
    elif tag == "graph":
        assert graphs[0] is not None and graphs[0] is graphs[1] is graphs[2]
    else:
        assert graphs == [None] * 3  # recompute_advantage runs the epochs eagerly
    sd = policy.state_dict()
    for k in z.files:
        if k.startswith(p + "final_actor.") or k.startswith(p + "final_critic."):
            # measured (round 3): <= 7.6e-8 abs after the Adam steps (round 2: 1e-3 / 1e-5)
            np.testing.assert_allclose(sd[k[len(p + "final_"):]].cpu().numpy(), z[k],
                                       rtol=1e-5, atol=1e-6, err_msg=k)
