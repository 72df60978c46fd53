"""NPGPolicy / TRPOPolicy (npg.py:68-181, trpo.py:74-160) vs the reference's recorded run
(tests/golden/npg.npz, tools/gen_goldens.py gen_npg): the reference collected a rollout with
its Collector on the synthetic env, ran process_fn (critic values, GAE with rew_norm,
logp_old, whole-batch advantage normalisation) and learn (2 repeats x 4 minibatches: vanilla
gradient, 10 CG steps on the KL Hessian, natural / KL-bounded step with line search, critic
Adam iterations).

CPU test: learn on the reference's process_fn output with torch on the host (the same
arithmetic as the reference, so tight tolerances).  GPU test: the device path end to end --
our collector's buffer holding the reference's rollout, process_fn through the fused MLP /
GAE kernels, learn on device tensors."""
import json
import os

import numpy as np
import pytest
import torch

CASES = ["npg", "trpo", "trpo_nonorm"]


def _policy(z, tag, dev, D, A):
    from tianshou_amd.env import Box
    from tianshou_amd.policy import NPGPolicy, TRPOPolicy
    from tianshou_amd.utils.models import fixed_std_normal, get_actor_critic, init_actor_critic
    p = tag + "_"
    cfg = json.loads(str(z[p + "cfg"]))
    cls = {"NPGPolicy": NPGPolicy, "TRPOPolicy": TRPOPolicy}[cfg.pop("cls")]
    actor, critic = get_actor_critic((D,), (64, 64), (A,), dev)
    actor, critic = actor.to(dev), critic.to(dev)
    init_actor_critic(actor, critic)
    optim = torch.optim.Adam(critic.parameters(), lr=1e-3)
    args = dict(discount_factor=0.99, gae_lambda=0.95, reward_normalization=True,
                advantage_normalization=True, optim_critic_iters=5, action_bound_method="clip",
                action_scaling=True)
    args.update(cfg)
    policy = cls(actor, critic, optim, fixed_std_normal, action_space=Box(-1.0, 1.0, (A,)),
                 **args).to(dev)
    policy.load_state_dict({k[len(p + "init_"):]: torch.as_tensor(z[k]) for k in z.files
                            if k.startswith(p + "init_")})
    return policy


def _check_learn(z, tag, res, policy, rtol, atol):
    p = tag + "_"
    keys = [k for k in z.files if k.startswith(p + "learn_")]
    assert keys
    for k in keys:
        name = k[len(p + "learn_"):]
        ours = res[{"loss_actor": "loss/actor", "loss_vf": "loss/vf"}.get(name, name)]
        np.testing.assert_allclose(ours, z[k], rtol=rtol, atol=atol, err_msg=name)
    sd = policy.state_dict()
    for k in z.files:
        if k.startswith(p + "final_actor.") or k.startswith(p + "final_critic."):
            np.testing.assert_allclose(sd[k[len(p + "final_"):]].cpu().numpy(), z[k],
                                       rtol=rtol, atol=atol, err_msg=k)


@pytest.mark.parametrize("tag", CASES)
def test_learn_cpu_matches_reference(golden_dir, tag):
    import warnings
    from tianshou_amd.data import Batch
    z = np.load(os.path.join(golden_dir, "npg.npz"))
    D, A = int(z["D"]), int(z["A"])
    policy = _policy(z, tag, torch.device("cpu"), D, A)
    p = tag + "_"
    idx = z[p + "indices"]
    t = lambda a: torch.as_tensor(np.asarray(a))  # noqa: E731
    batch = Batch(obs=t(z[p + "buf_obs"][idx]), act=t(z[p + "buf_act"][idx]).float(),
                  adv=t(z[p + "pf_adv"]), returns=t(z[p + "pf_returns"]),
                  v_s=t(z[p + "pf_v_s"]), logp_old=t(z[p + "pf_logp_old"]))
    np.random.seed(5)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        res = policy.learn(batch, batch_size=len(idx) // 4, repeat=2)
    _check_learn(z, tag, res, policy, rtol=1e-4, atol=2e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("tag", CASES)
def test_process_fn_and_learn_gpu_match_reference(golden_dir, tag):
    import warnings
    from tianshou_amd.data import Collector, VectorReplayBuffer
    from tianshou_amd.env import SyntheticVectorEnv, VectorEnvNormObs
    dev = torch.device("cuda", 0)
    z = np.load(os.path.join(golden_dir, "npg.npz"))
    E, D, A, L, T = (int(z[k]) for k in ("E", "D", "A", "L", "T"))
    policy = _policy(z, tag, dev, D, A)
    assert policy._fused and policy._mlp is not None
    env = VectorEnvNormObs(SyntheticVectorEnv(E, (D,), A, ep_len=L, device=dev))
    buf = VectorReplayBuffer(E * T, E, device=dev)
    c = Collector(policy, env, buf)
    c.collect(n_step=E * T)  # ring bookkeeping; the payload is replaced by the reference's
    p = tag + "_"
    m = buf._meta
    for k in ("obs", "obs_next", "act", "rew", "terminated", "truncated", "done"):
        getattr(m, k).copy_(torch.as_tensor(z[p + "buf_" + k], device=dev))
    batch, idx = buf.sample(0)
    assert idx.tolist() == z[p + "indices"].tolist()
    batch = policy.process_fn(batch, buf, idx)
    for k in ("v_s", "logp_old"):
        np.testing.assert_allclose(batch[k].cpu().numpy(), z[p + "pf_" + k], rtol=1e-4,
                                   atol=1e-5, err_msg=k)
    for k in ("returns", "adv"):
        np.testing.assert_allclose(batch[k].cpu().numpy(), z[p + "pf_" + k], rtol=1e-4,
                                   atol=1e-4, err_msg=k)
    np.random.seed(5)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        res = policy.learn(batch, batch_size=E * T // 4, repeat=2)
    _check_learn(z, tag, res, policy, rtol=2e-3, atol=2e-4)


def _dp_worker(rank, world, port, golden_dir, out):
    import sys
    import warnings
    import torch.distributed as dist
    from tests.conftest import PKG, ROOT
    for q in (ROOT, PKG):
        if q not in sys.path:
            sys.path.insert(0, q)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tianshou_amd.data import Batch
    z = np.load(os.path.join(golden_dir, "npg.npz"))
    D, A = int(z["D"]), int(z["A"])
    res = {}
    for tag in ("npg", "trpo"):
        policy = _policy(z, tag, torch.device("cpu"), D, A)
        assert policy.dp.active
        p = tag + "_"
        idx = z[p + "indices"]
        t = lambda a: torch.as_tensor(np.asarray(a))  # noqa: E731
        # identical batches on both ranks: every rank-average equals the local value, so
        # the data-parallel step must equal the single-process reference step
        batch = Batch(obs=t(z[p + "buf_obs"][idx]), act=t(z[p + "buf_act"][idx]).float(),
                      adv=t(z[p + "pf_adv"]), returns=t(z[p + "pf_returns"]),
                      v_s=t(z[p + "pf_v_s"]), logp_old=t(z[p + "pf_logp_old"]))
        np.random.seed(5)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            r = policy.learn(batch, batch_size=len(idx) // 4, repeat=2)
        res[tag] = (r, {k: v.clone() for k, v in policy.state_dict().items()})
    # whole-batch advantage normalisation over the ranks' shards
    a = torch.randn(64, generator=torch.Generator().manual_seed(4))
    res["adv"] = policy._normalize_adv(a[rank::world].clone())
    out[rank] = res
    dist.destroy_process_group()


def test_npg_trpo_data_parallel_gloo_two_ranks(golden_dir):
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = mp.Manager().dict()
    mp.spawn(_dp_worker, args=(2, port, golden_dir, out), nprocs=2, join=True)
    z = np.load(os.path.join(golden_dir, "npg.npz"))
    a = torch.randn(64, generator=torch.Generator().manual_seed(4))
    want_adv = ((a - a.mean()) / a.std()).numpy()
    for r in range(2):
        for tag in ("npg", "trpo"):
            res, sd = out[r][tag]

            class _P:  # state_dict holder for _check_learn
                def state_dict(self):
                    return sd
            _check_learn(z, tag, res, _P(), rtol=1e-4, atol=2e-5)
        np.testing.assert_allclose(out[r]["adv"].numpy(), want_adv[r::2], rtol=1e-5, atol=1e-6)
