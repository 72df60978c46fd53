"""ORACLE (bench cpu_baseline leg only) -- CPU port of one on-policy iteration:
synthetic env (NumPy) + VectorEnvNormObs (NumPy RunningMeanStd) + VectorReplayBuffer
storage (NumPy) + critic values / GAE (C oracle) + PPO learn (torch CPU fp32), i.e. the
reference algorithm (collector.py:184-402, a2c.py:83-117, ppo.py:87-162) restated for a
bounded sample of the bench workload.  Timed on the GPU box's host cores by bench.py;
never used by the product path.

``tests/test_oracle.py::test_cpu_port_matches_reference_collector`` runs it at config 2's
observation width (16 envs x 24 steps, D = 17) with the reference policy's initial weights
and checks its obs_rms, stored rows, rewards and process_fn returns / advantages against the
reference Collector + VectorEnvNormObs + process_fn goldens (``collector_d17.npz``): the
baseline the bench reports is a parity-checked restatement.
"""
import time

import numpy as np
import torch

from oracle import ref, synth_env


# reference state-dict keys (policy.state_dict(), utils/net/common.py Net.model, continuous.py
# ActorProb.mu / Critic.last) -> (net, layer index) of the nn.Sequential nets below
_REF_KEYS = {"actor.preprocess.model.model.0": ("actor", 0),
             "actor.preprocess.model.model.2": ("actor", 2),
             "actor.mu.model.0": ("actor", 4),
             "critic.preprocess.model.model.0": ("critic", 0),
             "critic.preprocess.model.model.2": ("critic", 2),
             "critic.last.model.0": ("critic", 4)}


def run_iteration(E, T, D, A, repeat=4, minibatches=32, ep_len=1000, threads=None, seed=0,
                  init=None, record=None):
    """One iteration; returns (env-steps/s, seconds).  ``init``: the reference policy's
    state-dict arrays (keys as _REF_KEYS + "actor.sigma_param") to start from; ``record``: a
    dict that receives obs_rms, the stored rows, rewards and process_fn's returns / adv."""
    if threads:
        torch.set_num_threads(threads)
    torch.manual_seed(seed)
    np.random.seed(seed)
    from torch import nn
    from torch.distributions import Independent, Normal

    def mlp(out):
        return nn.Sequential(nn.Linear(D, 64), nn.Tanh(), nn.Linear(64, 64), nn.Tanh(),
                             nn.Linear(64, out))
    actor, critic = mlp(A), mlp(1)
    sigma = nn.Parameter(torch.full((A,), -0.5))
    if init is not None:
        with torch.no_grad():
            nets = {"actor": actor, "critic": critic}
            for k, (net, i) in _REF_KEYS.items():
                nets[net][i].weight.copy_(torch.as_tensor(init[k + ".weight"]))
                nets[net][i].bias.copy_(torch.as_tensor(init[k + ".bias"]))
            sigma.copy_(torch.as_tensor(init["actor.sigma_param"]).reshape(-1))
    params = list(actor.parameters()) + list(critic.parameters()) + [sigma]
    optim = torch.optim.Adam(params, lr=3e-4)
    env = synth_env.SynthVecEnvNP(E, (D,), A, ep_len, seed=seed)
    rms = ref.RMS()
    ret_rms = ref.RMS()
    t0 = time.perf_counter()
    obs = env.reset()
    rms.update(obs)
    obs = rms.norm(obs)
    S_obs = np.zeros((E, T, D), np.float32)
    S_next = np.zeros((E, T, D), np.float32)
    S_act = np.zeros((E, T, A), np.float32)
    S_rew = np.zeros((E, T), np.float64)
    S_term = np.zeros((E, T), bool)
    S_trunc = np.zeros((E, T), bool)
    for t in range(T):
        with torch.no_grad():
            mu = actor(torch.as_tensor(obs))
            act = Independent(Normal(mu, sigma.exp().expand_as(mu)), 1).sample().numpy()
        _ = np.clip(act, -1.0, 1.0)
        nxt, rew, term, trunc = env.step()
        rms.update(nxt)
        nxt = rms.norm(nxt)
        S_obs[:, t], S_next[:, t], S_act[:, t] = obs, nxt, act
        S_rew[:, t], S_term[:, t], S_trunc[:, t] = rew, term, trunc
        obs = nxt.copy()
        done = np.flatnonzero(term | trunc)
        if len(done):
            r = env.reset(done)
            rms.update(r)
            obs[done] = rms.norm(r)
    n = E * T
    o = torch.as_tensor(S_obs.reshape(n, D))
    on = torch.as_tensor(S_next.reshape(n, D))
    act = torch.as_tensor(S_act.reshape(n, A))
    with torch.no_grad():
        v_s = critic(o).flatten().numpy()
        v_n = critic(on).flatten().numpy()
    scale = np.sqrt(ret_rms.var + 1e-8)
    ret, adv = ref.compute_episodic_return(S_rew.reshape(-1), S_term.reshape(-1),
                                           S_trunc.reshape(-1), np.arange(n),
                                           np.arange(T - 1, n, T), v_n * scale, v_s * scale,
                                           0.99, 0.95)
    returns = torch.as_tensor((ret / scale).astype(np.float32))
    adv_t = torch.as_tensor(adv.astype(np.float32))
    if record is not None:
        record.update(rms_mean=np.asarray(rms.mean), rms_var=np.asarray(rms.var),
                      rms_count=rms.count, obs=S_obs.reshape(n, D),
                      obs_next=S_next.reshape(n, D), rew=S_rew.reshape(-1), v_s=v_s,
                      returns=returns.numpy(), adv=adv_t.numpy())
    ret_rms.update(ret)
    with torch.no_grad():
        mu = actor(o)
        logp_old = Independent(Normal(mu, sigma.exp().expand_as(mu)), 1).log_prob(act)
    v_old = torch.as_tensor(v_s)
    bs = n // minibatches
    for _ in range(repeat):
        perm = torch.as_tensor(np.random.permutation(n))
        for s in range(0, n, bs):
            idx = perm[s:s + bs]
            mu = actor(o[idx])
            value = critic(o[idx]).flatten()
            a = adv_t[idx]
            a = (a - a.mean()) / (a.std() + 1e-8)
            dist = Independent(Normal(mu, sigma.exp().expand_as(mu)), 1)
            ratio = (dist.log_prob(act[idx]) - logp_old[idx]).exp()
            clip = -torch.min(ratio * a, ratio.clamp(0.8, 1.2) * a).mean()
            vf = (returns[idx] - value).pow(2).mean()
            loss = clip + 0.25 * vf
            optim.zero_grad()
            loss.backward()
            nn.utils.clip_grad_norm_(params, 0.5)
            optim.step()
    dt = time.perf_counter() - t0
    return n / dt, dt
