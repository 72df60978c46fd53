"""Pipelined exact obs_rms (csrc/collect.hip E): exact_obs_rms=True with
the action-independent env computes each step's env rows d launches ahead and the reference's
f32 statistic of those rows on a second graph branch (tsrl_rms_exact_stats), merged by the
next step launch.  The result must be the serial exact path's, bit for bit.

* tsrl_rms_exact_stats against NumPy's own np.mean / np.var over axis 0 of the f32 rows --
  the reference's arithmetic (statistics.py:93-101) -- for the step rows and the done rows of
  the reset array, bitwise, over row counts around the 64-row DMA instructions, the 2048-row
  LDS span and the 1024-row reset-list segment;
* whole collects (graph replay, several graph lengths and pipeline depths, short episodes so
  that many envs reset per step) against exact_pipeline = 0 (one tsrl_rms_exact_update
  between launches): buffer rows, flags, obs_rms state and the live obs identical.
The reference goldens of the fused exact path (test_gpu_rollout.py
test_exact_obs_rms_collect_bitwise, D = 8 / 376, graph_steps 4) run through this pipeline
too (it is the default)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    return torch.device("cuda", 0)


def _stats(x, xr, done, dev):
    from tianshou_amd import _C
    k, D = x.shape
    nb = int(_C.lib().tsrl_rms_exact_stats_bytes(D))
    out = torch.zeros(nb, dtype=torch.uint8, device=dev)
    xt = torch.as_tensor(x, device=dev)
    xrt = torch.as_tensor(xr, device=dev)
    dt = torch.as_tensor(done.astype(np.uint8), device=dev)
    _C.check(_C.lib().tsrl_rms_exact_stats(_C.ptr(xt), k, _C.ptr(xrt), _C.ptr(dt), D,
                                           _C.ptr(out), _C.stream_ptr(dev)),
             "tsrl_rms_exact_stats")
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    f = o[:16 * D].view(np.float32).reshape(4, D)
    off = (16 * D + 7) // 8 * 8
    n = o[off:off + 16].view(np.int64)
    return f, int(n[0]), int(n[1])


@pytest.mark.parametrize("k,D", [(1, 8), (15, 8), (16, 376), (257, 20), (4096, 376),
                                 (5000, 64)])
@pytest.mark.parametrize("p", [0.0, 0.003, 0.5, 1.0])
def test_exact_stats_equal_numpy(dev, k, D, p):
    rng = np.random.default_rng(k * 7 + D + int(p * 1000))
    # values on the synthetic env's grid and off it (arbitrary f32)
    x = (rng.standard_normal((k, D)) * 3 + 1).astype(np.float32)
    xr = (rng.standard_normal((k, D)) * 0.5 - 2).astype(np.float32)
    done = rng.random(k) < p
    f, n1, nd = _stats(x, xr, done, dev)
    assert n1 == k and nd == int(done.sum())
    assert np.array_equal(f[0], np.mean(x, axis=0)), "step-row mean"
    assert np.array_equal(f[1], np.var(x, axis=0)), "step-row var"
    if nd:
        assert np.array_equal(f[2], np.mean(xr[done], axis=0)), "reset-row mean"
        assert np.array_equal(f[3], np.var(xr[done], axis=0)), "reset-row var"


def _run(dev, depth, E, D, A, L, T, G, seed=3, group=1):
    """One collect of E * T steps at pipeline depth / statistics group (depth 0: serial)."""
    from tianshou_amd.data import Collector, VectorReplayBuffer
    from tianshou_amd.env import Box, SyntheticVectorEnv, VectorEnvNormObs
    from tianshou_amd.policy import PPOPolicy
    from tianshou_amd.utils.models import fixed_std_normal, get_actor_critic, init_and_get_optim
    torch.manual_seed(seed)
    actor, critic = get_actor_critic((D,), (64, 64), (A,), dev)
    optim = init_and_get_optim(actor, critic, 3e-4)
    policy = PPOPolicy(actor.to(dev), critic.to(dev), optim, fixed_std_normal,
                       action_space=Box(-1.0, 1.0, (A,)), action_bound_method="clip").to(dev)
    env = VectorEnvNormObs(SyntheticVectorEnv(E, (D,), A, ep_len=L, seed=seed, device=dev),
                           exact_obs_rms=True)
    buf = VectorReplayBuffer(E * T, E, device=dev)
    c = Collector(policy, env, buf)
    c.graph_steps = G
    c.exact_pipeline = depth
    c.exact_group = group
    torch.manual_seed(seed + 1)
    res = c.collect(n_step=E * T)
    assert c._step_on
    assert c._xpipe_ok() == (depth > 0)
    rms = env.get_obs_rms()
    m = buf._meta
    out = {k: getattr(m, k).cpu().numpy() for k in ("obs", "obs_next", "act", "rew",
                                                      "terminated", "truncated", "done")}
    out.update(mean=rms.mean, var=rms.var, count=rms.count, live=c.data.obs.cpu().numpy(),
               n_ep=res["n/ep"], rews=res["rews"])
    return out


@pytest.mark.parametrize("E,D,L,T,G", [(64, 8, 3, 12, 4), (512, 376, 5, 10, 4),
                                       (4096, 376, 7, 16, 8),
                                       # every env resets every step; a partial 16-row tile
                                       (100, 20, 1, 9, 2), (37, 12, 2, 7, 6)])
@pytest.mark.parametrize("depth", [1, 2, 3])
def test_pipelined_exact_collect_equals_serial(dev, E, D, L, T, G, depth):
    ref = _run(dev, 0, E, D, 6, L, T, G)
    got = _run(dev, depth, E, D, 6, L, T, G)
    for k in ref:
        assert np.array_equal(np.asarray(got[k]), np.asarray(ref[k])), k


@pytest.mark.parametrize("E,D,L,T,G", [(64, 8, 3, 12, 4), (512, 376, 5, 10, 6),
                                       (4096, 376, 7, 16, 8), (100, 20, 1, 9, 2)])
@pytest.mark.parametrize("depth,group", [(3, 2), (4, 2), (4, 3), (5, 2)])
def test_pipelined_exact_grouped_equals_serial(dev, E, D, L, T, G, depth, group):
    """Several steps' statistics per launch (tsrl_rms_exact_stats_n, Collector.exact_group):
    the same bits as the serial form, for graph lengths that do and do not divide evenly."""
    ref = _run(dev, 0, E, D, 6, L, T, G)
    got = _run(dev, depth, E, D, 6, L, T, G, group=group)
    for k in ref:
        assert np.array_equal(np.asarray(got[k]), np.asarray(ref[k])), k
