"""Atari-shaped on-policy path (BASELINE config 5 in miniature): uint8
4x84x84 frame stacks from the device env (frame_stack=4, gymnasium FrameStack semantics),
a save_only_last_obs / ignore_obs_next / stack_num=4 VectorReplayBuffer
(examples/atari/atari_ppo.py:183-189), the Nature-DQN trunk shared by a logits actor and a
critic (atari_ppo.py:104-137) and PPO with the fused Categorical loss.

Parity: the buffer stores exactly the last frame of every observation (bit-exact vs the
NumPy env restatement, oracle/synth_env.py), and the stacked observations the buffer
rebuilds through its episode-aware prev chain are exactly the frame stacks the collector saw
(bit-exact).  The PPO update must produce finite losses and the fused-loss learn() must
match the torch formulation of the same update (rtol 1e-4 on the losses)."""
import numpy as np
import pytest
import torch

from oracle import synth_env

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    return torch.device("cuda", 0)


def _setup(dev, E, T, L, seed=0):
    from tianshou_amd.data import Collector, VectorReplayBuffer
    from tianshou_amd.env import Discrete, SyntheticVectorEnv
    from tianshou_amd.policy import PPOPolicy
    from tianshou_amd.utils.net import ActorCritic, DiscreteActor, DiscreteCritic
    from tianshou_amd.utils.net_atari import DQN, layer_init
    torch.manual_seed(seed)
    env = SyntheticVectorEnv(E, (4, 84, 84), 6, ep_len=L, seed=3, device=dev,
                             obs_dtype=np.uint8, discrete=True, frame_stack=4)
    net = DQN(4, 84, 84, (6,), device=dev, features_only=True, output_dim=512,
              layer_init=layer_init).to(dev)
    actor = DiscreteActor(net, 6, softmax_output=False, device=dev).to(dev)
    critic = DiscreteCritic(net, device=dev).to(dev)
    optim = torch.optim.Adam(ActorCritic(actor, critic).parameters(), lr=2.5e-4)
    policy = PPOPolicy(actor, critic, optim,
                       lambda p: torch.distributions.Categorical(logits=p),
                       action_space=Discrete(6), action_scaling=False, discount_factor=0.99,
                       gae_lambda=0.95, max_grad_norm=0.5, vf_coef=0.25, ent_coef=0.01,
                       eps_clip=0.1, value_clip=True, advantage_normalization=False,
                       reward_normalization=True).to(dev)
    buf = VectorReplayBuffer(E * T, E, stack_num=4, ignore_obs_next=True,
                             save_only_last_obs=True, device=dev)
    return env, policy, buf, Collector(policy, env, buf, exploration_noise=True)


def test_atari_frame_stack_collect_and_update(dev):
    E, T, L = 8, 24, 11
    env, policy, buf, coll = _setup(dev, E, T, L)
    res = coll.collect(n_step=E * T)
    assert res["n/st"] == E * T
    assert buf.obs.shape == (buf.maxsize, 84, 84) and buf.obs.dtype == torch.uint8
    assert "obs_next" not in buf._meta.keys()
    # the observation stream of every env, from the NumPy env restatement
    ref = synth_env.SynthVecEnvNP(E, (4, 84, 84), 6, L, seed=3, u8=True, frame_stack=4)
    cur = ref.reset()
    seen = np.zeros((E, T, 4, 84, 84), np.uint8)
    dones = np.zeros((E, T), bool)
    for t in range(T):
        seen[:, t] = cur
        nxt, _, term, trunc = ref.step()
        done = term | trunc
        dones[:, t] = done
        if done.any():
            ids = np.flatnonzero(done)
            nxt[ids] = ref.reset(ids)
        cur = nxt
    stored = buf.obs.cpu().numpy().reshape(E, T, 84, 84)
    assert np.array_equal(stored, seen[:, :, -1])
    batch, idx = buf.sample(0)
    assert np.array_equal(idx, np.arange(E * T))
    assert batch.obs.shape == (E * T, 4, 84, 84)
    assert np.array_equal(batch.obs.cpu().numpy().reshape(E, T, 4, 84, 84), seen)
    # obs_next = get(next(idx), "obs"): the next observation inside an episode, the row's own
    # observation where the episode (or the stored data) ends (base.py:380-381)
    on = batch.obs_next.cpu().numpy().reshape(E, T, 4, 84, 84)
    inner = ~dones[:, :-1]
    assert np.array_equal(on[:, :-1][inner], seen[:, 1:][inner])
    assert np.array_equal(on[:, :-1][~inner], seen[:, :-1][~inner])
    assert np.array_equal(on[:, -1], seen[:, -1])
    assert np.array_equal(batch.info.env_id.cpu().numpy()[:, -1],
                          np.repeat(np.arange(E), T))
    out = policy.update(0, buf, batch_size=E * T // 4, repeat=2)
    assert len(out["loss"]) == 8 and np.all(np.isfinite(out["loss"]))


def test_atari_fused_cat_learn_matches_torch_formulation(dev):
    """The same collected batch and minibatch order through the fused Categorical loss and
    through the reference's torch formulation (_learn_generic)."""
    E, T, L = 8, 16, 7
    _, policy, buf, coll = _setup(dev, E, T, L, seed=1)
    coll.collect(n_step=E * T)
    batch, idx = buf.sample(0)
    batch = policy.process_fn(batch, buf, idx)
    sd = {k: v.clone() for k, v in policy.state_dict().items()}
    osd = policy.optim.state_dict()
    results = []
    for fused in (True, False):
        policy.load_state_dict(sd)
        policy.optim.load_state_dict(osd)
        np.random.seed(4)
        if fused:
            r = policy.learn(batch, batch_size=E * T // 2, repeat=2)
        else:
            r = policy._learn_generic(batch, batch_size=E * T // 2, repeat=2)
        results.append((r, {k: v.detach().cpu().clone() for k, v in
                            policy.state_dict().items()}))
    for k in ("loss", "loss/clip", "loss/vf", "loss/ent"):
        np.testing.assert_allclose(results[0][0][k], results[1][0][k], rtol=1e-4, atol=1e-5)
    # parameters after 4 Adam steps: Adam normalises each element's step to ~lr, so an
    # element whose gradient sits at the f32 noise level (summation order differs between the
    # two formulations and MIOpen's kernel choice) can move by up to lr per step either way;
    # allow that for at most 0.1 % of the elements, everything else within rtol 1e-3
    lr, steps = 2.5e-4, 4
    keys = list(results[0][1])
    a = np.concatenate([results[0][1][k].numpy().ravel() for k in keys])
    b = np.concatenate([results[1][1][k].numpy().ravel() for k in keys])
    bad = ~np.isclose(a, b, rtol=1e-3, atol=1e-5)
    assert bad.mean() <= 1e-3, bad.sum()
    assert np.abs(a - b).max() <= lr * steps


def test_atari_shared_trunk_process_fn_matches_separate_passes(dev):
    """process_fn with the shared DQN trunk (one trunk pass per row for V(s) and logp_old,
    V(s') read from V(s) through next(), base.py:380-381) against the reference's three
    separate passes (a2c.py:86-93 critic(obs), critic(obs_next); ppo.py:95-96 actor(obs))."""
    from tianshou_amd.policy.base import gae_device
    E, T, L = 8, 24, 9
    _, policy, buf, coll = _setup(dev, E, T, L, seed=2)
    policy._rew_norm = False
    assert policy._shared_trunk
    coll.collect(n_step=E * T)
    batch, idx = buf.sample(0)
    with torch.no_grad():
        v_ref = policy.critic(batch.obs).flatten()
        vn_ref = policy.critic(batch.obs_next).flatten()
        x, _ = policy.actor(batch.obs)
        lp_ref = torch.distributions.Categorical(logits=x).log_prob(batch.act.reshape(-1))
    p = policy._next_positions(buf, idx, dev)
    assert p is not None
    want_p = buf.next(idx)  # host next() over the same ring
    assert np.array_equal(p.cpu().numpy(), want_p)
    out = policy.process_fn(batch, buf, idx)
    # same weights, same rows; MIOpen may pick other kernels for the other call sequence
    vmax = float(v_ref.abs().max())
    np.testing.assert_allclose(out.v_s.cpu().numpy(), v_ref.cpu().numpy(), rtol=1e-5,
                               atol=1e-5 * vmax)
    np.testing.assert_allclose(out.logp_old.cpu().numpy(), lp_ref.cpu().numpy(), rtol=1e-5,
                               atol=1e-6)
    adv, ret, _, _ = gae_device(v_ref.contiguous(), vn_ref.contiguous(),
                                batch.rew.contiguous(), batch.terminated.contiguous(),
                                batch.truncated.contiguous(), 0.99, 0.95, T)
    np.testing.assert_allclose(out.adv.cpu().numpy(), adv.cpu().numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(out.returns.cpu().numpy(), ret.cpu().numpy(), rtol=1e-5,
                               atol=1e-5)
    # a partial sample whose next rows are missing falls back to evaluating obs_next
    sub = idx[::3]
    assert policy._next_positions(buf, sub, dev) is None


def test_frames_to_f32_nhwc_bit_exact(dev):
    """tsrl_frames_to_f32_nhwc = scale_obs (atari_network.py:18-30: obs / 255 in f64, then the
    trunk's f32 cast, :84) + the NHWC layout, bit for bit: the 4-channel vector path and the
    general path (odd plane sizes, other channel counts)."""
    from tianshou_amd.utils.net_atari import DQN, frames_to_f32_nhwc
    g = torch.Generator(device="cpu").manual_seed(0)
    lut = DQN(4, 84, 84, (6,), device=dev, features_only=True)._scale_lut(dev)
    for shape in ((37, 4, 84, 84), (5, 4, 7, 9), (3, 3, 84, 84), (2, 1, 5, 5), (0, 4, 84, 84)):
        obs = torch.randint(0, 256, shape, generator=g, dtype=torch.uint8)
        want = torch.as_tensor((obs.numpy() / 255.0).astype(np.float32))
        got = frames_to_f32_nhwc(obs.to(dev), lut)
        assert got.shape == shape and got.is_contiguous(memory_format=torch.channels_last)
        assert torch.equal(got.cpu(), want), shape


def test_dqn_nchw_input_scaling_bit_exact(dev):
    """The plain NCHW trunk (channels_last=False) scales uint8 frames through the same host-
    divided table as the NHWC path: its first layer sees scale_obs's f64 division + f32 cast
    bit for bit (atari_network.py:18-30, :84), so layout is the only difference between the
    two trunks."""
    from tianshou_amd.utils.net_atari import DQN
    b = DQN(4, 84, 84, (6,), device=dev, features_only=True, channels_last=False).to(dev)
    b.fused_conv1 = False
    seen = []
    h = b.net[0].register_forward_pre_hook(lambda m, inp: seen.append(inp[0].detach().clone()))
    g = torch.Generator(device="cpu").manual_seed(3)
    obs = torch.randint(0, 256, (9, 4, 84, 84), generator=g, dtype=torch.uint8)
    want = torch.as_tensor((obs.numpy() / 255.0).astype(np.float32))
    b(obs.to(dev))
    b(obs)  # host frames take the same table
    h.remove()
    assert len(seen) == 2
    for x in seen:
        assert x.dtype == torch.float32 and torch.equal(x.cpu(), want)


def test_dqn_nhwc_trunk_matches_nchw(dev):
    """The NHWC trunk fed by tsrl_frames_to_f32_nhwc against the plain NCHW module with the
    same weights (summation order only)."""
    from tianshou_amd.utils.net_atari import DQN, layer_init
    torch.manual_seed(0)
    a = DQN(4, 84, 84, (6,), device=dev, features_only=True, output_dim=512,
            layer_init=layer_init).to(dev)
    torch.manual_seed(0)
    b = DQN(4, 84, 84, (6,), device=dev, features_only=True, output_dim=512,
            layer_init=layer_init, channels_last=False).to(dev)
    a.fused_conv1 = b.fused_conv1 = False
    x = torch.randint(0, 256, (64, 4, 84, 84), dtype=torch.uint8, device=dev)
    ya, yb = a(x)[0], b(x)[0]
    torch.testing.assert_close(ya, yb, rtol=1e-4, atol=1e-5 * float(yb.abs().max()))
    g = torch.randn_like(ya)
    ya.backward(g)
    yb.backward(g)
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa.grad, pb.grad, rtol=1e-3,
                                   atol=1e-4 * float(pb.grad.abs().max()))


@pytest.mark.parametrize("n", [1, 37, 300])
def test_conv2_dgrad_kernel_vs_f64(dev, n):
    """tsrl_dqn_conv2_dgrad against fp64 conv_transpose (torch's conv2d input gradient) with
    the ReLU mask of z1: elementwise within 1e-6 of the absolute-value product (f32 GEMM
    error), masked entries exactly zero, ragged batches (tiles straddle samples)."""
    from tianshou_amd import _C
    torch.manual_seed(n)
    w = torch.randn(64, 32, 4, 4, device=dev).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(n, 9, 9, 64, device=dev)
    z1 = torch.relu(torch.randn(n, 20, 20, 32, device=dev))
    out = torch.empty(n, 20, 20, 32, device=dev)
    _C.check(_C.lib().tsrl_dqn_conv2_dgrad(_C.ptr(gy), n, w.data_ptr(), *w.stride(),
                                           _C.ptr(z1), _C.ptr(out), _C.stream_ptr(dev)), "dgrad")
    g64 = gy.permute(0, 3, 1, 2).double()
    ref = torch.nn.grad.conv2d_input((n, 32, 20, 20), w.double(), g64, stride=2)
    mag = torch.nn.grad.conv2d_input((n, 32, 20, 20), w.double().abs(), g64.abs(), stride=2)
    mask = (z1 > 0).permute(0, 3, 1, 2)
    got = out.permute(0, 3, 1, 2).double()
    assert bool((got[~mask] == 0).all())
    err = (got - ref)[mask].abs()
    assert bool((err <= 1e-6 * mag[mask] + 1e-12).all()), float((err / mag[mask]).max())
    # unmasked form
    _C.check(_C.lib().tsrl_dqn_conv2_dgrad(_C.ptr(gy), n, w.data_ptr(), *w.stride(), None,
                                           _C.ptr(out), _C.stream_ptr(dev)), "dgrad")
    err = (out.permute(0, 3, 1, 2).double() - ref).abs()
    assert bool((err <= 1e-6 * mag + 1e-12).all())


@pytest.mark.parametrize("rows,C", [(1, 64), (37 * 49, 64), (8192 * 81, 64), (1000, 4),
                                    (333, 32), (4097, 512)])
def test_relu_bwd_rows_vs_torch(dev, rows, C):
    """tsrl_relu_bwd_rows: gy bit-identical to threshold_backward, gb within 1e-6 of the f64
    column sum relative to the sum of magnitudes (f32 partials, f64 fold); in place
    (gy aliasing gz) and without gb; through relu_bwd_bias on channels_last activations."""
    from tianshou_amd import _C
    from tianshou_amd.utils.net_atari import relu_bwd_bias
    torch.manual_seed(rows + C)
    gz = torch.randn(rows, C, device=dev)
    z = torch.relu(torch.randn(rows, C, device=dev))
    ref = torch.ops.aten.threshold_backward(gz, z, 0.0)
    nb = int(_C.lib().tsrl_relu_bwd_rows_workspace_bytes(rows, C))
    ws = torch.full((nb,), 0xFF, dtype=torch.uint8, device=dev)
    gy = torch.full_like(gz, float("nan"))
    gb = torch.full((C,), float("nan"), device=dev)
    s_ = _C.stream_ptr(dev)
    _C.check(_C.lib().tsrl_relu_bwd_rows(_C.ptr(gz), _C.ptr(z), _C.ptr(gy), rows, C, _C.ptr(gb),
                                         ws.data_ptr(), nb, s_), "relu_bwd")
    assert torch.equal(gy, ref)
    r64 = ref.double()
    err = (gb.double() - r64.sum(0)).abs()
    assert bool((err <= 1e-6 * r64.abs().sum(0) + 1e-30).all()), float(err.max())
    g2 = gz.clone()
    _C.check(_C.lib().tsrl_relu_bwd_rows(_C.ptr(g2), _C.ptr(z), _C.ptr(g2), rows, C, None, None,
                                         0, s_), "relu_bwd in place")
    assert torch.equal(g2, ref)
    assert _C.lib().tsrl_relu_bwd_rows(_C.ptr(gz), _C.ptr(z), _C.ptr(gy), rows, C, _C.ptr(gb),
                                       ws.data_ptr(), nb - 16, s_) != 0
    if rows % 49 == 0:
        n = rows // 49
        to4 = lambda t: t.view(n, 7, 7, C).permute(0, 3, 1, 2)
        gy4, gb4 = relu_bwd_bias(to4(gz), to4(z), True)
        assert gy4.is_contiguous(memory_format=torch.channels_last)
        assert torch.equal(gy4, to4(ref)) and torch.equal(gb4, gb)


@pytest.mark.parametrize("n", [1, 5, 37, 300])
def test_conv1_wgrad_u8_vs_f64(dev, n):
    """tsrl_dqn_conv1_wgrad (bytes exact in bf16, gy split in 3 bf16 planes, per-workgroup
    partials folded in f64) against fp64 conv2d_weight of (frames / 255, gy): elementwise
    within 1e-6 of the absolute-value product (f32 GEMM error), bias gradient = sum of gy in
    f64 within 1e-6 relative; ragged batches (chunks of 32 pixels straddle samples, the last
    chunk partial); the channels_last weight gets a channels_last gradient."""
    from tianshou_amd.utils.net_atari import conv1_u8_wgrad
    torch.manual_seed(100 + n)
    x = torch.randint(0, 256, (n, 4, 84, 84), dtype=torch.uint8, device=dev)
    gy = torch.randn(n, 20, 20, 32, device=dev)
    gy[torch.rand_like(gy) < 0.4] = 0.0  # ReLU-masked rows
    w = torch.empty(32, 4, 8, 8, device=dev).contiguous(memory_format=torch.channels_last)
    gw, gb = conv1_u8_wgrad(x, gy, w, 255.0, True)
    assert gw.shape == (32, 4, 8, 8) and gw.is_contiguous(memory_format=torch.channels_last)
    x64 = x.double() / 255.0
    g64 = gy.permute(0, 3, 1, 2).double()
    ref = torch.nn.grad.conv2d_weight(x64, (32, 4, 8, 8), g64, stride=4)
    mag = torch.nn.grad.conv2d_weight(x64, (32, 4, 8, 8), g64.abs(), stride=4)
    err = (gw.double() - ref).abs()
    assert bool((err <= 1e-6 * mag + 1e-12).all()), float((err / (mag + 1e-30)).max())
    gb_ref = g64.sum(dim=(0, 2, 3))
    gb_mag = g64.abs().sum(dim=(0, 2, 3))
    assert bool(((gb.double() - gb_ref).abs() <= 1e-6 * gb_mag + 1e-12).all())
    # no bias: gb is None
    gw2, gb2 = conv1_u8_wgrad(x, gy, w.contiguous(), 255.0, False)
    assert gb2 is None and gw2.is_contiguous()
    assert torch.equal(gw2, gw.contiguous())


def test_conv1_wgrad_u8_production_size(dev):
    """tsrl_dqn_conv1_wgrad at the config-5 minibatch (8192 frame stacks: 512 workgroups x 50
    chunks, the full partial-slab fold) against MIOpen's f32 weight gradient of the f32 frames:
    within 2e-6 of the absolute-value product (both are f32 GEMMs of the same data)."""
    from tianshou_amd.utils.net_atari import conv1_u8_wgrad
    torch.manual_seed(7)
    n = 8192
    x = torch.randint(0, 256, (n, 4, 84, 84), dtype=torch.uint8, device=dev)
    gy = torch.randn(n, 20, 20, 32, device=dev)
    gy[torch.rand_like(gy) < 0.5] = 0.0
    w = torch.empty(32, 4, 8, 8, device=dev)
    gw, gb = conv1_u8_wgrad(x, gy, w, 255.0, True)
    xf = (x.float() / 255.0)
    g = gy.permute(0, 3, 1, 2)
    ref = torch.nn.grad.conv2d_weight(xf, (32, 4, 8, 8), g, stride=4)
    mag = torch.nn.grad.conv2d_weight(xf, (32, 4, 8, 8), g.abs(), stride=4)
    assert bool(((gw - ref).abs() <= 2e-6 * mag + 1e-9).all()), float(((gw - ref).abs() / mag).max())
    # bias: the f32 sum of 1.6M signed terms, within 1e-6 of the sum of their magnitudes
    gb_ref = g.double().sum(dim=(0, 2, 3))
    gb_mag = g.double().abs().sum(dim=(0, 2, 3))
    assert bool(((gb.double() - gb_ref).abs() <= 1e-6 * gb_mag).all())


@pytest.mark.parametrize("n", [1, 37, 1024])
def test_conv1_u8_kernel_vs_f64(dev, n):
    """tsrl_dqn_conv1_fwd (uint8 frames, bf16 byte operands x 3-plane split weights) against
    an fp64 relu(conv(frames / 255) + b): elementwise within 1e-6 of sum|w x| + |b| (f32 GEMM
    error), and in RMS no worse than 2x torch's own f32 convolution of the f32 frames; the
    weight is channels_last (strided access) and the batch ragged (tiles straddle
    samples)."""
    from tianshou_amd.utils.net_atari import DQN, conv1_u8, layer_init
    torch.manual_seed(n)
    net = DQN(4, 84, 84, (6,), device=dev, features_only=True, output_dim=512,
              layer_init=layer_init).to(dev)
    conv = net._conv1_parts()[0]
    assert net._conv1_parts()[1] is not None  # conv2 data gradient on the HIP path too
    with torch.no_grad():
        conv.bias.uniform_(-0.5, 0.5)
    x = torch.randint(0, 256, (n, 4, 84, 84), dtype=torch.uint8, device=dev)
    got = conv1_u8(x, conv, 255.0)
    assert got.shape == (n, 32, 20, 20) and got.is_contiguous(memory_format=torch.channels_last)
    w64, b64 = conv.weight.double(), conv.bias.double()
    x64 = x.double() / 255.0
    ref = torch.relu(torch.nn.functional.conv2d(x64, w64, b64, 4))
    mag = torch.nn.functional.conv2d(x64, w64.abs(), b64.abs(), 4)
    err = (got.double() - ref).abs()
    assert bool((err <= 1e-6 * mag + 1e-12).all()), float((err / (mag + 1e-30)).max())
    xf = net._scale_lut(dev)[x.long()]
    tref = torch.relu(torch.nn.functional.conv2d(xf, conv.weight, conv.bias, 4)).double()
    rms = lambda e: float(e.pow(2).mean().sqrt())  # noqa: E731
    assert rms(err) <= 2 * rms(tref - ref) + 1e-9, (rms(err), rms(tref - ref))


def test_dqn_fused_conv1_matches_miopen(dev):
    """The whole trunk with the uint8 first layer (forward: tsrl_dqn_conv1_fwd; backward:
    conv2's data gradient with conv1's ReLU mask from tsrl_dqn_conv2_dgrad, conv1's
    weight/bias gradient from the frames by tsrl_dqn_conv1_wgrad, MIOpen for the rest)
    against the same module on MIOpen throughout: outputs and every parameter gradient."""
    from tianshou_amd.utils.net_atari import DQN, layer_init
    torch.manual_seed(1)
    a = DQN(4, 84, 84, (6,), device=dev, features_only=True, output_dim=512,
            layer_init=layer_init).to(dev)
    x = torch.randint(0, 256, (96, 4, 84, 84), dtype=torch.uint8, device=dev)
    outs = []
    for fused in (True, False):
        a.fused_conv1 = fused
        a.zero_grad(set_to_none=True)
        y = a(x)[0]
        g = torch.randn(y.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(2))
        y.backward(g)
        outs.append((y.detach(), [p.grad.clone() for p in a.parameters()]))
    (ya, ga), (yb, gb) = outs
    torch.testing.assert_close(ya, yb, rtol=1e-4, atol=1e-5 * float(yb.abs().max()))
    for pa, pb in zip(ga, gb):
        torch.testing.assert_close(pa, pb, rtol=1e-3, atol=1e-4 * float(pb.abs().max()))


def test_dqn_relu_bwd_fused_path_taken(dev, monkeypatch):
    """The production trunk's conv2 and conv3 ReLU backward + bias gradient go through
    tsrl_relu_bwd_rows (one call each, NHWC rows n*81 and n*49 of 64 channels), and the result
    matches threshold_backward + the library bias gradient: outputs bit-identical, every
    gradient within f32 summation error (the same gy; the library's split-K weight gradients
    and the bias sums add in another order)."""
    from tianshou_amd import _C
    from tianshou_amd.utils import net_atari
    torch.manual_seed(3)
    a = net_atari.DQN(4, 84, 84, (6,), device=dev, features_only=True, output_dim=512,
                      layer_init=net_atari.layer_init).to(dev)
    x = torch.randint(0, 256, (96, 4, 84, 84), dtype=torch.uint8, device=dev)
    lib = _C.lib()
    real = lib.tsrl_relu_bwd_rows
    calls = []

    def spy(*args):
        calls.append((args[3], args[4]))
        return real(*args)

    monkeypatch.setattr(lib, "tsrl_relu_bwd_rows", spy)
    outs = []
    for fused in (True, False):
        monkeypatch.setattr(net_atari, "RELU_BWD_FUSED", fused)
        a.zero_grad(set_to_none=True)
        y = a(x)[0]
        g = torch.randn(y.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(4))
        y.backward(g)
        outs.append((y.detach(), [(n_, p.grad.clone()) for n_, p in a.named_parameters()]))
    assert sorted(calls) == [(96 * 49, 64), (96 * 81, 64)]
    (ya, ga), (yb, gb) = outs
    assert torch.equal(ya, yb)
    for (name, pa), (_, pb) in zip(ga, gb):
        torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-6 * float(pb.abs().max()),
                                   msg=name)


def test_dqn_conv1_only_path_matches_miopen(dev):
    """A trunk whose second convolution is not the Nature-DQN one (here grouped) takes the
    conv1-only autograd path (_Conv1U8: tsrl_dqn_conv1_fwd forward, ReLU mask +
    tsrl_dqn_conv1_wgrad backward): outputs and every parameter gradient against the same
    module on MIOpen throughout."""
    from torch import nn
    from tianshou_amd.utils.net_atari import DQN, layer_init
    torch.manual_seed(3)
    a = DQN(4, 84, 84, (6,), device=dev, features_only=True, output_dim=512,
            layer_init=layer_init).to(dev)
    a.net[0][2] = layer_init(nn.Conv2d(32, 64, 4, stride=2, groups=2)).to(dev).to(
        memory_format=torch.channels_last)
    a._conv1_split = None
    parts = a._conv1_parts()
    assert parts is not None and parts[1] is None  # conv1 only
    x = torch.randint(0, 256, (48, 4, 84, 84), dtype=torch.uint8, device=dev)
    outs = []
    for fused in (True, False):
        a.fused_conv1 = fused
        a.zero_grad(set_to_none=True)
        y = a(x)[0]
        g = torch.randn(y.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(4))
        y.backward(g)
        outs.append((y.detach(), [p.grad.clone() for p in a.parameters()]))
    (ya, ga), (yb, gb) = outs
    torch.testing.assert_close(ya, yb, rtol=1e-4, atol=1e-5 * float(yb.abs().max()))
    for pa, pb in zip(ga, gb):
        torch.testing.assert_close(pa, pb, rtol=1e-3, atol=1e-4 * float(pb.abs().max()))


def test_atari_shared_trunk_process_fn_wrapped_ring(dev):
    """As above on a ring that has wrapped (collect more steps than the buffer holds): the
    stacked obs / obs_next rows equal the env's FrameStack stream (oracle/synth_env.py) where
    the stack lies inside the retained window, next() positions equal the host next(), and
    process_fn's returns/advantages equal the GAE on the critic's V(obs) / V(obs_next).  On a
    random-index sample with duplicate indices, next() reuse either declines (None) or points
    at rows whose V(s) equals the critic on the batch's obs_next."""
    from tianshou_amd.policy.base import gae_device
    E, T, L, X = 6, 16, 7, 5
    _, policy, buf, coll = _setup(dev, E, T, L, seed=5)
    policy._rew_norm = False
    coll.collect(n_step=E * (T + X))  # X steps past the end of every sub-buffer
    ref = synth_env.SynthVecEnvNP(E, (4, 84, 84), 6, L, seed=3, u8=True, frame_stack=4)
    cur = ref.reset()
    seen = np.zeros((E, T + X, 4, 84, 84), np.uint8)
    dones = np.zeros((E, T + X), bool)
    for t in range(T + X):
        seen[:, t] = cur
        nxt, _, term, trunc = ref.step()
        done = term | trunc
        dones[:, t] = done
        if done.any():
            ids = np.flatnonzero(done)
            nxt[ids] = ref.reset(ids)
        cur = nxt
    seen, dones = seen[:, X:], dones[:, X:]  # the retained window, oldest first
    batch, idx = buf.sample(0)
    assert not np.array_equal(idx, np.arange(E * T))  # ring order, not storage order
    obs = batch.obs.cpu().numpy().reshape(E, T, 4, 84, 84)
    on = batch.obs_next.cpu().numpy().reshape(E, T, 4, 84, 84)
    # rows t >= 3 of the window: their frame stack never reaches past the oldest stored row
    assert np.array_equal(obs[:, 3:], seen[:, 3:])
    inner = ~dones[:, 3:-1]
    assert np.array_equal(on[:, 3:-1][inner], seen[:, 4:][inner])
    assert np.array_equal(on[:, 3:-1][~inner], seen[:, 3:-1][~inner])
    assert np.array_equal(on[:, -1], seen[:, -1])  # the newest row: its own observation
    p = policy._next_positions(buf, idx, dev)
    assert p is not None
    assert np.array_equal(idx[p.cpu().numpy()], buf.next(idx))
    with torch.no_grad():
        v_ref = policy.critic(batch.obs).flatten()
        vn_ref = policy.critic(batch.obs_next).flatten()
    out = policy.process_fn(batch, buf, idx)
    vmax = float(v_ref.abs().max())
    np.testing.assert_allclose(out.v_s.cpu().numpy(), v_ref.cpu().numpy(), rtol=1e-5,
                               atol=1e-5 * vmax)
    adv, ret, _, _ = gae_device(v_ref.contiguous(), vn_ref.contiguous(),
                                batch.rew.contiguous(), batch.terminated.contiguous(),
                                batch.truncated.contiguous(), 0.99, 0.95, T)
    np.testing.assert_allclose(out.adv.cpu().numpy(), adv.cpu().numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(out.returns.cpu().numpy(), ret.cpu().numpy(), rtol=1e-5,
                               atol=1e-5)
    # random-index sample with duplicates
    np.random.seed(11)
    _, ridx = buf.sample(40)
    ridx = np.concatenate([ridx, ridx[:8], idx[:4]])
    rb = buf[ridx]
    pr = policy._next_positions(buf, ridx, dev)
    with torch.no_grad():
        v = policy.critic(rb.obs).flatten()
        vn = policy.critic(rb.obs_next).flatten()
    if pr is not None:
        assert np.array_equal(ridx[pr.cpu().numpy()], buf.next(ridx))
        np.testing.assert_allclose(v[pr].cpu().numpy(), vn.cpu().numpy(), rtol=1e-5,
                                   atol=1e-5 * float(vn.abs().max()))


def test_gumbel_categorical_sample_distribution(dev):
    """gumbel_sample (tsrl_cat_gumbel_argmax) draws from Categorical(logits): empirical
    frequencies of 200k draws per row within 5 standard errors of softmax(logits), -inf
    logits never drawn, and the stream follows torch.manual_seed (reproducible)."""
    from tianshou_amd.policy.pg import gumbel_sample
    logits = torch.tensor([[0.0, 1.0, -1.0, 2.0, 0.5, -3.0],
                           [5.0, 5.0, 5.0, 5.0, 5.0, 5.0],
                           [0.0, float("-inf"), 1.0, float("-inf"), -2.0, 0.0]], device=dev)
    lg = torch.distributions.Categorical(logits=logits).logits
    m = 200000
    rep = lg.repeat(m, 1)
    torch.manual_seed(0)
    a = gumbel_sample(rep).view(m, 3)
    p = torch.softmax(logits, -1).double()
    for r in range(3):
        f = torch.bincount(a[:, r], minlength=6).double() / m
        se = (p[r] * (1 - p[r]) / m).sqrt()
        assert bool(((f - p[r]).abs() <= 5 * se + 1e-12).all()), (r, f, p[r])
    assert not bool(((a[:, 2] == 1) | (a[:, 2] == 3)).any())
    torch.manual_seed(0)
    assert torch.equal(gumbel_sample(rep).view(m, 3), a)


@pytest.mark.parametrize("n,rows_n", [(300, 257), (64, 64)])
def test_dqn_rows_in_place_matches_gathered(dev, n, rows_n):
    """DQN.forward(obs, rows=idx) -- the uint8 first-layer kernels reading the minibatch's
    frame stacks in place from the whole batch (tsrl_dqn_conv1_fwd / tsrl_dqn_conv1_wgrad with
    rows) -- against forward(obs[idx]) on the gathered copy: outputs and conv1's weight and
    bias gradients bit for bit (the same bytes reach the same kernels); the other gradients
    come from MIOpen / hipBLASLt, whose split-K weight gradients accumulate with atomics in a
    run-dependent order, so they are compared at rtol 1e-5 of their magnitude."""
    import copy
    from tianshou_amd.utils.net_atari import DQN, layer_init
    torch.manual_seed(7)
    net = DQN(4, 84, 84, (6,), device=dev, features_only=True, output_dim=512,
              layer_init=layer_init).to(dev)
    net2 = copy.deepcopy(net)
    g = torch.Generator(device=dev).manual_seed(n)
    obs = torch.randint(0, 256, (n, 4, 84, 84), dtype=torch.uint8, device=dev, generator=g)
    idx = torch.randint(0, n, (rows_n,), device=dev, generator=g)
    assert net.reads_rows(obs)
    y1, _ = net(obs, rows=idx)
    y2, _ = net2(obs[idx])
    gy = torch.randn(y1.shape, device=dev, generator=g)
    y1.backward(gy)
    y2.backward(gy)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
    conv1 = {n_ for n_, p in net.named_parameters() if p is net._conv1_parts()[0].weight or
             p is net._conv1_parts()[0].bias}
    assert len(conv1) == 2
    for (k, p1), (_, p2) in zip(net.named_parameters(), net2.named_parameters()):
        if k in conv1:
            assert torch.equal(p1.grad, p2.grad), k
        else:
            err = float((p1.grad - p2.grad).abs().max())
            assert err <= 1e-5 * float(p2.grad.abs().max()) + 1e-12, (k, err)


def test_dqn_fused_trunk_grads_accumulate(dev):
    """The fused trunk's gradients against the plain NCHW module over two backward passes:
    the first assigns every .grad, the second accumulates -- the Flatten + Linear weight
    gradient then goes straight into the existing .grad through its permuted view (round 6),
    and the bias gradient is the HIP column sum -- then a third behind FlatAdam's
    release_grads / gather_grads (the weight gradient written into its flat slot).
    Summation order only (rtol 1e-3)."""
    from tianshou_amd.utils import net_atari
    from tianshou_amd.utils.net_atari import DQN, layer_init
    torch.manual_seed(0)
    a = DQN(4, 84, 84, (6,), device=dev, features_only=True, output_dim=512,
            layer_init=layer_init).to(dev)
    torch.manual_seed(0)
    b = DQN(4, 84, 84, (6,), device=dev, features_only=True, output_dim=512,
            layer_init=layer_init, channels_last=False).to(dev)
    b.fused_conv1 = False
    taken = []
    orig = net_atari._FlattenLinear._grad_slot

    def spy(*args):
        s = orig(*args)
        taken.append((s[0] is not None, s[1]))
        return s

    def step(seed):
        g = torch.Generator(device=dev).manual_seed(seed)
        x = torch.randint(0, 256, (64, 4, 84, 84), dtype=torch.uint8, device=dev, generator=g)
        ya, yb = a(x)[0], b(x)[0]
        gy = torch.randn(ya.shape, device=dev, generator=g)
        ya.backward(gy)
        yb.backward(gy)

    def check():
        for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
            torch.testing.assert_close(pa.grad, pb.grad, rtol=1e-3,
                                       atol=1e-4 * float(pb.grad.abs().max()), msg=n)
    net_atari._FlattenLinear._grad_slot = staticmethod(spy)
    try:
        step(1)
        step(2)
        check()
        # FlatAdam's hand-over (release_grads / gather_grads): the Flatten + Linear weight
        # gradient is written into its published flat slot
        from tianshou_amd.policy.flat_adam import FlatAdam
        fa = FlatAdam(a.parameters())
        fa.release_grads()
        b.zero_grad()
        step(3)
        fa.gather_grads()
        assert all(p.grad.data_ptr() == v.data_ptr() for p, v in zip(fa.params, fa._views))
        check()
    finally:
        net_atari._FlattenLinear._grad_slot = staticmethod(orig)
    assert taken == [(False, False), (True, False), (True, True)]
