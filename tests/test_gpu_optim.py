"""tsrl_clip_adam (csrc/optim.hip) vs torch.nn.utils.clip_grad_norm_ + torch.optim.Adam on
the get_actor_critic parameters: 6 steps of random gradients (some clipped, some not), flat
storage bound through FusedActorCritic.bind_adam.  Tolerance rtol 1e-5 / atol 1e-7 (the
norm is summed in f64 here, in f32 partial norms by torch)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("max_norm", [0.5, None, 1e3])
def test_clip_adam_matches_torch(max_norm):
    from tianshou_amd.policy import fused_mlp
    from tianshou_amd.utils.models import get_actor_critic, init_actor_critic
    from tianshou_amd.utils.net import ActorCritic
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    nets = []
    for _ in range(2):
        a, c = get_actor_critic((24,), (64, 64), (5,), dev)
        a, c = a.to(dev), c.to(dev)
        nets.append((a, c))
    init_actor_critic(*nets[0])
    ac0, ac1 = ActorCritic(*nets[0]), ActorCritic(*nets[1])
    ac1.load_state_dict(ac0.state_dict())
    opt_ref = torch.optim.Adam(ac0.parameters(), lr=3e-4)
    opt = torch.optim.Adam(ac1.parameters(), lr=3e-4)
    fm = fused_mlp.FusedActorCritic(fused_mlp.match(*nets[1]), ac1.parameters())
    assert fm.bind_adam(opt) and fm.adam_bound(opt)
    g = torch.Generator(device=dev).manual_seed(1)
    for step in range(6):
        scale = 10.0 ** (step % 3 - 1)
        grads = [torch.randn(p.shape, device=dev, generator=g) * scale for p in ac0.parameters()]
        for p, gr in zip(ac0.parameters(), grads):
            p.grad = gr.clone()
        if max_norm:
            torch.nn.utils.clip_grad_norm_(ac0.parameters(), max_norm=max_norm)
        opt_ref.step()
        fm.bind_grads()
        for p, gr in zip(ac1.parameters(), grads):
            p.grad.copy_(gr)
        fm.clip_adam(max_norm)
        torch.cuda.synchronize()
        for (n0, p0), p1 in zip(ac0.named_parameters(), ac1.parameters()):
            np.testing.assert_allclose(p1.detach().cpu().numpy(), p0.detach().cpu().numpy(),
                                       rtol=1e-5, atol=1e-7, err_msg=f"step {step} {n0}")
            np.testing.assert_allclose(p1.grad.cpu().numpy(), p0.grad.cpu().numpy(), rtol=1e-5,
                                       atol=1e-9, err_msg=f"grad step {step} {n0}")
    for p0, p1 in zip(ac0.parameters(), ac1.parameters()):
        s0, s1 = opt_ref.state[p0], opt.state[p1]
        assert float(s1["step"]) == float(s0["step"]) == 6.0
        np.testing.assert_allclose(s1["exp_avg_sq"].cpu().numpy(), s0["exp_avg_sq"].cpu().numpy(),
                                   rtol=5e-5, atol=1e-12)
    # the state dict round-trips through torch
    sd = opt.state_dict()
    assert len(sd["state"]) == len(list(ac1.parameters()))


@pytest.mark.parametrize("max_norm", [0.5, None])
def test_clip_adam_nan_gradient_matches_torch(max_norm):
    """A NaN gradient element (what an invalid mu / sigma produces with validate_args=False,
    DESIGN.md section 7) takes the flat Adam state exactly where torch's takes it: with
    clipping the NaN norm reaches every gradient and every parameter (clip_grad_norm_'s
    clamp keeps the NaN), without clipping only that element's parameter, moments and later
    updates; finite elements stay equal to torch, the step counter advances the same way and
    the flat storage still backs the parameters afterwards."""
    from tianshou_amd.policy import fused_mlp
    from tianshou_amd.utils.models import get_actor_critic, init_actor_critic
    from tianshou_amd.utils.net import ActorCritic
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    nets = []
    for _ in range(2):
        a, c = get_actor_critic((24,), (64, 64), (5,), dev)
        nets.append((a.to(dev), c.to(dev)))
    init_actor_critic(*nets[0])
    ac0, ac1 = ActorCritic(*nets[0]), ActorCritic(*nets[1])
    ac1.load_state_dict(ac0.state_dict())
    opt_ref = torch.optim.Adam(ac0.parameters(), lr=3e-4)
    opt = torch.optim.Adam(ac1.parameters(), lr=3e-4)
    fm = fused_mlp.FusedActorCritic(fused_mlp.match(*nets[1]), ac1.parameters())
    assert fm.bind_adam(opt)
    g = torch.Generator(device=dev).manual_seed(2)
    for step in range(3):
        grads = [torch.randn(p.shape, device=dev, generator=g) for p in ac0.parameters()]
        if step == 1:
            grads[2].view(-1)[7] = float("nan")
        for p, gr in zip(ac0.parameters(), grads):
            p.grad = gr.clone()
        if max_norm:
            torch.nn.utils.clip_grad_norm_(ac0.parameters(), max_norm=max_norm)
        opt_ref.step()
        fm.bind_grads()
        for p, gr in zip(ac1.parameters(), grads):
            p.grad.copy_(gr)
        fm.clip_adam(max_norm)
        torch.cuda.synchronize()
        for (n0, p0), p1 in zip(ac0.named_parameters(), ac1.parameters()):
            x0, x1 = p0.detach().cpu().numpy(), p1.detach().cpu().numpy()
            np.testing.assert_array_equal(np.isnan(x1), np.isnan(x0), err_msg=f"{step} {n0}")
            np.testing.assert_allclose(x1[~np.isnan(x0)], x0[~np.isnan(x0)], rtol=1e-5,
                                       atol=1e-7, err_msg=f"step {step} {n0}")
    n_nan = sum(int(torch.isnan(p).sum()) for p in ac1.parameters())
    if max_norm:
        assert n_nan == sum(p.numel() for p in ac1.parameters())
    else:
        assert n_nan == 1
    for p0, p1 in zip(ac0.parameters(), ac1.parameters()):
        s0, s1 = opt_ref.state[p0], opt.state[p1]
        assert float(s1["step"]) == float(s0["step"]) == 3.0
        np.testing.assert_array_equal(torch.isnan(s1["exp_avg"]).cpu().numpy(),
                                      torch.isnan(s0["exp_avg"]).cpu().numpy())
    assert fm.adam_bound(opt)


@pytest.mark.parametrize("D", [376, 17, 24])
def test_clip_adam_split_epilogue_equals_split_w(D):
    """clip_adam(split_w1=True) leaves the bf16x6 planes of the UPDATED first-layer weights
    byte-identical to a fresh tsrl_mlp_split_w, and scale_grads=False leaves .grad
    unclipped while the parameter update is the same as with scaling."""
    from tianshou_amd import _C
    from tianshou_amd.policy import fused_mlp
    from tianshou_amd.utils.models import get_actor_critic, init_actor_critic
    from tianshou_amd.utils.net import ActorCritic
    dev = torch.device("cuda", 0)
    torch.manual_seed(3)
    a, c = get_actor_critic((D,), (64, 64), (6,), dev)
    a, c = a.to(dev), c.to(dev)
    init_actor_critic(a, c)
    ac = ActorCritic(a, c)
    opt = torch.optim.Adam(ac.parameters(), lr=1e-3)
    fm = fused_mlp.FusedActorCritic(fused_mlp.match(a, c), ac.parameters())
    assert fm.bind_adam(opt)
    g = torch.Generator(device=dev).manual_seed(5)
    L = _C.lib()
    nb = (int(L.tsrl_mlp_split_bytes(D)) + 3) // 4
    for step in range(3):
        fm.bind_grads()
        for p in ac.parameters():
            p.grad.copy_(torch.randn(p.shape, device=dev, generator=g) * 3.0)
        raw = [p.grad.clone() for p in ac.parameters()]
        fm.split_w1()
        fm.clip_adam(0.5, scale_grads=False, split_w1=True)
        torch.cuda.synchronize()
        got = fm._bufs["w1split"][:nb].clone()
        want = torch.empty(nb, dtype=torch.float32, device=dev)
        _C.check(L.tsrl_mlp_split_w(_C.ptr(fm.L["w1a"].weight), _C.ptr(fm.L["w1c"].weight), D,
                                    _C.ptr(want), _C.stream_ptr(dev)), "split")
        assert torch.equal(got.view(torch.int32), want.view(torch.int32)), f"step {step}"
        for p, r in zip(ac.parameters(), raw):
            assert torch.equal(p.grad, r)


def test_clip_adam_resumes_loaded_state():
    """optim.load_state_dict() on an optimiser whose storage the flat Adam pass owns: the
    loaded moments / step counts (not the flat buffers' later values) are what the next
    clip_adam continues from -- the same trajectory as torch Adam resumed from that state."""
    import copy
    from tianshou_amd.policy import fused_mlp
    from tianshou_amd.utils.models import get_actor_critic, init_actor_critic
    from tianshou_amd.utils.net import ActorCritic
    dev = torch.device("cuda", 0)
    torch.manual_seed(2)
    nets = []
    for _ in range(2):
        a, c = get_actor_critic((24,), (64, 64), (5,), dev)
        nets.append((a.to(dev), c.to(dev)))
    init_actor_critic(*nets[0])
    ac0, ac1 = ActorCritic(*nets[0]), ActorCritic(*nets[1])
    ac1.load_state_dict(ac0.state_dict())
    opt_ref = torch.optim.Adam(ac0.parameters(), lr=3e-4)
    opt = torch.optim.Adam(ac1.parameters(), lr=3e-4)
    fm = fused_mlp.FusedActorCritic(fused_mlp.match(*nets[1]), ac1.parameters())
    assert fm.bind_adam(opt)
    g = torch.Generator(device=dev).manual_seed(7)

    def grads():
        return [torch.randn(p.shape, device=dev, generator=g) for p in ac0.parameters()]

    def ref_step(gs):
        for p, gr in zip(ac0.parameters(), gs):
            p.grad = gr.clone()
        torch.nn.utils.clip_grad_norm_(ac0.parameters(), max_norm=0.5)
        opt_ref.step()

    def flat_step(gs):
        assert fm.adam_bound(opt)
        fm.bind_grads()
        for p, gr in zip(ac1.parameters(), gs):
            p.grad.copy_(gr)
        fm.clip_adam(0.5)

    for _ in range(3):
        gs = grads()
        ref_step(gs)
        flat_step(gs)
    torch.cuda.synchronize()
    saved_opt = copy.deepcopy(opt.state_dict())
    saved_par = copy.deepcopy(ac1.state_dict())
    for _ in range(2):  # steps the flat storage takes and then forgets
        flat_step(grads())
    ac1.load_state_dict(saved_par)
    opt.load_state_dict(saved_opt)
    assert fm.adam_bound(opt)  # re-binds the loaded state into the flat storage
    for p in ac1.parameters():
        assert opt.state[p]["exp_avg"].data_ptr() != 0
    for _ in range(3):
        gs = grads()
        ref_step(gs)
        flat_step(gs)
    torch.cuda.synchronize()
    for (n0, p0), p1 in zip(ac0.named_parameters(), ac1.parameters()):
        np.testing.assert_allclose(p1.detach().cpu().numpy(), p0.detach().cpu().numpy(),
                                   rtol=1e-5, atol=1e-7, err_msg=n0)
    for p0, p1 in zip(ac0.parameters(), ac1.parameters()):
        assert float(opt.state[p1]["step"]) == float(opt_ref.state[p0]["step"]) == 6.0


def test_flat_adam_refuses_mixed_step_counts():
    """A state dict where some parameters have Adam state and others none (per-parameter step
    counts differ): clip_adam applies ONE bias correction to every parameter, so the flat pass
    must not claim the optimiser (adam_bound / bind_adam False) -- torch's Adam then steps it,
    each parameter with its own count.  A uniform state dict still re-binds."""
    import copy
    from tianshou_amd.policy import fused_mlp
    from tianshou_amd.utils.models import get_actor_critic
    from tianshou_amd.utils.net import ActorCritic
    dev = torch.device("cuda", 0)
    torch.manual_seed(3)
    a, c = get_actor_critic((24,), (64, 64), (5,), dev)
    a, c = a.to(dev), c.to(dev)
    ac = ActorCritic(a, c)
    opt = torch.optim.Adam(ac.parameters(), lr=3e-4)
    fm = fused_mlp.FusedActorCritic(fused_mlp.match(a, c), ac.parameters())
    assert fm.bind_adam(opt)
    fm.bind_grads()
    for p in ac.parameters():
        p.grad.copy_(torch.randn_like(p))
    fm.clip_adam(0.5)
    torch.cuda.synchronize()
    full = copy.deepcopy(opt.state_dict())
    partial = copy.deepcopy(full)
    first = sorted(partial["state"])[0]
    del partial["state"][first]  # parameter 0 loses its state: step 0 vs 1 elsewhere
    opt.load_state_dict(partial)
    assert not fm.adam_bound(opt)
    assert not fm.bind_adam(opt)
    # torch's own Adam continues: parameter 0 from step 0, the others from step 1
    for p in ac.parameters():
        p.grad = torch.randn_like(p)
    opt.step()
    steps = [float(opt.state[p]["step"]) for p in ac.parameters()]
    assert steps[0] == 1.0 and all(s == 2.0 for s in steps[1:])
    # a uniform state dict binds again
    opt.load_state_dict(full)
    assert fm.bind_adam(opt)


def test_flat_adam_keeps_channels_last_conv_weights():
    """FlatAdam's flat slots keep each parameter's memory format (round 6): a channels_last
    conv weight stays channels_last as a parameter, as a .grad slot and in the Adam moments
    (MIOpen would otherwise copy it to the input's format on every convolution, and autograd
    would accumulate its channels_last gradient with a strided add).  Convolution backward
    into the slots + clip_adam over 4 steps = torch's clip_grad_norm_ + Adam on a twin;
    a loaded optimiser state re-binds into the same formats."""
    import copy
    from tianshou_amd.policy.flat_adam import FlatAdam
    dev = torch.device("cuda", 0)
    cl = torch.channels_last
    torch.manual_seed(4)

    def make():
        return torch.nn.Sequential(torch.nn.Conv2d(4, 8, 3, stride=2), torch.nn.ReLU(),
                                   torch.nn.Conv2d(8, 8, 3), torch.nn.Flatten(),
                                   torch.nn.Linear(8 * 4 * 4, 3)).to(dev).to(memory_format=cl)
    m0 = make()
    m1 = copy.deepcopy(m0)
    opt_ref = torch.optim.Adam(m0.parameters(), lr=1e-3)
    opt = torch.optim.Adam(m1.parameters(), lr=1e-3)
    fa = FlatAdam(m1.parameters())
    assert fa.bind_adam(opt) and fa.adam_bound(opt)
    for p0, p1 in zip(m0.parameters(), m1.parameters()):
        assert p1.stride() == p0.stride(), "memory format lost"
        assert torch.equal(p1.detach(), p0.detach())
        assert opt.state[p1]["exp_avg"].stride() == p0.stride()
    g = torch.Generator(device=dev).manual_seed(5)
    for step in range(4):
        x = torch.randn(16, 4, 13, 13, device=dev, generator=g).contiguous(memory_format=cl)
        opt_ref.zero_grad()
        m0(x).square().sum().backward()
        torch.nn.utils.clip_grad_norm_(m0.parameters(), max_norm=0.5)
        opt_ref.step()
        fa.zero_grad()
        m1(x).square().sum().backward()
        for p0, p1 in zip(m0.parameters(), m1.parameters()):
            assert p1.grad.stride() == p0.stride()
        fa.clip_adam(0.5)
        torch.cuda.synchronize()
        for (n0, p0), p1 in zip(m0.named_parameters(), m1.parameters()):
            np.testing.assert_allclose(p1.detach().cpu().numpy(), p0.detach().cpu().numpy(),
                                       rtol=1e-5, atol=1e-7, err_msg=f"step {step} {n0}")
    # a loaded state dict re-binds into the same (channels_last) slots
    sd = copy.deepcopy(opt.state_dict())
    opt.load_state_dict(sd)
    assert fa.bind_adam(opt)
    for p0, p1 in zip(m0.parameters(), m1.parameters()):
        assert opt.state[p1]["exp_avg_sq"].stride() == p0.stride()
        np.testing.assert_allclose(opt.state[p1]["exp_avg_sq"].cpu().numpy(),
                                   opt_ref.state[p0]["exp_avg_sq"].cpu().numpy(),
                                   rtol=5e-5, atol=1e-12)


def test_flat_adam_release_gather_grads():
    """release_grads() + backward + gather_grads() (the eager Categorical minibatch, round 6)
    leaves the same flat bucket as zero_grad() + backward: every gradient in its slot, a
    parameter that received no gradient zeroed, every .grad the slot view again."""
    from tianshou_amd.policy.flat_adam import FlatAdam
    dev = torch.device("cuda", 0)
    cl = torch.channels_last
    torch.manual_seed(6)
    m = torch.nn.Sequential(torch.nn.Conv2d(4, 8, 3, stride=2), torch.nn.ReLU(),
                            torch.nn.Flatten(), torch.nn.Linear(8 * 6 * 6, 3)).to(dev)
    m = m.to(memory_format=cl)
    unused = torch.nn.Parameter(torch.randn(5, device=dev))
    params = list(m.parameters()) + [unused]
    fa = FlatAdam(params)
    x = torch.randn(16, 4, 13, 13, device=dev).contiguous(memory_format=cl)
    fa.zero_grad()
    m(x).square().sum().backward()
    want = fa.flat_grad.clone()
    ptrs = [p.grad.data_ptr() for p in params]
    # stale values in the bucket must not leak into the gathered gradients
    fa.flat_grad.fill_(7.0)
    fa.release_grads()
    assert all(p.grad is None for p in params)
    m(x).square().sum().backward()
    fa.gather_grads()
    assert [p.grad.data_ptr() for p in params] == ptrs
    # (MIOpen's weight gradient may sum in another order run to run)
    torch.testing.assert_close(fa.flat_grad, want, rtol=1e-5,
                               atol=1e-6 * float(want.abs().max()))
    assert torch.count_nonzero(unused.grad) == 0
