"""Time the fused MLP kernels of one PPO minibatch at the benchmark shape (262144 rows,
Box(376)/Box(17), 64-64 tanh nets) with HIP events, and report achieved f32 MFMA TFLOP/s.

    python tools/mlp_kernel_bench.py [--rows 262144] [--D 376] [--A 17] [--iters 20] [--only NAME]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tianshou-fork_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=262144)
    ap.add_argument("--N", type=int, default=4096 * 2048)
    ap.add_argument("--D", type=int, default=376)
    ap.add_argument("--A", type=int, default=17)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default=None,
                    help="time one kernel only (l1_fwd, l1_fwd_x6, tail, dw, minibatch): PMC passes")
    ap.add_argument("--act", type=int, default=1, help="layer-1 activation: 1 tanh, 0 identity")
    ap.add_argument("--ld", type=int, default=0,
                    help="row pitch of the observation array in floats (0: D; e.g. 384 = "
                         "128-byte-aligned rows)")
    ap.add_argument("--contig", action="store_true",
                    help="minibatch rows contiguous (no permutation gather)")
    ap.add_argument("--sorted", action="store_true",
                    help="random minibatch rows, gathered in ascending row order")
    ap.add_argument("--eval-chunk", type=int, default=0,
                    help="rows per process_fn evaluation chunk (FusedActorCritic.EVAL_CHUNK)")
    a = ap.parse_args()
    from tianshou_amd import _C
    from tianshou_amd.dist import DataParallel
    from tianshou_amd.policy import fused_mlp
    from tianshou_amd.utils.models import get_actor_critic, init_actor_critic
    from tianshou_amd.utils.net import ActorCritic
    dev = torch.device("cuda", 0)
    actor, critic = get_actor_critic((a.D,), (64, 64), (a.A,), dev)
    actor, critic = actor.to(dev), critic.to(dev)
    init_actor_critic(actor, critic)
    layers = fused_mlp.match(actor, critic)
    fm = fused_mlp.FusedActorCritic(layers, ActorCritic(actor, critic).parameters())
    if a.eval_chunk:
        fm.EVAL_CHUNK = a.eval_chunk
    N, B, D, A = a.N, a.rows, a.D, a.A
    ld = a.ld or D
    obs = torch.randn(N, ld, device=dev)
    act = torch.randn(N, A, device=dev)
    logp_old = torch.randn(N, device=dev) - A
    adv = torch.randn(N, device=dev)
    ret = torch.randn(N, device=dev)
    v_s = torch.randn(N, device=dev)
    idx = None if a.contig else torch.randperm(N, device=dev)[:B]
    if a.sorted:
        idx = idx.sort().values
    p = _C.PPOParams()
    p.eps_clip, p.dual_clip, p.vf_coef, p.ent_coef, p.adv_eps = 0.2, 0.0, 0.25, 0.0, 1e-8
    p.b_global, p.value_clip, p.norm_adv = float(B), 0, 1
    dp = DataParallel()
    obs_v = obs[:, :D]  # the padded-storage view when ld > D (rows read in place)
    fm.minibatch(obs_v, idx, B, act, logp_old, adv, ret, v_s, p, dp)
    torch.cuda.synchronize()
    L = _C.lib()
    s = _C.stream_ptr(dev)
    h1 = fm._bufs["h1"]
    dz1 = fm._bufs["dz1"]
    W = layers
    flop_l1 = 2.0 * B * D * 128
    flop_tail = 2.0 * B * (64 * 64 * 2 * 3 + 64 * 32 * 3 + 64 * 2)
    sums = fm._bufs["sums"]
    ws = fm._bufs["tail_ws"]
    ws2 = fm._bufs["dw_ws"]
    adv_sums = fm._bufs["adv_sums"]

    def l1():
        _C.check(L.tsrl_mlp_l1_fwd(_C.ptr(obs), D, _C.ptr(idx), B, D, _C.ptr(W["w1a"].weight),
                                   _C.ptr(W["w1a"].bias), _C.ptr(W["w1c"].weight),
                                   _C.ptr(W["w1c"].bias), 1, _C.ptr(h1), 1, s))

    wsx = torch.empty((int(L.tsrl_mlp_split_bytes(D)) + 3) // 4, device=dev)

    def l1x6():
        _C.check(L.tsrl_mlp_split_w(_C.ptr(W["w1a"].weight), _C.ptr(W["w1c"].weight), D,
                                    _C.ptr(wsx), s))
        _C.check(L.tsrl_mlp_l1_fwd_x6(_C.ptr(obs), ld, _C.ptr(idx), B, D, _C.ptr(wsx),
                                      _C.ptr(W["w1a"].bias), _C.ptr(W["w1c"].bias), a.act,
                                      _C.ptr(h1), 1, s))

    rows_out = torch.empty(B, 128, device=dev)

    def l1x6_staged():  # the register-staged kernel (row-major output path)
        _C.check(L.tsrl_mlp_l1_fwd_x6(_C.ptr(obs), D, _C.ptr(idx), B, D, _C.ptr(wsx),
                                      _C.ptr(W["w1a"].bias), _C.ptr(W["w1c"].bias), 1,
                                      _C.ptr(rows_out), 0, s))

    def tail():
        _C.check(L.tsrl_ppo_tail(_C.ptr(h1), B, _C.ptr(idx), fm._tail_w, A, _C.ptr(act),
                                 _C.ptr(logp_old), _C.ptr(adv), _C.ptr(ret), _C.ptr(v_s),
                                 _C.ptr(adv_sums), p, _C.ptr(dz1), fm._tail_grads,
                                 _C.ptr(sums), _C.ptr(ws), ws.numel(), s))

    def dw():
        _C.check(L.tsrl_mlp_dw(_C.ptr(dz1), _C.ptr(obs), ld, _C.ptr(idx), B, D,
                               _C.ptr(W["w1a"].weight.grad), _C.ptr(W["w1a"].bias.grad),
                               _C.ptr(W["w1c"].weight.grad), _C.ptr(W["w1c"].bias.grad),
                               _C.ptr(ws2), ws2.numel(), s))

    def whole():
        fm.minibatch(obs_v, idx, B, act, logp_old, adv, ret, v_s, p, dp)

    EV = min(N, 1 << 21)
    flop_eval = 2.0 * EV * (D * 128 + 64 * 64 * 2 + 64 * (A + 1))

    def evaluate():  # process_fn: V(s) + logp_old of one 2M-row chunk (l1 + eval tail)
        fm.evaluate(obs_v[:EV], act[:EV])

    for name, fn, flop in (("l1_fwd", l1, flop_l1), ("l1_fwd_x6(+split)", l1x6, flop_l1),
                           ("l1_x6_staged(rows)", l1x6_staged, flop_l1),
                           ("tail(+reduce)", tail, flop_tail),
                           ("dw(+reduce)", dw, flop_l1), ("minibatch", whole, None),
                           ("eval(2M rows)", evaluate, flop_eval)):
        if a.only and not name.startswith(a.only):
            continue
        if ld != D and name in ("l1_fwd", "l1_x6_staged(rows)"):
            continue
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        tf = f"  {flop / us / 1e6:7.1f} TFLOP/s" if flop else ""
        print(f"{name:16s} {us:9.1f} us{tf}", flush=True)


if __name__ == "__main__":
    main()
