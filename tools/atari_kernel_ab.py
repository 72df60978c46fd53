"""A/B helper for the config-5 HIP trunk kernels (diagnostic, not a test): times
tsrl_dqn_conv1_fwd / tsrl_dqn_conv2_dgrad / tsrl_dqn_conv1_wgrad at --rows samples (HIP events,
--iters launches) and saves their outputs on seeded inputs to --save (a .pt of tensors), so two
library builds (TSRL_LIB_PATH) can be compared bit for bit with --compare A.pt B.pt.

python tools/atari_kernel_ab.py [--rows 8192] [--iters 20] [--save out.pt]
python tools/atari_kernel_ab.py --compare a.pt b.pt"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tianshou-fork_amd")]


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--save", default=None)
    ap.add_argument("--compare", nargs=2, default=None)
    a = ap.parse_args()
    if a.compare:
        x, y = (torch.load(p, weights_only=True) for p in a.compare)
        bad = 0
        for k in x:
            same = torch.equal(x[k], y[k])
            d = (x[k].double() - y[k].double()).abs()
            rel = float((d / x[k].double().abs().clamp_min(1e-30)).max())
            print(f"{k}: bit-identical {same} (max |diff| {float(d.max()):.3e}, "
                  f"max rel {rel:.3e}, differing {int((d > 0).sum())} of {d.numel()})")
            bad += not same
        sys.exit(1 if bad else 0)
    from tianshou_amd import _C
    from tianshou_amd.utils.net_atari import conv1_u8_wgrad
    dev = torch.device("cuda", 0)
    N = a.rows
    g = torch.Generator(device=dev).manual_seed(5)
    cl = torch.channels_last
    w1 = torch.randn(32, 4, 8, 8, device=dev, generator=g).contiguous(memory_format=cl)
    b1 = torch.randn(32, device=dev, generator=g)
    u8 = torch.randint(0, 256, (N, 4, 84, 84), dtype=torch.uint8, device=dev, generator=g)
    out1 = torch.empty(N, 20, 20, 32, device=dev)
    s_ = _C.stream_ptr(dev)
    lib = _C.lib()
    f1 = lambda: lib.tsrl_dqn_conv1_fwd(_C.ptr(u8), N, None, w1.data_ptr(), *w1.stride(),  # noqa
                                        _C.ptr(b1), 255.0, 1, _C.ptr(out1), s_)
    t1 = timed(f1, a.iters)
    flop1 = 2.0 * N * 400 * 32 * 256
    print(f"conv1 fwd     {t1 * 1e3:8.1f} us  {flop1 / t1 / 1e9:6.1f} TFLOP/s f32-equivalent",
          flush=True)
    w2 = torch.randn(64, 32, 4, 4, device=dev, generator=g).contiguous(memory_format=cl)
    gy2 = torch.randn(N, 9, 9, 64, device=dev, generator=g)
    z1 = torch.relu(torch.randn(N, 20, 20, 32, device=dev, generator=g))
    dx = torch.empty(N, 20, 20, 32, device=dev)
    f2 = lambda: lib.tsrl_dqn_conv2_dgrad(_C.ptr(gy2), N, w2.data_ptr(), *w2.stride(),  # noqa
                                          _C.ptr(z1), _C.ptr(dx), s_)
    t2 = timed(f2, a.iters)
    flop2 = 2.0 * N * 81 * 64 * 32 * 16
    print(f"conv2 dgrad   {t2 * 1e3:8.1f} us  {flop2 / t2 / 1e9:6.1f} TFLOP/s f32-equivalent",
          flush=True)
    gy1 = torch.randn(N, 20, 20, 32, device=dev, generator=g)
    res = {}
    f3 = lambda: res.__setitem__("w", conv1_u8_wgrad(u8, gy1, w1, 255.0, True))  # noqa: E731
    t3 = timed(f3, a.iters)
    print(f"conv1 wgrad   {t3 * 1e3:8.1f} us  {flop1 / t3 / 1e9:6.1f} TFLOP/s f32-equivalent",
          flush=True)
    torch.cuda.synchronize()
    if a.save:
        gw, gb = res["w"]
        torch.save({"conv1_fwd": out1.cpu(), "conv2_dgrad": dx.cpu(), "conv1_wgrad_w": gw.cpu(),
                    "conv1_wgrad_b": gb.cpu()}, a.save)


if __name__ == "__main__":
    main()
