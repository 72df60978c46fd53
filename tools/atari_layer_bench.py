"""Per-layer timing of the config-5 Nature-DQN trunk on MI355X (diagnostic, not a test):
every convolution's forward, data gradient and weight gradient (MIOpen, channels_last f32,
the layers of examples/atari/atari_network.py:53-90), the bias / ReLU elementwise passes
around them, and the two linear layers, for one PPO minibatch (default 8192 rows).
Reports ms and the f32 TFLOP/s of each GEMM-shaped op.

python tools/atari_layer_bench.py [--rows 8192] [--iters 10]"""
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
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    N = a.rows
    cl = torch.channels_last
    layers = [(4, 32, 8, 4, 84), (32, 64, 4, 2, 20), (64, 64, 3, 1, 9)]
    total = 0.0
    for cin, cout, k, s, hw in layers:
        ho = (hw - k) // s + 1
        x = torch.randn(N, cin, hw, hw, device=dev).contiguous(memory_format=cl)
        w = torch.randn(cout, cin, k, k, device=dev).contiguous(memory_format=cl)
        b = torch.randn(cout, device=dev)
        y = torch.nn.functional.conv2d(x, w, None, s)
        gy = torch.randn_like(y)
        flop = 2.0 * N * ho * ho * cout * cin * k * k
        res = {}
        res["fwd"] = timed(lambda: torch.nn.functional.conv2d(x, w, None, s), a.iters)
        res["fwd+bias"] = timed(lambda: torch.nn.functional.conv2d(x, w, b, s), a.iters)
        res["dgrad"] = timed(lambda: torch.ops.aten.convolution_backward(
            gy, x, w, None, (s, s), (0, 0), (1, 1), False, (0, 0), 1, (True, False, False)),
            a.iters)
        res["wgrad"] = timed(lambda: torch.ops.aten.convolution_backward(
            gy, x, w, None, (s, s), (0, 0), (1, 1), False, (0, 0), 1, (False, True, False)),
            a.iters)
        res["relu_"] = timed(lambda: torch.relu_(y), a.iters)
        res["relu_bwd"] = timed(lambda: torch.ops.aten.threshold_backward(gy, y, 0.0), a.iters)
        res["bias_grad"] = timed(lambda: gy.sum((0, 2, 3)), a.iters)
        from tianshou_amd.utils.net_atari import relu_bwd_bias
        gyc = gy.contiguous(memory_format=cl)
        yc = y.contiguous(memory_format=cl)
        res["relu_bwd+bias_grad fused"] = timed(lambda: relu_bwd_bias(gyc, yc, True), a.iters)
        line = " ".join(f"{kk} {v:7.3f} ms" for kk, v in res.items())
        print(f"conv {cin}->{cout} k{k} s{s} out {ho}x{ho}: {line}  | fwd "
              f"{flop / res['fwd'] / 1e9:6.1f} dgrad {flop / res['dgrad'] / 1e9:6.1f} "
              f"wgrad {flop / res['wgrad'] / 1e9:6.1f} TFLOP/s", flush=True)
        total += res["fwd+bias"] + res["dgrad"] + res["wgrad"] + res["relu_"] + \
            res["relu_bwd"] + res["bias_grad"]
    # the uint8 first layer (tsrl_dqn_conv1_fwd) vs frames -> f32 NHWC + MIOpen conv + ReLU
    from tianshou_amd.utils.net_atari import DQN, conv1_u8, frames_to_f32_nhwc, layer_init
    net = DQN(4, 84, 84, (6,), device=dev, features_only=True, output_dim=512,
              layer_init=layer_init).to(dev)
    conv = net._conv1_parts()[0]
    u8 = torch.randint(0, 256, (N, 4, 84, 84), dtype=torch.uint8, device=dev)
    lut = net._scale_lut(dev)
    t_fused = timed(lambda: conv1_u8(u8, conv, 255.0), a.iters)
    t_lib = timed(lambda: torch.relu_(conv(frames_to_f32_nhwc(u8, lut))), a.iters)
    flop = 2.0 * N * 400 * 32 * 256
    print(f"conv1 from u8: tsrl_dqn_conv1_fwd {t_fused:7.3f} ms ({flop / t_fused / 1e9:6.1f} "
          f"TFLOP/s f32-equivalent) vs frames+MIOpen+ReLU {t_lib:7.3f} ms", flush=True)
    from tianshou_amd import _C
    w2 = torch.randn(64, 32, 4, 4, device=dev).contiguous(memory_format=cl)
    gy2 = torch.randn(N, 9, 9, 64, device=dev)
    z1 = torch.relu(torch.randn(N, 20, 20, 32, device=dev))
    dx = torch.empty(N, 20, 20, 32, device=dev)
    s_ = _C.stream_ptr(dev)
    t_dg = timed(lambda: _C.lib().tsrl_dqn_conv2_dgrad(_C.ptr(gy2), N, w2.data_ptr(),
                                                        *w2.stride(), _C.ptr(z1), _C.ptr(dx),
                                                        s_), a.iters)
    gy2c = gy2.permute(0, 3, 1, 2)
    z1c = z1.permute(0, 3, 1, 2)
    t_lib = timed(lambda: torch.ops.aten.threshold_backward(torch.ops.aten.convolution_backward(
        gy2c, z1c, w2, None, (2, 2), (0, 0), (1, 1), False, (0, 0), 1,
        (True, False, False))[0], z1c, 0.0), a.iters)
    flop = 2.0 * N * 81 * 64 * 32 * 16
    print(f"conv2 data gradient + conv1 ReLU mask: tsrl_dqn_conv2_dgrad {t_dg:7.3f} ms "
          f"({flop / t_dg / 1e9:6.1f} TFLOP/s f32-equivalent) vs MIOpen + threshold_backward "
          f"{t_lib:7.3f} ms", flush=True)
    for fin, fout in ((3136, 512), (512, 7)):
        x = torch.randn(N, fin, device=dev)
        lin = torch.nn.Linear(fin, fout).to(dev)
        gy = torch.randn(N, fout, device=dev)
        flop = 2.0 * N * fin * fout

        def fb():
            xx = x.requires_grad_(True)
            out = lin(xx)
            out.backward(gy)
        t = timed(fb, a.iters)
        print(f"linear {fin}->{fout} fwd+bwd {t:7.3f} ms  {3 * flop / t / 1e9:6.1f} TFLOP/s",
              flush=True)
        total += t
    print(f"sum of the parts {total:7.3f} ms per {N}-row minibatch")


if __name__ == "__main__":
    main()
