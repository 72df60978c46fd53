"""Round-6 probe (diagnostic): torch.ops.aten.miopen_convolution_relu (MIOpen conv + bias +
ReLU) vs this repo's F.conv2d (no bias) + tsrl_bias_relu_rows for the config-5 conv2 / conv3
shapes, channels_last f32: time per call and max |difference|."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tianshou-fork_amd")]


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    from tianshou_amd.utils.net_atari import bias_relu_
    dev = torch.device("cuda", 0)
    cl = torch.channels_last
    for cin, cout, k, s, hw in [(32, 64, 4, 2, 20), (64, 64, 3, 1, 9)]:
        for n in (1024, 8192):
            x = torch.relu(torch.randn(n, cin, hw, hw, device=dev)).contiguous(memory_format=cl)
            w = (0.05 * torch.randn(cout, cin, k, k, device=dev)).contiguous(memory_format=cl)
            b = 0.1 * torch.randn(cout, device=dev)
            ref = lambda: bias_relu_(torch.nn.functional.conv2d(x, w, None, s), b)  # noqa
            fus = lambda: torch.ops.aten.miopen_convolution_relu(x, w, b, [s, s], [0, 0],  # noqa
                                                                 [1, 1], 1)
            try:
                y1, y2 = ref(), fus()
                d = float((y1 - y2).abs().max())
                print(f"conv {cin}->{cout} k{k} s{s} n {n}: unfused {timed(ref):7.1f} us  "
                      f"fused {timed(fus):7.1f} us  max|diff| {d:.3g}  fused cl "
                      f"{y2.is_contiguous(memory_format=cl)}", flush=True)
            except Exception as e:  # noqa: BLE001
                print(f"conv {cin}->{cout} n {n}: fused op failed: {e}", flush=True)


if __name__ == "__main__":
    main()
