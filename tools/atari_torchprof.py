"""Config-5 glue attribution: torch.profiler over one collect + update of bench.py's atari
workload (after warm-up iterations), printing the device time of the small torch kernels
(copies, adds, fills, clamps, reductions) grouped by the Python stack that launched them.

    python tools/atari_torchprof.py [--envs 1024] [--T 256] [--stack 6]
"""
import argparse
import os
import sys
import types

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "tianshou-fork_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=1024)
    ap.add_argument("--T", type=int, default=256)
    ap.add_argument("--stack", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    import bench
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    np.random.seed(0)
    args = types.SimpleNamespace(envs=a.envs, T=a.T, act=6, ep_len=256, perm="numpy")
    coll, policy, buf = bench.build_atari(args, dev, 0)
    n = a.envs * a.T

    def iteration():
        coll.collect(n_step=n)
        policy.update(0, buf, batch_size=8192, repeat=4)
        coll.reset_buffer(keep_statistics=True)
        torch.cuda.synchronize()

    for _ in range(a.warmup):
        iteration()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                 record_shapes=True) as prof:
        iteration()
    want = ("aten::copy_", "aten::add_", "aten::fill_", "aten::zero_", "aten::clamp",
            "aten::clamp_", "aten::sum", "aten::add", "aten::mul", "aten::where")
    agg = {}
    tot = 0.0
    for ev in prof.events():
        dt = getattr(ev, "device_time_total", None)
        if dt is None:
            dt = ev.cuda_time_total
        if ev.name not in want:
            continue
        # device time of the op's kernels
        chain = []
        p = ev.cpu_parent
        while p is not None and len(chain) < a.stack:
            chain.append(p.name)
            p = p.cpu_parent
        key = (ev.name, str(ev.input_shapes)[:120], " < ".join(chain))
        c = agg.setdefault(key, [0.0, 0])
        c[0] += dt
        c[1] += 1
        tot += dt
    rows = sorted(agg.items(), key=lambda kv: -kv[1][0])
    print(f"device time of {len(want)} small-op kinds: {tot / 1e3:.2f} ms per iteration")
    for (name, shapes, chain), (dt, cnt) in rows[:a.top]:
        print(f"{dt / 1e3:8.2f} ms {cnt:5d}x {name} {shapes}\n           < {chain}")


if __name__ == "__main__":
    main()
