"""Config-5 collect diagnostics (GPU): per-step time of Collector.collect for the u8
frame-stack env with the Nature-DQN policy, eager vs HIP-graph replay, and whether graphs
were captured.  python tools/atari_collect_probe.py"""
import os
import sys
import time
from types import SimpleNamespace

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tianshou-fork_amd")]

import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    args = SimpleNamespace(envs=1024, T=256, act=6, ep_len=256, perm="sorted")
    for g in (0, 64):
        coll, policy, buf = bench.build_atari(args, dev, 0)
        coll.graph_steps = g
        for it in range(3):
            coll.reset_buffer(keep_statistics=True)
            torch.cuda.synchronize()
            t = time.perf_counter()
            coll.collect(n_step=args.envs * args.T)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
        print(f"graph_steps={g}: collect {dt * 1e3:.1f} ms ({dt / args.T * 1e6:.0f} us/step), "
              f"graphs captured {sorted(getattr(coll, '_graphs', {}) or {})}, "
              f"fused_act {coll._fused_act_on}", flush=True)


if __name__ == "__main__":
    main()
