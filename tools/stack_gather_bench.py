"""Config-5 frame-stack gather timing: bench.py's atari workload collects one 1024 x 256 batch,
then buf.sample(0) (the minibatch stacks, tsrl_stack_gather) is timed with HIP events; prints
ms per sample(0) and a checksum of the stacked obs (equal across builds = same bytes).

    python tools/stack_gather_bench.py [--reps 5]
"""
import argparse
import os
import sys
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tianshou-fork_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import bench
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    np.random.seed(0)
    args = types.SimpleNamespace(envs=1024, T=256, act=6, ep_len=256, perm="numpy")
    coll, policy, buf = bench.build_atari(args, dev, 0)
    coll.collect(n_step=1024 * 256)
    torch.cuda.synchronize()
    batch, idx = buf.sample(0)
    obs = torch.as_tensor(batch.obs)
    ck = int(obs.view(-1, 4096).to(torch.int64).sum(1).mul(torch.arange(
        obs.numel() // 4096, device=obs.device) % 1009 + 1).sum())
    print(f"obs {tuple(obs.shape)} {obs.dtype} checksum {ck}", flush=True)
    ts = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        b2, _ = buf.sample(0)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
        del b2
    print("sample(0) ms: " + " ".join(f"{t:.2f}" for t in ts), flush=True)


if __name__ == "__main__":
    main()
