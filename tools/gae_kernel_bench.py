"""Stand-alone tsrl_gae launch loop at the bench shape (4096 envs x 2048 steps, rew_norm f64
path with ret_rms partials, as bench.py's process_fn runs it) for rocprofv3 kernel-trace and
PMC passes.  Prints the HIP-event mean per launch and the algorithmic HBM rate."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tianshou-fork_amd"))

import torch  # noqa: E402

from tianshou_amd import _C  # noqa: E402
from tianshou_amd.policy.base import gae_device  # noqa: E402


def main(envs=4096, steps=2048, iters=int(os.environ.get("ITERS", "50")),
         mode=os.environ.get("MODE", "rew_norm")):
    dev = torch.device("cuda", 0)
    n = envs * steps
    g = torch.Generator(device=dev).manual_seed(0)
    v_s = torch.randn(n, device=dev, generator=g)
    v_n = torch.randn(n, device=dev, generator=g)
    rew = torch.rand(n, device=dev, dtype=torch.float64, generator=g)
    u = torch.rand(n, device=dev, generator=g)
    term, trunc = u < 0.001, u > 0.999
    scale = torch.tensor([1.25], dtype=torch.float64, device=dev) if mode == "rew_norm" else None
    nparts = int(_C.lib().tsrl_gae_num_partials(n, steps))
    parts = torch.empty(nparts * 3, dtype=torch.float64, device=dev) if scale is not None else None
    for _ in range(3):
        gae_device(v_s, v_n, rew, term, trunc, 0.99, 0.95, steps, None, scale, ret_partials=parts)
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        gae_device(v_s, v_n, rew, term, trunc, 0.99, 0.95, steps, None, scale, ret_partials=parts)
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    med = ts[len(ts) // 2]
    print(f"tsrl_gae {mode} n={n}: median {med:.2f} us, mean {sum(ts) / len(ts):.2f} us, "
          f"{26 * n / med / 1e3:.1f} GB/s algorithmic (26 B/transition), "
          f"{26 * n / med / 1e3 / 8000:.3f} of 8 TB/s")


if __name__ == "__main__":
    main()
