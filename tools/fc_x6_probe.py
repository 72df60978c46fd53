"""Probe: config 5's FC layer (Linear 3136 -> 512 over 8192-row minibatches) as bf16x6 products
on hipBLASLt's bf16 GEMMs with f32 output (torch mm / addmm with out_dtype), against the f32
GEMMs it runs today: time of the forward, data-gradient and weight-gradient GEMMs, and the
error of each against an f64 product.

The six products a_i b_j (i + j <= 2) of the 3-way bf16 splits are grouped into three GEMMs per
product by concatenating split planes along K: [a0|a1|a2] . [b0|b0|b0], [a0|a1] . [b1|b1],
a0 . b2 -- K' = 6 K in total, every product exact in f32, accumulated in f32.  The weight
gradient reuses the forward's [x0|x1|x2] planes as the N side (output blocks summed after).

    python tools/fc_x6_probe.py [--rows 8192] [--iters 20]
"""
import argparse

import torch


def split3(t):
    a0 = t.to(torch.bfloat16)
    r = t - a0.float()
    a1 = r.to(torch.bfloat16)
    a2 = (r - a1.float()).to(torch.bfloat16)
    return a0, a1, a2


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def x6_mm(A3, B3, K):
    """sum over i + j <= 2 of A_i @ B_j: A3 = [A0|A1|A2] ([M, 3K] bf16), B3 = (B0, B1, B2) as
    [K, N] bf16 each."""
    B0, B1, B2 = B3
    y = torch.mm(A3, torch.cat([B0, B0, B0], 0), out_dtype=torch.float32)
    y = torch.addmm(y, A3[:, :2 * K], torch.cat([B1, B1], 0), out_dtype=torch.float32)
    return torch.addmm(y, A3[:, :K], B2, out_dtype=torch.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    N, K, O = a.rows, 3136, 512
    x = torch.relu(torch.randn(N, K, device=dev, generator=g))
    w = torch.randn(O, K, device=dev, generator=g) * 0.02
    gy = torch.randn(N, O, device=dev, generator=g) * 1e-3
    xs, ws, gs = split3(x), split3(w), split3(gy)
    X3 = torch.cat(xs, 1).contiguous()                  # [N, 3K]
    WT = tuple(t.t().contiguous() for t in ws)          # [K, O] each
    G3 = torch.cat(gs, 1).contiguous()                  # [N, 3O]
    Wp = tuple(t.contiguous() for t in ws)              # [O, K] each

    def wgrad_x6():
        """gy^T x from the same [x0|x1|x2] planes: gy_i^T @ X3 gives the blocks
        [gy_i^T x0 | gy_i^T x1 | gy_i^T x2]; the six needed blocks are summed after."""
        o1 = torch.mm(gs[0].t(), X3, out_dtype=torch.float32)
        o2 = torch.mm(gs[1].t(), X3[:, :2 * K], out_dtype=torch.float32)
        o3 = torch.mm(gs[2].t(), X3[:, :K], out_dtype=torch.float32)
        return o1[:, :K] + o1[:, K:2 * K] + o1[:, 2 * K:] + o2[:, :K] + o2[:, K:] + o3

    def report(name, f32fn, x6fn, ref, flop):
        t32 = timed(f32fn, a.iters)
        t6 = timed(x6fn, a.iters)
        e32 = ((f32fn().double() - ref).abs().max() / ref.abs().max()).item()
        e6 = ((x6fn().double() - ref).abs().max() / ref.abs().max()).item()
        print(f"{name:6s} f32 {t32:8.1f} us ({flop / t32 / 1e6:6.1f} TF/s)  x6 {t6:8.1f} us "
              f"({flop / t6 / 1e6:6.1f} TF/s f32-eq, {6 * flop / t6 / 1e6:7.1f} TF/s bf16)  "
              f"max err / max |ref|: f32 {e32:.2e} x6 {e6:.2e}", flush=True)

    xd, wd, gd = x.double(), w.double(), gy.double()
    report("fwd", lambda: x @ w.t(), lambda: x6_mm(X3, WT, K), xd @ wd.t(), 2.0 * N * K * O)
    report("dgrad", lambda: gy @ w, lambda: x6_mm(G3, Wp, O), gd @ wd, 2.0 * N * K * O)
    report("wgrad", lambda: gy.t() @ x, wgrad_x6, gd.t() @ xd,
           2.0 * N * K * O)
    t_split = timed(lambda: torch.cat(split3(x), 1), a.iters)
    print(f"torch split of x into [x0|x1|x2]: {t_split:.1f} us (a fused kernel writes the same "
          f"{N * 3 * K * 2 / 1e6:.0f} MB)")


if __name__ == "__main__":
    main()
