"""Probe the skinny MLP GEMMs of the PPO minibatch (B = 262144 rows, D = 376, H = 64) under
the available BLAS back-ends and a split-K formulation.  GPU only; prints one line per
variant (median of 20 runs, HIP events)."""
import sys

import torch


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2] * 1e3


def main():
    dev = torch.device("cuda", 0)
    B, D, H = 262144, 376, 64
    x = torch.randn(B, D, device=dev)
    w = torch.randn(H, D, device=dev)
    w2 = torch.randn(2 * H, D, device=dev)
    bias = torch.randn(H, device=dev)
    dy = torch.randn(B, H, device=dev)
    dy2 = torch.randn(B, 2 * H, device=dev)
    h = torch.randn(B, H, device=dev)
    w_hh = torch.randn(H, H, device=dev)
    for lib in ("default", "cublas", "cublaslt"):
        if lib != "default":
            try:
                torch.backends.cuda.preferred_blas_library(lib)
            except Exception as e:
                print(lib, "unavailable", e)
                continue
        res = {
            "fwd_L1 addmm [B,376]x[376,64]": timeit(lambda: torch.addmm(bias, x, w.t())),
            "fwd_L1 fused a+c [B,376]x[376,128]": timeit(lambda: x @ w2.t()),
            "dW1 [64,B]x[B,376]": timeit(lambda: dy.t() @ x),
            "dW1 fused [128,B]x[B,376]": timeit(lambda: dy2.t() @ x),
            "db1 dy.sum(0)": timeit(lambda: dy.sum(0)),
            "fwd_L2 [B,64]x[64,64]": timeit(lambda: h @ w_hh.t()),
            "dW2 [64,B]x[B,64]": timeit(lambda: dy.t() @ h),
        }
        for k, v in res.items():
            print(f"{lib:9s} {k:40s} {v:9.1f} us", flush=True)
    torch.backends.cuda.preferred_blas_library("default")
    for s in (16, 64, 256):
        xs = x.view(s, B // s, D)
        dys = dy.view(s, B // s, H)
        t = timeit(lambda: torch.bmm(dys.transpose(1, 2), xs).sum(0))
        print(f"splitK{s:<4d} dW1 bmm+sum                          {t:9.1f} us", flush=True)
        t = timeit(lambda: torch.bmm(dys.transpose(1, 2), xs))
        print(f"splitK{s:<4d} dW1 bmm only                         {t:9.1f} us", flush=True)
    ones = torch.ones(B, device=dev)
    print(f"db1 ones@dy {timeit(lambda: ones @ dy):9.1f} us")


if __name__ == "__main__":
    main()
