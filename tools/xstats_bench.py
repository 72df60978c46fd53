"""Stand-alone timing of the exact obs_rms kernels at the headline shape (4096 x 376 f32 rows,
~0.1 % reset rows): tsrl_rms_exact_stats (the pipelined form's batch moments, streamed) and
tsrl_rms_exact_update (the serial form's LDS-resident chains + merge), each alone on the
device, HIP-event mean per launch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tianshou-fork_amd"))

import torch  # noqa: E402

from tianshou_amd import _C  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main(k=4096, D=376):
    dev = torch.device("cuda", 0)
    lib = _C.lib()
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(k, D, device=dev, generator=g)
    xr = torch.randn(k, D, device=dev, generator=g)
    done = (torch.rand(k, device=dev, generator=g) < 0.001).to(torch.uint8)
    st = torch.zeros(int(lib.tsrl_rms_exact_stats_bytes(D)), dtype=torch.uint8, device=dev)
    s = _C.stream_ptr(dev)
    t1 = timeit(lambda: lib.tsrl_rms_exact_stats(_C.ptr(x), k, _C.ptr(xr), _C.ptr(done), D,
                                                 _C.ptr(st), s))
    mean = torch.zeros(D, device=dev)
    var = torch.ones(D, device=dev)
    cnt = torch.zeros(1, dtype=torch.float64, device=dev)
    sm, sv = torch.zeros_like(mean), torch.zeros_like(var)
    ticket = torch.zeros(1, dtype=torch.int32, device=dev)
    t2 = timeit(lambda: lib.tsrl_rms_exact_update(
        _C.ptr(x), None, k, _C.ptr(xr), _C.ptr(done), k, D, _C.ptr(mean), _C.ptr(var),
        _C.ptr(cnt), _C.ptr(sm), _C.ptr(sv), _C.ptr(ticket), s))
    print(f"k={k} D={D}: tsrl_rms_exact_stats {t1:.1f} us, tsrl_rms_exact_update {t2:.1f} us")


if __name__ == "__main__":
    main()
