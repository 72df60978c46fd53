"""Host timing of the threaded np.random.permutation draws (tsrl_np_shuffle_draws_mt) against
the sequential loop (tsrl_np_shuffle_draws), with equality checks:
    python tools/perm_mt_bench.py [n ...] [--threads T]"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tianshou-fork_amd"))
import numpy as np  # noqa: E402

from tianshou_amd import _C  # noqa: E402


def run(fn, key, pos, n, *extra):
    k = np.ascontiguousarray(key, dtype=np.uint32).copy()
    p = ctypes.c_int32(int(pos))
    d = np.empty(n, np.uint32)
    t = time.perf_counter()
    _C.check(fn(k.ctypes.data, ctypes.addressof(p), n, d.ctypes.data, *extra))
    return k, p.value, d, time.perf_counter() - t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("n", type=int, nargs="*", default=[8388608, 67108864])
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--device", action="store_true", help="device permutation end to end")
    ap.add_argument("--plan", action="store_true",
                    help="PPOPolicy's pipelined global minibatch plans, rank 3 of 8")
    a = ap.parse_args()
    if a.plan:
        plan_bench()
        return
    if a.device:
        device_bench(a.n)
        return
    L = _C.lib()
    rng = np.random.RandomState(7)
    print("cpus", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)), flush=True)
    for n in a.n:
        for r in range(a.reps):
            st = rng.get_state()
            k1, p1, d1, t1 = run(L.tsrl_np_shuffle_draws, st[1], st[2], n)
            k2, p2, d2, t2 = run(L.tsrl_np_shuffle_draws_mt, st[1], st[2], n, a.threads)
            ok = np.array_equal(d1, d2) and np.array_equal(k1, k2) and p1 == p2
            print(f"n={n} rep {r}: sequential {t1 * 1e3:.1f} ms, threaded {t2 * 1e3:.1f} ms, "
                  f"equal {ok}", flush=True)
            rng.set_state(("MT19937", k1, p1, 0, 0.0))


def device_bench(n_list, world=8):
    """End-to-end np_permutation(n) on the device (host draws + copy + tsrl_shuffle_apply) and
    the data-parallel share selection of _minibatch_plan for rank 0 of `world`."""
    import torch
    from tianshou_amd.utils.np_perm import LegacyPermutation, _draws
    dev = torch.device("cuda", 0)
    lp = LegacyPermutation()
    for n in n_list:
        np.random.seed(1)
        ref_state = np.random.get_state()
        for r in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            perm = lp(n, dev)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            st = np.random.get_state()
            buf = torch.empty(n, dtype=torch.int32, pin_memory=True)
            th = time.perf_counter()
            _draws(st[1], st[2], n, buf.numpy().view(np.uint32))
            td = time.perf_counter()
            lp._apply(buf, n, dev)
            torch.cuda.synchronize()
            ta = time.perf_counter()
            d = torch.empty(n, dtype=torch.int32, device=dev)
            d.copy_(buf, non_blocking=True)
            torch.cuda.synchronize()
            tc = time.perf_counter()
            print(f"   host draws {1e3 * (td - th):.1f} ms, copy+apply {1e3 * (ta - td):.1f} ms, "
                  f"copy alone {1e3 * (tc - ta):.1f} ms", flush=True)
            nl, B = n // world, n // 32
            pos = torch.nonzero((perm >= 0) & (perm < nl)).squeeze(1)
            idx = (perm[pos]).contiguous()
            lab = torch.div(pos, B, rounding_mode="floor")
            counts = torch.bincount(lab, minlength=32).cpu()
            t2 = time.perf_counter()
            print(f"device n={n} rep {r}: permutation {1e3 * (t1 - t0):.1f} ms, rank share "
                  f"selection + counts {1e3 * (t2 - t1):.1f} ms", flush=True)
        if n <= 8388608:
            np.random.set_state(ref_state)
            want = np.random.permutation(n)
            np.random.set_state(ref_state)
            got = lp(n, dev).cpu().numpy()
            print("  equals np.random.permutation:", np.array_equal(want, got), flush=True)


def plan_bench(world=8, rank=3, n=4096 * 2048, repeat=4):
    """One update's plans (repeat x np.random.permutation(world x n) + this rank's share) as
    _learn issues them: draws prefetched (as during the collect), side-stream device work.
    Reports the host time per plan and the side-stream GPU time per plan."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import dist_worker as w
    from test_gpu_perm import _FakeDP
    dev = torch.device("cuda", 0)
    policy = w.build_policy(376, 17, dev)
    policy.dp = _FakeDP(world, rank)
    np.random.seed(0)
    for it in range(3):
        policy._np_perm.prefetch(world * n, repeat)
        time.sleep(0.3)  # the collect phase the draws hide behind
        policy._np_perm_used = False
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        plans = policy._plan_pipeline(n, dev, n // 32, repeat, True)
        host = []
        for k in range(repeat):
            th = time.perf_counter()
            idx, chunks = plans(k)
            host.append(1e3 * (time.perf_counter() - th))
        torch.cuda.synchronize()
        tot = 1e3 * (time.perf_counter() - t0)
        print(f"iter {it}: {repeat} plans of rank {rank}/{world}, n={n}: host per plan "
              f"{', '.join(f'{h:.1f}' for h in host)} ms; all plans done {tot:.1f} ms; "
              f"rows {idx.numel()} in {len(chunks)} minibatches", flush=True)


if __name__ == "__main__":
    main()
