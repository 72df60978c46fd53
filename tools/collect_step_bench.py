"""Time the Collector's vector step at the headline shape (4096 envs, Box 376 / 17, the
bench's actor): one-launch fused step (csrc/collect.hip) vs the four-launch step.

python tools/collect_step_bench.py [--steps 256] [--envs 4096]
TSRL_LIB_PATH=<variant .so> selects a variant build (tools/build_variant.sh; e.g.
-DCOLLECT_TRACE=1 with --trace: per-workgroup phase stamps of the fused kernel)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tianshou-fork_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=256)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--obs", type=int, default=376)
    ap.add_argument("--act", type=int, default=17)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--ep-len", type=int, default=1000)
    ap.add_argument("--trace", action="store_true",
                    help="read the per-workgroup phase stamps of a -DCOLLECT_TRACE=1 build")
    args = ap.parse_args()
    from tianshou_amd.data import Collector, VectorReplayBuffer
    from tianshou_amd.env import SyntheticVectorEnv, VectorEnvNormObs
    from tianshou_amd.policy import PPOPolicy
    from tianshou_amd.utils.models import fixed_std_normal, get_actor_critic, init_and_get_optim
    dev = torch.device("cuda", 0)
    E, D, A, T = args.envs, args.obs, args.act, args.steps
    for fused in (True, False):
        torch.manual_seed(0)
        actor, critic = get_actor_critic((D,), (64, 64), (A,), dev)
        optim = init_and_get_optim(actor, critic, 3e-4)
        pol = PPOPolicy(actor, critic, optim, fixed_std_normal,
                        action_space=SyntheticVectorEnv(1, (D,), A, device=dev).action_space,
                        action_bound_method="clip").to(dev)
        env = VectorEnvNormObs(SyntheticVectorEnv(E, (D,), A, ep_len=args.ep_len, device=dev))
        buf = VectorReplayBuffer(E * T, E, device=dev)
        c = Collector(pol, env, buf)
        c.use_fused_step = fused
        c.collect(n_step=E * T)  # warm-up: graph captures
        best = 1e9
        for _ in range(args.reps):
            buf.reset(keep_statistics=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            c.collect(n_step=E * T)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        print(f"fused_step={fused} (on={c._step_on}): {best * 1e3:.2f} ms per {T} steps = "
              f"{best / T * 1e6:.2f} us per step", flush=True)
        if args.trace and fused:
            trace_report(c, E, D)


def trace_report(c, E, D):
    """Phase stamps of the last 16 fused launches (s_memrealtime, 100 MHz): per-phase times
    inside a launch and the idle time between consecutive launches."""
    import numpy as np
    ws = c._scratch["collect_ws"].cpu().numpy()
    nblk = -(-E // 16)
    rup = lambda x: -(-x // 256) * 256  # noqa: E731
    # collect.hip make_ws: tickets, 2 totals slots, 2 state slots, then the trace
    off = 256 + 3 * rup((4 * 512 + 2) * 8) + 2 * rup(2 * 512 * 4 + 8 * 8)
    tr = ws[off:off + 16 * nblk * 64].view(np.uint64).reshape(16, nblk, 8).astype(np.int64)
    tr2 = ws[off + 16 * nblk * 64:off + 32 * nblk * 64].view(np.uint64).reshape(16, nblk, 8)
    stamp_rel = (tr[:, :, :4] - tr[:, :, :1]) / 100.0
    print("  stamps (all launches, median after the workgroup start): add "
          f"{np.median(stamp_rel[:, :, 1]):5.2f}, env {np.median(stamp_rel[:, :, 2]):5.2f}, "
          f"actor {np.median(stamp_rel[:, :, 3]):5.2f} us")
    tr2 = tr2.astype(np.int64)
    if tr2.any():
        # prologue detail stamps (wave 0): relative to the workgroup's own start stamp
        rel = (tr2[:, :, :8] - tr[:, :, :1]) / 100.0
        chained = tr2[:, :, 3].min(axis=1) > 0
        rel = rel[chained]
        for i, nm in enumerate(["A1 loads issued", "merge loads issued", "reset rows issued",
                                "merge math done", "after LDS barrier", "actor layer 1 done",
                                "h1 in LDS", "mu head done"]):
            print(f"  prologue {nm:>20s}: median {np.median(rel[:, :, i]):5.2f} p90 "
                  f"{np.percentile(rel[:, :, i], 90):5.2f} us after the workgroup start")
    order = np.argsort(tr[:, :, 0].min(1))
    tr = tr[order]
    names = ["start", "add", "env", "actor", "unused", "unused"]
    spans, gaps = [], []
    for j in range(16):
        t0 = tr[j, :, 0].min()
        end = tr[j, :, :6].max()
        spans.append((end - t0) / 100.0)
        if j:
            gaps.append((t0 - tr[j - 1, :, :6].max()) / 100.0)
    us = (tr[-1] - tr[-1, :, 0].min()) / 100.0
    for i in range(4):
        print(f"  stamp {names[i]:>9}: min {us[:, i].min():7.2f}  median {np.median(us[:, i]):7.2f}"
              f"  max {us[:, i].max():7.2f} us")
    for i in range(1, 4):
        d = us[:, i] - us[:, i - 1]
        print(f"  phase {names[i]:>9}: median {np.median(d):6.2f}  max {d.max():6.2f} us")
    allu = (tr[:, :, :6] - tr[:, :, :1].min(axis=1, keepdims=True)) / 100.0
    mg = allu[:, :, 4] - allu[:, :, 0]
    ad = allu[:, :, 1] - allu[:, :, 4]
    print(f"  all launches: prologue merge median {np.median(mg):5.2f} p90 {np.percentile(mg, 90):5.2f}"
          f" max {mg.max():5.2f} us; add after merge median {np.median(ad):5.2f} p90 "
          f"{np.percentile(ad, 90):5.2f} max {ad.max():5.2f} us")
    for j in range(16):
        print(f"   launch {j:2d}: span {spans[j]:6.2f} us, merge max {mg[j].max():5.2f}, add max "
              f"{ad[j].max():5.2f}, env end max {allu[j, :, 2].max():6.2f}" +
              (f", gap before {gaps[j - 1]:6.2f}" if j else ""))
    tl = []
    for j in range(16):
        t0 = tr[j, :, 0].min()
        env = (tr[j, :, 3].max() - t0) / 100.0
        gf = tr[j, :, 4]
        gfd = (gf[gf > 0].max() - t0) / 100.0 if (gf > 0).any() else np.nan
        mg = tr[j, :, 5]
        mgd = (mg[mg > 0].max() - t0) / 100.0 if (mg > 0).any() else np.nan
        tl.append((env, gfd, mgd))
    tl = np.asarray(tl)
    print(f"  per launch (median): last env {np.median(tl[:, 0]):6.2f}, last group fold "
          f"{np.nanmedian(tl[:, 1]):6.2f}, merge done {np.nanmedian(tl[:, 2]):6.2f} us")
    j = int(np.argsort(tl[:, 0])[8])  # a median launch: its slowest workgroups
    t0 = tr[j, :, 0].min()
    u = (tr[j, :, :4] - t0) / 100.0
    for b in np.argsort(u[:, 3])[-8:]:
        print(f"  launch {j} wg {b:4d} xcc {tr[j, b, 6] & 15} hwid {tr[j, b, 7]:#x}: start "
              f"{u[b, 0]:6.2f} add {u[b, 1]:6.2f} actor {u[b, 2]:6.2f} env {u[b, 3]:6.2f} us")
    add = u[:, 1] - u[:, 0]
    xcc = tr[j, :, 6] & 15
    for x in range(8):
        m = xcc == x
        if m.any():
            print(f"  xcc {x}: {m.sum():3d} wgs, add median {np.median(add[m]):5.2f} max "
                  f"{add[m].max():5.2f} us")
    print(f"  launch span (first stamp -> last stamp): median {np.median(spans):6.2f} us; "
          f"gap between launches (last stamp -> next first stamp): median {np.median(gaps):6.2f} "
          f"min {np.min(gaps):6.2f} max {np.max(gaps):6.2f} us")


if __name__ == "__main__":
    main()
