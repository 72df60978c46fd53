"""Per-kernel totals from a rocprofv3 rocpd database (the sqlite *_results.db it writes):
python tools/rocpd_top.py <db> [N] [--last-ms MS]  -> name, calls, total ms, mean us (top N by
total); --last-ms keeps only the kernels that start in the last MS milliseconds of the trace
(a steady-state window: e.g. the last timed iteration, after warm-up and MIOpen's find).
Whatever the top-N cut, the kernels the bench line and DESIGN.md cite are always listed
afterwards (ALWAYS: the GAE kernel of `roofline`, the fused collect step, the minibatch
kernels), with min / max durations, so the roofline is reproducible from the summary alone."""
import os
import sqlite3
import sys

args = [a for a in sys.argv[1:]]
last_ms = None
if "--last-ms" in args:
    i = args.index("--last-ms")
    last_ms = float(args[i + 1])
    del args[i:i + 2]
db = args[0]
if not os.path.isfile(db):
    sys.exit(__doc__)
n = int(args[1]) if len(args) > 1 else 30
c = sqlite3.connect(db)
where, params = "", ()
if last_ms is not None:
    t_end = c.execute("select max(end) from kernels").fetchone()[0]
    where, params = "where start >= ?", (t_end - last_ms * 1e6,)
    t0 = c.execute(f"select min(start) from kernels {where}", params).fetchone()[0]
    print(f"window: last {last_ms:.0f} ms of the trace ({(t_end - t0) / 1e6:.1f} ms of kernels)")
tot = c.execute(f"select sum(duration)/1e6 from kernels {where}", params).fetchone()[0]
print(f"total kernel time {tot:.2f} ms")
for name, cnt, ms, us in c.execute(
        f"select name, count(*), sum(duration)/1e6, avg(duration)/1e3 from kernels {where} "
        "group by name order by sum(duration) desc limit ?", params + (n,)):
    print(f"{ms:10.2f} ms {cnt:7d} x {us:10.1f} us  {name[:140]}")
ALWAYS = ("gae_rows_staged_kernel", "collect_box_step_kernel", "l1_ring_kernel",
          "dw_x6_kernel", "dw_reduce_kernel", "ppo_tail_kernel", "tail_reduce_kernel",
          "clip_adam_kernel", "rms_exact_kernel", "eval_tail_kernel", "rms_exact_stats_kernel",
          "spec_step_kernel", "xpipe_finalize_kernel", "ppo_tail16_kernel")
print("cited kernels (every launch in the window): total ms, calls, mean / min / max us")
for pat in ALWAYS:
    for name, cnt, ms, us, lo, hi in c.execute(
            "select name, count(*), sum(duration)/1e6, avg(duration)/1e3, min(duration)/1e3, "
            f"max(duration)/1e3 from kernels {where + (' and' if where else 'where')} "
            "name like ? group by name order by name", params + (f"%{pat}%",)):
        print(f"{ms:10.2f} ms {cnt:7d} x {us:10.2f} us (min {lo:.2f}, max {hi:.2f})  "
              f"{name[:120]}")
# the layer-1 kernel serves both the minibatch (learn) and process_fn's evaluation chunks:
# split its launches by grid size when the database records it
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
gcol = next((x for x in ("grid_size", "grid_size_x", "grid_x", "grid") if x in cols), None)
if gcol:
    print(f"l1_ring_kernel by {gcol}: calls, mean / min / max us")
    for g, cnt, us, lo, hi in c.execute(
            f"select {gcol}, count(*), avg(duration)/1e3, min(duration)/1e3, max(duration)/1e3 "
            f"from kernels {where + (' and' if where else 'where')} name like ? "
            f"group by {gcol} order by {gcol}", params + ("%l1_ring_kernel%",)):
        print(f"  {gcol} {g}: {cnt:6d} x {us:10.2f} us (min {lo:.2f}, max {hi:.2f})")
