"""Kernel durations and launch gaps from a rocprofv3 rocpd database:
python tools/rocpd_gaps.py <db> <kernel-name-substring> -> per-launch duration and the idle time
between consecutive kernels around it (median / p90)."""
import sqlite3
import sys

import numpy as np

db, sub = sys.argv[1], sys.argv[2]
c = sqlite3.connect(db)
rows = c.execute("select name, start, end from kernels order by start").fetchall()
dur, gap_before, gap_after = [], [], []
for i, (n, s, e) in enumerate(rows):
    if sub in n:
        dur.append(e - s)
        if i > 0:
            gap_before.append(s - rows[i - 1][2])
        if i + 1 < len(rows):
            gap_after.append(rows[i + 1][1] - e)
for name, v in (("duration", dur), ("gap before", gap_before), ("gap after", gap_after)):
    v = np.asarray(v) / 1e3
    print(f"{name:>10}: n {len(v)}  median {np.median(v):8.2f} us  p10 {np.percentile(v, 10):8.2f}"
          f"  p90 {np.percentile(v, 90):8.2f}")
