"""Per-kernel means of rocprofv3 --pmc counters from its rocpd database:
python tools/pmc_summary.py <results.db> [kernel-name-substring]."""
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
c = sqlite3.connect(db)
acc = defaultdict(lambda: defaultdict(list))
dur = defaultdict(dict)
for name, cn, v, disp, d in c.execute(
        "select kernel_name, counter_name, value, dispatch_id, duration from counters_collection"):
    if sub in name:
        acc[name[:70]][cn].append(v)
        dur[name[:70]][disp] = d
for n, cs in acc.items():
    ds = list(dur[n].values())
    print(f"{n}  (dispatches {len(ds)}, mean duration {sum(ds) / len(ds) / 1e3:.1f} us)")
    for cn, v in sorted(cs.items()):
        print(f"  {cn:28s} {sum(v) / len(v):18.1f}")
