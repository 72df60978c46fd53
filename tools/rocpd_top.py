"""Per-kernel totals from a rocprofv3 rocpd database (the sqlite *_results.db it writes):
python tools/rocpd_top.py <db> [N]  -> name, calls, total ms, mean us (top N by total)."""
import sqlite3
import sys

db = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
c = sqlite3.connect(db)
tot = c.execute("select sum(duration)/1e6 from kernels").fetchone()[0]
print(f"total kernel time {tot:.2f} ms")
for name, cnt, ms, us in c.execute(
        "select name, count(*), sum(duration)/1e6, avg(duration)/1e3 from kernels "
        "group by name order by sum(duration) desc limit ?", (n,)):
    print(f"{ms:10.2f} ms {cnt:7d} x {us:10.1f} us  {name[:140]}")
