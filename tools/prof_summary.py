"""Summarise a rocprofv3 kernel-trace database (.db) into a per-kernel stats table."""
import sqlite3
import sys

db = sys.argv[1]
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
rows = c.execute("select * from kernels").fetchall()
ki = {n: i for i, n in enumerate(cols)}
name_col = "name" if "name" in ki else "kernel_name"
agg = {}
for r in rows:
    n = r[ki[name_col]]
    d = (r[ki["end"]] - r[ki["start"]]) / 1e3  # us
    a = agg.setdefault(n, [0, 0.0, 1e30, 0.0])
    a[0] += 1
    a[1] += d
    a[2] = min(a[2], d)
    a[3] = max(a[3], d)
tot = sum(a[1] for a in agg.values())
print("%-110s %7s %12s %10s %10s %10s %6s" % ("kernel", "calls", "total_us", "avg_us", "min_us", "max_us", "pct"))
for n, a in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print("%-110s %7d %12.1f %10.2f %10.2f %10.2f %6.2f" % (n[:110], a[0], a[1], a[1] / a[0], a[2], a[3], 100 * a[1] / tot))
print("total kernel time %.1f us over %d dispatches" % (tot, sum(a[0] for a in agg.values())))
