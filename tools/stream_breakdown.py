"""Per-stream kernel breakdown of the last full training step in a rocprofv3 kernel-trace DB.

    python tools/stream_breakdown.py <run_results.db> [top=28]
"""
import collections
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 28
rows = db.execute("select name,start,end,stream_id from kernels order by start").fetchall()
ends = [i for i, r in enumerate(rows) if r[0].startswith('philox_normal_kernel')]  # one per step (forward start)
step = rows[ends[-2] + 1:ends[-1] + 1]
print("step span %.1f us, %d launches" % ((step[-1][2] - step[0][1]) / 1e3, len(step)))
for sid in sorted({r[3] for r in step}):
    tot = collections.defaultdict(float)
    c = collections.Counter()
    for n, s, e, st in step:
        if st != sid:
            continue
        k = n.replace('void ', '').replace('(anonymous namespace)::', '').split('(')[0][:50]
        tot[k] += (e - s) / 1e3
        c[k] += 1
    print("stream", sid, "launches", sum(c.values()), "busy %.1f us" % sum(tot.values()))
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:top]:
        print("  %-50s %4d %8.1f  avg %6.1f" % (k, c[k], v, v / c[k]))
