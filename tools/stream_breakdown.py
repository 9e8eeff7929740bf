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

# main-stream idle gaps: launch boundaries (~1.5-2 us) vs waits on the side streams' events
main = max({r[3] for r in step}, key=lambda sid: sum(1 for r in step if r[3] == sid))
ms = [r for r in step if r[3] == main]
gaps = [(ms[i + 1][1] - ms[i][2]) / 1e3 for i in range(len(ms) - 1)]
bins = [(0, 2), (2, 4), (4, 10), (10, 50), (50, 1e9)]
print("main stream %d idle gaps, total %.1f us" % (len(gaps), sum(gaps)))
for lo, hi in bins:
    sel = [g for g in gaps if lo <= g < hi]
    print("  gap [%g, %g) us: %4d gaps, %8.1f us" % (lo, hi, len(sel), sum(sel)))
name = lambda n: n.replace('void ', '').replace('(anonymous namespace)::', '').split('(')[0][:40]
# which transitions the 4-10 us gaps follow (launch boundaries after event records vs plain dependencies)
mid = collections.Counter()
mid_t = collections.defaultdict(float)
for i, gp in enumerate(gaps):
    if 4 <= gp < 10:
        k = "%s -> %s" % (name(ms[i][0]).split('<')[0], name(ms[i + 1][0]).split('<')[0])
        mid[k] += 1
        mid_t[k] += gp
print("  4-10 us gaps by transition:")
for k, v in mid.most_common(14):
    print("    %4d %8.1f us  %s" % (v, mid_t[k], k))
order = sorted(range(len(gaps)), key=lambda i: -gaps[i])[:int(sys.argv[3]) if len(sys.argv) > 3 else 20]
for i in sorted(order):
    print("  %7.1f us after %-40s before %-40s" % (gaps[i], name(ms[i][0]), name(ms[i + 1][0])))

# what the other streams ran during the largest main-stream gaps (cross-stream waits vs CU contention)
if len(sys.argv) > 4:
    for i in sorted(order)[:int(sys.argv[4])]:
        g0, g1 = ms[i][2], ms[i + 1][1]
        if g1 - g0 < 15e3:
            continue
        print("gap %.1f us after %s:" % ((g1 - g0) / 1e3, name(ms[i][0])))
        for n, s, e, sid in step:
            if sid != main and s < g1 and e > g0:
                print("    stream %d %-40s %8.1f .. %8.1f us" % (sid, name(n), (s - g0) / 1e3, (e - g0) / 1e3))
