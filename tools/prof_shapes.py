"""Per (kernel, grid, stream) duration summary from a rocprofv3 --kernel-trace results db.
    python tools/prof_shapes.py run_results.db [name-regex]"""
import collections
import re
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
d = collections.defaultdict(list)
q = "select name, grid_x, grid_y, grid_z, workgroup_x, lds_size, duration, stream from kernels"
for n, gx, gy, gz, wx, lds, dur, st in c.execute(q):
    short = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    if pat and not pat.search(short):
        continue
    d[(short, gx // max(wx, 1), gy, gz, lds, st)].append(dur)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print("%-58s grid(%5d,%3d,%3d) lds %6d %-15s n %4d avg %7.2f tot %8.1f" % (
        k[0][:58], k[1], k[2], k[3], k[4], k[5][:15], len(v), sum(v) / len(v) / 1e3, sum(v) / 1e3))
