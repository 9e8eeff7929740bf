"""Per-launch view of one training step from a rocprofv3 kernel-trace database.

    python tools/prof_launches.py <run_results.db> [step_from_end=1] [min_us=0] [name_filter]

Steps are delimited by adam_kernel launches.  Prints launch order, kernel (short name),
grid in workgroups, and duration, plus a per-kernel total for that step.
"""
import sqlite3
import sys
from collections import defaultdict


def short(n):
    n = n.replace("void ", "")
    return n.split("(")[0][:48]


def main():
    db = sqlite3.connect(sys.argv[1])
    back = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
    filt = sys.argv[4] if len(sys.argv) > 4 else ""
    rows = db.execute("select name, start, end, grid_x, grid_y, grid_z, workgroup_x, workgroup_y, workgroup_z "
                      "from kernels order by start").fetchall()
    ends = [i for i, r in enumerate(rows) if r[0].startswith("adam_kernel")]
    if len(ends) < back + 1:
        raise SystemExit("not enough steps")
    lo, hi = ends[-back - 1] + 1, ends[-back] + 1
    step = rows[lo:hi]
    tot = defaultdict(float)
    cnt = defaultdict(int)
    span = (step[-1][2] - step[0][1]) / 1e3
    busy = 0.0
    for i, (name, s, e, gx, gy, gz, wx, wy, wz) in enumerate(step):
        us = (e - s) / 1e3
        busy += us
        k = short(name)
        tot[k] += us
        cnt[k] += 1
        if us >= min_us and filt in name:
            print("%5d %-48s grid %5d x %3d x %3d  %8.2f us" % (i, k, gx // max(wx, 1), gy // max(wy, 1),
                                                               gz // max(wz, 1), us))
    print("\nstep: %d launches, span %.1f us, kernel-busy %.1f us (%.1f%%)" % (len(step), span, busy,
                                                                               100 * busy / span))
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:25]:
        print("  %-48s %5d  %9.1f us" % (k, cnt[k], v))


if __name__ == "__main__":
    main()
