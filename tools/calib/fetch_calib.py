"""FETCH_SIZE per dispatch of tools/calib/fetch_calib against the known bytes it reads.
    python tools/calib/fetch_calib.py <rocprofv3 csv dir>"""
import collections
import csv
import glob
import sys

BYTES = {"k16": 768 << 20, "k8": 768 << 20, "k4": 768 << 20, "seg64": 384 << 20}
rows = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != "FETCH_SIZE":
            continue
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
        rows[k].append(float(r["Counter_Value"]) * 1024.0)
print("%-8s %6s %14s %14s %8s" % ("kernel", "disp", "FETCH_bytes", "read_bytes", "ratio"))
for k, v in sorted(rows.items()):
    avg = sum(v) / len(v)
    print("%-8s %6d %14.0f %14d %8.3f" % (k, len(v), avg, BYTES.get(k, 0), avg / BYTES.get(k, 1)))
