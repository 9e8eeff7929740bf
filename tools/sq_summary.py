"""Per-kernel SQ counter summary from a rocprofv3 --pmc csv (SQ_WAVES, SQ_WAVE_CYCLES,
SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY, SQ_INSTS_VALU, SQ_INSTS_MFMA).
    python tools/sq_summary.py <dir>"""
import collections
import csv
import glob
import sys

files = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in files:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:90]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
rows = sorted(agg.items(), key=lambda kv: -kv[1]["SQ_WAVE_CYCLES"])
if any("SQ_LDS_BANK_CONFLICT" in v for v in agg.values()):  # second pass: LDS / wait breakdown
    print("%-90s %6s %12s %12s %12s %12s %10s %10s" % ("kernel", "disp", "lds_bconf/w", "wait_lds/w", "lds_inst/w",
                                                       "wcyc/w", "vmem_rd/w", "vmem_wr/w"))
    for k, v in rows[:30]:
        w = max(v["SQ_WAVES"], 1)
        print("%-90s %6d %12.0f %12.0f %12.0f %12.0f %10.0f %10.0f" % (
            k, len(disp[k]), v["SQ_LDS_BANK_CONFLICT"] / w, v["SQ_WAIT_INST_LDS"] / w, v["SQ_INSTS_LDS"] / w,
            v["SQ_WAVE_CYCLES"] / w, v.get("SQ_INSTS_VMEM_RD", 0) / w, v.get("SQ_INSTS_VMEM_WR", 0) / w))
    sys.exit(0)
print("%-90s %6s %9s %7s %7s %7s %9s %7s" % ("kernel", "disp", "wcyc/w", "wait%", "winst%", "act%", "valu/w", "mfma/w"))
for k, v in rows[:30]:
    w = max(v["SQ_WAVES"], 1)
    wc = max(v["SQ_WAVE_CYCLES"], 1)
    print("%-90s %6d %9.0f %7.1f %7.1f %7.1f %9.0f %7.1f" % (k, len(disp[k]), wc / w, 100 * v["SQ_WAIT_ANY"] / wc,
                                                            100 * v["SQ_WAIT_INST_ANY"] / wc,
                                                            100 * v["SQ_ACTIVE_INST_ANY"] / wc, v["SQ_INSTS_VALU"] / w,
                                                            v["SQ_INSTS_MFMA"] / w))
