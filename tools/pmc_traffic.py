"""Per-kernel HBM traffic from two rocprofv3 PMC passes (CSV output).

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d <fetch_dir> -o run -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d <write_dir> -o run -- python3 bench.py ...
    python tools/pmc_traffic.py <fetch_dir> <write_dir> <out.json> [label]

FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  FETCH_SIZE is corrected per kernel by the
calibrated rule of fetch_rule() below (tools/calib/fetch_calib.hip, profiles/r03_fetch_calib.txt:
whole-128-B-line reads count half, 64-B-segment reads count exactly); WRITE_SIZE is taken as is.
Each kernel's entry records the rule applied.  The two counters cannot share a pass (TCC slots),
hence two runs of the same command; per-kernel averages are matched by kernel name.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _short(name):
    name = name.strip()
    if name.startswith("void "):
        name = name[5:]
    name = name.replace("(anonymous namespace)::", "")
    depth = 0
    for i, ch in enumerate(name):  # cut the argument list, keep template arguments
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return name[:i]
    return name


# Calibration (tools/calib/fetch_calib.hip, profiles/r03_fetch_calib.txt, 768 MiB streamed past the
# Infinity Cache): FETCH_SIZE counts HALF the bytes of fully coalesced reads of whole 128-B lines,
# at 16, 8 and 4 B per lane alike, and EXACTLY the bytes of reads that take 64-B halves of lines.
# So the factor follows each operand's contiguous span per row, not the lane width:
#   >= 128 B per row segment -> x2;  64 B segments -> x1.
# kernels whose HBM operand rows are >= 128 B (fp32 rows of >= 32 channels, 16 B/lane streams)
WIDE16 = ("wgrad_halo_kernel", "igemm_halo_kernel", "igemm_bf16_kernel", "wgrad_bf16_kernel", "igemm_fwd_kernel",
          "wgrad_kernel", "wgrad_reduce_kernel<", "splitk_reduce_kernel", "bn_apply_kernel", "bn_bwd_reduce_kernel",
          "bn_bwd_apply_kernel", "adam_kernel", "shadow_n_kernel", "shadow_t_kernel", "loss_reduce_kernel",
          "dense_kw_kernel")


def _targs(k, name):
    return [t.strip() for t in k[len(name) + 1:k.rindex(">")].split(",")]


def _wh2_factor(targs):
    """wgrad_halo2_kernel<WO, CP, KYR, WN, WK, DB, OPB, NSW, PF, S[, NSP]>: the G window rows are 32
    channels (64 B bf16 -> x1, 128 B fp32 -> x2), the D rows 32*WN*NSW channels; the factor is the
    byte-weighted harmonic mix of the two operands' factors (algorithmic bytes per chunk)."""
    WO, CP, WN, OPB, NSW = int(targs[0]), int(targs[1]), int(targs[3]), int(targs[6]), int(targs[7])
    S = int(targs[9]) if len(targs) > 9 else 1
    per = WO * WO
    img = 1 if CP <= per else CP // per
    R = CP // WO if CP <= per else WO
    npix = img * (S * (R - 1) + 4) * (S * (WO - 1) + 4)
    gb, db = (2 if OPB & 1 else 4), (2 if OPB & 2 else 4)
    DN = 32 * WN * NSW
    g_bytes, d_bytes = npix * 32 * gb, CP * DN * db
    fg = 2.0 if 32 * gb >= 128 else 1.0
    fd = 2.0 if DN * db >= 128 else 1.0
    return (g_bytes + d_bytes) / (g_bytes / fg + d_bytes / fd)


def fetch_rule(kernel):
    k = kernel.replace("(anonymous namespace)::", "").split("(")[0]
    if k.startswith("igemm_halo_kw_kernel<"):
        abf = _targs(k, "igemm_halo_kw_kernel")[3] == "true"
        if abf:
            return 1.0, "FETCH_SIZE x1 (bf16 window rows of 32 channels = 64-B line halves: calibrated exact)"
        return 2.0, "FETCH_SIZE x2 (fp32 window rows of 32 channels = whole 128-B lines: calibrated half-count)"
    if k.startswith("wgrad_halo2_kernel<"):
        f = _wh2_factor(_targs(k, "wgrad_halo2_kernel"))
        return f, "FETCH_SIZE x%.3f (G window / D row mix of 64-B (x1) and >= 128-B (x2) segments, calibrated)" % f
    for w in WIDE16:
        if k.startswith(w) or (w.endswith("<") and k.startswith(w[:-1])):
            return 2.0, "FETCH_SIZE x2 (rows of >= 128 B: calibrated half-count)"
    return 1.0, "FETCH_SIZE x1 (row segments below 128 B or unknown: as counted)"


def _load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit("no counter_collection.csv under %s" % d)
    acc = defaultdict(lambda: [0, 0.0])
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter:
                    continue
                a = acc[_short(row["Kernel_Name"])]
                a[0] += 1
                a[1] += float(row["Counter_Value"])
    return acc


def main():
    fdir, wdir, out = sys.argv[1:4]
    label = sys.argv[4] if len(sys.argv) > 4 else ""
    fe, wr = _load(fdir, "FETCH_SIZE"), _load(wdir, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fe) & set(wr)):
        nf, kf = fe[k]
        nw, kw = wr[k]
        mult, rule = fetch_rule(k)
        fetch = mult * kf * 1024.0 / nf
        write = kw * 1024.0 / nw
        kernels[k] = dict(dispatches_fetch_pass=nf, dispatches_write_pass=nw, fetch_rule=rule,
                          fetch_bytes_per_launch=round(fetch), write_bytes_per_launch=round(write),
                          hbm_bytes_per_launch=round(fetch + write))
    doc = dict(label=label, source="rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), csv",
               correction="per kernel (fetch_rule, calibrated on known byte counts: tools/calib/fetch_calib.hip, "
                          "profiles/r03_fetch_calib.txt): FETCH_SIZE x2 where the operand rows are whole 128-B lines "
                          "(counted half), x1 for 64-B line halves (counted exactly), byte-weighted mixes for the "
                          "weight-GEMMs; each kernel's fetch_rule names its factor; KiB->bytes x1024",
               kernels=kernels)
    with open(out, "w") as fh:
        json.dump(doc, fh, indent=1, sort_keys=True)
    top = sorted(kernels.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"] * kv[1]["dispatches_fetch_pass"])
    for k, v in top[:15]:
        print("%-60s %6d  %10.2f MB/launch" % (k[:60], v["dispatches_fetch_pass"], v["hbm_bytes_per_launch"] / 1e6))


if __name__ == "__main__":
    main()
