"""Per-kernel HBM traffic from two rocprofv3 PMC passes (CSV output).

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d <fetch_dir> -o run -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d <write_dir> -o run -- python3 bench.py ...
    python tools/pmc_traffic.py <fetch_dir> <write_dir> <out.json> [label]

FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  MI355X_MICROARCH.md (HBM section): on
gfx950 FETCH_SIZE reports 1/2 of the bytes of WIDE (16 B/lane) coalesced streaming reads, so it
is doubled only for kernels whose HBM operand loads are 16 B/lane (WIDE16 below, from the
kernel sources); other access widths are uncalibrated and are reported as counted ("x1,
uncalibrated").  WRITE_SIZE is taken as is.  Each kernel's entry records the rule applied.  The two counters cannot share a pass (TCC slots),
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


# kernels whose operand loads from HBM are 16 B per lane (f32x4 / bf16x8 / int4 vectors)
WIDE16 = ("wgrad_halo_kernel", "igemm_halo_kernel", "igemm_bf16_kernel", "wgrad_bf16_kernel", "igemm_fwd_kernel",
          "wgrad_kernel", "wgrad_reduce_kernel<", "splitk_reduce_kernel", "bn_apply_kernel", "bn_bwd_reduce_kernel",
          "bn_bwd_apply_kernel", "adam_kernel", "shadow_n_kernel", "shadow_t_kernel", "loss_reduce_kernel")


# kernels whose operand width follows their storage template parameter (opload.h): OPB (last
# template argument at OPB_POS) 0 = both operands fp32 (16 B/lane loads), else a bf16 operand loads 8 B/lane
OPB_POS = {"wgrad_halo2_kernel": 6, "wgrad_halo_kernel": 2}
# 16 B/lane whatever the storage (8 fp32 = two 16-B loads, 8 bf16 = one)
WIDE16_ANY = ("igemm_halo_kw_kernel",)


def fetch_rule(kernel):
    k = kernel.replace("(anonymous namespace)::", "").split("(")[0]
    for w in WIDE16_ANY:
        if k.startswith(w):
            return 2.0, "FETCH_SIZE x2 (16 B/lane loads: gfx950 half-count)"
    for w, pos in OPB_POS.items():
        if k.startswith(w + "<"):
            targs = k[len(w) + 1:].rstrip(">").split(",")
            opb = targs[pos].strip() if pos < len(targs) else targs[-1].strip()
            if opb == "0":
                return 2.0, "FETCH_SIZE x2 (fp32 operands, 16 B/lane loads: gfx950 half-count)"
            return 1.0, "FETCH_SIZE x1 (a bf16 operand loads 8 B/lane: uncalibrated, as counted)"
    for w in WIDE16:
        if k.startswith(w) or (w.endswith("<") and k.startswith(w[:-1])):
            return 2.0, "FETCH_SIZE x2 (16 B/lane loads: gfx950 half-count)"
    return 1.0, "FETCH_SIZE x1 (loads narrower than 16 B/lane: uncalibrated, as counted)"


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
               correction="per kernel (fetch_rule): FETCH_SIZE x2 only for 16 B/lane loads (gfx950 half-count), "
                          "x1 otherwise (uncalibrated); KiB->bytes x1024",
               kernels=kernels)
    with open(out, "w") as fh:
        json.dump(doc, fh, indent=1, sort_keys=True)
    top = sorted(kernels.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"] * kv[1]["dispatches_fetch_pass"])
    for k, v in top[:15]:
        print("%-60s %6d  %10.2f MB/launch" % (k[:60], v["dispatches_fetch_pass"], v["hbm_bytes_per_launch"] / 1e6))


if __name__ == "__main__":
    main()
