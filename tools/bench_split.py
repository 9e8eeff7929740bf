"""Time single split-bf16 (dtype bf16x6) gather-GEMM launches on the CelebA B=128 step's shapes.

    python tools/bench_split.py [--iters N] [--check] [--set main|all]

Every forward conv / conv-T of the decoder, encoder and recognition ladders and the input gradient of
each (as the gather it is: a conv's input gradient is the transposed gather and vice versa), weighted
by its launches per step (decoder 8, encoder 7, recognition one T-batched launch of 8 x 128 images).
--check compares every output with an fp64 torch reference (rel L2; the split mode is fp32-grade).
Run a variant build with SVAE_LIB=path/to/lib.so."""
import argparse
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
L = importlib.import_module("sequential-variational-autoencoder_amd._lib")

# (name, n, h_in, cin, cout, stride, transpose, launches per step)
FWD = [
    ("dec.s1.32", 128, 32, 64, 32, 1, 1, 8), ("dec.s1.16", 128, 16, 128, 64, 1, 1, 8),
    ("dec.s1.8", 128, 8, 256, 128, 1, 1, 8), ("dec.s2.16>32", 128, 16, 64, 32, 2, 1, 8),
    ("dec.s2.8>16", 128, 8, 128, 64, 2, 1, 8), ("dec.s2.4>8", 128, 4, 384, 128, 2, 1, 8),
    ("enc.b.32", 128, 32, 32, 32, 1, 0, 7), ("enc.b.16", 128, 16, 64, 64, 1, 0, 7),
    ("enc.b.8", 128, 8, 128, 128, 1, 0, 7), ("enc.a.32>16", 128, 32, 32, 64, 2, 0, 7),
    ("enc.a.16>8", 128, 16, 64, 128, 2, 0, 7), ("enc.c.8>4", 128, 8, 128, 128, 2, 0, 7),
    ("rec.b.32", 1024, 32, 32, 32, 1, 0, 1), ("rec.b.16", 1024, 16, 64, 64, 1, 0, 1),
    ("rec.b.8", 1024, 8, 128, 128, 1, 0, 1), ("rec.a.32>16", 1024, 32, 32, 64, 2, 0, 1),
    ("rec.a.16>8", 1024, 16, 64, 128, 2, 0, 1),
]


def dgrad_shape(name, n, h, cin, cout, s, tr, cnt):
    ho = h * s if tr else h // s
    return ("d:" + name, n, ho, cout, cin, s, 1 - tr, cnt)


ALL = FWD + [dgrad_shape(*f) for f in FWD]
MAIN = [f for f in ALL if f[0] in ("dec.s1.32", "dec.s1.16", "dec.s1.8", "d:dec.s1.32", "d:dec.s1.16",
                                   "d:dec.s1.8", "rec.b.32", "d:enc.b.16", "dec.s2.8>16", "d:enc.a.32>16")]


H16 = False  # --h16: the shadows also hold the scaled fp16 pair (halo_kw NS = 2, path bit 5)


def split3(w):
    p0 = w.to(torch.bfloat16)
    r = w - p0.float()
    p1 = r.to(torch.bfloat16)
    p2 = (r - p1.float()).to(torch.bfloat16)
    pl = [p0, p1, p2]
    if H16:  # csrc/common.h h16_pair: w * 2^10 as fp16 hi / lo (stored as raw 16-bit words)
        s = w * 1024.0
        h0 = s.to(torch.float16)
        h1 = (s - h0.float()).to(torch.float16)
        pl += [h0.view(torch.bfloat16), h1.view(torch.bfloat16)]
    return torch.stack(pl)


def path_bits():
    return 2 | 16 | (32 if H16 else 0)


def ref_conv(x, w_tnk, cin, cout, s, tr):
    """fp64 TF-SAME conv (transpose=0) / conv_transpose (1) of NHWC x with w[tap][cout][cin]."""
    import torch.nn.functional as F
    xd = x.double().permute(0, 3, 1, 2)
    wd = w_tnk.double().view(4, 4, cout, cin)
    n, _, h, _ = xd.shape
    if not tr:
        ho = h // s
        pad = max((ho - 1) * s + 4 - h, 0)
        pb = pad // 2
        xp = F.pad(xd, (pb, pad - pb, pb, pad - pb))
        y = F.conv2d(xp, wd.permute(2, 3, 0, 1), stride=s)
    else:
        ho = h * s
        pad = max((h - 1) * s + 4 - ho, 0)
        pb = pad // 2
        y = F.conv_transpose2d(xd, wd.permute(3, 2, 0, 1), stride=s)  # [cin, cout, kh, kw] -> in=cin
        y = y[:, :, pb:pb + ho, pb:pb + ho]
    return y.permute(0, 2, 3, 1)


def stamps(names):
    """Per-wave phase stamps (s_memtime, halo_kw.hip KW_STAMP) of one launch per shape: 0 entry,
    1 prologue issued, 2+2c chunk c staged (after its barrier), 3+2c chunk c MFMAs done, 10 chunk loop
    done, 11 partial tiles in LDS, 12 epilogue done."""
    import numpy as np
    scratch = torch.zeros(64 << 20, device="cuda")
    for (name, n, h, cin, cout, s, tr, cnt) in ALL:
        if name not in names:
            continue
        x = torch.randn(n, h, h, cin, device="cuda")
        wp = split3(torch.randn(16, cout, cin, device="cuda") * 0.05).contiguous()
        ho = h * s if tr else h // s
        y = torch.empty(n, ho, ho, cout, device="cuda")
        a = (L.ptr(x), n, h, cin, L.ptr(wp), cout, s, tr, path_bits(), L.ptr(y), L.ptr(scratch), scratch.numel() * 4,
             L.stream_ptr())
        for _ in range(3):
            L.lib().svae_op_gather_bf16(*a)
        torch.cuda.synchronize()
        scratch.zero_()
        L.lib().svae_op_gather_bf16(*a)
        torch.cuda.synchronize()
        st = scratch.view(torch.int64).cpu().numpy()
        nz = np.nonzero(st)[0]
        nblk = (nz.max() // 64 + 1) if len(nz) else 0
        t = st[:nblk * 64].reshape(nblk, 4, 16).astype(np.float64)
        t0 = t[:, :, 0].min()
        span = t[:, :, 12].max() - t0
        print("%s %s: %d blocks, span %.0f clk" % (name, (n, h, cin, cout, s, tr), nblk, span))
        names_ = {1: "prologue", 2: "stage0", 3: "mfma0", 4: "stage1", 5: "mfma1", 6: "stage2", 7: "mfma2",
                  8: "stage3", 9: "mfma3", 10: "loopend", 11: "red", 12: "epi", 13: "args", 14: "issued",
                  15: "stores"}
        rows = []
        for i in range(1, 16):
            cur = t[:, :, i]
            ok = cur > 0
            if ok.any():
                rows.append(((cur - t[:, :, 0])[ok].mean(), i))
        for off, i in sorted(rows):
            print("  %-9s at %8.0f clk after entry" % (names_[i], off))
        life = (t[:, :, 12] - t[:, :, 0]).mean()
        starts = np.sort(t[:, 0, 0] - t0)
        print("  lifetime mean %.0f clk; block starts p25/p50/p75 %.0f/%.0f/%.0f" % (
            life, np.percentile(starts, 25), np.percentile(starts, 50), np.percentile(starts, 75)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--set", default="all", choices=["all", "main"])
    ap.add_argument("--h16", action="store_true", help="the scaled fp16 planes (halo_kw NS = 2)")
    ap.add_argument("--stamps", default=None,
                    help="comma-separated shape names: per-phase stamps of a -DSVAE_EXP_STAMPS build (halo_kw)")
    args = ap.parse_args()
    global H16
    H16 = args.h16
    if args.stamps:
        return stamps(args.stamps.split(","))
    torch.manual_seed(0)
    shapes = ALL if args.set == "all" else MAIN
    scratch = torch.empty(64 << 20, device="cuda")
    tot_f = tot_t = 0.0
    for (name, n, h, cin, cout, s, tr, cnt) in shapes:
        x = torch.randn(n, h, h, cin, device="cuda")
        w = torch.randn(16, cout, cin, device="cuda") * 0.05
        wp = split3(w).contiguous()
        ho = h * s if tr else h // s
        y = torch.empty(n, ho, ho, cout, device="cuda")
        a = (L.ptr(x), n, h, cin, L.ptr(wp), cout, s, tr, path_bits(), L.ptr(y), L.ptr(scratch), scratch.numel() * 4,
             L.stream_ptr())
        rc = L.lib().svae_op_gather_bf16(*a)
        if rc != 0:
            print("%-14s %s: not eligible (%d)" % (name, (n, h, cin, cout, s, tr), rc))
            continue
        err = None
        if args.check:
            torch.cuda.synchronize()
            r = ref_conv(x, w, cin, cout, s, tr)
            err = float((y.double() - r).norm() / r.norm())
        for _ in range(3):
            L.lib().svae_op_gather_bf16(*a)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            L.lib().svae_op_gather_bf16(*a)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.iters
        fl = 2.0 * n * ho * ho * cout * cin * (4 if (tr and s == 2) else 16)
        tot_f += fl * cnt
        tot_t += us * cnt
        print("%-14s %-28s %8.2f us %7.1f TF/s useful x%d%s" % (name, (n, h, cin, cout, s, tr), us, fl / us / 1e6, cnt,
                                                           "" if err is None else "  rel %.2e" % err), flush=True)
    k = 3 if H16 else 6
    print("per step: %.1f us, %.1f TF/s useful (%.1f issued)" % (tot_t, tot_f / tot_t / 1e6, k * tot_f / tot_t / 1e6))


if __name__ == "__main__":
    main()
