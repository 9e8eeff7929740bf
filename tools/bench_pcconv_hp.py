"""Per-shape timing of the split mode's fused fp16-plane conv (svae_pcnn_conv_planes with two scaled fp16
planes, pc_conv3 HP / the row-staged pc_conv3r) at the c_pixelvae head's geometry (B = 128, 160 filters):
the resnet convs of the three resolutions, their input gradients and the 1x1 nin layers.  Also checks the
result against the first library's output (bitwise expected between pc_conv3 HP and pc_conv3r).
    SVAE_LIB=... python tools/bench_pcconv_hp.py [--batch B] [--reps R]   (knobs build: SVAE_PC_RS=0|1)"""
import argparse
import ctypes
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
L = importlib.import_module("sequential-variational-autoencoder_amd._lib")


def shapes():
    out = []
    for res in (64, 32, 16):
        for (kh, kw, pl) in ((2, 3, 1), (2, 2, 1)):
            out.append((res, 160, 160, kh, kw, 1, pl, 0))   # c1
            out.append((res, 160, 320, kh, kw, 1, pl, 0))   # c2 (2F)
            out.append((res, 320, 160, kh, kw, 1, pl, 1))   # c2's input gradient
            out.append((res, 160, 160, kh, kw, 1, pl, 1))   # c1's input gradient
        out.append((res, 160, 160, 1, 1, 0, 0, 0))          # nin
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--save", default=None, help="write the outputs (.pt) for a bitwise comparison")
    ap.add_argument("--compare", default=None, help="compare with outputs saved by --save")
    a = ap.parse_args()
    lib = L.lib()
    st = L.stream_ptr()
    p = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    ref = torch.load(a.compare, weights_only=True) if a.compare else None
    saved = {}
    tot_t = tot_f = 0.0
    for (res, cin, cout, kh, kw, pt, pl, mode) in shapes():
        n = a.batch
        rows = n * res * res
        n_, hi, ho = (rows, 1, 1) if kh == 1 and kw == 1 else (n, res, res)
        taps = kh * kw
        kpad = (cin + 31) // 32 * 32
        x = torch.rand(rows, cin, device="cuda", generator=g) * 2 - 1
        xs = torch.empty(2, rows, cin, dtype=torch.bfloat16, device="cuda")
        xsc = torch.empty(2, device="cuda")
        L.check(lib.svae_pcnn_split_planes(p(x), rows, cin, cin, 2, p(xs), cin, 1, p(xsc), st))
        V = torch.randn(taps, cin, cout, device="cuda", generator=g) * 0.05
        gg = torch.rand(cout, device="cuda", generator=g) + 0.5
        norm = torch.empty(cout, device="cuda")
        kd = (cout + 31) // 32 * 32
        wkf = torch.empty(2 * taps * cout * kpad, dtype=torch.bfloat16, device="cuda")
        wkd = torch.empty(2 * taps * cin * kd, dtype=torch.bfloat16, device="cuda")
        wsc = torch.empty(2, device="cuda")
        L.check(lib.svae_pcnn_wnorm_planes(p(V), p(gg), taps, cin, cout, p(norm), p(wkf), kpad, p(wkd), kd, 2, p(wsc), st))
        y = torch.empty(rows, cout, device="cuda")
        args = (p(xs), n_, hi, hi, cin, cin, 1, rows * cin, p(wkf), kpad, 2, p(xsc), p(wsc), None, p(y), ho, ho, cout,
                cout, kh, kw, 1, pt, pl, mode, 0, 0, st)
        fn = lib.svae_pcnn_conv_planes
        for _ in range(2):
            L.check(fn(*args))
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn(*args)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        fl = 2.0 * rows * cout * cin * taps
        key = "%d_%d_%d_%dx%d_m%d" % (res, cin, cout, kh, kw, mode)
        cmp = ""
        if ref is not None:
            d = (y - ref[key].cuda()).abs().max().item()
            cmp = " max|diff| vs saved %.3g" % d
        if a.save:
            saved[key] = y.cpu()
        print("%-22s %9.1f us %7.1f TF/s useful%s" % (key, us, fl / us / 1e6, cmp), flush=True)
        tot_t += us
        tot_f += fl
    print("all shapes: %.1f us, %.1f TF/s useful" % (tot_t, tot_f / tot_t / 1e6))
    if a.save:
        torch.save(saved, a.save)


if __name__ == "__main__":
    main()
