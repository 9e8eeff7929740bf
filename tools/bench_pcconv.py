"""Per-shape timing of svae_pcnn_conv at the c_pixelvae head's geometry (B = 128, 160 filters):
the resnet convs of the three resolutions, their input gradients and the 1x1 nin layers.
    SVAE_PC3=0|1|2 python tools/bench_pcconv.py [--batch B] [--reps R]"""
import argparse
import ctypes
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
L = importlib.import_module("sequential-variational-autoencoder_amd._lib")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--xb", action="store_true", help="bf16 input for the forward (mode 0) convs")
    ap.add_argument("--wgrad", action="store_true", help="time svae_pcnn_conv_wgrad of the forward (mode 0) shapes")
    ap.add_argument("--shape", default=None, help="only res,cin,cout,kh,kw,mode (e.g. 64,160,160,2,3,0)")
    a = ap.parse_args()
    lib = L.lib()
    st = L.stream_ptr()
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    shapes = []
    for res in (64, 32, 16):
        for (kh, kw, pl) in ((2, 3, 1), (2, 2, 1)):
            shapes.append((res, 160, 160, kh, kw, 1, pl, 0))   # c1
            shapes.append((res, 160, 320, kh, kw, 1, pl, 0))   # c2 (2F)
            shapes.append((res, 320, 160, kh, kw, 1, pl, 1))   # c2's input gradient
        shapes.append((res, 160, 160, 1, 1, 0, 0, 0))          # nin
    if a.shape:
        res, cin, cout, kh, kw, mode = (int(v) for v in a.shape.split(","))
        shapes = [(res, cin, cout, kh, kw, 0 if kh == 1 else 1, (kw - 1) // 2 if kw == 3 else kw - 1, mode)]
    tot_t = tot_f = 0.0
    for (res, cin, cout, kh, kw, pt, pl, mode) in shapes:
        n = a.batch
        rows = n * res * res
        if kh == 1 and kw == 1:  # dense view: rows x 1 x 1
            n_, hi, ho = rows, 1, 1
        else:
            n_, hi, ho = n, res, res
        kpad = (cin + 31) // 32 * 32
        xb = a.xb and mode == 0
        x = torch.randn(rows, cin, device="cuda").to(torch.bfloat16 if xb else torch.float32)
        wk = (torch.randn(kh * kw, cout, kpad, device="cuda") * 0.05).to(torch.bfloat16)
        y = torch.empty(rows, cout, device="cuda")
        if a.wgrad:
            if mode != 0:
                continue
            dy = torch.randn(rows, cout, device="cuda")
            dW = torch.empty(kh * kw * cin * cout, device="cuda")
            sc = torch.empty(1 << 26, device="cuda")
            fn = lib.svae_pcnn_conv_wgrad
            db = torch.empty(cout, device="cuda")
            args = (p(x), n_, hi, hi, cin, cin, int(xb), p(dy), cout, 0, ho, ho, cout, kh, kw, 1, pt, pl, mode, p(dW), p(db),
                    p(sc), sc.numel(), st)
        else:
            fn = lib.svae_pcnn_conv
            args = (p(x), n_, hi, hi, cin, cin, int(xb), p(wk), kpad, None, p(y), ho, ho, cout, cout, kh, kw, 1, pt, pl, mode,
                    0, 0, st)
        for _ in range(2):
            L.check(fn(*args))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            L.check(fn(*args))
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        fl = 2.0 * rows * cin * cout * kh * kw
        tot_t += us
        tot_f += fl
        print("res %2d %3d->%3d k%dx%d mode %d: %8.1f us  %7.1f TF/s" % (res, cin, cout, kh, kw, mode, us, fl / us / 1e6),
              flush=True)
    print("%s SVAE_PC3=%s xb=%d total %.1f us, %.1f TF/s" % ("wgrad" if a.wgrad else "conv", os.environ.get("SVAE_PC3", "1"), int(a.xb), tot_t, tot_f / tot_t / 1e6))


if __name__ == "__main__":
    main()
