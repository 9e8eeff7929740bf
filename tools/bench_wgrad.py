"""Time single bf16 weight-gradient launches (svae_op_wgrad_bf16) on the CelebA B=128 layer
shapes of the stride-1 halo weight-GEMM (wgrad_halo_kernel<32,1>, bench.py's dominant kernel)
and its stride-2 sibling.  Prints avg us per call (kernel + slab reduce when split) and TFLOP/s
of the algorithmic 2*16*M*N*pixels.
    python tools/bench_wgrad.py [iters] [path]      path 2 = halo (default), 0 = tap-merged"""
import ctypes
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
L = importlib.import_module("sequential-variational-autoencoder_amd._lib")

SHAPES = [  # (n, h_in, cin, cout, stride, transpose, name)
    (128, 32, 64, 32, 1, 1, "dec s1 lvl0 conv-T"), (128, 16, 128, 64, 1, 1, "dec s1 lvl1 conv-T"),
    (128, 8, 256, 128, 1, 1, "dec s1 lvl2 conv-T"),
    (128, 32, 32, 32, 1, 0, "enc b lvl0 conv"), (128, 16, 64, 64, 1, 0, "enc b lvl1 conv"),
    (128, 8, 128, 128, 1, 0, "enc b lvl2 conv"),
    (1024, 32, 32, 32, 1, 0, "inf b lvl0 x8"), (1024, 16, 64, 64, 1, 0, "inf b lvl1 x8"),
    (1024, 8, 128, 128, 1, 0, "inf b lvl2 x8"),
    (128, 64, 3, 32, 2, 0, "enc a lvl0 conv s2"), (128, 32, 32, 64, 2, 0, "enc a lvl1 conv s2"),
    (128, 16, 64, 128, 2, 0, "enc a lvl2 conv s2"), (128, 16, 64, 32, 2, 1, "dec s2 lvl0 conv-T"),
    (128, 8, 128, 64, 2, 1, "dec s2 lvl1 conv-T"), (128, 4, 384, 128, 2, 1, "dec s2 lvl2 conv-T"),
]


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    path = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    store = sys.argv[3] if len(sys.argv) > 3 else "fp32"  # "step": the engine's bf16 operand storage
    torch.manual_seed(0)
    scratch = torch.empty(64 << 20, device="cuda")
    tot_f = tot_t = 0.0
    for (n, h, cin, cout, s, tr, name) in SHAPES:
        ho = h * s if tr else h // s
        # "step": dY (BN-backward output) is bf16; x is bf16 except the decoder s1 conv-T's concat input
        xb = store == "step" and not (tr and s == 1)
        db = store == "step" and cin % 4 == 0
        x = torch.randn(n, h, h, cin, device="cuda").to(torch.bfloat16 if xb else torch.float32)
        dy = torch.randn(n, ho, ho, cout, device="cuda").to(torch.bfloat16 if db else torch.float32)
        dw = torch.empty(16 * cin * cout, device="cuda")
        p2 = path | (16 if xb else 0) | (32 if db else 0)
        args = (ctypes.c_void_p(x.data_ptr()), n, h, cin, ctypes.c_void_p(dy.data_ptr()), cout, s, tr, p2,
                L.ptr(dw), L.ptr(scratch), scratch.numel() * 4, L.stream_ptr())
        L.check(L.lib().svae_op_wgrad_bf16(*args))
        for _ in range(3):
            L.lib().svae_op_wgrad_bf16(*args)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            L.lib().svae_op_wgrad_bf16(*args)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / iters
        pix = n * (h * h if tr else ho * ho)
        fl = 2.0 * 16 * cin * cout * pix
        tot_f += fl
        tot_t += us
        print("%-22s %-26s %9.2f us  %8.1f TFLOP/s" % (name, str((n, h, cin, cout, s, tr)), us, fl / us / 1e6),
              flush=True)
    print("total %.1f us, %.1f TFLOP/s" % (tot_t, tot_f / tot_t / 1e6))


if __name__ == "__main__":
    main()
