"""Time the small-N stride-2 conv-T gather (layer-0 conv input gradient, CelebA B=128) in
isolation through svae_op_conv_dgrad."""
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
L = importlib.import_module("sequential-variational-autoencoder_amd._lib")

for n in (128, 64, 32):
    dy = torch.randn(n, 32, 32, 32, device="cuda")
    w = torch.randn(4, 4, 3, 32, device="cuda") * 0.05
    dx = torch.empty(n, 64, 64, 3, device="cuda")
    args = (L.ptr(dy), n, 64, 3, L.ptr(w), 32, 2, 0, L.ptr(dx), L.stream_ptr())
    for _ in range(3):
        L.check(L.lib().svae_op_conv_dgrad(*args))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        L.lib().svae_op_conv_dgrad(*args)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 20
    mb = (dy.numel() + dx.numel()) * 4 / 1e6
    print("n=%d: %.2f us  (%.1f MB -> %.2f TB/s)" % (n, us, mb, mb / us / 1e6 * 1e6 / 1e6))
