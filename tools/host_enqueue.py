"""Host enqueue cost of the training step: wall time of the launch calls alone (GPU not waited
for) vs the GPU time per step.  python tools/host_enqueue.py [steps]"""
import importlib
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "sequential-variational-autoencoder_amd"
cfgmod = importlib.import_module(PKG + ".config")
SV = importlib.import_module(PKG + ".sequential_vae").SequentialVAE
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
cfg = cfgmod.preset("celeba", dtype="bf16")
net = SV(cfg, seed=0)
x = (torch.rand(cfg.batch, cfg.height, cfg.width, cfg.channels, device="cuda") * 2 - 1).contiguous()


def step(it):
    net.forward(x, x, None, 1.0 - math.exp(-it / cfg.reg_coeff_rate))
    net.backward_apply(cfg.learning_rate, it)


for it in range(1, 6):
    step(it)
torch.cuda.synchronize()
per = []
t0 = time.perf_counter()
for it in range(6, 6 + steps):
    a = time.perf_counter()
    step(it)
    per.append(time.perf_counter() - a)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print("host enqueue per step: mean %.2f ms, min %.2f ms, max %.2f ms" %
      (1e3 * sum(per) / steps, 1e3 * min(per), 1e3 * max(per)))
print("loop %.2f ms/step, drain after loop %.2f ms, total %.2f ms/step" %
      (1e3 * (t1 - t0) / steps, 1e3 * (t2 - t1), 1e3 * (t2 - t0) / steps))
