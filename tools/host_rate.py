"""Host enqueue rate vs GPU rate of the training step (is the host the bottleneck?).

For k = 1..K steps enqueued from an empty queue: host time to enqueue them (no sync) and the
wall time until the GPU has drained them. If host_ms/step approaches gpu_ms/step the launch
path (not the kernels) bounds the step.
"""
import importlib
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = "sequential-variational-autoencoder_amd"


def main():
    cfgmod = importlib.import_module(PKG + ".config")
    SV = importlib.import_module(PKG + ".sequential_vae").SequentialVAE
    cfg = cfgmod.preset(sys.argv[1] if len(sys.argv) > 1 else "celeba", dtype="bf16")
    net = SV(cfg, seed=0)
    x = torch.rand(cfg.batch, cfg.height, cfg.width, cfg.channels, device="cuda")

    def step(it):
        net.forward(x, x, None, 1.0 - math.exp(-it / cfg.reg_coeff_rate))
        net.backward()
        net.apply_gradients(cfg.learning_rate, it)

    it = 0
    for _ in range(5):
        it += 1
        step(it)
    torch.cuda.synchronize()
    for k in (1, 2, 5, 10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            it += 1
            step(it)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print("k=%2d host enqueue %.2f ms/step   wall %.2f ms/step" % (k, (t1 - t0) * 1e3 / k, (t2 - t0) * 1e3 / k),
              flush=True)
    # split of the host cost
    torch.cuda.synchronize()
    t0 = time.perf_counter(); net.forward(x, x, None, 0.5); t1 = time.perf_counter()
    net.backward(); t2 = time.perf_counter(); net.apply_gradients(cfg.learning_rate, it + 1); t3 = time.perf_counter()
    torch.cuda.synchronize()
    print("host: forward %.2f ms, backward %.2f ms, adam %.2f ms" % ((t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3))


if __name__ == "__main__":
    main()
