"""Probe: how much would capturing the whole training step in a hipGraph save?

Captures one bench step (forward + backward_apply) with torch.cuda.graph on a side stream and
replays it; compares ms/step with the eager enqueue of the same step.  The replay repeats the
captured Philox offset and Adam step (timing only: the values are not what training needs).

    python tools/graph_probe.py [--steps 30]
"""
import argparse
import importlib
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "sequential-variational-autoencoder_amd"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--config", default="celeba")
    args = ap.parse_args()
    cfgmod = importlib.import_module(PKG + ".config")
    SV = importlib.import_module(PKG + ".sequential_vae").SequentialVAE
    cfg = cfgmod.preset(args.config, dtype="bf16")
    net = SV(cfg, seed=0)
    g = torch.Generator(device="cuda")
    g.manual_seed(1234)
    lo, hi = cfg.range
    x = (torch.rand(cfg.batch, cfg.height, cfg.width, cfg.channels, device="cuda", generator=g) * (hi - lo) + lo)

    def step(it):
        net.forward(x, x, None, 1.0 - math.exp(-it / cfg.reg_coeff_rate))
        net.backward_apply(cfg.learning_rate, it)

    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for it in range(1, 6):
            step(it)
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        t0 = time.perf_counter()
        for it in range(6, 6 + args.steps):
            step(it)
        torch.cuda.synchronize()
        eager = (time.perf_counter() - t0) / args.steps * 1e3
    print("eager   %.3f ms/step  %.1f img/s" % (eager, cfg.batch / eager * 1e3), flush=True)

    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        step(100)
    torch.cuda.synchronize()
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        graph.replay()
    torch.cuda.synchronize()
    rep = (time.perf_counter() - t0) / args.steps * 1e3
    print("graph   %.3f ms/step  %.1f img/s  (%.1f%% of eager)" % (rep, cfg.batch / rep * 1e3, 100 * rep / eager),
          flush=True)
    print("loss after replays", net.loss_value(), flush=True)


if __name__ == "__main__":
    main()
