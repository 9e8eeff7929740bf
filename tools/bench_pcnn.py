"""Throughput of the PixelCNN++ head training step on the GPU: forward + NLL +
backward + Adam at the pixelvae.py geometry (64x64, nr_resnet 3, 160 filters, 10 mixtures,
conditioned on a 48-d latent), synthetic U[-1,1] images.  Prints one JSON line.
    python tools/bench_pcnn.py [--batch B] [--steps K] [--warmup W] [--cpu]"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PC = importlib.import_module("sequential-variational-autoencoder_amd.pixelcnn")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu", action="store_true", help="also time the fp32 torch-CPU oracle on one step")
    a = ap.parse_args()
    spec = PC.make_spec(H=64, W=64, K=48)
    net = PC.PixelCNNpp(spec, seed=0)
    rng = np.random.default_rng(0)
    x = torch.tensor(rng.uniform(-1, 1, (a.batch, 64, 64, 3)), dtype=torch.float32, device="cuda")
    h = torch.tensor(rng.normal(size=(a.batch, 48)), dtype=torch.float32, device="cuda")
    net.data_init(x, h)
    for _ in range(a.warmup):
        net.train_step(x, h, lr=1e-4)
    torch.cuda.synchronize()
    net.conv_flops = 0.0
    t0 = time.perf_counter()
    nll = 0.0
    for _ in range(a.steps):
        nll = net.train_step(x, h, lr=1e-4)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    fl = 3.0 * net.conv_flops / a.steps  # forward + input gradient + weight gradient
    line = dict(metric="images/sec (PixelCNN++ head 64x64 fwd+bwd+Adam step)", value=round(a.batch / dt, 2),
                unit="images/sec", ms_per_step=round(dt * 1e3, 3), batch=a.batch, dtype="bf16 MFMA, fp32 accumulate",
                bits_per_dim=round(nll / (a.batch * 64 * 64 * 3 * np.log(2)), 4), conv_tflop_per_step=round(fl / 1e12, 3),
                conv_tflops_achieved=round(fl / dt / 1e12, 2), params=net.n_params,
                config="nr_resnet 3, nr_filters 160, nr_logistic_mix 10, relu, K=48 (pixelvae.py:54-63)")
    if a.cpu:
        from oracle import pcnn as opc
        torch.set_num_threads(min(16, os.cpu_count() or 1))
        params = net.params()
        ospec = opc.make_spec(H=64, W=64, K=48)
        xb, hb = x[:2].cpu().double().numpy(), h[:2].cpu().double().numpy()
        t0 = time.perf_counter()
        opc.loss_and_grads(ospec, params, xb, hb)
        line["cpu_baseline"] = dict(value=round(2 / (time.perf_counter() - t0), 3), unit="images/sec", kind="port",
                                    cores=torch.get_num_threads(),
                                    sample="1 fwd+bwd of 2 images with oracle/pcnn.py (fp64 torch CPU)")
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
