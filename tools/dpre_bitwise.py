"""bf16 mode: the BN-backward outputs (SVAE_DPRE_F32=1 keeps them fp32) and the post-activation
tensors read only by GEMMs (SVAE_ACT_F32=1) stored as bf16 (default) vs fp32 must give bitwise the
same gradients and losses -- every consumer rounds them to bf16 identically.  Runs the engine in a
child process per setting and compares the gradient buffers and the per-step losses.
    python tools/dpre_bitwise.py [preset] [batch] [env var, default SVAE_DPRE_F32]"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, importlib, numpy as np, torch
sys.path.insert(0, %r)
cfg = importlib.import_module("sequential-variational-autoencoder_amd.config").preset(%r, batch=%d, dtype="bf16")
net = importlib.import_module("sequential-variational-autoencoder_amd.sequential_vae").SequentialVAE(cfg, seed=0)
g = torch.Generator(device="cuda"); g.manual_seed(5)
x = torch.rand(cfg.batch, cfg.height, cfg.width, cfg.channels, device="cuda", generator=g) * 2 - 1
eps = torch.randn(cfg.mc_steps, cfg.batch, cfg.latent_dim, device="cuda", generator=g)
net.forward(x, x, eps, 0.7); net.backward(); torch.cuda.synchronize()
st = net.step_stats().cpu().numpy().astype(np.float32).ravel()
np.save(%r, np.concatenate([net.grads.cpu().numpy().ravel(), st]))
'''


def run(preset, batch, f32, out, var="SVAE_DPRE_F32"):
    env = dict(os.environ)
    if f32:  # "NAME" -> NAME=1, or an explicit "NAME=VALUE"
        k, _, v = var.partition("=")
        env[k] = v or "1"
    subprocess.run([sys.executable, "-c", CHILD % (ROOT, preset, batch, out)], env=env, check=True)
    return np.load(out)


if __name__ == "__main__":
    preset = sys.argv[1] if len(sys.argv) > 1 else "celeba"
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    var = sys.argv[3] if len(sys.argv) > 3 else "SVAE_DPRE_F32"
    a = run(preset, batch, False, "/tmp/g_bf.npy", var)
    b = run(preset, batch, True, "/tmp/g_f32.npy", var)
    diff = int(np.sum(a.view(np.uint32) != b.view(np.uint32)))
    print("%s B=%d %s: gradient/loss words differing between bf16 and fp32 storage: %d of %d (max |d| %.3e)" % (
        preset, batch, var, diff, a.size, float(np.abs(a - b).max())))
    sys.exit(0 if diff == 0 else 1)
