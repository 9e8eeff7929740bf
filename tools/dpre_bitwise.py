"""bf16 mode: the BN-backward outputs stored as bf16 (default) vs fp32 (SVAE_DPRE_F32=1) must give
bitwise the same gradients -- every consumer rounds them to bf16 identically.  Runs the engine in
a child process per setting and compares the gradient buffers.
    python tools/dpre_bitwise.py [preset] [batch]"""
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
np.save(%r, net.grads.cpu().numpy())
'''


def run(preset, batch, f32, out):
    env = dict(os.environ)
    if f32:
        env["SVAE_DPRE_F32"] = "1"
    subprocess.run([sys.executable, "-c", CHILD % (ROOT, preset, batch, out)], env=env, check=True)
    return np.load(out)


if __name__ == "__main__":
    preset = sys.argv[1] if len(sys.argv) > 1 else "celeba"
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    a = run(preset, batch, False, "/tmp/g_bf.npy")
    b = run(preset, batch, True, "/tmp/g_f32.npy")
    diff = int(np.sum(a.view(np.uint32) != b.view(np.uint32)))
    print("%s B=%d: gradient words differing between bf16 and fp32 dpre storage: %d of %d (max |d| %.3e)" % (
        preset, batch, diff, a.size, float(np.abs(a - b).max())))
    sys.exit(0 if diff == 0 else 1)
