"""Localise halo-vs-plain differences inside the bf16 step (run on the GPU box).
    python tools/dbg_halo.py            # spawns both variants, prints per-quantity diffs"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = r'''
import sys, numpy as np, torch, importlib
sys.path.insert(0, %r)
cfgmod = importlib.import_module("sequential-variational-autoencoder_amd.config")
SV = importlib.import_module("sequential-variational-autoencoder_amd.sequential_vae").SequentialVAE
from oracle import spec
T = int(sys.argv[2])
cfg = cfgmod.preset("celeba", batch=8, mc_steps=T, dtype="bf16")
net = SV(cfg, seed=0)
cd = spec.make_config("celeba", batch=8, mc_steps=T)
x, tgt, eps = spec.make_inputs(cd, batch=8)
net.forward(x, tgt, eps, 1.0)
net.backward()
torch.cuda.synchronize()
out = {"loss": np.array(net.loss_value())}
for t in range(T):
    out["xhat%%d" %% t] = net.xhat(t).cpu().numpy()
    out["mu%%d" %% t] = net.latent(1, t).cpu().numpy()
    out["sig%%d" %% t] = net.latent(2, t).cpu().numpy()
    out["stats%%d" %% t] = net.copy_out(4, t, 2).cpu().numpy()
for k, v in net.grad_dict().items():
    out["g:" + k] = v
np.savez(sys.argv[1], **out)
'''


def run(no_halo, T):
    out = "/tmp/dbg_%d_%d.npz" % (no_halo, T)
    env = dict(os.environ)
    env["SVAE_NO_HALO"] = "1" if no_halo else "0"
    r = subprocess.run([sys.executable, "-c", SCRIPT % ROOT, out, str(T)], env=env, capture_output=True, text=True)
    if r.returncode:
        print(r.stderr[-3000:])
        sys.exit(1)
    return np.load(out)


for T in (1, 2):
    a, b = run(0, T), run(1, T)
    print("==== T=%d" % T)
    rows = []
    for k in a.files:
        u, v = a[k].astype(np.float64), b[k].astype(np.float64)
        n = np.linalg.norm(v)
        d = np.linalg.norm(u - v) / n if n > 0 else np.linalg.norm(u - v)
        rows.append((d, k))
    for d, k in rows:
        if not k.startswith("g:"):
            print("  %-12s %.3e" % (k, d))
    rows = sorted([r for r in rows if r[1].startswith("g:")], reverse=True)
    for d, k in rows[:25]:
        print("  %.3e %s" % (d, k))
