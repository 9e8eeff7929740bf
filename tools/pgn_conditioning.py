"""Predicted-noise chains are ill-conditioned: a 1e-6 input move shifts the float64 oracle's d loss / d z_t
by percent (relu / lrelu kinks weighted by the NLL's 1/sd^2 .. 1/sd^3).  Prints engine-vs-oracle and
perturbed-vs-unperturbed dz for a homogeneous tiny chain (tests/test_chain_variants_gpu.py bounds on this)."""
import sys, os
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_chain_variants_gpu as T
from conftest import pkg_mod
from oracle import spec, model

over = dict(add_noise_to_chain=True, predict_generator_noise=True, share_theta_weights=True, share_phi_weights=True)
seed, reg, T_ = 2, 0.3, 3
cfg = pkg_mod("config").preset("tiny", batch=4, mc_steps=T_, **over)
net = pkg_mod("sequential_vae").SequentialVAE(cfg, seed=seed)
cd = spec.make_config("tiny", batch=4, mc_steps=T_, add_noise_to_chain=True, predict_generator_noise=True)
x, tgt, eps = spec.make_inputs(cd, seed_x=seed, seed_eps=seed + 1)
noise = spec.make_chain_noise(cd, batch=4, seed=seed + 2)
rng = np.random.default_rng(0)
outs = []
for k in range(4):
    xp = (x + (0 if k == 0 else 1e-6 * rng.standard_normal(x.shape))).astype(np.float32)
    net.forward(xp, xp, eps, reg, noise=noise)
    net.backward()
    torch.cuda.synchronize()
    dz_e = [net.latent(pkg_mod("_lib").BUF_DZ, t).cpu().numpy().astype(np.float64) for t in range(T_)]
    o = T._oracle(net, cd, (True, True), xp, xp, eps, noise, reg)
    outs.append((dz_e, o["dz"]))
    print("k=%d  engine vs oracle dz rel: %s" % (k, ["%.2e" % T._rel(dz_e[t], o["dz"][t]) for t in range(T_)]), flush=True)
for k in range(1, 4):
    print("perturbation %d: engine dz moves %s, oracle dz moves %s" % (
        k, ["%.2e" % T._rel(outs[k][0][t], outs[0][0][t]) for t in range(T_)],
        ["%.2e" % T._rel(outs[k][1][t], outs[0][1][t]) for t in range(T_)]))
