"""Generate the golden fixtures under tests/golden/ from the fp64 oracle (oracle/model.py).

The reference (TF 1.x, tf.contrib) cannot run in this image and ships no tests or
vectors, so these fixtures are regression anchors produced by the
CPU restatement, not reference outputs: parity stays "unpinned" by the reference.
Weights are not stored; they come from the seeded splitmix64 generator
(oracle/weightgen.py, re-implemented independently in the product's weights.py).

    python tools/make_golden.py            # rewrites tests/golden/*.npz

Each .npz holds (all float64 unless noted, no pickled objects):
  x, target [B,H,W,C] f32, eps [T,B,Dz] f32, reg
  loss, final_loss, recon [T], kl [T], recon_img [T,B], kl_img [T,B], elbo_img [B]
  mu, sig [T,B,Dz]
  xhat_final [B,H,W,C]; xhat_norm [T]; xhat_sample [T,S] (every k-th element of x_hat_t)
  grad_names (unicode), grad_norm [P]; small_names, small_offsets, small_grads (tensors <= 1024 elems)
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import model, spec  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")

CASES = {
    # name: (preset, overrides, reg)
    "tiny_b4": ("tiny", dict(batch=4), 1.0),
    "tiny_b4_reg2e-4": ("tiny", dict(batch=4), 2e-4),
    "mnist_1step_b4": ("mnist_1step", dict(batch=4), 1.0),
    "celeba_b4": ("celeba", dict(batch=4), 1.0),
    "lsun_b4": ("lsun", dict(batch=4), 1.0),
}
# generative-mode fixtures (oracle.model.generate): z ~ N(0,1) PCG64 seed 2, [T,B,Dz]
GEN_CASES = {
    "gen_tiny_b4": ("tiny", dict(batch=4)),
    "gen_mnist_1step_b4": ("mnist_1step", dict(batch=4)),
}
SAMPLES = 512
SMALL = 1024


def make(name):
    preset, over, reg = CASES[name]
    cfg = spec.make_config(preset, **over)
    # fp32-rounded weights (what any fp32 implementation holds), evaluated in float64
    table, struct, params = spec.init_params(cfg, seed=0, dtype=np.float32)
    params = {k: v.astype(np.float64) for k, v in params.items()}
    x, tgt, eps = spec.make_inputs(cfg)
    t0 = time.time()
    o = model.forward_backward(cfg, struct, params, x, tgt, eps, reg, want_grads=True)
    dt = time.time() - t0
    T = cfg["mc_steps"]
    xh = np.stack(o["xhat"])
    flat = xh.reshape(T, -1)
    step = max(1, flat.shape[1] // SAMPLES)
    names = [p["name"] for p in table]
    small = [n for n in names if o["grads"][n].size <= SMALL]
    offs = np.cumsum([0] + [o["grads"][n].size for n in small])
    rec = dict(
        preset=np.array(preset), reg=np.float64(reg), batch=np.int64(cfg["batch"]),
        x=x, target=tgt, eps=eps,
        loss=np.float64(o["loss"]), final_loss=np.float64(o["final_loss"]),
        recon=np.array(o["recon"]), kl=np.array(o["kl"]),
        recon_img=np.stack(o["recon_img"]), kl_img=np.stack(o["kl_img"]), elbo_img=o["elbo_img"],
        mu=np.stack(o["mu"]), sig=np.stack(o["sig"]),
        xhat_final=xh[-1], xhat_norm=np.linalg.norm(flat, axis=1), xhat_sample=flat[:, ::step][:, :SAMPLES],
        xhat_sample_stride=np.int64(step),
        grad_names=np.array(names), grad_norm=np.array([np.linalg.norm(o["grads"][n]) for n in names]),
        small_names=np.array(small), small_offsets=offs.astype(np.int64),
        small_grads=np.concatenate([o["grads"][n].ravel() for n in small]),
    )
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **rec)
    print("%-18s loss=%.10f  %.1fs  %d KB" % (name, o["loss"], dt, os.path.getsize(path) // 1024))


def make_gen(name):
    preset, over = GEN_CASES[name]
    cfg = spec.make_config(preset, **over)
    table, struct, params = spec.init_params(cfg, seed=0, dtype=np.float32)
    params = {k: v.astype(np.float64) for k, v in params.items()}
    z = np.random.default_rng(2).standard_normal((cfg["mc_steps"], cfg["batch"], cfg["latent_dim"])).astype(np.float32)
    xs = model.generate(cfg, struct, params, z)
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, preset=np.array(preset), batch=np.int64(cfg["batch"]), z=z, xhat=np.stack(xs))
    print("%-18s |x_T|=%.6f  %d KB" % (name, np.linalg.norm(xs[-1]), os.path.getsize(path) // 1024))


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    for n in (sys.argv[1:] or list(CASES) + list(GEN_CASES)):
        (make_gen if n in GEN_CASES else make)(n)
