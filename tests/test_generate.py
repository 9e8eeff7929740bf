"""Generative mode of the oracle (oracle.model.generate; sequential_vae.py:947-952, :1025,
generate_mc_samples :1393-1428) -- CPU checks.

The generative branch reuses the training branch's variables (reuse=True, :1070-1073), so the
generator fed with the training chain's own latents z_t = mu_t + sigma_t eps_t must reproduce the
training chain's x_hat_t exactly; and the committed generative fixtures re-derive bit-for-bit."""
import glob
import os

import numpy as np
import pytest

from oracle import model, spec

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("preset,batch", [("tiny", 4), ("mnist_1step", 4)])
def test_generator_on_training_latents_reproduces_training_chain(preset, batch):
    cfg = spec.make_config(preset, batch=batch)
    _, struct, params = spec.init_params(cfg, seed=0)
    x, tgt, eps = spec.make_inputs(cfg)
    o = model.forward_backward(cfg, struct, params, x, tgt, eps, 1.0, want_grads=False)
    xs = model.generate(cfg, struct, params, np.stack(o["z"]))
    for t in range(cfg["mc_steps"]):
        np.testing.assert_array_equal(xs[t], o["xhat"][t])


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "gen_*.npz"))),
                         ids=lambda p: os.path.basename(p)[:-4])
def test_generate_golden(path):
    g = np.load(path)
    cfg = spec.make_config(str(g["preset"]), batch=int(g["batch"]))
    _, struct, params = spec.init_params(cfg, seed=0, dtype=np.float32)
    params = {k: v.astype(np.float64) for k, v in params.items()}
    xs = np.stack(model.generate(cfg, struct, params, g["z"]))
    np.testing.assert_allclose(xs, g["xhat"], rtol=0, atol=1e-12)
