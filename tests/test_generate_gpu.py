"""Generative mode of the HIP engine (svae_generate) against the oracle's generator chain
(oracle.model.generate) and the committed generative fixtures.  fp32: x_hat_t within 1e-4 rel
(L2) and 1e-3 max-abs (BASELINE north_star decoder-output bound)."""
import glob
import os

import numpy as np
import pytest
import torch

from conftest import pkg_mod
from oracle import model, spec

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _rel(a, b):
    return float(np.linalg.norm(np.ravel(a) - np.ravel(b)) / np.linalg.norm(np.ravel(b)))


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "gen_*.npz"))),
                         ids=lambda p: os.path.basename(p)[:-4])
def test_generate_matches_golden(path):
    g = np.load(path)
    cfg = pkg_mod("config").preset(str(g["preset"]), batch=int(g["batch"]))
    net = pkg_mod("sequential_vae").SequentialVAE(cfg, seed=0)
    xs = net.generate(g["z"])
    torch.cuda.synchronize()
    for t, x in enumerate(xs):
        x = x.cpu().numpy()
        assert _rel(x, g["xhat"][t]) <= 1e-4, t
        assert np.abs(x - g["xhat"][t]).max() <= 1e-3, t


def test_generate_api_and_state():
    cfg = pkg_mod("config").preset("tiny", batch=4)
    net = pkg_mod("sequential_vae").SequentialVAE(cfg, seed=0)
    out = net.generate_mc_samples()
    assert len(out) == cfg.mc_steps + 1
    assert out[0].shape == (4, 32, 32, 3) and (out[0] >= 0).all() and (out[0] < 1).all()
    for x in out[1:]:
        assert x.shape == (4, 32, 32, 3) and np.isfinite(x).all() and np.abs(x).max() <= 1.0 + 1e-6
    with pytest.raises(RuntimeError):  # no training forward state after generate
        net.backward()
    cd = spec.make_config("tiny", batch=4)
    x, tgt, eps = spec.make_inputs(cd)
    net.forward(x, tgt, eps, 1.0)
    net.backward()  # valid again
    torch.cuda.synchronize()
    assert torch.isfinite(net.grads).all()


def test_generate_celeba_bf16_and_fp32():
    """CelebA geometry, both dtypes: finite, in range; bf16 within a loose bound of fp32 on the
    first chain step (bf16 operands, fp32 accumulation)."""
    z = np.random.default_rng(3).standard_normal((2, 8, 12)).astype(np.float32)
    outs = {}
    for dt in ("fp32", "bf16"):
        cfg = pkg_mod("config").preset("celeba", batch=8, mc_steps=2, dtype=dt)
        net = pkg_mod("sequential_vae").SequentialVAE(cfg, seed=0)
        outs[dt] = [x.cpu().numpy() for x in net.generate(z)]
        for x in outs[dt]:
            assert np.isfinite(x).all() and np.abs(x).max() <= 1.0 + 1e-6
    assert _rel(outs["bf16"][0], outs["fp32"][0]) <= 5e-2
    cd = spec.make_config("celeba", batch=8, mc_steps=2)
    _, struct, params = spec.init_params(cd, seed=0, dtype=np.float32)
    ref = model.generate(cd, struct, {k: v.astype(np.float64) for k, v in params.items()}, z)
    assert _rel(outs["fp32"][0], ref[0]) <= 1e-4
