"""The committed golden fixtures (tests/golden/*.npz, made by tools/make_golden.py) against
a fresh run of the fp64 oracle and the seeded input/weight generators.

The reference ships no vectors (TF 1.x, no tests, cannot run here), so
these fixtures pin the oracle against itself across commits/machines: a change to the
restatement, the weight stream (oracle/weightgen.py) or the input recipe shows up here.
"""
import glob
import os

import numpy as np
import pytest

from oracle import model, spec

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FILES = sorted(f for f in glob.glob(os.path.join(GOLD, "*.npz")) if not os.path.basename(f).startswith("gen_"))


def _rel(a, b):
    return float(np.linalg.norm(np.ravel(a) - np.ravel(b)) / max(np.linalg.norm(np.ravel(b)), 1e-30))


def test_fixtures_present():
    names = {os.path.basename(f)[:-4] for f in FILES}
    assert {"tiny_b4", "tiny_b4_reg2e-4", "mnist_1step_b4", "celeba_b4", "lsun_b4"} <= names


@pytest.mark.parametrize("path", FILES, ids=lambda p: os.path.basename(p)[:-4])
def test_oracle_reproduces_golden(path):
    g = np.load(path)  # allow_pickle=False: plain arrays only
    cfg = spec.make_config(str(g["preset"]), batch=int(g["batch"]))
    x, tgt, eps = spec.make_inputs(cfg)
    assert np.array_equal(x, g["x"]) and np.array_equal(tgt, g["target"]) and np.array_equal(eps, g["eps"])
    table, struct, params = spec.init_params(cfg, seed=0, dtype=np.float32)
    params = {k: v.astype(np.float64) for k, v in params.items()}
    assert [p["name"] for p in table] == list(g["grad_names"])
    o = model.forward_backward(cfg, struct, params, x, tgt, eps, float(g["reg"]))
    assert abs(o["loss"] - g["loss"]) <= 1e-10 * abs(g["loss"])
    assert abs(o["final_loss"] - g["final_loss"]) <= 1e-10 * abs(g["final_loss"])
    np.testing.assert_allclose(o["recon"], g["recon"], rtol=1e-10)
    np.testing.assert_allclose(o["kl"], g["kl"], rtol=1e-10)
    np.testing.assert_allclose(np.stack(o["recon_img"]), g["recon_img"], rtol=1e-9)
    np.testing.assert_allclose(o["elbo_img"], g["elbo_img"], rtol=1e-9)
    assert _rel(np.stack(o["mu"]), g["mu"]) <= 1e-9 and _rel(np.stack(o["sig"]), g["sig"]) <= 1e-9
    T = len(g["recon"])
    flat = np.stack(o["xhat"]).reshape(T, -1)
    s = int(g["xhat_sample_stride"])
    assert _rel(flat[:, ::s][:, :g["xhat_sample"].shape[1]], g["xhat_sample"]) <= 1e-9
    assert _rel(o["xhat"][-1], g["xhat_final"]) <= 1e-9
    names = list(g["grad_names"])
    gn = np.array([np.linalg.norm(o["grads"][n]) for n in names])
    assert _rel(gn, g["grad_norm"]) <= 1e-8
    small = np.concatenate([o["grads"][n].ravel() for n in g["small_names"]])
    assert _rel(small, g["small_grads"]) <= 1e-8


@pytest.mark.parametrize("path", FILES, ids=lambda p: os.path.basename(p)[:-4])
def test_golden_internal_consistency(path):
    """Loss bookkeeping of compute_and_accumulate_loss (sequential_vae.py:1163-1176):
    loss = sum_t 16*recon_t + reg*KL_t (intermediate_reconstruction, coeff 1) and the
    per-image terms average to the batch terms."""
    g = np.load(path)
    reg = float(g["reg"])
    assert abs(16 * g["recon"].sum() + reg * g["kl"].sum() - g["loss"]) <= 1e-12 * abs(g["loss"])
    np.testing.assert_allclose(g["recon_img"].mean(1), g["recon"], rtol=1e-12)
    np.testing.assert_allclose(g["kl_img"].mean(1), g["kl"], rtol=1e-12)
    assert abs(g["elbo_img"].mean() - g["loss"]) <= 1e-12 * abs(g["loss"])
    assert g["final_loss"] == g["recon"][-1]
    assert (g["sig"] > 0).all() and (g["sig"] < 1).all()
