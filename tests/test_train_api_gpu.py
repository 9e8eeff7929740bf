"""The reference training interface over several iterations (sequential_vae.py:1341-1375):
``train(input, target)`` advances ``iteration``, feeds reg_coeff = 1 - exp(-it/5000) (:1357),
runs [train_op, loss, final_loss] and returns final_loss / H / W; train_op is compute_gradients
(:1273) -> clip(+-10) (:1274-1275) -> Adam (:1267, :1276).

Three train() calls with injected eps on the tiny geometry (fp32) are compared with the float64
oracle run the same way: oracle forward/backward at the same reg schedule, then the oracle's
clip + TF Adam on the oracle's own gradients (moments carried across iterations)."""
import math

import numpy as np
import pytest
import torch

from conftest import pkg_mod
from oracle import model, spec

pytestmark = pytest.mark.gpu


def test_train_three_iterations_against_oracle():
    cfg = pkg_mod("config").preset("tiny", batch=4)
    net = pkg_mod("sequential_vae").SequentialVAE(cfg, seed=0)
    cd = spec.make_config("tiny", batch=4)
    _, struct = spec.build_params(cd)
    x, tgt, eps0 = spec.make_inputs(cd, batch=4)
    rng = np.random.default_rng(11)
    P = {k: v.astype(np.float64) for k, v in net.param_dict().items()}
    P0 = {k: v.copy() for k, v in P.items()}
    M = {k: np.zeros_like(v) for k, v in P.items()}
    V = {k: np.zeros_like(v) for k, v in P.items()}
    H, W = cfg.height, cfg.width
    lr = cfg.learning_rate
    for it in (1, 2, 3):
        eps = eps0 if it == 1 else rng.standard_normal(eps0.shape).astype(np.float32)
        before = {k: v.astype(np.float64) for k, v in net.param_dict().items()}
        got = net.train(x, tgt, eps=eps)
        torch.cuda.synchronize()
        assert net.iteration == it
        reg = 1.0 - math.exp(-it / 5000.0)
        # the return convention, on the engine's own pre-update weights
        o_same = model.forward_backward(cd, struct, before, x, tgt, eps, reg, want_grads=False)
        assert abs(got - o_same["final_loss"] / H / W) <= 1e-4 * abs(o_same["final_loss"] / H / W), (it, got)
        assert abs(net.loss_value() - o_same["loss"]) <= 1e-4 * abs(o_same["loss"])   # reg schedule
        # the oracle's own trajectory (its weights, gradients and Adam moments)
        o = model.forward_backward(cd, struct, P, x, tgt, eps, reg)
        ret_oracle = o["final_loss"] / H / W
        P, M, V = model.adam_update(P, o["grads"], M, V, it, lr=lr, clip=cfg.clip_grad_value)
        now = net.param_dict()
        d = np.concatenate([np.ravel(now[k] - P[k]) for k in P])
        frac = float(np.mean(np.abs(d) > 1e-6))
        # cumulative update since initialisation, engine vs oracle trajectory
        du_e = np.concatenate([np.ravel(now[k] - P0[k]) for k in P])
        du_o = np.concatenate([np.ravel(P[k] - P0[k]) for k in P])
        upd = float(np.linalg.norm(du_e - du_o) / np.linalg.norm(du_o))
        print("iteration %d: train() %.8f  oracle %.8f  (rel %.2e); params max|d| %.2e, "
              "fraction > 1e-6: %.2e, cumulative update rel L2 %.2e" % (
                  it, got, ret_oracle, abs(got - ret_oracle) / ret_oracle, np.abs(d).max(), frac, upd))
        assert abs(got - ret_oracle) <= 1e-4 * abs(ret_oracle)
        # Adam's m/sqrt(v) is sign-like where the gradient is ~0 (and at step 1 everywhere: the
        # first update is lr*sign(g)), so an fp32 gradient of the other sign, or a slightly different
        # ratio, moves that weight by up to ~lr: bound the size of such moves and the update as a whole
        assert np.abs(d).max() <= 2.5 * lr * it
        assert upd <= 0.1
    out = net.test(x)
    assert out.shape == (4, H, W, 3) and np.isfinite(out).all()
    net.close()
