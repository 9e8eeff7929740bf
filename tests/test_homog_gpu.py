"""Homogeneous chains (share_theta_weights / share_phi_weights, sequential_vae.py:107-113;
scopes :1573-1577, :1683-1687, :1757-1761; netnames c_homog_v1 :316-321, c_homog_one_step
:281-288) against the fp32 oracle: the oracle runs its per-step graph with every step's copy
aliasing the shared tensor, and a shared tensor's gradient is the sum over the steps that use it.
Bounds as tests/test_engine_gpu.py (loss 1e-4, x_hat 1e-4 L2, gradients vector 1e-3, median 1e-4)."""
import numpy as np
import pytest
import torch

from conftest import pkg_mod
from oracle import model, spec

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float(np.linalg.norm(np.ravel(a) - np.ravel(b)) / max(np.linalg.norm(np.ravel(b)), 1e-30))


@pytest.mark.parametrize("theta,phi", [(True, True), (True, False), (False, True)])
def test_homog_matches_oracle(theta, phi):
    cfg = pkg_mod("config").preset("tiny", batch=4, share_theta_weights=theta, share_phi_weights=phi)
    net = pkg_mod("sequential_vae").SequentialVAE(cfg, seed=0)
    cd = spec.make_config("tiny", batch=4)
    x, tgt, eps = spec.make_inputs(cd)
    reg = 0.8
    net.forward(x, tgt, eps, reg)
    net.backward()
    torch.cuda.synchronize()
    pub = {k: v.astype(np.float64) for k, v in net.param_dict().items()}
    assert set(pub) == {p["name"] for p in spec.shared_table(cd, theta, phi)}
    _, struct = spec.build_params(cd)
    o = model.forward_backward(cd, struct, spec.expand_shared(pub, cd, theta, phi), x, tgt, eps, reg)
    loss = net.loss_value(reg_coeff=reg)
    assert abs(loss - o["loss"]) <= 1e-4 * abs(o["loss"]), (loss, o["loss"])
    for t in range(cd["mc_steps"]):
        assert _rel(net.xhat(t).cpu().numpy(), o["xhat"][t]) <= 1e-4
    gref = spec.sum_shared_grads(o["grads"], theta, phi)
    g = net.grad_dict()
    live = [k for k, v in gref.items() if np.linalg.norm(v) > 1e-7]
    cat = lambda d: np.concatenate([np.ravel(d[k]) for k in live])
    gvec = _rel(cat(g), cat(gref))
    gmed = float(np.median([_rel(g[k], gref[k]) for k in live]))
    assert gvec <= 1e-3 and gmed <= 1e-4, (gvec, gmed)


def test_homog_after_adam_steps_matches_oracle():
    """Adam updates the public (shared) tensors; the next forward re-broadcasts them into the
    per-step copies, so parity with the oracle holds on the updated weights."""
    cfg = pkg_mod("config").preset("tiny_homog", batch=4)
    net = pkg_mod("sequential_vae").SequentialVAE(cfg, seed=0)
    cd = spec.make_config("tiny", batch=4)
    x, tgt, eps = spec.make_inputs(cd)
    p0 = net.params.clone()
    for _ in range(2):
        net.train(x, tgt)
    assert float((net.params - p0).abs().max()) > 0
    net.forward(x, tgt, eps, 0.5)
    net.backward()
    torch.cuda.synchronize()
    pub = {k: v.astype(np.float64) for k, v in net.param_dict().items()}
    _, struct = spec.build_params(cd)
    o = model.forward_backward(cd, struct, spec.expand_shared(pub, cd), x, tgt, eps, 0.5)
    assert abs(net.loss_value(reg_coeff=0.5) - o["loss"]) <= 1e-4 * abs(o["loss"])
    gref = spec.sum_shared_grads(o["grads"])
    g = net.grad_dict()
    live = [k for k, v in gref.items() if np.linalg.norm(v) > 1e-7]
    cat = lambda d: np.concatenate([np.ravel(d[k]) for k in live])
    assert _rel(cat(g), cat(gref)) <= 1e-3


@pytest.mark.parametrize("preset", ["c_homog_v1", "c_homog_one_step"])
def test_celeba_homog_presets_run(preset):
    """The reference's homogeneous CelebA netnames at B=16: one bf16 training step, finite loss
    and gradients, every live public gradient written."""
    cfg = pkg_mod("config").preset(preset, batch=16, dtype="bf16")
    net = pkg_mod("sequential_vae").SequentialVAE(cfg, seed=0)
    x = torch.rand(16, 64, 64, 3, device="cuda") * 2 - 1
    net.forward(x, x, None, 1.0)
    net.backward()
    torch.cuda.synchronize()
    assert np.isfinite(net.loss_value())
    g = net.grads[:net.n_live]
    assert torch.isfinite(g).all()
    assert float(g.abs().max()) > 0
