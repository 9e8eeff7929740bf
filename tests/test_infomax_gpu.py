"""Latent InfoMax chains (predict_latent_code, sequential_vae.py:129-131, :1013-1020): step t >= 1
encodes q(z_t | x_{t-1}) from the previous sample, so the recognition backward feeds d loss /
d x_{t-1}; KL only at step 0 unless predict_latent_code_with_regularization (:1170-1172);
regularized_steps (:1154).  Engine vs the fp32 oracle, tiny geometry (T=3, B=4); bounds as
tests/test_engine_gpu.py (loss 1e-4, x_hat 1e-4 L2, gradients vector 1e-3 / median 1e-4)."""
import numpy as np
import pytest
import torch

from conftest import pkg_mod
from oracle import model, spec

pytestmark = pytest.mark.gpu

CASES = {
    "infomax": dict(predict_latent_code=True),
    "infomax_reg": dict(predict_latent_code=True, predict_latent_code_with_regularization=True),
    "infomax_homog": dict(predict_latent_code=True, share_theta_weights=True, share_phi_weights=True),
    "regularized_steps": dict(regularized_steps=(0, 2)),
}


def _rel(a, b):
    return float(np.linalg.norm(np.ravel(a) - np.ravel(b)) / max(np.linalg.norm(np.ravel(b)), 1e-30))


@pytest.mark.parametrize("name", list(CASES))
def test_infomax_matches_oracle(name):
    over = CASES[name]
    cfg = pkg_mod("config").preset("tiny", batch=4, **over)
    net = pkg_mod("sequential_vae").SequentialVAE(cfg, seed=0)
    sh_t, sh_p = over.get("share_theta_weights", False), over.get("share_phi_weights", False)
    cd = spec.make_config("tiny", batch=4, **{k: v for k, v in over.items() if "share" not in k})
    x, tgt, eps = spec.make_inputs(cd)
    reg = 0.6
    net.forward(x, tgt, eps, reg)
    net.backward()
    torch.cuda.synchronize()
    pub = {k: v.astype(np.float64) for k, v in net.param_dict().items()}
    _, struct = spec.build_params(cd)
    params = spec.expand_shared(pub, cd, sh_t, sh_p) if (sh_t or sh_p) else pub
    o = model.forward_backward(cd, struct, params, x, tgt, eps, reg)
    loss = net.loss_value(reg_coeff=reg)
    assert abs(loss - o["loss"]) <= 1e-4 * abs(o["loss"]), (loss, o["loss"])
    np.testing.assert_allclose(net.elbo_per_image().cpu().numpy(), o["elbo_img"], rtol=1e-4)
    for t in range(cd["mc_steps"]):
        assert _rel(net.xhat(t).cpu().numpy(), o["xhat"][t]) <= 1e-4
        assert _rel(net.latent(pkg_mod("_lib").BUF_MU, t).cpu().numpy(), o["mu"][t]) <= 1e-4
    gref = spec.sum_shared_grads(o["grads"], sh_t, sh_p, cd["predict_latent_code"]) if (sh_t or sh_p) else o["grads"]
    g = net.grad_dict()
    live = [k for k, v in gref.items() if np.linalg.norm(v) > 1e-7]
    cat = lambda d: np.concatenate([np.ravel(d[k]) for k in live])
    gvec = _rel(cat(g), cat(gref))
    gmed = float(np.median([_rel(g[k], gref[k]) for k in live]))
    assert gvec <= 1e-3 and gmed <= 1e-4, (gvec, gmed)


@pytest.mark.parametrize("preset", ["c_homog_reg_pred_latent", "c_homog_no_reg_pred_latent"])
def test_celeba_infomax_presets_run(preset):
    """The reference's Latent InfoMax CelebA netnames at B=16 in bf16: a finite training step."""
    cfg = pkg_mod("config").preset(preset, batch=16, dtype="bf16")
    net = pkg_mod("sequential_vae").SequentialVAE(cfg, seed=0)
    x = torch.rand(16, 64, 64, 3, device="cuda") * 2 - 1
    losses = [net.train(x, x) for _ in range(2)]
    torch.cuda.synchronize()
    assert all(np.isfinite(losses))
    assert torch.isfinite(net.grads[:net.n_live]).all()
