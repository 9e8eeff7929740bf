"""Loss / latent / highway knobs of the reference's argument set against the fp32 oracle (tiny
geometry, T=3, B=4): intermediate_reconstruction=False (sequential_vae.py:725, :1167),
first_step_loss_coeff (:227, :1175-1176), latent_prior_stddev (:232, KL :1156-1158),
latent_mean_clip (:230, heads :1594/:1607) and min/max highway (:243-244, :1727-1729).
Bounds as tests/test_engine_gpu.py: loss / per-step terms 1e-4, x_hat 1e-4 (L2), gradients
vector 1e-3 and per-tensor median 1e-4 (fp32 kink flips: no per-tensor max)."""
import numpy as np
import pytest
import torch

from conftest import pkg_mod
from oracle import model, spec

pytestmark = pytest.mark.gpu

VARIANTS = {
    "no_intermediate_recon": dict(intermediate_reconstruction=False),
    "first_step_coeff": dict(first_step_loss_coeff=0.3),
    "prior_stddev": dict(latent_prior_stddev=0.5),
    "mean_clip": dict(latent_mean_clip=0.05),
    "highway_range": dict(min_highway=0.2, max_highway=0.9),
}


def _rel(a, b):
    return float(np.linalg.norm(np.ravel(a) - np.ravel(b)) / max(np.linalg.norm(np.ravel(b)), 1e-30))


@pytest.mark.parametrize("name", list(VARIANTS))
def test_variant_matches_oracle(name):
    over = VARIANTS[name]
    cfg = pkg_mod("config").preset("tiny", batch=4, **over)
    net = pkg_mod("sequential_vae").SequentialVAE(cfg, seed=0)
    cd = spec.make_config("tiny", batch=4, **over)
    x, tgt, eps = spec.make_inputs(cd)
    reg = 0.7
    net.forward(x, tgt, eps, reg)
    net.backward()
    torch.cuda.synchronize()
    _, struct = spec.build_params(cd)
    params = {k: v.astype(np.float64) for k, v in net.param_dict().items()}
    o = model.forward_backward(cd, struct, params, x, tgt, eps, reg)
    loss = net.loss_value(reg_coeff=reg)
    assert abs(loss - o["loss"]) <= 1e-4 * abs(o["loss"]), (loss, o["loss"])
    stats = net.step_stats().cpu().numpy()
    for t in range(cd["mc_steps"]):
        assert abs(stats[t, 0] - o["recon"][t]) <= 1e-4 * abs(o["recon"][t])
        assert abs(stats[t, 1] - o["kl"][t]) <= 1e-4 * abs(o["kl"][t])
        assert _rel(net.xhat(t).cpu().numpy(), o["xhat"][t]) <= 1e-4
    g = net.grad_dict()
    live = [k for k, v in o["grads"].items() if np.linalg.norm(v) > 1e-7]
    cat = lambda d: np.concatenate([np.ravel(d[k]) for k in live])
    gvec = _rel(cat(g), cat(o["grads"]))
    gmed = float(np.median([_rel(g[k], o["grads"][k]) for k in live]))
    assert gvec <= 1e-3 and gmed <= 1e-4, (gvec, gmed)
    if name == "mean_clip":  # the clip is active: some means sit on the bound
        mu = np.concatenate([np.ravel(m) for m in o["mu"]])
        assert (np.abs(mu) == 0.05).mean() > 0.05
