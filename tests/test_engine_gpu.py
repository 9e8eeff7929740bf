"""End-to-end parity of the HIP training step against the CPU oracle (oracle/model.py,
numpy float64), same seeded inputs / injected eps / identical weights.

Tolerances (BASELINE.json north_star: 1e-4 relative fp32 on ELBO and decoder output):
  loss / per-step recon & KL : |d|/|ref| <= 1e-4
  x_hat_t (decoder output)   : ||d||2/||ref||2 <= 1e-4 and max-abs <= 1e-3
  gradients                  : per tensor ||d||/||ref|| <= 1e-3 (tensors with ||ref|| > 1e-7)
"""
import math

import numpy as np
import pytest
import torch

from conftest import pkg_mod
from oracle import model, spec, torch_twin

pytestmark = pytest.mark.gpu


def _engine(preset, batch, **over):
    cfgmod = pkg_mod("config")
    SV = pkg_mod("sequential_vae").SequentialVAE
    cfg = cfgmod.preset(preset, batch=batch, **over)
    return SV(cfg, seed=0), cfg


def _oracle_run(net, cfg_dict, x, tgt, eps, reg):
    _, struct = spec.build_params(cfg_dict)
    params = {k: v.astype(np.float64) for k, v in net.param_dict().items()}
    return model.forward_backward(cfg_dict, struct, params, x, tgt, eps, reg)


def _rel(a, b):
    return float(np.linalg.norm(np.ravel(a) - np.ravel(b)) / max(np.linalg.norm(np.ravel(b)), 1e-30))


@pytest.mark.parametrize("preset,batch,reg", [("tiny", 4, 0.37), ("mnist_1step", 4, 1.0), ("celeba", 4, 1.0),
                                              ("tiny", 7, 1e-3)])
def test_fwd_bwd_matches_oracle(preset, batch, reg):
    net, cfg = _engine(preset, batch)
    cd = spec.make_config(preset, batch=batch)
    x, tgt, eps = spec.make_inputs(cd, batch=batch)
    if preset == "tiny" and batch == 7:
        tgt = np.clip(x + 0.1 * np.random.default_rng(9).standard_normal(x.shape).astype(np.float32), -1, 1)
    net.forward(x, tgt, eps, reg)
    net.backward()
    torch.cuda.synchronize()
    o = _oracle_run(net, cd, x, tgt, eps, reg)
    stats = net.step_stats().cpu().numpy()
    loss = net.loss_value(stats, reg)
    assert abs(loss - o["loss"]) <= 1e-4 * abs(o["loss"]), (loss, o["loss"])
    for t in range(cfg.mc_steps):
        assert abs(stats[t, 0] - o["recon"][t]) <= 1e-4 * abs(o["recon"][t])
        assert abs(stats[t, 1] - o["kl"][t]) <= 1e-4 * abs(o["kl"][t])
        xh = net.xhat(t).cpu().numpy()
        assert _rel(xh, o["xhat"][t]) <= 1e-4
        assert np.abs(xh - o["xhat"][t]).max() <= 1e-3
        np.testing.assert_allclose(net.latent(1, t).cpu().numpy(), o["mu"][t], rtol=1e-3, atol=1e-5)
    elbo = net.elbo_per_image().cpu().numpy()
    np.testing.assert_allclose(elbo, o["elbo_img"], rtol=1e-4)
    g = net.grad_dict()
    worst = (0.0, "")
    for name, ref in o["grads"].items():
        n = np.linalg.norm(ref)
        if n <= 1e-7:
            assert np.abs(g[name]).max() <= 1e-5 + 1e-3 * n, name
            continue
        r = _rel(g[name], ref)
        worst = max(worst, (r, name))
    assert worst[0] <= 1e-3, worst


def test_train_step_adam_matches_oracle():
    """train() = forward + backward + clip + TF Adam; two iterations vs the oracle."""
    net, cfg = _engine("tiny", 4)
    cd = spec.make_config("tiny", batch=4)
    x, tgt, eps = spec.make_inputs(cd, batch=4)
    table, struct = spec.build_params(cd)
    params = {k: v.astype(np.float64) for k, v in net.param_dict().items()}
    m = {k: np.zeros_like(v) for k, v in params.items()}
    v = {k: np.zeros_like(p) for k, p in params.items()}
    for it in (1, 2):
        reg = 1.0 - math.exp(-it / 5000.0)
        net.forward(x, tgt, eps[::-1].copy() if it == 2 else eps, reg)
        net.backward()
        net.apply_gradients(2e-4, it)
        o = model.forward_backward(cd, struct, params, x, tgt, eps[::-1].copy() if it == 2 else eps, reg)
        params, m, v = model.adam_update(params, o["grads"], m, v, it, lr=2e-4, clip=10.0)
    torch.cuda.synchronize()
    got = net.param_dict()
    for k in params:
        d = np.abs(got[k] - params[k]).max()
        assert d <= 2e-6 + 1e-4 * np.abs(params[k]).max(), (k, d)


def test_reference_api_train_and_test():
    net, cfg = _engine("tiny", 4)
    x, tgt, _ = spec.make_inputs(spec.make_config("tiny", batch=4), batch=4)
    losses = [net.train(x, tgt) for _ in range(3)]
    assert net.iteration == 3
    assert all(np.isfinite(losses))
    out = net.test(x)
    assert out.shape == (4, 32, 32, 3) and np.isfinite(out).all()
    assert out.min() >= -1.0 - 1e-6 and out.max() <= 1.0 + 1e-6   # highway of dataset-range outputs


def test_celeba_b128_forward_matches_twin():
    """Headline geometry (CelebA 64x64, B=128, T=8): ELBO and decoder output vs the
    float64 CPU restatement of the same graph (forward only)."""
    net, cfg = _engine("celeba", 128)
    cd = spec.make_config("celeba")
    x, tgt, eps = spec.make_inputs(cd)
    net.forward(x, tgt, eps, 1.0)
    torch.cuda.synchronize()
    _, struct = spec.build_params(cd)
    tw = torch_twin.Twin(cd, struct, net.param_dict(), dtype=torch.float64, requires_grad=False)
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    with torch.no_grad():
        o = tw.step(x, tgt, eps, 1.0, backward=False)
    loss = net.loss_value(reg_coeff=1.0)
    assert abs(loss - o["loss"]) <= 1e-4 * abs(o["loss"]), (loss, o["loss"])
    xh = net.xhat(-1).cpu().numpy()
    assert _rel(xh, o["xhat"][-1]) <= 1e-4


def test_full_size_properties():
    """Size-independent properties at the bench geometry: determinism, ELBO mean ==
    loss, zero gradient on the frozen (dead / pre-BN bias) region."""
    net, cfg = _engine("celeba", 128)
    cd = spec.make_config("celeba")
    x, tgt, eps = spec.make_inputs(cd)
    net.forward(x, tgt, eps, 1.0)
    net.backward()
    g1 = net.grads.clone()
    l1 = net.loss_value()
    e1 = net.elbo_per_image().mean().item()
    net.forward(x, tgt, eps, 1.0)
    net.backward()
    torch.cuda.synchronize()
    assert torch.equal(g1, net.grads), "backward not deterministic"
    assert abs(e1 - l1) <= 1e-5 * abs(l1)
    assert torch.isfinite(net.grads).all()
    assert net.grads[net.n_live:].abs().max().item() == 0.0
