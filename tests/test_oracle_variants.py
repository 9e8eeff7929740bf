"""Oracle restatements of the §8(f3) chain variants (TEST INFRASTRUCTURE checks, CPU):

* use_uniform_prior: KL_b = mean_d(-log sigma)                       sequential_vae.py:1159-1160
* add_noise_to_chain with the fixed noise_stddevs                      :239-240, :1088-1090, :1665-1666
* predict_generator_noise: stddevs_prediction + Gaussian NLL          :1147-1150, :1667, :1848-1875
* add_improvement_maximization_loss (own gradient over phi)           :1182-1201, :1299-1316

Each is checked two ways: the numpy fp64 tape against the independent torch float64 twin
(values and gradients), and the tape's gradients against central finite differences of its own
loss (h = 1e-7; ReLU/lrelu kinks make the loss only piecewise smooth).  The reference cannot run
here (no TensorFlow), so these variants are parity-unpinned like the rest.
"""
import numpy as np
import pytest
import torch

from oracle import model, spec, torch_twin

VARIANTS = {
    "uniform_prior": dict(use_uniform_prior=True),
    "noise_fixed": dict(add_noise_to_chain=True),
    "noise_pred": dict(add_noise_to_chain=True, predict_generator_noise=True),
    "noise_pred_infomax": dict(add_noise_to_chain=True, predict_generator_noise=True, predict_latent_code=True,
                               regularized_steps=(0,)),
    "imp_max": dict(predict_latent_code=True, add_improvement_maximization_loss=True, latent_pred_loss_coeff=0.01),
}


def _setup(over, T=3, seed=0, batch=4):
    cfg = spec.make_config("tiny", mc_steps=T, **over)
    _, struct, params = spec.init_params(cfg, seed=seed)
    x, tgt, eps = spec.make_inputs(cfg, batch=batch, seed_x=seed + 5, seed_eps=seed + 6)
    noise = spec.make_chain_noise(cfg, batch=batch) if cfg["add_noise_to_chain"] else None
    return cfg, struct, params, x, tgt, eps, noise


def test_default_noise_stddevs_follow_reference_list():
    c = spec.make_config("celeba", add_noise_to_chain=True)
    assert c["noise_stddevs"] == [0.5, 0.25, 0.125, 0.0625, 0.03125, 0.015625, 0.0078125, 0.0]
    c = spec.make_config("tiny", add_noise_to_chain=True)
    assert c["noise_stddevs"] == [0.5, 0.25, 0.125]
    with pytest.raises(AssertionError):
        spec.make_config("tiny", predict_generator_noise=True)


def test_stddev_network_variables_follow_tf_naming():
    """stddevs_prediction's layers are created in the generator scope after the output / ratio
    conv-T: Conv..Conv_4 + BatchNorm_k continuing the scope's count, then Conv_5 (1x1)."""
    cfg = spec.make_config("tiny", add_noise_to_chain=True, predict_generator_noise=True)
    table, _ = spec.build_params(cfg)
    names = [p["name"] for p in table if p["name"].startswith("theta/generative_step_1/")]
    tail = names[-17:]
    assert tail[0] == "theta/generative_step_1/Conv/weights"
    assert tail[-2:] == ["theta/generative_step_1/Conv_5/weights", "theta/generative_step_1/Conv_5/biases"]
    shapes = {p["name"]: p["shape"] for p in table}
    assert shapes["theta/generative_step_1/Conv/weights"] == (4, 4, 3, 5)
    assert shapes["theta/generative_step_1/Conv_4/weights"] == (4, 4, 5, 5)
    assert shapes["theta/generative_step_1/Conv_5/weights"] == (1, 1, 5, 1)
    # tiny: 4 split + 1 top + 3x2 decoder BatchNorms before the stddev network's
    assert "theta/generative_step_1/BatchNorm_11/beta" in shapes
    assert "theta/generative_step_1/BatchNorm_15/beta" in shapes


@pytest.mark.parametrize("name", list(VARIANTS))
def test_variant_oracle_matches_torch_twin(name):
    cfg, struct, params, x, tgt, eps, noise = _setup(VARIANTS[name])
    o = model.forward_backward(cfg, struct, params, x, tgt, eps, reg_coeff=0.37, noise=noise)
    p = torch_twin.Twin(cfg, struct, params, dtype=torch.float64).step(x, tgt, eps, reg_coeff=0.37, noise=noise)
    assert abs(o["loss"] - p["loss"]) <= 1e-12 * abs(o["loss"])
    for t in range(cfg["mc_steps"]):
        np.testing.assert_allclose(o["xhat"][t], p["xhat"][t], rtol=1e-10, atol=1e-12)
    # zero-gradient tensors (pre-BN biases) hold roundoff at the scale of the largest gradient
    for gk in ("grads", "imp_grads") if "imp_loss" in o else ("grads",):
        gmax = max(np.abs(g).max() for g in o[gk].values())
        for k, g in o[gk].items():
            np.testing.assert_allclose(g, p[gk][k], rtol=1e-8, atol=1e-11 * (1 + gmax), err_msg=k)
    if "imp_loss" in o:
        assert abs(o["imp_loss"] - p["imp_loss"]) <= 1e-12 * abs(o["imp_loss"])


def _fd_check(cfg, struct, params, x, tgt, eps, noise, key, gkey, names, reg=0.8, min_checked=5):
    o = model.forward_backward(cfg, struct, params, x, tgt, eps, reg, noise=noise)
    checked = 0
    for name in names:
        g = o[gkey][name]
        if np.abs(g).max() == 0:
            continue
        idx = np.unravel_index(np.argmax(np.abs(g)), g.shape)
        h = 1e-7
        pp = {k: v.copy() for k, v in params.items()}
        pp[name][idx] += h
        lp = model.forward_backward(cfg, struct, pp, x, tgt, eps, reg, want_grads=False, noise=noise)[key]
        pp[name][idx] -= 2 * h
        lm = model.forward_backward(cfg, struct, pp, x, tgt, eps, reg, want_grads=False, noise=noise)[key]
        fd = (lp - lm) / (2 * h)
        assert abs(fd - g[idx]) <= 1e-4 * max(1.0, abs(g[idx])), (name, fd, g[idx])
        checked += 1
    assert checked >= min_checked, checked
    return o


@pytest.mark.parametrize("name", ["uniform_prior", "noise_fixed", "noise_pred"])
def test_variant_finite_differences(name):
    cfg, struct, params, x, tgt, eps, noise = _setup(VARIANTS[name], T=2, seed=3)
    rng = np.random.default_rng(1)
    names = [n for n in params if not n.endswith("biases") or "fully_connected" in n or "Conv_5" in n]
    pick = list(rng.choice(sorted(names), size=10, replace=False))
    if name == "noise_pred":  # every stddev-network tensor of the last step
        pick += [n for n in params if n.startswith("theta/generative_step_1/") and
                 any(("/%s/" % k) in n for k in ("Conv", "Conv_2", "Conv_4", "Conv_5", "BatchNorm_15"))]
    _fd_check(cfg, struct, params, x, tgt, eps, noise, "loss", "grads", pick)


def test_improvement_loss_finite_differences():
    """d improvement_maximization_loss / d phi (the only variables its optimiser updates)."""
    cfg, struct, params, x, tgt, eps, noise = _setup(VARIANTS["imp_max"], T=3, seed=5)
    rng = np.random.default_rng(2)
    phi = sorted(n for n in params if n.startswith("phi/") and (not n.endswith("biases") or "fully_connected" in n))
    o = _fd_check(cfg, struct, params, x, tgt, eps, noise, "imp_loss", "imp_grads",
                  list(rng.choice(phi, size=10, replace=False)))
    assert o["imp_loss"] < 0  # maximises the step-to-step change
    # step 0's recognition only reaches the loss through x_0 -> x_1; it has a gradient as well
    assert np.abs(o["imp_grads"]["phi/inference_step_0/fully_connected/weights"]).max() > 0


def test_noise_changes_only_the_chain_input():
    """Fixed-noise chain: the step-0 MLE is unchanged, later steps see mle + reg*sd*noise."""
    cfg, struct, params, x, tgt, eps, noise = _setup(VARIANTS["noise_fixed"])
    base = spec.make_config("tiny", mc_steps=3)
    a = model.forward_backward(base, struct, params, x, tgt, eps, 0.5, want_grads=False)
    b = model.forward_backward(cfg, struct, params, x, tgt, eps, 0.5, want_grads=False, noise=noise)
    np.testing.assert_allclose(a["xhat"][0], b["xhat"][0], rtol=0, atol=0)
    np.testing.assert_allclose(b["sample"][1], b["xhat"][1] + 0.5 * 0.25 * noise[1].astype(np.float64), rtol=1e-12)
    assert np.abs(a["xhat"][1] - b["xhat"][1]).max() > 1e-3
