"""oracle/pixelvae.py (the c_pixelvae chain restatement, PARITY UNPINNED) against central finite
differences of its own loss: autograd through the recognition network, step 0's ladder, the head's
model_spec, the reparameterised mixture draw and the highway mix (fp64, no bf16 rounding)."""
import numpy as np
import pytest

from oracle import pcnn as opc
from oracle import pixelvae as opv
from oracle import spec


def _setup():
    cd = spec.make_config("tiny", H=16, W=16, C=3, levels=4, filter_sizes=[3, 4, 4, 8, 8, 8],
                          latent_dims=[2, 2, 2, 2], mc_steps=2, batch=2, latent_mean_clip=4.0, min_highway=0.2,
                          max_highway=0.8, regularized_steps=(0,), first_step_loss_coeff=2.0)
    cd["share_theta"] = cd["share_phi"] = True
    _, _, per = spec.init_params(cd, seed=0)
    pub = {}
    for k, v in per.items():
        pub.setdefault(spec.shared_name(k, True, True, False), v)
    ospec = opc.make_spec(H=16, W=16, K=8, nr_resnet=1, nr_filters=4, nr_mix=2)
    hp = opc.init_params(ospec, 3)
    x, tgt, eps = spec.make_inputs(cd, batch=2)
    rng = np.random.default_rng(7)
    um = rng.uniform(0.05, 0.95, (2, 16, 16, 2))
    ul = rng.uniform(0.2, 0.8, (2, 16, 16, 3))
    return cd, pub, ospec, hp, x, tgt, eps, um, ul


@pytest.mark.parametrize("which", ["phi", "theta0", "head_conv", "highway"])
def test_pixelvae_oracle_gradient_vs_finite_differences(which):
    cd, pub, ospec, hp, x, tgt, eps, um, ul = _setup()
    o = opv.forward_backward(cd, pub, ospec, hp, x, tgt, eps, 0.7, um, ul, None, bf16_head=False)
    rng = np.random.default_rng(1)
    if which == "phi":
        name, src, grads = "phi/inference_network/Conv_1/weights", pub, o["grads"]
    elif which == "theta0":
        name, src, grads = "theta/generative_step_0/Conv2d_transpose_1/weights", pub, o["grads"]
    elif which == "head_conv":
        name, src, grads = "conv2d_1/V", hp, o["head_grads"]
    else:
        name, src, grads = "highway/W", hp, o["head_grads"]
    assert name in src, sorted(src)[:20]
    base = np.array(src[name], np.float64)
    idx = [tuple(rng.integers(0, s) for s in base.shape) for _ in range(3)]
    h = 1e-6
    for ix in idx:
        vals = []
        for sgn in (1, -1):
            p = np.array(base, copy=True)
            p[ix] += sgn * h
            s2 = dict(src)
            s2[name] = p
            args = (s2, hp) if src is pub else (pub, s2)
            vals.append(opv.forward_backward(cd, args[0], ospec, args[1], x, tgt, eps, 0.7, um, ul, None,
                                             bf16_head=False)["loss"])
        fd = (vals[0] - vals[1]) / (2 * h)
        g = float(np.asarray(grads[name])[ix])
        assert abs(fd - g) <= 1e-5 * max(1.0, abs(g)) + 1e-7, (which, ix, fd, g)


def test_pixelvae_oracle_loss_bookkeeping():
    """loss = first_step_loss_coeff * (16 rec_0 + reg KL_0) + 16 rec_1 (regularized_steps = [0])."""
    cd, pub, ospec, hp, x, tgt, eps, um, ul = _setup()
    o = opv.forward_backward(cd, pub, ospec, hp, x, tgt, eps, 0.7, um, ul, None, bf16_head=False)
    want = 2.0 * (16 * o["rec"][0] + 0.7 * o["kl"][0]) + 16 * o["rec"][1]
    assert abs(o["loss"] - want) <= 1e-12 * abs(want)
    assert np.abs(o["xhat"][1]).max() <= 1.0 + 1e-12  # a mix of two images in [-1, 1]
