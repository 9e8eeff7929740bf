"""CPU checks of the PixelCNN++ head's oracle (oracle/pcnn.py, PARITY UNPINNED: no runnable
reference) and of the product's pure-host parameter table.

What pins the restatement instead of reference outputs:
  * the autoregressive property model_spec exists for (model.py:37-40 shifts, nn.py:292-320):
    the output at a pixel depends only on pixels strictly before it in raster order;
  * the discretized-logistic loss against an independent scalar restatement of nn.py:46-87;
  * autograd against central finite differences."""
import math

import numpy as np
import torch

from conftest import pkg_mod
from oracle import pcnn as opc

SPEC = dict(H=8, W=8, K=3, nr_resnet=1, nr_filters=4, nr_mix=2)


def test_product_param_table_matches_oracle():
    PC = pkg_mod("pixelcnn")
    for nl in ("relu", "concat_elu"):
        kw = dict(SPEC, nonlinearity=nl, nr_resnet=2)
        assert list(PC.param_shapes(PC.make_spec(**kw)).items()) == list(opc.param_shapes(opc.make_spec(**kw)).items())
    # the reference's layer count at nr_resnet 3 (pixelvae.py Args): 3 + 3*3*2 + 2*2 up convs, 21 gated
    # resnets down, 4 deconvs; every gated resnet has 2 convs and a conditional projection
    sh = opc.param_shapes(opc.make_spec())
    n_conv = len([k for k in sh if k.startswith("conv2d_") and k.endswith("/V")])
    n_hw = len([k for k in sh if k.endswith("/hw")])
    assert n_hw == 3 * 3 * 2 + (3 + 4 + 4) * 2 and n_conv == 3 + 4 + 2 * n_hw
    assert sh["dense_%d/V" % (len([k for k in sh if k.startswith("dense_") and k.endswith("/V")]) - 1)] == (160, 100)


def test_autoregressive_property():
    """l at raster position q depends on x only through positions < q (the receptive field that
    the down / down-right shifts build, model.py:37-40)."""
    spec = opc.make_spec(**SPEC)
    P = opc.to_tensors(opc.init_params(spec, 0), requires_grad=False)
    rng = np.random.default_rng(0)
    x = torch.tensor(rng.uniform(-1, 1, (1, 8, 8, 3)))
    h = torch.tensor(rng.normal(size=(1, 3)))
    base = opc.Net(spec, P).model(x, h)
    for q in (0, 9, 27, 63):
        yi, xi = divmod(q, 8)
        x2 = x.clone()
        x2[0, yi, xi] += 0.5
        d = (opc.Net(spec, P).model(x2, h) - base).abs().amax(dim=-1)[0].reshape(-1)
        assert float(d[:q + 1].max()) == 0.0, q  # nothing at or before the perturbed position changes
        if q < 63:
            assert float(d[q + 1:].max()) > 0.0


def _scalar_logp(x, lp, M):
    """Independent per-pixel restatement of nn.py:46-87 in plain Python floats."""
    sig = lambda v: 1.0 / (1.0 + math.exp(-v)) if v >= 0 else math.exp(v) / (1.0 + math.exp(v))
    sp = lambda v: max(v, 0.0) + math.log1p(math.exp(-abs(v)))
    logit = lp[:M]
    mx = max(logit)
    lse_logit = mx + math.log(sum(math.exp(v - mx) for v in logit))
    terms = []
    for j in range(M):
        tot = logit[j] - lse_logit
        for c in range(3):
            base = M + c * 3 * M
            mean = lp[base + j]
            coef = [math.tanh(lp[M + cc * 3 * M + 2 * M + j]) for cc in range(3)]
            if c == 1:
                mean += coef[0] * x[0]
            if c == 2:
                mean += coef[1] * x[0] + coef[2] * x[1]
            ls = max(lp[base + M + j], -7.0)
            inv = math.exp(-ls)
            cx = x[c] - mean
            pin, mnin = inv * (cx + 1 / 255.0), inv * (cx - 1 / 255.0)
            if x[c] < -0.999:
                v = pin - sp(pin)
            elif x[c] > 0.999:
                v = -sp(mnin)
            else:
                cd = sig(pin) - sig(mnin)
                if cd > 1e-5:
                    v = math.log(max(cd, 1e-12))
                else:
                    mid = inv * cx
                    v = mid - ls - 2 * sp(mid) - math.log(127.5)
            tot += v
        terms.append(tot)
    mx = max(terms)
    return mx + math.log(sum(math.exp(t - mx) for t in terms))


def test_mix_logistic_matches_scalar_restatement():
    rng = np.random.default_rng(5)
    M = 3
    x = rng.uniform(-1, 1, (1, 2, 3, 3))
    x[0, 0, 0] = [-1.0, 1.0, 0.2]
    l = rng.normal(size=(1, 2, 3, 10 * M))
    l[0, 1, 2, M + M:M + 2 * M] = -9.0  # clamp to -7 and the tiny-bin branch
    got = opc.mix_logistic_logprob(torch.tensor(x), torch.tensor(l)).numpy()
    for i in range(2):
        for j in range(3):
            ref = _scalar_logp(list(x[0, i, j]), list(l[0, i, j]), M)
            assert abs(got[0, i, j] - ref) < 1e-9 * max(1.0, abs(ref))


def test_oracle_gradient_finite_differences():
    spec = opc.make_spec(**dict(SPEC, H=4, W=4))
    params = opc.init_params(spec, 1)
    rng = np.random.default_rng(2)
    x = rng.uniform(-0.9, 0.9, (2, 4, 4, 3))
    h = rng.normal(size=(2, 3))
    _, _, g = opc.loss_and_grads(spec, params, x, h)
    for name, idx in (("conv2d_0/V", (1, 2, 3, 1)), ("conv2d_4/g", (2,)), ("deconv2d_1/V", (0, 1, 2, 3)),
                      ("conditional_weights_3/hw", (1, 5)), ("dense_13/b", (7,)), ("dense_4/V", (5, 2))):
        eps = 1e-5
        p1 = {k: v.copy() for k, v in params.items()}
        p2 = {k: v.copy() for k, v in params.items()}
        p1[name][idx] += eps
        p2[name][idx] -= eps
        fd = (opc.loss_and_grads(spec, p1, x, h)[0] - opc.loss_and_grads(spec, p2, x, h)[0]) / (2 * eps)
        assert abs(fd - g[name][idx]) < 1e-5 * max(1.0, abs(fd)), (name, fd, g[name][idx])
