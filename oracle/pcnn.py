"""PyTorch-CPU fp64 restatement of the PixelCNN++ decoder head -- TEST
INFRASTRUCTURE ONLY: imported by tests/ and nothing in the product path.

PARITY UNPINNED.  The reference path cannot run: TensorFlow is absent here, and the glue
pixel_cnn/pixelvae.py:68-158 is broken as written (``tf_vars`` / ``substr`` undefined and a stray
``return subset`` at :108-112, ``min_highway_ratio`` undefined at :136, ``x_sample[i]`` indexing a
placeholder at :126).  There are no golden vectors for it in the reference.  This module is the
documented *repaired* restatement the HIP path is checked against:

  * model_spec(x, h)                       pixel_cnn_pp/model.py:11-117 (conditional on h)
  * conv2d / deconv2d / dense (weight norm) nn.py:160-252, incl. the data-dependent init pass
  * gated_resnet                            nn.py:264-288
  * down/right shifts, shifted (de)convs    nn.py:292-320
  * discretized_mix_logistic_loss           nn.py:46-87
  * sample_from_discretized_mix_logistic    nn.py:89-109 (uniforms injected)
  * pixelvae glue (repaired)                pixelvae.py:123-137: the head's output for the chain is
    the sample, mixed per IMAGE with the previous chain sample by the highway ratio
    min + (max - min) * sigmoid(fc(latents)); its training loss is the PixelCNN++ NLL.

Parameter layout (canonical, not TF's): conv and deconv V [kh, kw, Cin, Cout]; dense / nin V
[in, out]; conditional weights hw [K, 2F]; every weight-normed layer has g [Cout], b [Cout].
Weight norm: W = g * V / ||V|| with the norm over every axis but Cout (nn.py:173, :201, :236).
Layer names follow the reference's counters (nn.py:151-157), e.g. ``conv2d_3``.

``bf16=True`` rounds every conv / nin operand (input activations and normalised weights) to bf16
before the fp64 product, as the HIP path's bf16 MFMA does (fp32 accumulation is then the only
difference).
"""
import math

import numpy as np
import torch
import torch.nn.functional as Fn

DT = torch.float64


def _bf(t):
    return t.to(torch.bfloat16).to(t.dtype)


# ---------------------------------------------------------------------------------------------
# layer specs (the network as a list, so the HIP host code and this oracle build the same graph)
# ---------------------------------------------------------------------------------------------
def make_spec(H=64, W=64, C=3, K=48, nr_resnet=3, nr_filters=160, nr_mix=10, nonlinearity="relu"):
    """Hyper-parameters (pixelvae.py:54-63: nr_resnet 3, nr_filters 160, nr_logistic_mix 10,
    resnet_nonlinearity 'relu', dropout_p 0.3).  K = latent width (the h of model_spec)."""
    assert H % 4 == 0 and W % 4 == 0
    return dict(H=H, W=W, C=C, K=K, R=nr_resnet, F=nr_filters, M=nr_mix, nl=nonlinearity)


class Names:
    """nn.get_name counters (nn.py:151-157) -> parameter names in creation order."""

    def __init__(self):
        self.c = {}

    def __call__(self, kind):
        i = self.c.get(kind, 0)
        self.c[kind] = i + 1
        return "%s_%d" % (kind, i)


def param_shapes(spec):
    """Ordered {name: shape} of every variable model_spec creates, plus the highway FC."""
    shapes = {}
    nm = Names()
    F, R, K, M = spec["F"], spec["R"], spec["K"], spec["M"]
    cat = spec["nl"] == "concat_elu"
    nlc = lambda c: 2 * c if cat else c  # channels after the resnet nonlinearity

    def conv(cin, cout, kh, kw, kind="conv2d"):
        n = nm(kind)
        shapes[n + "/V"] = (kh, kw, cin, cout)
        shapes[n + "/g"] = (cout,)
        shapes[n + "/b"] = (cout,)

    def dense(cin, cout):
        n = nm("dense")
        shapes[n + "/V"] = (cin, cout)
        shapes[n + "/g"] = (cout,)
        shapes[n + "/b"] = (cout,)

    def resnet(kh, kw, a_ch=None):
        conv(nlc(F), F, kh, kw)
        if a_ch is not None:
            dense(nlc(a_ch), F)
        conv(nlc(F), 2 * F, kh, kw)
        shapes[nm("conditional_weights") + "/hw"] = (K, 2 * F)

    # up pass (model.py:37-58); the counter order follows the TF construction order
    conv(spec["C"] + 1, F, 2, 3)
    conv(spec["C"] + 1, F, 1, 3)
    conv(spec["C"] + 1, F, 2, 1)
    for stage in range(3):
        for _ in range(R):
            resnet(2, 3)
            resnet(2, 2, F)
        if stage < 2:
            conv(F, F, 2, 3)
            conv(F, F, 2, 2)
    # down pass (model.py:65-89)
    for stage in range(3):
        n = R if stage == 0 else R + 1
        for _ in range(n):
            resnet(2, 3, F)
            resnet(2, 2, 2 * F)
        if stage < 2:
            conv(F, F, 2, 3, "deconv2d")
            conv(F, F, 2, 2, "deconv2d")
    dense(F, 10 * M)  # nin(elu(ul), 10 * nr_mix)
    shapes["highway/W"] = (K, 1)  # pixelvae.py:136 fully_connected(latents, 1, sigmoid)
    shapes["highway/b"] = (1,)
    return shapes


def init_params(spec, seed=0):
    """nn.py initialisers: V ~ N(0, 0.05), g = 1, b = 0, hw ~ N(0, 0.05); highway FC Xavier."""
    rng = np.random.default_rng(seed)
    out = {}
    for name, shp in param_shapes(spec).items():
        leaf = name.split("/")[-1]
        if leaf in ("V", "hw"):
            out[name] = rng.normal(0.0, 0.05, size=shp)
        elif leaf == "g":
            out[name] = np.ones(shp)
        elif name == "highway/W":
            lim = math.sqrt(6.0 / (shp[0] + shp[1]))
            out[name] = rng.uniform(-lim, lim, size=shp)
        else:
            out[name] = np.zeros(shp)
    return out


# ---------------------------------------------------------------------------------------------
# ops (NHWC tensors, fp64)
# ---------------------------------------------------------------------------------------------
def _wn(V, g, axes):
    n = torch.sqrt((V * V).sum(dim=axes, keepdim=True))
    return V * (g / n)


def _nonlin(x, kind):
    if kind == "concat_elu":  # nn.py:12-15
        return Fn.elu(torch.cat([x, -x], dim=-1))
    if kind == "elu":
        return Fn.elu(x)
    return torch.relu(x)


class Net:
    """model_spec + loss + sample on explicit parameters (dict name -> fp64 tensor)."""

    def __init__(self, spec, params, bf16=False, init=False):
        self.s = spec
        self.p = params
        self.bf16 = bf16
        self.init = init  # data-dependent init pass (nn.py:176-180, :206-210): updates g, b
        self.nm = Names()
        self.updates = {}

    def _r(self, t):
        return _bf(t) if self.bf16 else t

    def _out_init(self, x, n, scale):
        if self.init:  # moments over every axis but the channel; the returned x is NOT normalised
            m = x.mean(dim=tuple(range(x.dim() - 1)))
            v = ((x - m) ** 2).mean(dim=tuple(range(x.dim() - 1)))
            si = scale / torch.sqrt(v + 1e-10)
            self.updates[n + "/g"] = (self.p[n + "/g"] * si).detach()
            self.updates[n + "/b"] = (self.p[n + "/b"] - m * si).detach()
        return x

    def conv(self, x, kh, kw, stride, pt, pl, init_scale=1.0):
        """nn.conv2d (:189-216) on an explicitly padded input: out(oy,ox) = sum in(oy*s - pt + ky,
        ox*s - pl + kx) W[ky,kx], VALID over the pad (pt top, pl left, the rest bottom/right)."""
        n = self.nm("conv2d")
        V, g, b = self.p[n + "/V"], self.p[n + "/g"], self.p[n + "/b"]
        Wt = self._r(_wn(V, g, (0, 1, 2)))
        xc = self._r(x).permute(0, 3, 1, 2)
        H, Wd = x.shape[1], x.shape[2]
        Ho, Wo = (H - 1) // stride + 1, (Wd - 1) // stride + 1
        pb = (Ho - 1) * stride + kh - H - pt
        pr = (Wo - 1) * stride + kw - Wd - pl
        xp = Fn.pad(xc, (pl, max(pr, 0), pt, max(pb, 0)))
        y = Fn.conv2d(xp, Wt.permute(3, 2, 0, 1), stride=stride).permute(0, 2, 3, 1) + b
        return self._out_init(y, n, init_scale)

    def deconv(self, x, kh, kw, cl):
        """nn.deconv2d VALID stride 2 (:219-252) cropped as down(_right)_shifted_deconv2d
        (:306-320): out(y, x) = full(y, x + cl), full(Y, X) = sum in(iy, ix) W[ky, kx] over
        Y = 2 iy + ky, X = 2 ix + kx."""
        n = self.nm("deconv2d")
        V, g, b = self.p[n + "/V"], self.p[n + "/g"], self.p[n + "/b"]
        Wt = self._r(_wn(V, g, (0, 1, 2)))  # canonical [kh, kw, Cin, Cout]
        xc = self._r(x).permute(0, 3, 1, 2)
        full = Fn.conv_transpose2d(xc, Wt.permute(2, 3, 0, 1), stride=2)
        H, Wd = x.shape[1], x.shape[2]
        y = full[:, :, :2 * H, cl:cl + 2 * Wd].permute(0, 2, 3, 1) + b
        return self._out_init(y, n, 1.0)

    def dense(self, x, init_scale=1.0):
        """nn.dense (:160-186) over the last axis (nin, :255-260)."""
        n = self.nm("dense")
        V, g, b = self.p[n + "/V"], self.p[n + "/g"], self.p[n + "/b"]
        Wt = self._r(_wn(V, g, (0,)))
        y = self._r(x) @ Wt + b
        return self._out_init(y, n, init_scale)

    def ds_conv(self, x, kh, kw, stride=1):
        return self.conv(x, kh, kw, stride, kh - 1, (kw - 1) // 2)

    def drs_conv(self, x, kh, kw, stride=1):
        return self.conv(x, kh, kw, stride, kh - 1, kw - 1)

    def gated_resnet(self, x, h, kh, kw, a=None, dmask=None):
        """nn.py:264-288 (dropout off unless a keep-mask is injected)."""
        nl = self.s["nl"]
        pad = (kh - 1, (kw - 1) // 2) if kw == 3 else (kh - 1, kw - 1)
        c1 = self.conv(_nonlin(x, nl), kh, kw, 1, *pad)
        if a is not None:
            c1 = c1 + self.dense(_nonlin(a, nl))
        c1 = _nonlin(c1, nl)
        if dmask is not None:
            c1 = c1 * dmask
        c2 = self.conv(c1, kh, kw, 1, *pad, init_scale=0.1)
        hw = self.p[self.nm("conditional_weights") + "/hw"]
        c2 = c2 + (h @ hw)[:, None, None, :]
        F = x.shape[-1]
        return x + c2[..., :F] * torch.sigmoid(c2[..., F:])

    def model(self, x, h, masks=None):
        """model_spec(x, h) (model.py:11-117) -> l [B, H, W, 10 M].  masks: the training pass's
        dropout keep-masks (1 / keep_prob or 0), one per gated resnet in construction order."""
        R = self.s["R"]
        mk = iter(masks) if masks is not None else None
        grn = self.gated_resnet

        def gr(x_, h_, kh, kw, a=None):
            m = None if mk is None else torch.as_tensor(next(mk), dtype=x_.dtype).reshape(x_.shape)
            return grn(x_, h_, kh, kw, a=a, dmask=m)
        ones = torch.ones(x.shape[:-1] + (1,), dtype=x.dtype)
        xp = torch.cat([x, ones], dim=-1)
        u = [down_shift(self.ds_conv(xp, 2, 3))]
        ul = [down_shift(self.ds_conv(xp, 1, 3)) + right_shift(self.drs_conv(xp, 2, 1))]
        for stage in range(3):
            for _ in range(R):
                u.append(gr(u[-1], h, 2, 3))
                ul.append(gr(ul[-1], h, 2, 2, a=u[-1]))
            if stage < 2:
                u.append(self.ds_conv(u[-1], 2, 3, stride=2))
                ul.append(self.drs_conv(ul[-1], 2, 2, stride=2))
        uu, uul = u.pop(), ul.pop()
        for stage in range(3):
            for _ in range(R if stage == 0 else R + 1):
                uu = gr(uu, h, 2, 3, a=u.pop())
                uul = gr(uul, h, 2, 2, a=torch.cat([uu, ul.pop()], dim=-1))
            if stage < 2:
                uu = self.deconv(uu, 2, 3, 1)
                uul = self.deconv(uul, 2, 2, 0)
        assert not u and not ul
        return self.dense(Fn.elu(uul))


def down_shift(x):
    """nn.py:292-294."""
    return torch.cat([torch.zeros_like(x[:, :1]), x[:, :-1]], dim=1)


def right_shift(x):
    """nn.py:296-298."""
    return torch.cat([torch.zeros_like(x[:, :, :1]), x[:, :, :-1]], dim=2)


def mix_logistic_logprob(x, l):
    """Per-pixel log p(x) (the negated summand of discretized_mix_logistic_loss, nn.py:46-87)."""
    B, H, W, C = x.shape
    M = l.shape[-1] // 10
    logit = l[..., :M]
    p = l[..., M:].reshape(B, H, W, C, 3 * M)
    means = p[..., :M]
    log_scales = torch.clamp(p[..., M:2 * M], min=-7.0)
    coeffs = torch.tanh(p[..., 2 * M:3 * M])
    xr = x[..., None].expand(B, H, W, C, M)
    m2 = means[:, :, :, 1] + coeffs[:, :, :, 0] * xr[:, :, :, 0]
    m3 = means[:, :, :, 2] + coeffs[:, :, :, 1] * xr[:, :, :, 0] + coeffs[:, :, :, 2] * xr[:, :, :, 1]
    means = torch.stack([means[:, :, :, 0], m2, m3], dim=3)
    cx = xr - means
    inv = torch.exp(-log_scales)
    plus_in = inv * (cx + 1.0 / 255.0)
    min_in = inv * (cx - 1.0 / 255.0)
    cdf_plus = torch.sigmoid(plus_in)
    cdf_min = torch.sigmoid(min_in)
    log_cdf_plus = plus_in - Fn.softplus(plus_in)
    log_one_minus_cdf_min = -Fn.softplus(min_in)
    cdf_delta = cdf_plus - cdf_min
    mid_in = inv * cx
    log_pdf_mid = mid_in - log_scales - 2.0 * Fn.softplus(mid_in)
    lp = torch.where(xr < -0.999, log_cdf_plus,
                     torch.where(xr > 0.999, log_one_minus_cdf_min,
                                 torch.where(cdf_delta > 1e-5, torch.log(torch.clamp(cdf_delta, min=1e-12)),
                                             log_pdf_mid - np.log(127.5))))
    lp = lp.sum(dim=3) + torch.log_softmax(logit, dim=-1)
    return torch.logsumexp(lp, dim=-1)


def mix_logistic_loss(x, l):
    """discretized_mix_logistic_loss(x, l, sum_all=True) (nn.py:46-87)."""
    return -mix_logistic_logprob(x, l).sum()


def mix_logistic_sample(l, u_mix, u_log):
    """sample_from_discretized_mix_logistic (nn.py:89-109) with its uniforms injected:
    u_mix [B,H,W,M] (Gumbel argmax), u_log [B,H,W,3] (logistic draw), both in (1e-5, 1-1e-5)."""
    B, H, W = l.shape[:3]
    M = l.shape[-1] // 10
    logit = l[..., :M]
    p = l[..., M:].reshape(B, H, W, 3, 3 * M)
    sel = Fn.one_hot(torch.argmax(logit - torch.log(-torch.log(u_mix)), dim=-1), M).to(l.dtype)[:, :, :, None, :]
    means = (p[..., :M] * sel).sum(-1)
    log_scales = torch.clamp((p[..., M:2 * M] * sel).sum(-1), min=-7.0)
    coeffs = (torch.tanh(p[..., 2 * M:3 * M]) * sel).sum(-1)
    xs = means + torch.exp(log_scales) * (torch.log(u_log) - torch.log(1.0 - u_log))
    x0 = torch.clamp(xs[..., 0], -1.0, 1.0)
    x1 = torch.clamp(xs[..., 1] + coeffs[..., 0] * x0, -1.0, 1.0)
    x2 = torch.clamp(xs[..., 2] + coeffs[..., 1] * x0 + coeffs[..., 2] * x1, -1.0, 1.0)
    return torch.stack([x0, x1, x2], dim=-1)


def highway_mix(sample, prev, latents, Wh, bh, lo, hi):
    """pixelvae.py:135-137 (repaired: min/max_highway_connection): per-image ratio."""
    r = lo + (hi - lo) * torch.sigmoid(latents @ Wh + bh)  # [B, 1]
    r = r[:, :, None, None]
    return r * sample + (1.0 - r) * prev, r


def to_tensors(params, requires_grad=True):
    return {k: torch.tensor(v, dtype=DT, requires_grad=requires_grad) for k, v in params.items()}


def loss_and_grads(spec, params, x, h, bf16=False):
    """NLL (sum over the batch) and d NLL / d every parameter (name -> ndarray)."""
    P = to_tensors(params)
    net = Net(spec, P, bf16=bf16)
    xt = torch.tensor(x, dtype=DT)
    ht = torch.tensor(h, dtype=DT)
    l = net.model(xt, ht)
    loss = mix_logistic_loss(xt, l)
    names = [k for k in P if not k.startswith("highway/")]
    gs = torch.autograd.grad(loss, [P[k] for k in names], allow_unused=True)
    grads = {k: (np.zeros(params[k].shape) if g is None else g.numpy()) for k, g in zip(names, gs)}
    return float(loss), l.detach().numpy(), grads


def data_init(spec, params, x, h, masks=None, bf16=False):
    """The init pass (model(..., init=True), pixelvae.py:103-105): new g, b of every weight-normed
    layer in construction order, each from its own (un-normalised) output moments.  masks: the
    pass's dropout keep-masks (pixelvae.py:103-105 passes dropout_p to the init model too);
    bf16: the HIP head's operand rounding."""
    P = to_tensors(params, requires_grad=False)
    net = Net(spec, P, bf16=bf16, init=True)
    net.model(torch.tensor(np.asarray(x), dtype=DT), torch.tensor(np.asarray(h), dtype=DT), masks=masks)
    out = dict(params)
    for k, v in net.updates.items():
        out[k] = v.numpy()
    return out
