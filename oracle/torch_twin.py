"""PyTorch-CPU autograd twin of the Sequential-VAE training subgraph — TEST INFRASTRUCTURE.

Second, independent restatement of the executed graph (sequential_vae.py:877-1212,
1537-1842; abstract_network.py:8-71), NCHW internally with explicit NHWC
flatten order for every FC input.  Used (a) to cross-check oracle/model.py and
(b) as the CPU throughput baseline in bench.py (``cpu_baseline.kind = "port"``):
the reference's own TF-CPU path cannot run here (no TensorFlow).
"""
import math
import os

import torch
import torch.nn.functional as Fn
from . import spec as _spec


def _same(n_in, k, s):
    n_out = -(-n_in // s)
    total = max((n_out - 1) * s + k - n_in, 0)
    return n_out, total // 2, total - total // 2


def conv2d_same(x, w_tf, s):
    """TF conv2d SAME; w_tf [kh,kw,Cin,Cout]; x NCHW."""
    k = w_tf.shape[0]
    _, pb, pa = _same(x.shape[2], k, s)
    xp = Fn.pad(x, (pb, pa, pb, pa))
    return Fn.conv2d(xp, w_tf.permute(3, 2, 0, 1), stride=s)


def conv2d_t_same(x, w_tf, s):
    """TF conv2d_transpose SAME; w_tf [kh,kw,Cout,Cin]; out = full[pb : pb + H*s]."""
    k = w_tf.shape[0]
    Ho = x.shape[2] * s
    _, pb, _ = _same(Ho, k, s)
    full = Fn.conv_transpose2d(x, w_tf.permute(3, 2, 0, 1), stride=s)
    return full[:, :, pb:pb + Ho, pb:pb + Ho]


def _bf(t):
    return t.to(torch.bfloat16).to(t.dtype)


def _split(t):
    """bf16 hi/lo split of an operand (the engine's dtype='bf16x3' staging): t ~ hi + lo."""
    hi = _bf(t)
    return hi, _bf(t - hi)


def _x3(f, a, b):
    """f bilinear in (a, b), evaluated as the engine's split-bf16 MFMA mode does:
    a_hi*b_hi + a_hi*b_lo + a_lo*b_hi (the a_lo*b_lo term dropped), summed in the working dtype."""
    ah, al = _split(a)
    bh, bl = _split(b)
    return f(ah, bh) + f(ah, bl) + f(al, bh)


class _RoundSTE(torch.autograd.Function):
    """bf16 storage of a pre-BN conv output (the engine's bf16 mode, DESIGN §5 "bf16 pre"): the value is
    rounded (RNE) where the GEMM epilogue stores it; the gradient passes unchanged (the engine's dpre is
    the gradient at the stored tensor and flows into the conv's backward as is)."""

    @staticmethod
    def forward(ctx, x):
        return _bf(x)

    @staticmethod
    def backward(ctx, g):
        return g


class _RoundedOp(torch.autograd.Function):
    """y = op(x, w) whose GEMM operands are rounded to bf16 exactly where the engine's
    dtype='bf16' path rounds them (fp32 accumulation everywhere):
      fwd   : round(x), round(w)       (gather-GEMM staging)
      dgrad : round(dy), round(w)      (gather-GEMM staging)
      wgrad : round(x), round(dy)      (weight-GEMM staging)
    each leg individually switchable (output conv-T / layer-0 dgrad run in fp32)."""

    @staticmethod
    def forward(ctx, x, w, fn, rf, rd, rw, split=False):
        ctx.fn, ctx.rd, ctx.rw, ctx.split = fn, rd, rw, split
        ctx.save_for_backward(x, w)
        if split:
            return _x3(fn, x, w) if rf else fn(x, w)
        return fn(_bf(x) if rf else x, _bf(w) if rf else w)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        if ctx.split:  # vjp_x(w, gy) and vjp_w(x, gy) are bilinear: split both operands of each
            def vx(ww, g):
                with torch.enable_grad():
                    xa = x.detach().requires_grad_(True)
                    return torch.autograd.grad(ctx.fn(xa, ww), xa, g)[0]

            def vw(xx, g):
                with torch.enable_grad():
                    wa = w.detach().requires_grad_(True)
                    return torch.autograd.grad(ctx.fn(xx, wa), wa, g)[0]
            gx = _x3(vx, w, gy) if ctx.rd else vx(w, gy)
            gw = _x3(vw, x, gy) if ctx.rw else vw(x, gy)
            return gx, gw, None, None, None, None, None
        with torch.enable_grad():
            xa = (_bf(x) if ctx.rd else x).detach().requires_grad_(True)
            wa = (_bf(w) if ctx.rd else w).detach().requires_grad_(True)
            gx, = torch.autograd.grad(ctx.fn(xa, wa), xa, _bf(gy) if ctx.rd else gy)
            xw = (_bf(x) if ctx.rw else x).detach().requires_grad_(True)
            ww = (_bf(w) if ctx.rw else w).detach().requires_grad_(True)
            gw, = torch.autograd.grad(ctx.fn(xw, ww), ww, _bf(gy) if ctx.rw else gy)
        return gx, gw, None, None, None, None, None


def bn_train(x, beta, eps=1e-3):
    dims = [0, 2, 3] if x.dim() == 4 else [0]
    m = x.mean(dim=dims, keepdim=True)
    v = ((x - m) ** 2).mean(dim=dims, keepdim=True)
    shape = [1, -1, 1, 1] if x.dim() == 4 else [1, -1]
    return (x - m) / torch.sqrt(v + eps) + beta.view(shape)


def lrelu(x):
    return torch.maximum(torch.minimum(x * 0.1, torch.zeros_like(x)), x)


def nhwc_flatten(x):
    return x.permute(0, 2, 3, 1).reshape(x.shape[0], -1)


def nhwc_unflatten(x, S, C):
    return x.reshape(x.shape[0], S, S, C).permute(0, 3, 1, 2)


class Twin:
    def __init__(self, cfg, struct, params, dtype=torch.float32, requires_grad=True, emulate_bf16=False,
                 emulate_split=False, pre_bf16=None):
        self.cfg, self.struct = cfg, struct
        self.P = {k: torch.tensor(v, dtype=dtype, requires_grad=requires_grad) for k, v in params.items()}
        self.dtype = dtype
        self.bf16 = emulate_bf16 or emulate_split
        self.split = emulate_split  # dtype='bf16x3': every rounded leg as hi/lo split products
        # bf16 mode stores every conv layer's pre-BN output as bf16 (the engine's SVAE_PRE_F32=1 keeps fp32)
        if pre_bf16 is None:
            pre_bf16 = emulate_bf16 and not emulate_split and os.environ.get("SVAE_PRE_F32", "0") != "1"
        self.pre_bf16 = pre_bf16

    def _op(self, fn, x, w, rf=True, rd=True, rw=True):
        if not self.bf16:
            return fn(x, w)
        return _RoundedOp.apply(x, w, fn, rf, rd, rw, self.split)

    def _conv(self, x, w, s, transpose):
        fn = (lambda a, b: conv2d_t_same(a, b, s)) if transpose else (lambda a, b: conv2d_same(a, b, s))
        # every conv / conv-T leg is a bf16 gather- or weight-GEMM (the layer-0 input gradient,
        # N = image channels, included: bf16 halo gather)
        return self._op(fn, x, w)

    def _cba(self, x, lay, s, act, transpose=False, residual=None):
        P = self.P
        y = self._conv(x, P[lay["w"]], s, transpose)
        if self.pre_bf16:
            y = _RoundSTE.apply(y)
        y = y + P[lay["b"]].view(1, -1, 1, 1)
        y = bn_train(y, P[lay["beta"]])
        if residual is not None:
            y = y + residual
        if act == "lrelu":
            y = lrelu(y)
        elif act == "relu":
            y = torch.relu(y)
        return y

    def _fcbn(self, x, lay, gemm=True):
        P = self.P
        mm = self._op(lambda a, b: a @ b, x, P[lay["w"]]) if gemm else x @ P[lay["w"]]
        return lrelu(bn_train(mm + P[lay["b"]], P[lay["beta"]]))

    def _fc(self, x, lay):
        return x @ self.P[lay["w"]] + self.P[lay["b"]]

    def inference(self, st, x):
        L, clip = self.cfg["levels"], self.cfg["latent_mean_clip"]
        cur, means, stds, ladder = x, [], [], None
        for lvl in range(L - 1):
            lv = st["levels"][lvl]
            cur = self._cba(self._cba(cur, lv["a"], 2, "lrelu"), lv["b"], 1, "lrelu")
            ladder = nhwc_flatten(cur)
            means.append(self._fc(ladder, lv["mean"]).clamp(-clip, clip))
            stds.append(torch.sigmoid(self._fc(ladder, lv["std"])))
        means.append(self._fc(ladder, st["last_mean"]).clamp(-clip, clip))
        stds.append(torch.sigmoid(self._fc(ladder, st["last_std"])))
        return torch.cat(means, 1), torch.cat(stds, 1)

    def encodings(self, st, xprev):
        L = self.cfg["levels"]
        cur, encs = xprev, [xprev]
        for lvl in range(L - 1):
            lv = st["levels"][lvl]
            cur = self._cba(self._cba(cur, lv["a"], 2, "lrelu"), lv["b"], 1, "lrelu")
            encs.append(cur)
        cur = nhwc_flatten(self._cba(cur, st["last_conv"], 2, "lrelu"))
        encs.append(self._fcbn(cur, st["last_fc"]))
        return encs

    def generator(self, st, xprev, z, enc_st):
        cfg = self.cfg
        L, F, S = cfg["levels"], cfg["filter_sizes"], cfg["image_sizes"]
        encs = self.encodings(enc_st, xprev) if xprev is not None else None
        parts = torch.split(z, cfg["latent_dims"], dim=1)
        lad = [nhwc_unflatten(self._fcbn(parts[i], st["split"][i], gemm=False), S[i + 1], F[i + 1])
               for i in range(L - 1)]
        lad.append(self._fcbn(parts[L - 1], st["split"][L - 1], gemm=False))
        cur = torch.cat([encs[L], lad[L - 1]], 1) if encs is not None else lad[L - 1]
        cur = nhwc_unflatten(self._fcbn(cur, st["top"]), S[L], F[L])
        for dl in st["levels"]:
            lvl = dl["level"]
            res = encs[lvl + 1] if encs is not None else None
            d = self._cba(cur, dl["s2"], 2, "relu", transpose=True, residual=res)
            cur = self._cba(torch.cat([d, lad[lvl]], 1), dl["s1"], 1, "relu", transpose=True)
        lo, hi = cfg["range"]
        P = self.P
        oc = lambda a, b: conv2d_t_same(a, b, 2)
        # output / ratio conv-T: bf16 forward (halo gather, N = C+1), fp32 input gradient (small-C
        # gather over the 4-channel packed gradient), bf16 weight gradient
        o = torch.sigmoid(self._op(oc, cur, P[st["out"]["w"]], rd=False) + P[st["out"]["b"]].view(1, -1, 1, 1))
        self._conv_output = o  # stddevs_prediction input (sequential_vae.py:1734)
        out = (hi - lo) * o + lo
        if encs is not None:
            r = torch.sigmoid(self._op(oc, cur, P[st["ratio"]["w"]], rd=False) +
                              P[st["ratio"]["b"]].view(1, -1, 1, 1))
            r = cfg["min_highway"] + (cfg["max_highway"] - cfg["min_highway"]) * r.expand(-1, cfg["C"], -1, -1)
            out = r * out + (1 - r) * encs[0]
        return out

    def stddevs(self, sst, o):
        """stddevs_prediction (sequential_vae.py:1866-1875): fp32 (no bf16 legs in the engine)."""
        cur = o
        for lay in sst["convs"]:
            P = self.P
            y = conv2d_same(cur, P[lay["w"]], 1) + P[lay["b"]].view(1, -1, 1, 1)
            cur = lrelu(bn_train(y, P[lay["beta"]]))
        s = torch.sigmoid(conv2d_same(cur, self.P[sst["out"]["w"]], 1) + self.P[sst["out"]["b"]].view(1, -1, 1, 1))
        return self.cfg["predict_generator_stddev_max"] * s

    def step(self, x_nhwc, target_nhwc, eps, reg_coeff=1.0, backward=True, noise=None):
        cfg = self.cfg
        x = torch.as_tensor(x_nhwc, dtype=self.dtype).permute(0, 3, 1, 2)
        tgt = torch.as_tensor(target_nhwc, dtype=self.dtype).permute(0, 3, 1, 2)
        eps = torch.as_tensor(eps, dtype=self.dtype)
        Tn, p2 = cfg["mc_steps"], cfg["latent_prior_stddev"] ** 2
        loss, prev, recs, kls, xhats = 0.0, None, [], [], []
        noisy, pgn = cfg.get("add_noise_to_chain", False), cfg.get("predict_generator_noise", False)
        imp, prev_mle = 0.0, None
        for t in range(Tn):
            st = self.struct[t]
            rin = prev if (cfg.get("predict_latent_code", False) and t >= 1) else x  # :1013-1016
            mu, sig = self.inference(st["inference"], rin)
            z = mu + sig * eps[t]
            xh = self.generator(st["generator"], prev, z, st.get("encoder"))
            sample = xh
            if noisy:  # :1088-1090
                nt = torch.as_tensor(noise[t], dtype=self.dtype).permute(0, 3, 1, 2)
                sd = self.stddevs(st["generator"]["stddev"], self._conv_output) if pgn else cfg["noise_stddevs"][t]
                sample = xh + reg_coeff * sd * nt
            if pgn:  # :1149-1150
                rec = (torch.log(sd) + 0.5 * math.log(2 * math.pi) + 0.5 * ((xh - tgt) / sd) ** 2).mean()
            else:
                rec = ((xh - tgt) ** 2).mean()
            if cfg.get("use_uniform_prior", False):  # :1159-1160
                kl = (-torch.log(sig)).mean(1).mean()
            else:
                kl = (-0.5 - torch.log(sig) + 0.5 * sig ** 2 / p2 + 0.5 * mu ** 2 / p2).mean(1).mean()
            if cfg.get("add_improvement_maximization_loss", False) and prev_mle is not None:  # :1189-1199
                imp = imp - reg_coeff * cfg["latent_pred_loss_coeff"] * ((xh - prev_mle) ** 2).sum(dim=(1, 2, 3)).mean()
            prev_mle = xh
            c = cfg["first_step_loss_coeff"] if t == 0 else 1.0
            if cfg["intermediate_reconstruction"] or t == Tn - 1:
                loss = loss + 16.0 * c * rec
            loss = loss + reg_coeff * c * _spec.kl_on(cfg, t) * kl  # :1154, :1170-1172
            recs.append(rec.detach())
            kls.append(kl.detach())
            xhats.append(xh.detach().permute(0, 2, 3, 1))
            prev = sample
        out = dict(loss=float(loss.detach()), final_loss=float(recs[-1]), recon=[float(r) for r in recs],
                   kl=[float(k) for k in kls], xhat=[h.numpy() for h in xhats])
        if backward:
            for p in self.P.values():
                p.grad = None
            loss.backward(retain_graph=torch.is_tensor(imp))
            out["grads"] = {k: (p.grad.numpy() if p.grad is not None else torch.zeros_like(p).numpy())
                            for k, p in self.P.items()}
            if torch.is_tensor(imp):
                for p in self.P.values():
                    p.grad = None
                imp.backward()
                out["imp_grads"] = {k: (p.grad.numpy() if p.grad is not None else torch.zeros_like(p).numpy())
                                    for k, p in self.P.items()}
        if torch.is_tensor(imp):
            out["imp_loss"] = float(imp.detach())
        return out
