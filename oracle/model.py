"""numpy float64 restatement of the executed Sequential-VAE training subgraph — TEST INFRASTRUCTURE.

Mirrors, function for function, the reference graph built by
``SequentialVAE.construct_network`` (sequential_vae.py:877-984) for the
configurations in BASELINE.json (inhomogeneous chain, concat noise, intermediate
reconstruction) and the chain variants of SURVEY §8(f3): Latent InfoMax, chain noise
with fixed or predicted stddevs (:1088-1091, :1147-1150, :1848-1875), the uniform
prior (:1159-1160) and the improvement-maximisation loss (:1182-1201).  ε is
injected ([T,B,Dz]) instead of drawn by ``tf.random_normal`` (:1023), and so is
the chain noise ([T,B,H,W,C], ``tf.random_normal(image_batch_shape)`` :1090).
"""
import numpy as np

from . import tape as T
from . import spec as S


def _conv_bn_act(tp, P, x, layer, stride, act, transpose=False, residual=None):
    """conv2d_bn_lrelu / conv2d_t_bn(_relu) (abstract_network.py:17-61).

    The pre-BN bias is added as in TF (it is zero-initialised and BN removes it)."""
    w = P[layer["w"]]
    y = (T.conv2d_transpose if transpose else T.conv2d)(tp, x, w, stride)
    y = T.bias_add(tp, y, P[layer["b"]])
    y = T.batch_norm(tp, y, P[layer["beta"]])
    if residual is not None:  # generator_ladder shortcut, sequential_vae.py:1712-1713
        y = T.add(tp, y, residual)
    if act == "lrelu":
        y = T.lrelu(tp, y)
    elif act == "relu":
        y = T.relu(tp, y)
    return y


def _fc_bn_lrelu(tp, P, x, layer):
    """fc_bn_lrelu (abstract_network.py:64-71)."""
    y = T.matmul(tp, x, P[layer["w"]])
    y = T.bias_add(tp, y, P[layer["b"]])
    y = T.batch_norm(tp, y, P[layer["beta"]])
    return T.lrelu(tp, y)


def _fc(tp, P, x, layer):
    return T.bias_add(tp, T.matmul(tp, x, P[layer["w"]]), P[layer["b"]])


def _flatten(tp, x):
    return T.reshape(tp, x, (x.v.shape[0], -1))  # NHWC flatten, (h*W+w)*C+c


def inference_ladder(tp, P, cfg, st, x):
    """sequential_vae.py:1579-1630 (phi/inference_step_t)."""
    L = cfg["levels"]
    clip = cfg["latent_mean_clip"]
    cur = x
    means, stds = [], []
    ladder = None
    for lvl in range(L - 1):
        lv = st["levels"][lvl]
        hidden = _conv_bn_act(tp, P, cur, lv["a"], 2, "lrelu")
        cur = _conv_bn_act(tp, P, hidden, lv["b"], 1, "lrelu")
        ladder = _flatten(tp, cur)
        m = _fc(tp, P, ladder, lv["mean"])
        if np.isfinite(clip):
            m = T.clip(tp, m, -clip, clip)
        s = T.sigmoid(tp, _fc(tp, P, ladder, lv["std"]))
        means.append(m)
        stds.append(s)
    # :1602-1605 — last conv + fc_bn_lrelu: output unused (dead) -> not evaluated.
    # :1607-1609 — the last heads read `ladder` (level L-2 flatten).
    m = _fc(tp, P, ladder, st["last_mean"])
    if np.isfinite(clip):
        m = T.clip(tp, m, -clip, clip)
    s = T.sigmoid(tp, _fc(tp, P, ladder, st["last_std"]))
    means.append(m)
    stds.append(s)
    return T.concat_last(tp, means), T.concat_last(tp, stds)


def compute_encodings(tp, P, cfg, st, xprev):
    """sequential_vae.py:1764-1777."""
    L = cfg["levels"]
    cur = xprev
    encs = [xprev]
    for lvl in range(L - 1):
        lv = st["levels"][lvl]
        hidden = _conv_bn_act(tp, P, cur, lv["a"], 2, "lrelu")
        cur = _conv_bn_act(tp, P, hidden, lv["b"], 1, "lrelu")
        encs.append(cur)
    cur = _conv_bn_act(tp, P, cur, st["last_conv"], 2, "lrelu")
    cur = _flatten(tp, cur)
    encs.append(_fc_bn_lrelu(tp, P, cur, st["last_fc"]))
    return encs


def split_latent(tp, P, cfg, st, z):
    """sequential_vae.py:1796-1808."""
    L, F, S = cfg["levels"], cfg["filter_sizes"], cfg["image_sizes"]
    parts = T.split_last(tp, z, cfg["latent_dims"])
    ladder = []
    for i in range(L - 1):
        y = _fc_bn_lrelu(tp, P, parts[i], st["split"][i])
        ladder.append(T.reshape(tp, y, (-1, S[i + 1], S[i + 1], F[i + 1])))
    ladder.append(_fc_bn_lrelu(tp, P, parts[L - 1], st["split"][L - 1]))
    return ladder


def generator_ladder(tp, P, cfg, st, xprev, z, enc_st, rec=None):
    """sequential_vae.py:1679-1739 with combine_noise('concat') (:1833-1834)."""
    L, F, S = cfg["levels"], cfg["filter_sizes"], cfg["image_sizes"]
    encodings = compute_encodings(tp, P, cfg, enc_st, xprev) if xprev is not None else None
    ladder = split_latent(tp, P, cfg, st, z)
    if encodings is not None:
        cur = T.concat_last(tp, [encodings[L], ladder[L - 1]])
    else:
        cur = ladder[L - 1]
    cur = _fc_bn_lrelu(tp, P, cur, st["top"])
    if rec is not None:
        rec["top_act"] = cur
    cur = T.reshape(tp, cur, (-1, S[L], S[L], F[L]))
    for dl in st["levels"]:
        lvl = dl["level"]
        res = encodings[lvl + 1] if encodings is not None else None
        deconv = _conv_bn_act(tp, P, cur, dl["s2"], 2, "relu", transpose=True, residual=res)
        deconv = T.concat_last(tp, [deconv, ladder[lvl]])
        cur = _conv_bn_act(tp, P, deconv, dl["s1"], 1, "relu", transpose=True)
        if rec is not None:
            rec["s1_act_%d" % lvl] = cur
            rec["cat_%d" % lvl] = deconv
    lo, hi = cfg["range"]
    o = T.conv2d_transpose(tp, cur, P[st["out"]["w"]], 2)
    o = T.sigmoid(tp, T.bias_add(tp, o, P[st["out"]["b"]]))
    if rec is not None:
        rec["conv_output"] = o  # input of stddevs_prediction (:1734)
    output = T.affine(tp, o, hi - lo, lo)
    if encodings is not None:
        r = T.conv2d_transpose(tp, cur, P[st["ratio"]["w"]], 2)
        r = T.sigmoid(tp, T.bias_add(tp, r, P[st["ratio"]["b"]]))
        mn, mx = cfg["min_highway"], cfg["max_highway"]
        r = T.affine(tp, T.tile_last(tp, r, cfg["C"]), mx - mn, mn)
        one_minus = T.affine(tp, r, -1.0, 1.0)
        output = T.add(tp, T.mul(tp, r, output), T.mul(tp, one_minus, encodings[0]))
    return output


def stddevs_prediction(tp, P, cfg, sst, o):
    """sequential_vae.py:1866-1875: conv2d_bn_lrelu (4x4, stride 1) per filter size, a 1x1
    conv2d with sigmoid, times predict_generator_stddev_max -> [B,H,W,1]."""
    cur = o
    for lay in sst["convs"]:
        cur = _conv_bn_act(tp, P, cur, lay, 1, "lrelu")
    s = T.conv2d(tp, cur, P[sst["out"]["w"]], 1)
    s = T.sigmoid(tp, T.bias_add(tp, s, P[sst["out"]["b"]]))
    return T.affine(tp, s, cfg["predict_generator_stddev_max"], 0.0)


def forward_backward(cfg, struct, params, x, target, eps, reg_coeff=1.0, want_grads=True, noise=None):
    """One training iteration's fwd (+bwd) — the value of ``self.loss``,
    ``self.final_loss`` and d loss / d every trainable variable
    (sequential_vae.py:1273 ``compute_gradients``, before clipping).  With the chain noise on,
    ``noise`` [T,B,H,W,C] is the N(0,1) draw of :1090 per step.  With the improvement-maximisation
    loss on, ``imp_loss`` and ``imp_grads`` (its gradient, :1302-1303) are returned as well."""
    tp = T.Tape()
    P = {k: tp.leaf(v) for k, v in params.items()}
    xin = tp.leaf(np.asarray(x, np.float64))
    target = np.asarray(target, np.float64)
    Tn = cfg["mc_steps"]
    terms, coeffs = [], []
    out = dict(recon=[], kl=[], recon_img=[], kl_img=[], xhat=[], mu=[], sig=[], z=[])
    znodes, xnodes, recs = [], [], []
    out.update(sample=[], sd=[])
    noisy = cfg.get("add_noise_to_chain", False)
    pgn = cfg.get("predict_generator_noise", False)
    imp_terms = []
    prev, prev_mle = None, None   # training_samples[t-1], training_mles[t-1]
    for t in range(Tn):
        st = struct[t]
        # recognition input: x, or x_{t-1} in Latent InfoMax mode (sequential_vae.py:1013-1016)
        rin = prev if (cfg.get("predict_latent_code", False) and t >= 1) else xin
        mu, sig = inference_ladder(tp, P, cfg, st["inference"], rin)
        e = tp.leaf(np.asarray(eps[t], np.float64))
        z = T.add(tp, mu, T.mul(tp, sig, e))                       # :1023
        recd = {}
        xhat = generator_ladder(tp, P, cfg, st["generator"], prev, z, st.get("encoder"), recd)
        recs.append(recd)
        sd = None
        sample = xhat
        if noisy:  # training_sample = mle + reg * stddevs * N(0,1)  (:1088-1090)
            nt = np.asarray(noise[t], np.float64)
            if pgn:
                sd = stddevs_prediction(tp, P, cfg, st["generator"]["stddev"], recd["conv_output"])
                sample = T.add_scaled_noise(tp, xhat, sd, nt, reg_coeff)
            else:
                sample = T.add_scaled_noise(tp, xhat, cfg["noise_stddevs"][t], nt, reg_coeff)
        if pgn:
            rec = T.nll_per_row(tp, xhat, target, sd)              # :1149-1150
        else:
            rec = T.mean_sq_err_per_row(tp, xhat, target)          # :1146
        if cfg.get("use_uniform_prior", False):
            kl = T.kl_uniform_per_row(tp, sig)                     # :1159-1160
        else:
            kl = T.kl_per_row(tp, mu, sig, cfg["latent_prior_stddev"])  # :1156-1158
        if cfg.get("add_improvement_maximization_loss", False) and prev_mle is not None:
            # reg * latent_pred_loss_coeff * -reduce_mean(||x_t - x_{t-1}||^2)  (:1189-1199)
            imp_terms.append(T.mean_all(tp, T.sq_norm_diff_per_row(tp, xhat, prev_mle)))
        rec_m, kl_m = T.mean_all(tp, rec), T.mean_all(tp, kl)      # :1163-1164
        c_first = cfg["first_step_loss_coeff"] if t == 0 else 1.0  # :1175-1176 (applies to step-0 terms)
        if cfg["intermediate_reconstruction"] or t == Tn - 1:       # :1167-1168
            terms.append(rec_m)
            coeffs.append(16.0 * c_first)
        terms.append(kl_m)                                          # :1154, :1170-1172
        coeffs.append(reg_coeff * c_first * S.kl_on(cfg, t))
        out["recon"].append(float(rec_m.v))
        out["kl"].append(float(kl_m.v))
        out["recon_img"].append(rec.v.copy())
        out["kl_img"].append(kl.v.copy())
        out["xhat"].append(xhat.v.copy())
        out["mu"].append(mu.v.copy())
        out["sig"].append(sig.v.copy())
        out["z"].append(z.v.copy())
        out["sample"].append(sample.v.copy())
        out["sd"].append(None if sd is None else sd.v.copy())
        znodes.append(z)
        xnodes.append(xhat)
        prev, prev_mle = sample, xhat
    loss = T.scalar_sum(tp, terms, coeffs)
    out["loss"] = float(loss.v)
    out["final_loss"] = out["recon"][-1]                            # :1204
    # ELBO per image: sum_t [16*recon_t + reg*KL_t] with the same coefficients
    elbo_img = np.zeros(x.shape[0])
    for t in range(Tn):
        c_first = cfg["first_step_loss_coeff"] if t == 0 else 1.0
        if cfg["intermediate_reconstruction"] or t == Tn - 1:
            elbo_img += 16.0 * c_first * out["recon_img"][t]
        elbo_img += reg_coeff * c_first * S.kl_on(cfg, t) * out["kl_img"][t]
    out["elbo_img"] = elbo_img
    if want_grads:
        tp.backward(loss)
        out["grads"] = {k: (n.g if n.g is not None else np.zeros_like(n.v)) for k, n in P.items()}
        out["dz"] = [n.g.copy() for n in znodes]          # d loss / d z_t
        out["dxhat"] = [n.g.copy() for n in xnodes]       # d loss / d x_hat_t (total)
        out["dec_grads"] = [{k: (n.g.copy() if n.g is not None else None) for k, n in r.items()} for r in recs]
    if imp_terms:
        c = -reg_coeff * cfg["latent_pred_loss_coeff"]
        imp = T.scalar_sum(tp, imp_terms, [c] * len(imp_terms))
        out["imp_loss"] = float(imp.v)
        if want_grads:
            T.zero_grads(tp)
            tp.backward(imp)
            out["imp_grads"] = {k: (n.g if n.g is not None else np.zeros_like(n.v)) for k, n in P.items()}
    return out


def generate(cfg, struct, params, z):
    """Generative mode (sequential_vae.py:947-952, :1025, :1070-1073): the generator chain on
    given latents z [T,B,Dz] (N(0,1) at generation time, generate_mc_samples :1393-1428), no
    recognition network, x_0 = generator_first_step(z_0), x_t = generator(x_{t-1}, z_t), the same
    (reused) variables, BatchNorm in training mode on the generated batch.  Returns [x_hat_t]."""
    tp = T.Tape()
    P = {k: tp.leaf(v) for k, v in params.items()}
    out, prev = [], None
    for t in range(cfg["mc_steps"]):
        st = struct[t]
        zt = tp.leaf(np.asarray(z[t], np.float64))
        xhat = generator_ladder(tp, P, cfg, st["generator"], prev, zt, st.get("encoder"))
        out.append(xhat.v.copy())
        prev = xhat
    return out


def adam_update(params, grads, m, v, step, lr=2e-4, clip=10.0, b1=0.9, b2=0.999, eps=1e-8):
    """clip_by_value(±10) (sequential_vae.py:1274-1275) + tf.train.AdamOptimizer
    (:1267,1276): lr_t = lr*sqrt(1-b2^t)/(1-b1^t); w -= lr_t*m/(sqrt(v)+eps)."""
    lr_t = lr * np.sqrt(1.0 - b2 ** step) / (1.0 - b1 ** step)
    for k in params:
        g = np.clip(grads[k], -clip, clip)
        m[k] = b1 * m[k] + (1.0 - b1) * g
        v[k] = b2 * v[k] + (1.0 - b2) * g * g
        params[k] = params[k] - lr_t * m[k] / (np.sqrt(v[k]) + eps)
    return params, m, v
