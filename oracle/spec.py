"""Model geometry + TF-variable table of the executed graph (oracle copy) — TEST INFRASTRUCTURE.

Restates the variable scopes/creation order of the reference so that the
product's C-ABI layout (``svae_param_layout``) can be checked against it:

* ``phi/inference_step_t``            — inference_ladder (sequential_vae.py:1573-1609)
* ``theta/generative_encoder_step_t`` — compute_encodings (sequential_vae.py:1757-1775), t >= 1
* ``theta/generative_step_t``         — split_latent + generator_ladder (sequential_vae.py:1683-1727)

Names follow tf.contrib.layers' default scope naming (``Conv``, ``Conv_1``,
``BatchNorm``, ``fully_connected_2``, ``Conv2d_transpose_3`` …).  ``dead`` marks
variables created by the reference but never on the executed path (the last
inference level's conv + fc_bn_lrelu, sequential_vae.py:1602-1605, whose output
is unused because the level-3 heads read ``ladder``); ``zero_grad`` marks the
conv/FC biases that sit in front of a BatchNorm (their gradient is identically
zero: BN subtracts the batch mean).
"""
import numpy as np

PRESETS = {
    # sequential_vae.py:201-258 defaults == netname c_inhomog (:727) / sequential_vae_celebA_inhomog (:671)
    "celeba": dict(H=64, W=64, C=3, levels=4, filter_sizes=[3, 32, 64, 128, 384, 512],
                   latent_dims=[3, 3, 3, 3], mc_steps=8, batch=128, range=(-1.0, 1.0)),
    # sequential_vae_lsun (:712-714)
    "lsun": dict(H=64, W=64, C=3, levels=4, filter_sizes=[3, 32, 64, 128, 384, 512],
                 latent_dims=[20, 30, 30, 30], mc_steps=8, batch=256, range=(-1.0, 1.0)),
    # m_* 3-level geometry (:842-848), latent [8,8,8] (:815), one step
    "mnist_1step": dict(H=32, W=32, C=1, levels=3, filter_sizes=[1, 64, 128, 192, 256],
                        latent_dims=[8, 8, 8], mc_steps=1, batch=64, range=(0.0, 1.0)),
    # small geometry for fast parity tests (same code path as celeba: 4 levels)
    "tiny": dict(H=32, W=32, C=3, levels=4, filter_sizes=[3, 8, 8, 16, 24, 16],
                 latent_dims=[2, 2, 3, 2], mc_steps=3, batch=4, range=(-1.0, 1.0)),
}

DEFAULTS = dict(intermediate_reconstruction=True, first_step_loss_coeff=1.0,
                latent_prior_stddev=1.0, latent_mean_clip=float("inf"),
                min_highway=0.0, max_highway=1.0, predict_latent_code=False,
                predict_latent_code_with_regularization=False, regularized_steps=None,
                # chain-noise variants (sequential_vae.py:232-240): noise added to the sample fed to
                # the next step, fixed per-step stddevs or predicted by a per-step conv network
                use_uniform_prior=False, add_noise_to_chain=False, noise_stddevs=None,
                predict_generator_noise=False, predict_generator_stddev_max=1.0,
                stddev_filter_sizes=(5, 5, 5, 5, 5),
                # improvement maximisation (:227, :253, :1182-1201, own optimiser :1299-1316)
                add_improvement_maximization_loss=False, latent_pred_loss_coeff=0.001)

# sequential_vae.py:239 (exactly mc_steps long; the last entry 0 so the chain ends on its MLE)
DEFAULT_NOISE_STDDEVS = [0.5 ** 1, 0.5 ** 2, 0.5 ** 3, 0.5 ** 4, 0.5 ** 5, 0.5 ** 6, 0.5 ** 7, 0.0]


def kl_on(cfg, t):
    """Does step t's KL term enter self.loss?  sequential_vae.py:1154 (``step in
    self.regularized_steps``) and :1170-1172 (Latent InfoMax: step 0 only, unless
    predict_latent_code_with_regularization)."""
    rs = cfg.get("regularized_steps")
    if rs is not None and t not in rs:
        return 0.0
    plc = cfg.get("predict_latent_code", False)
    return 1.0 if (not plc or cfg.get("predict_latent_code_with_regularization", False) or t == 0) else 0.0


def make_config(preset="celeba", **over):
    cfg = dict(DEFAULTS)
    cfg.update(PRESETS[preset])
    cfg.update(over)
    L = cfg["levels"]
    cfg["image_sizes"] = [cfg["H"] // (2 ** i) for i in range(L + 1)]
    cfg["latent_dim"] = int(sum(cfg["latent_dims"]))
    if cfg["add_noise_to_chain"] and not cfg["predict_generator_noise"] and cfg["noise_stddevs"] is None:
        nd = DEFAULT_NOISE_STDDEVS
        assert cfg["mc_steps"] <= len(nd), "noise_stddevs must be given for mc_steps > 8"
        cfg["noise_stddevs"] = list(nd[:cfg["mc_steps"]])  # the reference indexes noise_stddevs[step]
    if cfg["predict_generator_noise"]:
        # stddevs = 0 without the chain noise (:1664-1671), and the NLL then takes log(0)
        assert cfg["add_noise_to_chain"], "predict_generator_noise needs add_noise_to_chain"
    assert len(cfg["filter_sizes"]) == L + 2 and len(cfg["latent_dims"]) == L
    return cfg


class _Scope:
    def __init__(self, prefix, out):
        self.prefix, self.out = prefix, out
        self.cnt = {}

    def _name(self, kind):
        i = self.cnt.get(kind, 0)
        self.cnt[kind] = i + 1
        return kind if i == 0 else "%s_%d" % (kind, i)

    def add(self, kind, entries, dead=False):
        base = self._name(kind)
        names = []
        for suffix, shape, init, zero_grad in entries:
            n = "%s/%s/%s" % (self.prefix, base, suffix)
            self.out.append(dict(name=n, shape=tuple(int(s) for s in shape), init=init,
                                 dead=dead, zero_grad=zero_grad or dead))
            names.append(n)
        return names

    # abstract_network.py:17-24 / 55-71
    def conv_bn(self, shape, transpose=False, dead=False):
        kind = "Conv2d_transpose" if transpose else "Conv"
        cout = shape[2] if transpose else shape[3]
        w, b = self.add(kind, [("weights", shape, "normal0.02", False), ("biases", (cout,), "zeros", True)], dead)
        (beta,) = self.add("BatchNorm", [("beta", (cout,), "zeros", False)], dead)
        return dict(w=w, b=b, beta=beta)

    def fc_bn(self, nin, nout, dead=False):
        w, b = self.add("fully_connected", [("weights", (nin, nout), "normal0.02", False),
                                            ("biases", (nout,), "zeros", True)], dead)
        (beta,) = self.add("BatchNorm", [("beta", (nout,), "zeros", False)], dead)
        return dict(w=w, b=b, beta=beta)

    def fc(self, nin, nout):  # layers.fully_connected default init (xavier)
        w, b = self.add("fully_connected", [("weights", (nin, nout), "glorot", False),
                                            ("biases", (nout,), "zeros", False)])
        return dict(w=w, b=b)

    def convt_plain(self, shape):  # conv2d_t with default (xavier) init, sequential_vae.py:1720,1727
        w, b = self.add("Conv2d_transpose", [("weights", shape, "glorot", False),
                                             ("biases", (shape[2],), "zeros", False)])
        return dict(w=w, b=b)


def build_params(cfg):
    """Returns (table, struct): ``table`` is the ordered variable list, ``struct``
    the per-step name map used by model.py / torch_twin.py."""
    L, F, D, S = cfg["levels"], cfg["filter_sizes"], cfg["latent_dims"], cfg["image_sizes"]
    C = cfg["C"]
    table, struct = [], []
    for t in range(cfg["mc_steps"]):
        st = {}
        # ---- phi: inference_ladder (sequential_vae.py:1585-1609)
        sc = _Scope("phi/inference_step_%d" % t, table)
        inf = []
        cin = F[0]
        for lvl in range(L - 1):
            a = sc.conv_bn((4, 4, cin, F[lvl + 1]))
            b = sc.conv_bn((4, 4, F[lvl + 1], F[lvl + 1]))
            nflat = S[lvl + 1] * S[lvl + 1] * F[lvl + 1]
            hm = sc.fc(nflat, D[lvl])
            hs = sc.fc(nflat, D[lvl])
            inf.append(dict(a=a, b=b, mean=hm, std=hs))
            cin = F[lvl + 1]
        dead_conv = sc.conv_bn((4, 4, F[L - 1], F[L - 1]), dead=True)
        dead_fc = sc.fc_bn(S[L] * S[L] * F[L - 1], F[L], dead=True)
        nflat = S[L - 1] * S[L - 1] * F[L - 1]
        hm = sc.fc(nflat, D[L - 1])
        hs = sc.fc(nflat, D[L - 1])
        st["inference"] = dict(levels=inf, last_mean=hm, last_std=hs, dead=[dead_conv, dead_fc])
        # ---- theta: compute_encodings (sequential_vae.py:1764-1775), only for t >= 1
        if t >= 1:
            sc = _Scope("theta/generative_encoder_step_%d" % t, table)
            enc = []
            cin = F[0]
            for lvl in range(L - 1):
                a = sc.conv_bn((4, 4, cin, F[lvl + 1]))
                b = sc.conv_bn((4, 4, F[lvl + 1], F[lvl + 1]))
                enc.append(dict(a=a, b=b))
                cin = F[lvl + 1]
            c = sc.conv_bn((4, 4, F[L - 1], F[L - 1]))
            fcl = sc.fc_bn(S[L] * S[L] * F[L - 1], F[L])
            st["encoder"] = dict(levels=enc, last_conv=c, last_fc=fcl)
        # ---- theta: split_latent + generator_ladder (sequential_vae.py:1689-1727)
        sc = _Scope("theta/generative_step_%d" % t, table)
        split = []
        for i in range(L - 1):
            split.append(sc.fc_bn(D[i], S[i + 1] * S[i + 1] * F[i + 1]))
        split.append(sc.fc_bn(D[L - 1], F[L + 1]))
        top_in = F[L + 1] + (F[L] if t >= 1 else 0)
        top = sc.fc_bn(top_in, S[L] * S[L] * F[L])
        dec = []
        cin = F[L]
        for lvl in range(L - 2, -1, -1):
            s2 = sc.conv_bn((4, 4, F[lvl + 1], cin), transpose=True)
            s1 = sc.conv_bn((4, 4, F[lvl + 1], 2 * F[lvl + 1]), transpose=True)
            dec.append(dict(level=lvl, s2=s2, s1=s1))
            cin = F[lvl + 1]
        out = sc.convt_plain((4, 4, C, F[1]))
        ratio = sc.convt_plain((4, 4, 1, F[1])) if t >= 1 else None
        st["generator"] = dict(split=split, top=top, levels=dec, out=out, ratio=ratio)
        if cfg.get("add_noise_to_chain") and cfg.get("predict_generator_noise"):
            # stddevs_prediction (:1866-1875), created after the output / ratio conv-T: conv2d_bn_lrelu
            # 4x4 s1 per entry of predict_generator_stddev_filter_sizes, then a 1x1 conv2d (default
            # xavier init, bias) with sigmoid
            convs, cin = [], C
            for f in cfg["stddev_filter_sizes"]:
                convs.append(sc.conv_bn((4, 4, cin, f)))
                cin = f
            w, b = sc.add("Conv", [("weights", (1, 1, cin, 1), "glorot", False), ("biases", (1,), "zeros", False)])
            st["generator"]["stddev"] = dict(convs=convs, out=dict(w=w, b=b))
        struct.append(st)
    return table, struct


def init_params(cfg, seed=0, dtype=np.float64):
    from .weightgen import generate
    table, struct = build_params(cfg)
    params = {p["name"]: generate(p["name"], p["shape"], p["init"], seed).astype(dtype) for p in table}
    return table, struct, params


def make_inputs(cfg, batch=None, seed_x=0, seed_eps=1):
    """Synthetic batch of SURVEY §8d: x ~ U[range] (PCG64 seed 0), target = x,
    eps ~ N(0,1) [T,B,Dz] (PCG64 seed 1)."""
    B = batch or cfg["batch"]
    lo, hi = cfg["range"]
    rx = np.random.default_rng(seed_x)
    x = rx.uniform(lo, hi, size=(B, cfg["H"], cfg["W"], cfg["C"])).astype(np.float32)
    re = np.random.default_rng(seed_eps)
    eps = re.standard_normal(size=(cfg["mc_steps"], B, cfg["latent_dim"])).astype(np.float32)
    return x, x.copy(), eps


def make_chain_noise(cfg, batch=None, seed=2):
    """N(0,1) chain noise [T,B,H,W,C] of training_sample = mle + reg*stddevs*noise
    (sequential_vae.py:1090), PCG64 seed 2 (injected like eps)."""
    B = batch or cfg["batch"]
    r = np.random.default_rng(seed)
    return r.standard_normal(size=(cfg["mc_steps"], B, cfg["H"], cfg["W"], cfg["C"])).astype(np.float32)


# ---- homogeneous chains: TF variable sharing (sequential_vae.py:107-113) ----
def shared_name(name, share_theta, share_phi, plc=False):
    """Scope a per-step variable takes under weight sharing:
    share_phi   -> "phi/inference_network" for every step (:1573-1577, predict_latent_code off);
    share_theta -> "theta/generative_encoder_network" (:1757-1761) and, for steps >= 1 only,
                   "theta/generative_network" (:1683-1687; step 0 keeps generative_step_0)."""
    head, _, rest = name.partition("/")
    scope, _, tail = rest.partition("/")
    if share_phi and head == "phi" and scope.startswith("inference_step_") and not (plc and scope == "inference_step_0"):
        return "phi/inference_network/" + tail
    if share_theta and head == "theta" and scope.startswith("generative_encoder_step_"):
        return "theta/generative_encoder_network/" + tail
    if share_theta and head == "theta" and scope.startswith("generative_step_") and int(scope.split("_")[-1]) >= 1:
        return "theta/generative_network/" + tail
    return name


def shared_table(cfg, share_theta=True, share_phi=True):
    plc = cfg.get("predict_latent_code", False)
    """Variables of the homogeneous model in TF creation order (first use creates, AUTO_REUSE
    reuses): one entry per shared name."""
    table, _ = build_params(cfg)
    seen, out = set(), []
    for p in table:
        n = shared_name(p["name"], share_theta, share_phi, plc)
        if n not in seen:
            seen.add(n)
            out.append(dict(p, name=n))
    return out


def expand_shared(params_pub, cfg, share_theta=True, share_phi=True):
    """Per-step (inhomogeneous-layout) parameter dict whose copies alias the shared tensors."""
    table, _ = build_params(cfg)
    plc = cfg.get("predict_latent_code", False)
    return {p["name"]: params_pub[shared_name(p["name"], share_theta, share_phi, plc)] for p in table}


def sum_shared_grads(grads, share_theta=True, share_phi=True, plc=False):
    """Gradient of each shared variable = sum over the steps that use it (TF's gradient of a
    variable read in several places)."""
    out = {}
    for n, g in grads.items():
        k = shared_name(n, share_theta, share_phi, plc)
        out[k] = out[k] + g if k in out else np.array(g, copy=True)
    return out
