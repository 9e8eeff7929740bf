"""PixelCNN++ decoder head over the HIP kernels of include/svae_pcnn.h.

Mirrors the reference's interface for this head:
  * ``PixelCNNpp.model(x, h)``      pixel_cnn_pp/model.py:11-117 (model_spec, conditional on h)
  * ``PixelCNNpp.loss(x, h)``       + nn.discretized_mix_logistic_loss (nn.py:46-87), sum_all
  * ``PixelCNNpp.data_init(x, h)``  the init pass (pixelvae.py:103-105; nn.py:176-180, :206-210)
  * ``PixelCNNpp.sample(h, ...)``   sample_from_model's autoregressive loop (pixelvae.py:170-194)
                                    with nn.sample_from_discretized_mix_logistic (nn.py:89-109)
  * ``make_pixel_cnn(...)``         pixelvae.py:68-158, repaired: returns
                                    (highway_train_out, 0, cache) like the reference.

Every tensor op runs in libsvae_hip.so (bf16-MFMA gather convolutions and weight gradients, fused
elementwise kernels, the mixture loss with its analytic gradient); torch only allocates device
memory.  The backward is an explicit tape of the forward's primitive ops in reverse.

Parameters live in one flat fp32 buffer (canonical layouts: conv / deconv V [kh, kw, Cin, Cout],
dense V [in, out], hw [K, 2F]); names follow the reference's layer counters (nn.py:151-157).
"""
import ctypes
import math

import numpy as np
import torch

from . import _lib

NL_KIND = {"relu": 0, "elu": 1, "concat_elu": 2}


def _p(t, off=0):
    """Device pointer of fp32 tensor ``t`` at element offset ``off`` (None-safe)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr() + 4 * off)


def _ck(rc):
    _lib.check(rc)


def _r16(c):
    """K padding of the bf16 weight copies: 32 (the LDS-staged conv's K chunk)."""
    return (c + 31) // 32 * 32


class DropMask:
    """A dropout keep-mask drawn inside the nonlinearity kernels from (seed, keep) instead of stored:
    ``shape`` (rows, channels); ``tensor(net)`` writes the same mask out (svae_pcnn_dropout_mask)."""
    __slots__ = ("shape", "keep", "seed")

    def __init__(self, rows, c, keep, seed):
        self.shape, self.keep, self.seed = (rows, c), float(keep), int(seed)

    def tensor(self, net):
        m = torch.empty(self.shape, dtype=torch.float32, device=net.dev)
        _ck(net.L.svae_pcnn_dropout_mask(m.numel(), self.keep, self.seed, _p(m), _lib.stream_ptr()))
        return m


class Act:
    """An NHWC activation: ``buf`` [n*h*w][ld] fp32 (or bf16: a nonlinearity output read only by the
    bf16-MFMA convs), channels [off, off + c)."""
    __slots__ = ("buf", "off", "c", "ld", "n", "h", "w", "amax", "planes")

    def __init__(self, buf, c, n, h, w, off=0, ld=None, amax=None):
        self.buf, self.c, self.n, self.h, self.w, self.off = buf, c, n, h, w, off
        self.ld = c if ld is None else ld
        self.amax = amax  # (split mode) [2] floats, [1] = max|this activation| from its producer, or None
        self.planes = None  # (split mode) its fp16 planes written by its producer (PixelCNNpp._planes' tuple)

    @property
    def rows(self):
        return self.n * self.h * self.w

    @property
    def bf(self):
        return self.buf.dtype == torch.bfloat16

    def ptr(self):
        return ctypes.c_void_p(self.buf.data_ptr() + self.buf.element_size() * self.off)


def param_shapes(spec):
    """Ordered {name: shape} of every variable model_spec creates (model.py:35-112 in TF
    construction order; counters nn.py:151-157), plus the highway FC (pixelvae.py:136)."""
    shapes = {}
    cnt = {}

    def nm(kind):
        i = cnt.get(kind, 0)
        cnt[kind] = i + 1
        return "%s_%d" % (kind, i)

    F, R, K, M = spec["F"], spec["R"], spec["K"], spec["M"]
    nlc = (lambda c: 2 * c) if spec["nl"] == "concat_elu" else (lambda c: c)

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
    for stage in range(3):
        for _ in range(R if stage == 0 else R + 1):
            resnet(2, 3, F)
            resnet(2, 2, 2 * F)
        if stage < 2:
            conv(F, F, 2, 3, "deconv2d")
            conv(F, F, 2, 2, "deconv2d")
    dense(F, 10 * M)
    shapes["highway/W"] = (K, 1)
    shapes["highway/b"] = (1,)
    return shapes


def make_spec(H=64, W=64, C=3, K=48, nr_resnet=3, nr_filters=160, nr_mix=10, nonlinearity="relu"):
    """pixelvae.py Args (:54-63): nr_resnet 3, nr_filters 160, nr_logistic_mix 10, 'relu'."""
    if H % 4 or W % 4:
        raise ValueError("H and W must be multiples of 4 (two stride-2 stages)")
    if C != 3:
        raise ValueError("the discretized logistic mixture models RGB (nn.py:57-59)")
    if nonlinearity not in NL_KIND:
        raise ValueError("resnet nonlinearity %r is not supported (model.py:24-31)" % nonlinearity)
    if nr_filters % 4 or nr_mix > 16:
        raise ValueError("nr_filters must be a multiple of 4 and nr_logistic_mix <= 16")
    return dict(H=H, W=W, C=C, K=K, R=nr_resnet, F=nr_filters, M=nr_mix, nl=nonlinearity)


class PixelCNNpp:
    """Conditional PixelCNN++ on libsvae_hip.so.  One instance owns its parameters, gradients,
    Adam moments and Polyak averages (flat fp32 device buffers)."""

    def __init__(self, spec, params=None, seed=0, device="cuda", scratch_elems=1 << 26, planes=1, bf16_grads=False,
                 fuse_absmax=True, im2col=True):
        if not torch.cuda.is_available():
            raise RuntimeError("PixelCNNpp needs a GPU (HIP kernels in libsvae_hip.so); there is no CPU fallback")
        self.s = spec
        self.L = _lib.lib()
        self.dev = torch.device(device)
        shapes = param_shapes(spec)
        self.table = {}
        off = 0
        for k, shp in shapes.items():
            n = int(np.prod(shp))
            self.table[k] = (off, shp, n)
            off += (n + 63) // 64 * 64
        self.n_params = off
        self.P = torch.zeros(off, dtype=torch.float32, device=self.dev)
        self.G = torch.zeros_like(self.P)
        self.m = torch.zeros_like(self.P)
        self.v = torch.zeros_like(self.P)
        self.ema = None
        if params is None:
            params = self.init_values(seed)
        self.set_params(params)
        self.scratch = torch.empty(scratch_elems, dtype=torch.float32, device=self.dev)
        self.iteration = 0
        self._dh = None
        self._tape, self._g, self._keep, self._same, self._cnt = [], {}, [], {}, {}
        self._record = self._init = False
        self._dropout_p, self._masks, self.last_masks = 0.0, None, []
        self.keep_masks = False  # drawn masks: record their tensors in last_masks (else DropMask descriptors)
        # relu / elu backward in the consuming conv's input-gradient epilogue (svae_pcnn_conv_act_bwd):
        # bitwise the same gradients, but 800 -> 765 img/s on c_pixelvae (the one-block-per-CU halo conv
        # exposes the epilogue's extra loads), so off by default
        self.fuse_act_bwd = False
        # the gradients of the resnet convs' outputs, read only as bf16 MFMA operands, stored bf16 (their
        # bias gradients summed in fp32 by the op that writes them)
        # (opt-in: measured slower, 804 vs 882 img/s; bf16 head only)
        self.bf16_grads = bool(bf16_grads)
        self._nl_src, self._bias_of, self._bf16_grad = {}, {}, set()
        self._mask_max = {}
        # operand planes of the conv / nin GEMMs: 1 = bf16 MFMA operands; 3 = the split mode (include/svae_pcnn.h):
        # fp32-grade products, nn.py:189-252 in fp32 -- two scaled fp16 planes per operand (3 fp16-MFMA
        # products) for the layers whose channel counts allow 16-bit storage (h16), else 3 bf16 planes (6)
        # (2 bf16 planes would be neither the bf16 head nor fp32-grade on the layers without fp16 planes)
        if planes not in (1, 3):
            raise ValueError("planes must be 1 (bf16 MFMA operands) or 3 (the fp32-grade split mode)")
        self.planes = planes
        self.h16 = True
        # (split mode) the nonlinearity kernels also leave max|y| of their outputs, which are conv inputs, so
        # the fp16-plane split skips its absmax pass (bitwise; fuse_absmax=False: the separate pass, for A/Bs)
        self.fuse_absmax = bool(fuse_absmax)
        # the split mode's small-channel input convs as 1x1 convs over their im2col (K = kh * kw * cin <= 32)
        self.im2col = bool(im2col)
        if planes > 1:  # every activation and gradient stays fp32 (split into planes at each GEMM)
            self.bf16_grads = False
        self.probe, self.probe_cap = None, 0  # [(flops, event, event)] of timed forward conv launches
        self.conv_flops = 0.0  # running total of forward conv FLOPs (tools/bench_pcnn.py)

    # ---------------- parameters ----------------
    def init_values(self, seed=0):
        """nn.py initialisers: V, hw ~ N(0, 0.05); g = 1; b = 0; highway FC Xavier-uniform."""
        rng = np.random.default_rng(seed)
        out = {}
        for k, (_, shp, _) in self.table.items():
            leaf = k.split("/")[-1]
            if leaf in ("V", "hw"):
                out[k] = rng.normal(0.0, 0.05, size=shp)
            elif leaf == "g":
                out[k] = np.ones(shp)
            elif k == "highway/W":
                lim = math.sqrt(6.0 / (shp[0] + shp[1]))
                out[k] = rng.uniform(-lim, lim, size=shp)
            else:
                out[k] = np.zeros(shp)
        return out

    def set_params(self, params):
        host = np.zeros(self.n_params, np.float32)
        for k, (off, shp, n) in self.table.items():
            host[off:off + n] = np.asarray(params[k], np.float32).reshape(-1)
        self.P.copy_(torch.from_numpy(host))

    def get(self, buf, name):
        off, shp, n = self.table[name]
        return buf[off:off + n].view(*shp)

    def params(self):
        host = self.P.cpu().numpy()
        return {k: host[off:off + n].reshape(shp).copy() for k, (off, shp, n) in self.table.items()}

    def grads(self):
        host = self.G.cpu().numpy()
        return {k: host[off:off + n].reshape(shp).copy() for k, (off, shp, n) in self.table.items()}

    # ---------------- tape primitives ----------------
    def _new(self, rows, c):
        return torch.empty(rows, c, dtype=torch.float32, device=self.dev)

    def _grad(self, a):
        """Gradient buffer of activation ``a`` ([rows][c], zero on first use); a reshaped view
        (``_view``) shares its source's buffer."""
        while id(a) in self._same:
            a = self._same[id(a)]
        g = self._g.get(id(a))
        if g is None:
            g = torch.zeros(a.rows, a.c, dtype=torch.float32, device=self.dev)
            self._g[id(a)] = g
            self._keep.append(a)
        return g

    def _root(self, a):
        while id(a) in self._same:
            a = self._same[id(a)]
        return a

    def _gout(self, a):
        """(gradient buffer of ``a``, accumulate flag) for an op that adds its contribution: the first
        contribution WRITES a fresh buffer (no zero fill, no read-modify-write), later ones accumulate."""
        while id(a) in self._same:
            a = self._same[id(a)]
        g = self._g.get(id(a))
        if g is not None:
            return g, 1
        g = torch.empty(a.rows, a.c, dtype=torch.float32, device=self.dev)
        self._g[id(a)] = g
        self._keep.append(a)
        return g, 0

    def _galias(self, a, g):
        """Make ``g`` (a dead gradient buffer of ``a``'s shape) the gradient of ``a`` if it has none yet;
        returns False if ``a`` already has one (the caller then accumulates into it)."""
        while id(a) in self._same:
            a = self._same[id(a)]
        if id(a) in self._g or tuple(g.shape) != (a.rows, a.c):
            return False
        self._g[id(a)] = g
        self._keep.append(a)
        return True

    def _has_grad(self, a):
        while id(a) in self._same:
            a = self._same[id(a)]
        return id(a) in self._g

    def _view(self, a, n, h, w):
        """``a`` reshaped to another row space (same buffer and gradient)."""
        v = Act(a.buf, a.c, n, h, w, a.off, a.ld, a.amax if n * h * w == a.rows else None)
        if n * h * w == a.rows:
            v.planes = a.planes  # (the same [rows][c] planes)
        self._same[id(v)] = a
        self._keep.append(v)
        return v

    def _st(self):
        return _lib.stream_ptr()

    def _wconv(self, x, name, cout, kh, kw, s, pt, pl, mode=0, ho=None, wo=None, zero_edge=0, out=None,
               init_scale=1.0, amax=False):
        """Weight-normed conv / deconv / dense (nn.py:160-252) as a gather GEMM; returns the output Act
        (or accumulates into ``out``, whose existing values it adds to)."""
        L = self.L
        st = self._st()
        taps, cin = kh * kw, x.c
        off_v, _, _ = self.table[name + "/V"]
        off_g, _, _ = self.table[name + "/g"]
        off_b, _, _ = self.table[name + "/b"]
        kf, kd = _r16(cin), _r16(cout)
        if (self.planes > 1 and self.h16 and self.im2col and cin % 8 and cout % 8 == 0 and s == 1 and mode == 0
                and taps * cin <= 32 and not self._init and id(x) in self._nograd and not x.bf):
            return self._wconv_col(x, name, cout, kh, kw, pt, pl, zero_edge, out)
        h16 = self.planes > 1 and self.h16 and cin % 8 == 0 and cout % 8 == 0  # this layer's plane format
        P = 2 if h16 else self.planes
        norm = torch.empty(cout, dtype=torch.float32, device=self.dev)
        wkf = torch.empty(P * taps * cout * kf, dtype=torch.bfloat16, device=self.dev)
        wkd = torch.empty(P * taps * cin * kd, dtype=torch.bfloat16, device=self.dev)
        wsc = torch.empty(2, dtype=torch.float32, device=self.dev) if h16 else None  # [2^-s, max|W|]
        _ck(L.svae_pcnn_wnorm_planes(_p(self.P, off_v), _p(self.P, off_g), taps, cin, cout, _p(norm), _p(wkf), kf,
                                     ctypes.c_void_p(wkd.data_ptr()), kd, P, _p(wsc), st))
        xs = self._planes(x, h16) if self.planes > 1 else None  # (the split mode's planes of x, kept for the backward)
        if ho is None:
            ho, wo = (x.h - 1) // s + 1, (x.w - 1) // s + 1
        # algorithmic FLOPs of the forward gather GEMM (valid taps only for the stride-2 deconvs)
        self.conv_flops += 2.0 * x.n * ho * wo * cout * cin * taps / (s * s if mode == 1 else 1)
        acc = out is not None
        if out is None:
            out = Act(self._new(x.n * ho * wo, cout), cout, x.n, ho, wo)
        pr = self.probe is not None and len(self.probe) < self.probe_cap
        if pr:  # bench.py's live roofline probe: an event pair around this forward conv launch
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        if amax and xs is not None and wsc is not None and out.off == 0:
            # (the last writer of an activation a split-mode nonlinearity reads: max |out| for its planes' bound)
            out.amax = torch.empty(2, dtype=torch.float32, device=self.dev)
            buf, ld, bf, pst, P_, xsc = xs
            _ck(L.svae_pcnn_conv_planes_amax(ctypes.c_void_p(buf.data_ptr()), x.n, x.h, x.w, x.c, ld, bf, pst,
                                             ctypes.c_void_p(wkf.data_ptr()), kf, P_, _p(xsc), _p(wsc),
                                             _p(self.P, off_b), out.ptr(), ho, wo, cout, out.ld, kh, kw, s, pt, pl, mode,
                                             1 if acc else 0, zero_edge, _p(out.amax), st))
        else:
            self._conv(x, xs, wkf, kf, wsc, _p(self.P, off_b), out.ptr(), ho, wo, cout, out.ld, kh, kw, s, pt, pl, mode,
                       1 if acc else 0, zero_edge)
        if pr:
            e1.record()
            nprod = 1 if xs is None else xs[4] * (xs[4] + 1) // 2  # MFMA launches per algorithmic product
            self.probe.append((2.0 * x.n * ho * wo * cout * cin * taps / (s * s if mode == 1 else 1), e0, e1, nprod))
        if self._init:  # data-dependent init: this layer's g, b from the moments of its own output
            # (before any shift or sum), which is passed on un-normalised (tf.identity of the old x)
            src = out
            if acc or zero_edge:
                src = Act(self._new(x.n * ho * wo, cout), cout, x.n, ho, wo)
                self._conv(x, xs, wkf, kf, wsc, _p(self.P, off_b), src.ptr(), ho, wo, cout, cout, kh, kw, s,
                           pt - (zero_edge == 1), pl - (zero_edge == 2), mode, 0, 0)
            _ck(L.svae_pcnn_wn_init(src.ptr(), src.rows, cout, src.ld, float(init_scale), _p(self.P, off_g),
                                    _p(self.P, off_b), _p(self.scratch), st))
        if self._record:
            geo = (kh, kw, s, pt, pl, mode, zero_edge, kf, kd, off_v, off_g, off_b, (taps, cin))
            self._tape.append(lambda: self._wconv_bwd(x, out, norm, wkd, geo, xs, wsc))
            self._bias_of.setdefault(id(self._root(out)), []).append(off_b)  # (every conv summed into it)
        return out

    def _wconv_col(self, x, name, cout, kh, kw, pt, pl, zero_edge, out):
        """A small-channel stride-1 conv of the split mode (the head's 4-channel input convs, no input gradient) as
        the 1x1 fp16-plane conv of its im2col: K = kh * kw * cin columns in one 32-wide chunk (svae_pcnn_im2col_h16,
        the weights V viewed as [kh * kw * cin][cout]); the weight gradient is the 1x1 one over the same planes."""
        L = self.L
        st = self._st()
        taps, cin = kh * kw, x.c
        K = taps * cin
        off_v, _, _ = self.table[name + "/V"]
        off_g, _, _ = self.table[name + "/g"]
        off_b, _, _ = self.table[name + "/b"]
        ho, wo = x.h, x.w
        rows = x.n * ho * wo
        norm = torch.empty(cout, dtype=torch.float32, device=self.dev)
        wkf = torch.empty(2 * cout * 32, dtype=torch.bfloat16, device=self.dev)
        wsc = torch.empty(2, dtype=torch.float32, device=self.dev)
        _ck(L.svae_pcnn_wnorm_planes(_p(self.P, off_v), _p(self.P, off_g), 1, K, cout, _p(norm), _p(wkf), 32, None, 0, 2,
                                     _p(wsc), st))
        xcol = torch.empty(2 * rows * 32, dtype=torch.bfloat16, device=self.dev)
        xsc = torch.empty(2, dtype=torch.float32, device=self.dev)
        _ck(L.svae_pcnn_im2col_h16(x.ptr(), x.n, x.h, x.w, cin, x.ld, ho, wo, kh, kw, pt, pl,
                                   ctypes.c_void_p(xcol.data_ptr()), 32, _p(xsc), st))
        xc = Act(xcol, 32, x.n, ho, wo)  # (the planes' operand as the 1x1 conv's input: x.c = 32 columns)
        self._nograd.add(id(xc))
        self._keep.append(xc)
        xs = (xcol, 32, 1, rows * 32, 2, xsc)
        self.conv_flops += 2.0 * rows * cout * cin * taps
        acc = out is not None
        if out is None:
            out = Act(self._new(rows, cout), cout, x.n, ho, wo)
        pr = self.probe is not None and len(self.probe) < self.probe_cap
        if pr:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        self._conv(xc, xs, wkf, 32, wsc, _p(self.P, off_b), out.ptr(), ho, wo, cout, out.ld, 1, 1, 1, 0, 0, 0,
                   1 if acc else 0, zero_edge)
        if pr:
            e1.record()
            self.probe.append((2.0 * rows * cout * cin * taps, e0, e1, 3))
        if self._record:
            geo = (1, 1, 1, 0, 0, 0, zero_edge, 32, 0, off_v, off_g, off_b, (1, K))
            self._tape.append(lambda: self._wconv_bwd(xc, out, norm, None, geo, xs, wsc))
            self._bias_of.setdefault(id(self._root(out)), []).append(off_b)
        return out

    def _planes(self, a, h16):
        """The split mode's operand planes of activation (or [rows][c] gradient) ``a``: (buffer, ld, 16-bit flag,
        plane stride, planes, scale) -- the two scaled fp16 planes (h16; scale = [2^-s, max|a|]), else
        ``self.planes`` bf16 planes (16-bit where the bf16-operand kernels take them: c % 8 == 0, else fp32)."""
        if isinstance(a, Act):
            if a.planes is not None:  # written as planes by its producer (svae_pcnn_nonlin_h16)
                if not h16:
                    raise RuntimeError("an fp16-plane activation read by a non-fp16-plane layer")
                return a.planes
            assert not a.bf, "split mode: activations are fp32"
            src, rows, c, ld = a.ptr(), a.rows, a.c, a.ld
            if h16 and a.amax is not None:  # its producer left max|a| (svae_pcnn_nonlin_absmax): no absmax pass
                out = torch.empty(2 * rows * c, dtype=torch.bfloat16, device=self.dev)
                _ck(self.L.svae_pcnn_split_h16_premax(src, rows, c, ld, ctypes.c_void_p(out.data_ptr()), c,
                                                      _p(a.amax), self._st()))
                return out, c, 1, rows * c, 2, a.amax
        else:
            assert a.dtype == torch.float32 and a.is_contiguous()
            src, rows, c, ld = _p(a), a.shape[0], a.shape[1], a.shape[1]
        bf = h16 or c % 8 == 0
        P = 2 if h16 else self.planes
        out = torch.empty(P * rows * c, dtype=torch.bfloat16 if bf else torch.float32, device=self.dev)
        sc = torch.empty(2, dtype=torch.float32, device=self.dev) if h16 else None
        _ck(self.L.svae_pcnn_split_planes(src, rows, c, ld, P, ctypes.c_void_p(out.data_ptr()), c, int(bf), _p(sc),
                                          self._st()))
        return out, c, int(bf), rows * c, P, sc

    def _conv(self, x, xs, wk, kpad, wsc, bias, y, ho, wo, cout, ldy, kh, kw, s, pt, pl, mode, acc, zero_edge):
        """One gather conv of ``x`` (an Act; ``xs`` its split-mode planes, or None) with the weight copy ``wk``
        (``wsc``: its fp16 planes' scale)."""
        if xs is None:
            _ck(self.L.svae_pcnn_conv(x.ptr(), x.n, x.h, x.w, x.c, x.ld, int(x.bf), ctypes.c_void_p(wk.data_ptr()), kpad,
                                      bias, y, ho, wo, cout, ldy, kh, kw, s, pt, pl, mode, acc, zero_edge, self._st()))
            return
        buf, ld, bf, pst, P, xsc = xs
        _ck(self.L.svae_pcnn_conv_planes(ctypes.c_void_p(buf.data_ptr()), x.n, x.h, x.w, x.c, ld, bf, pst,
                                         ctypes.c_void_p(wk.data_ptr()), kpad, P, _p(xsc), _p(wsc), bias, y, ho, wo,
                                         cout, ldy, kh, kw, s, pt, pl, mode, acc, zero_edge, self._st()))

    def _wconv_bwd(self, x, y, norm, wkd, geo, xs=None, wsc=None):
        L = self.L
        st = self._st()
        kh, kw, s, pt, pl, mode, zero_edge, kf, kd, off_v, off_g, off_b, _ = geo
        taps, cin, cout = kh * kw, x.c, y.c
        dy = self._grad(y)
        dyb = dy.dtype == torch.bfloat16  # (its consumer wrote it bf16 and this conv's bias gradient with it)
        if zero_edge:  # the zeroed shifted outputs pass no gradient
            dy = dy.clone()
            _ck(L.svae_pcnn_mask_edge(_p(dy), y.n, y.h, y.w, cout, cout, zero_edge, st))
        dW = torch.empty(taps * cin * cout, dtype=torch.float32, device=self.dev)
        sc = self.scratch
        if xs is not None:
            self._wconv_bwd_split(x, y, dy, norm, wkd, geo, xs, wsc, dW)
            return
        # dW and (fp32 dy) the bias gradient, written into G, from one pass over dy
        _ck(L.svae_pcnn_conv_wgrad(x.ptr(), x.n, x.h, x.w, cin, x.ld, int(x.bf), ctypes.c_void_p(dy.data_ptr()), cout,
                                   int(dyb), y.h, y.w, cout, kh, kw, s, pt, pl, mode, _p(dW),
                                   None if dyb else _p(self.G, off_b), _p(sc), sc.numel(), st))
        _ck(L.svae_pcnn_wnorm_bwd(_p(self.P, off_v), _p(self.P, off_g), _p(norm), _p(dW), taps, cin, cout,
                                  _p(self.G, off_v), _p(self.G, off_g), st))
        if id(x) in self._nograd:
            return
        root = x
        while id(root) in self._same:
            root = self._same[id(root)]
        nl = None if dyb else self._nl_src.get(id(root))
        if nl is not None:  # x = f(src) * mask: the input gradient's epilogue writes d src (no d x, no f' pass)
            src, k, mp, keep, seed = nl
            ds, dacc = self._gout(src)
            _ck(L.svae_pcnn_conv_act_bwd(_p(dy), y.n, y.h, y.w, cout, cout, ctypes.c_void_p(wkd.data_ptr()), kd, _p(ds),
                                         x.h, x.w, cin, cin, kh, kw, s, pt, pl, 1 - mode, dacc, src.ptr(), src.ld, k, mp,
                                         keep, seed, st))
            return
        dx, dacc = self._gout(x)
        # the input gradient: the transposed gather over dy with the [tap][Cin][Cout] copy
        _ck(L.svae_pcnn_conv(ctypes.c_void_p(dy.data_ptr()), y.n, y.h, y.w, cout, cout, int(dyb),
                             ctypes.c_void_p(wkd.data_ptr()), kd, None, _p(dx), x.h, x.w, cin, cin, kh, kw, s, pt, pl,
                             1 - mode, dacc, 0, st))

    def _wconv_bwd_split(self, x, y, dy, norm, wkd, geo, xs, wsc, dW):
        """_wconv_bwd in the split mode: dW and the input gradient as plane-product sums over the planes of x
        and of dy (fp32, split in the layer's plane format; the bias gradient its column sums)."""
        L = self.L
        st = self._st()
        kh, kw, s, pt, pl, mode, zero_edge, kf, kd, off_v, off_g, off_b, (wn_taps, wn_cin) = geo
        taps, cin, cout = kh * kw, x.c, y.c
        xb, xld, xbf, xpst, P, xsc = xs
        sc = self.scratch
        if xsc is not None and self.fuse_absmax and cout % 4 == 0 and dy.dtype == torch.float32:
            # the fp16 planes of dy: the bias gradient's column sums and max|dy| from one pass, then the premax split
            dsc = torch.empty(2, dtype=torch.float32, device=self.dev)
            _ck(L.svae_pcnn_colsum_absmax(_p(dy), y.rows, cout, cout, _p(self.G, off_b), 0, _p(sc), _p(dsc), st))
            ds = torch.empty(2 * y.rows * cout, dtype=torch.bfloat16, device=self.dev)
            _ck(L.svae_pcnn_split_h16_premax(_p(dy), y.rows, cout, cout, ctypes.c_void_p(ds.data_ptr()), cout, _p(dsc),
                                             st))
            dld, dbf, dpst = cout, 1, y.rows * cout
        else:
            ds, dld, dbf, dpst, _, dsc = self._planes(dy, xsc is not None)
            _ck(L.svae_pcnn_colsum(_p(dy), y.rows, cout, cout, 0, 0, 0, _p(self.G, off_b), 0, _p(sc), st))
        _ck(L.svae_pcnn_conv_wgrad_planes(ctypes.c_void_p(xb.data_ptr()), x.n, x.h, x.w, cin, xld, xbf, xpst,
                                          ctypes.c_void_p(ds.data_ptr()), dld, dbf, dpst, P, _p(xsc), _p(dsc), y.h, y.w,
                                          cout, kh, kw, s, pt, pl, mode, _p(dW), _p(sc), sc.numel(), st))
        # (an im2col layer, _wconv_col: dW's first wn_taps * wn_cin rows are the [tap][cin] ones of V)
        _ck(L.svae_pcnn_wnorm_bwd(_p(self.P, off_v), _p(self.P, off_g), _p(norm), _p(dW), wn_taps, wn_cin, cout,
                                  _p(self.G, off_v), _p(self.G, off_g), st))
        if id(x) in self._nograd:
            return
        dx, dacc = self._gout(x)
        _ck(L.svae_pcnn_conv_planes(ctypes.c_void_p(ds.data_ptr()), y.n, y.h, y.w, cout, dld, dbf, dpst,
                                    ctypes.c_void_p(wkd.data_ptr()), kd, P, _p(dsc), _p(wsc), None, _p(dx), x.h, x.w,
                                    cin, cin, kh, kw, s, pt, pl, 1 - mode, dacc, 0, st))

    def _dense(self, x, name, cout, init_scale=1.0):
        """nn.nin / dense over the channel axis (nn.py:255-260): a 1x1 gather GEMM over every pixel."""
        y = self._wconv(self._view(x, x.rows, 1, 1), name, cout, 1, 1, 1, 0, 0, init_scale=init_scale)
        return self._view(y, x.n, x.h, x.w)

    def _nonlin(self, x, kind, mask=None, planes_out=False):
        """y = f(x) (* the dropout keep-mask, fused).  Every nonlinearity output of the network is read
        only by convolutions (bf16 MFMA operands), so y is stored as bf16 when its channels allow it:
        the conv result is bitwise the one from fp32 storage (nn.py:270-274: dropout before the conv)."""
        k = NL_KIND[kind]
        c = 2 * x.c if k == 2 else x.c
        bf = self.planes == 1 and c % 8 == 0 and x.c % 4 == 0 and x.ld % 4 == 0
        if isinstance(mask, DropMask):  # drawn in the kernel from (seed, keep)
            mp, keep, seed = None, mask.keep, mask.seed
        else:
            mp, keep, seed = _p(mask), 1.0, 0
        # planes_out: the caller's consumer is an fp16-plane conv (channels % 8 == 0 both ways), so y may exist as
        # its planes only
        if (planes_out and self.planes > 1 and self.h16 and self.fuse_absmax and x.amax is not None and c % 8 == 0
                and x.c % 4 == 0
                and x.ld % 4 == 0 and x.buf.dtype == torch.float32 and not self._init
                and x.buf.data_ptr() % 16 == 0 and x.off % 4 == 0):
            # the split mode's conv input straight as its fp16 planes: the exponent from x's producer's max |x|
            # (no fp32 y, no absmax, no split pass; y is read only by the consuming conv)
            pl = torch.empty(2 * x.rows * c, dtype=torch.bfloat16, device=self.dev)
            psc = torch.empty(2, dtype=torch.float32, device=self.dev)
            mmax = self._mask_max.get(id(mask), 0.0) if mp is not None else 0.0
            _ck(self.L.svae_pcnn_nonlin_h16(x.ptr(), x.rows, x.c, x.ld, k, mp, float(mmax), keep, seed, _p(x.amax),
                                            ctypes.c_void_p(pl.data_ptr()), c, _p(psc), self._st()))
            y = Act(pl, c, x.n, x.h, x.w)
            y.planes = (pl, c, 1, x.rows * c, 2, psc)
            self._keep.append(y)
            buf = None
        else:
            buf = torch.empty(x.rows, c, dtype=torch.bfloat16 if bf else torch.float32, device=self.dev)
            y = Act(buf, c, x.n, x.h, x.w)
        if buf is None:
            pass
        elif (self.planes > 1 and self.h16 and self.fuse_absmax and c % 8 == 0 and x.c % 4 == 0 and x.ld % 4 == 0
                and x.buf.dtype == torch.float32):
            # the split mode's conv input: the kernel also leaves max|y| for its fp16 planes (bitwise the pass)
            y.amax = torch.empty(2, dtype=torch.float32, device=self.dev)
            _ck(self.L.svae_pcnn_nonlin_absmax(x.ptr(), x.rows, x.c, x.ld, k, mp, keep, seed, y.ptr(), y.ld,
                                               _p(y.amax), self._st()))
        else:
            _ck(self.L.svae_pcnn_nonlin(x.ptr(), x.rows, x.c, x.ld, k, mp, keep, seed, y.ptr(), y.ld, int(bf),
                                        self._st()))
        if self._record and k != 2 and self.fuse_act_bwd and self.planes == 1:  # its consuming conv applies f' (svae_pcnn_conv_act_bwd)
            self._nl_src[id(y)] = (x, k, mp, keep, seed)
            self._keep.append(x)
        if self._record:
            def bwd():
                if not self._has_grad(y):
                    return
                rx = self._root(x)
                if (id(rx) in self._bf16_grad and not self._has_grad(x) and k != 2 and x.c % 8 == 0
                        and x.ld % 4 == 0):
                    # x's only consumer: its gradient is written here whole, as bf16 (the producing convs read
                    # it only as an MFMA operand), with the fp32 column sums = their bias gradients
                    dx = torch.empty(x.rows, x.c, dtype=torch.bfloat16, device=self.dev)
                    self._g[id(rx)] = dx
                    self._keep.append(rx)
                    offs = self._bias_of[id(rx)]
                    _ck(self.L.svae_pcnn_nonlin_bwd(x.ptr(), x.rows, x.c, x.ld, k, mp, keep, seed, _p(self._grad(y)),
                                                    c, ctypes.c_void_p(dx.data_ptr()), x.c, 1, 0,
                                                    _p(self.G, offs[0]), _p(self.scratch), self._st()))
                    for o in offs[1:]:
                        self.G[o:o + x.c].copy_(self.G[offs[0]:offs[0] + x.c])
                    return
                dx, dacc = self._gout(x)
                _ck(self.L.svae_pcnn_nonlin_bwd(x.ptr(), x.rows, x.c, x.ld, k, mp, keep, seed, _p(self._grad(y)), c,
                                                _p(dx), x.c, 0, dacc, None, None, self._st()))
            self._tape.append(bwd)
        return y

    def _cat(self, a, b):
        c = a.c + b.c
        y = Act(self._new(a.rows, c), c, a.n, a.h, a.w)
        st = self._st()
        _ck(self.L.svae_pcnn_copy(a.ptr(), a.ld, a.rows, a.c, y.ptr(), c, 0, st))
        _ck(self.L.svae_pcnn_copy(b.ptr(), b.ld, b.rows, b.c, _p(y.buf, a.c), c, 0, st))
        if self._record:
            def bwd():
                if not self._has_grad(y):
                    return
                dy = self._grad(y)
                da, aacc = self._gout(a)
                _ck(self.L.svae_pcnn_copy(_p(dy), c, a.rows, a.c, _p(da), a.c, aacc, self._st()))
                db, bacc = self._gout(b)
                _ck(self.L.svae_pcnn_copy(_p(dy, a.c), c, b.rows, b.c, _p(db), b.c, bacc, self._st()))
            self._tape.append(bwd)
        return y

    def _gate(self, x, c2, h, hw_name):
        """out = x + a * sigmoid(b), [a | b] = c2 + h . hw (nn.py:277-288)."""
        F = x.c
        st = self._st()
        off_hw, _, _ = self.table[hw_name]
        K = self.s["K"]
        hp = torch.empty(x.n, 2 * F, dtype=torch.float32, device=self.dev)
        _ck(self.L.svae_pcnn_gemm_small(_p(h), K, 0, _p(self.P, off_hw), 2 * F, 0, _p(hp), 2 * F, x.n, 2 * F, K, 0.0,
                                        st))
        y = Act(self._new(x.rows, F), F, x.n, x.h, x.w)
        if self.planes > 1 and self.h16 and self.fuse_absmax:  # max |y|: the next nonlinearity writes fp16 planes
            y.amax = torch.empty(2, dtype=torch.float32, device=self.dev)
            _ck(self.L.svae_pcnn_gate_amax(x.ptr(), x.ld, c2.ptr(), _p(hp), x.rows, x.h * x.w, F, y.ptr(), F,
                                           _p(y.amax), st))
        else:
            _ck(self.L.svae_pcnn_gate(x.ptr(), x.ld, c2.ptr(), _p(hp), x.rows, x.h * x.w, F, y.ptr(), F, st))
        if self._record:
            def bwd():
                if not self._has_grad(y):
                    return
                st2 = self._st()
                dy = self._grad(y)
                dhp = torch.empty(x.n, 2 * F, dtype=torch.float32, device=self.dev)  # per-image sums of dc2
                rc = self._root(c2)
                offs = self._bias_of.get(id(rc), [])
                if id(rc) in self._bf16_grad and len(offs) == 1 and (x.h * x.w) % 64 == 0 and F % 4 == 0:
                    # c2's only consumer: dc2 written bf16 (its conv reads it only as an MFMA operand) with
                    # the fp32 sums over all rows, the conv's bias gradient
                    dc2 = torch.empty(c2.rows, c2.c, dtype=torch.bfloat16, device=self.dev)
                    self._g[id(rc)] = dc2
                    self._keep.append(rc)
                    _ck(self.L.svae_pcnn_gate_bwd(c2.ptr(), _p(hp), _p(dy), F, x.rows, x.h * x.w, F,
                                                  ctypes.c_void_p(dc2.data_ptr()), 1, _p(dhp), _p(self.G, offs[0]),
                                                  _p(self.scratch), st2))
                else:
                    dc2, _ = self._gout(c2)  # (c2's only consumer: written)
                    _ck(self.L.svae_pcnn_gate_bwd(c2.ptr(), _p(hp), _p(dy), F, x.rows, x.h * x.w, F, _p(dc2), 0,
                                                  _p(dhp), None, _p(self.scratch), st2))
                # the residual's gradient is dy itself: y's gradient is complete and dead after this
                # op, so x takes the buffer over when it has no gradient yet (else one accumulating copy)
                if not self._galias(x, dy):
                    _ck(self.L.svae_pcnn_copy(_p(dy), F, x.rows, F, _p(self._grad(x)), F, 1, st2))
                # d hw [K][2F] = h^T . dhp
                _ck(self.L.svae_pcnn_gemm_small(_p(h), K, 1, _p(dhp), 2 * F, 0, _p(self.G, off_hw), 2 * F, K, 2 * F,
                                                x.n, 0.0, st2))
                if self._dh is not None:  # d h += dhp . hw^T
                    _ck(self.L.svae_pcnn_gemm_small(_p(dhp), 2 * F, 0, _p(self.P, off_hw), 2 * F, 1, _p(self._dh), K,
                                                    x.n, K, 2 * F, 1.0, st2))
            self._tape.append(bwd)
        return y

    # ---------------- the network ----------------
    def _gated_resnet(self, x, h, kh, kw, a=None):
        nl = self.s["nl"]
        pt, pl = kh - 1, (kw - 1) // 2 if kw == 3 else kw - 1
        # (the split mode: c1's last writer leaves max |c1|, so the dropout nonlinearity below writes its fp16
        #  planes directly, svae_pcnn_nonlin_h16)
        hp = x.c % 8 == 0  # (every conv of the resnet on fp16 planes: F and 2F channels)
        c1 = self._wconv(self._nonlin(x, nl, planes_out=hp), self._nm("conv2d"), x.c, kh, kw, 1, pt, pl,
                         amax=a is None)
        if a is not None:
            v = self._dense_into(self._nonlin(a, nl, planes_out=hp), self._nm("dense"), c1, amax=True)
            c1.amax = v.amax
        # training-pass dropout (nn.py:273-274) fused into the nonlinearity
        mask = self._next_mask(c1.rows, 2 * c1.c if nl == "concat_elu" else c1.c)
        t2 = self._nonlin(c1, nl, mask, planes_out=hp)
        c2 = self._wconv(t2, self._nm("conv2d"), 2 * x.c, kh, kw, 1, pt, pl, init_scale=0.1)
        if self.bf16_grads:  # c1 / c2 feed one op each: their gradients may be written bf16 by it
            self._bf16_grad.update((id(self._root(c1)), id(self._root(c2))))
        return self._gate(x, c2, h, self._nm("conditional_weights") + "/hw")

    def _next_mask(self, rows, c):
        """The next gated resnet's dropout mask (1 / keep_prob where kept, else 0; tf.nn.dropout,
        nn.py:273-274): from the injected list (parity), else, when dropout_p > 0, a DropMask the
        nonlinearity kernels draw from a seed (the seeds come from torch's CPU generator, so
        torch.manual_seed fixes them).  Every mask used is appended to ``self.last_masks`` (a
        DropMask, or its tensor when ``keep_masks`` is set)."""
        if self._masks is not None:
            m = next(self._masks)
            if not isinstance(m, DropMask):
                mx = float(np.max(m)) if isinstance(m, np.ndarray) else float(torch.as_tensor(m).max())
                m = torch.as_tensor(m, dtype=torch.float32, device=self.dev).reshape(rows, c).contiguous()
                self._mask_max[id(m)] = mx  # (its largest factor: the planes' bound of svae_pcnn_nonlin_h16)
        elif self._dropout_p > 0.0:
            m = DropMask(rows, c, 1.0 - self._dropout_p, int(torch.randint(0, 2 ** 62, (1,)).item()))
            if self.keep_masks:
                m = m.tensor(self)
        else:
            return None
        self.last_masks.append(m)
        return m

    def _dense_into(self, x, name, out, amax=False):
        v = self._view(out, out.rows, 1, 1)
        self._wconv(self._view(x, x.rows, 1, 1), name, out.c, 1, 1, 1, 0, 0, out=v, amax=amax)
        return v

    def _nm(self, kind):
        i = self._cnt.get(kind, 0)
        self._cnt[kind] = i + 1
        return "%s_%d" % (kind, i)

    def _run(self, x, h, record, init=False, dropout_p=0.0, masks=None):
        """model_spec(x, h) (model.py:11-117) -> l Act [rows][10 M].  dropout_p > 0: the training
        pass's dropout in every gated resnet, masks injected (``masks``, in gated-resnet order) or
        drawn on the device."""
        s = self.s
        self._record, self._init = record, init
        self._dropout_p = float(dropout_p)
        self._masks = iter(masks) if masks is not None else None
        self.last_masks = []
        self._tape, self._g, self._keep, self._same, self._cnt = [], {}, [], {}, {}
        self._nograd = set()
        self._nl_src, self._bias_of, self._bf16_grad = {}, {}, set()
        self._mask_max = {}
        B, H, W = x.shape[0], s["H"], s["W"]
        F, R = s["F"], s["R"]
        rows = B * H * W
        xp = Act(self._new(rows, 4), 4, B, H, W)
        _ck(self.L.svae_pcnn_pad_ones(_p(x), rows, 3, xp.ptr(), 4, self._st()))
        self._nograd.add(id(xp))
        self._keep.append(xp)
        # u: down_shift(down_shifted_conv2d(x_pad, [2, 3])): pt + 1 and the first row zeroed
        u = [self._wconv(xp, self._nm("conv2d"), F, 2, 3, 1, 2, 1, zero_edge=1)]
        # ul: down_shift(ds_conv [1, 3]) + right_shift(drs_conv [2, 1])
        ul0 = self._wconv(xp, self._nm("conv2d"), F, 1, 3, 1, 1, 1, zero_edge=1)
        self._wconv(xp, self._nm("conv2d"), F, 2, 1, 1, 1, 1, zero_edge=2, out=ul0)
        ul = [ul0]
        for stage in range(3):
            for _ in range(R):
                u.append(self._gated_resnet(u[-1], h, 2, 3))
                ul.append(self._gated_resnet(ul[-1], h, 2, 2, a=u[-1]))
            if stage < 2:
                u.append(self._wconv(u[-1], self._nm("conv2d"), F, 2, 3, 2, 1, 1))
                ul.append(self._wconv(ul[-1], self._nm("conv2d"), F, 2, 2, 2, 1, 1))
        uu, uul = u.pop(), ul.pop()
        for stage in range(3):
            for _ in range(R if stage == 0 else R + 1):
                uu = self._gated_resnet(uu, h, 2, 3, a=u.pop())
                uul = self._gated_resnet(uul, h, 2, 2, a=self._cat(uu, ul.pop()))
            if stage < 2:  # down_shifted_deconv2d / down_right_shifted_deconv2d (stride 2, VALID, cropped)
                uu = self._wconv(uu, self._nm("deconv2d"), F, 2, 3, 2, 0, 1, mode=1, ho=2 * uu.h, wo=2 * uu.w)
                uul = self._wconv(uul, self._nm("deconv2d"), F, 2, 2, 2, 0, 0, mode=1, ho=2 * uul.h, wo=2 * uul.w)
        assert not u and not ul
        e = self._nonlin(uul, "elu")
        return self._dense(e, self._nm("dense"), 10 * s["M"])

    def _inputs(self, x, h):
        s = self.s
        x = torch.as_tensor(x, dtype=torch.float32, device=self.dev).contiguous()
        h = torch.as_tensor(h, dtype=torch.float32, device=self.dev).contiguous()
        if tuple(x.shape[1:]) != (s["H"], s["W"], 3) or h.shape != (x.shape[0], s["K"]):
            raise ValueError("x must be [B, %d, %d, 3] and h [B, %d]" % (s["H"], s["W"], s["K"]))
        return x, h

    def model(self, x, h):
        """l = model_spec(x, h): [B, H, W, 10 M] (no tape)."""
        x, h = self._inputs(x, h)
        l = self._run(x, h, record=False)
        self._drop()
        return l.buf.view(x.shape[0], self.s["H"], self.s["W"], 10 * self.s["M"])

    def _drop(self):
        self._tape, self._g, self._keep, self._same, self._nl_src = [], {}, [], {}, {}
        self._bias_of, self._bf16_grad = {}, set()

    def loss(self, x, h, backward=True, grad_h=False, coef=1.0):
        """NLL = discretized_mix_logistic_loss(x, model(x, h)) summed (nn.py:84-85).  With
        ``backward``, d(coef * NLL)/d every parameter lands in ``self.G`` (written) and, with
        ``grad_h``, d/dh is returned too."""
        x, h = self._inputs(x, h)
        st = self._st()
        l = self._run(x, h, record=backward)
        pix = l.rows
        logp = torch.empty(pix, dtype=torch.float32, device=self.dev)
        dl = self._gout(l)[0] if backward else None  # (written whole by the mixture kernel)
        _ck(self.L.svae_pcnn_mixlogistic(_p(x), l.ptr(), pix, self.s["M"], _p(logp), _p(dl), float(coef), st))
        tot = torch.empty(1, dtype=torch.float64, device=self.dev)
        _ck(self.L.svae_pcnn_sum(_p(logp), pix, None, ctypes.c_void_p(tot.data_ptr()), st))
        dh = None
        if backward:
            self.G.zero_()
            self._dh = torch.zeros(x.shape[0], self.s["K"], dtype=torch.float32, device=self.dev) if grad_h else None
            for fn in reversed(self._tape):
                fn()
            dh = self._dh
            self._dh = None
        self._drop()
        nll = -float(tot.item())
        return (nll, dh) if grad_h else nll

    def forward_train(self, x, h, dropout_p=0.0, masks=None):
        """l = model_spec(x, h) of the training pass (dropout in the gated resnets), with the tape
        kept for backward_from.  Returns l [B, H, W, 10 M] (the tape's own buffer)."""
        x, h = self._inputs(x, h)
        self._fw_in = (x, h)
        l = self._run(x, h, record=True, dropout_p=dropout_p, masks=masks)
        self._fw_l = l
        return l.buf.view(x.shape[0], self.s["H"], self.s["W"], 10 * self.s["M"])

    def backward_from(self, dl, grad_h=True):
        """Backward of the last forward_train from dl = d loss / d l ([rows][10 M] device tensor): every
        parameter's gradient is WRITTEN into ``self.G`` (zeroed first); returns d loss / d h [B, K]."""
        x, _ = self._fw_in
        self.G.zero_()
        self._gout(self._fw_l)[0].copy_(dl.reshape(self._fw_l.rows, self._fw_l.c))
        self._dh = torch.zeros(x.shape[0], self.s["K"], dtype=torch.float32, device=self.dev) if grad_h else None
        for fn in reversed(self._tape):
            fn()
        dh, self._dh = self._dh, None
        self._drop()
        self._fw_in = self._fw_l = None
        return dh

    def data_init(self, x, h, dropout_p=0.0, masks=None):
        """The data-dependent init pass (pixelvae.py:103-105): every weight-normed layer's g, b from
        its own output moments, in construction order (nn.py:176-180, :206-210)."""
        x, h = self._inputs(x, h)
        self._run(x, h, record=False, init=True, dropout_p=dropout_p, masks=masks)
        self._init = False
        self._drop()

    def adam(self, lr, step=None, clip=float("inf")):
        """One Adam update of every parameter from ``self.G`` (TF AdamOptimizer, the optimiser
        sequential_vae.py:1246-1276 applies to every trainable variable)."""
        self.iteration = self.iteration + 1 if step is None else step
        _ck(self.L.svae_pcnn_adam(_p(self.P), _p(self.G), _p(self.m), _p(self.v), self.n_params, float(lr),
                                  int(self.iteration), float(clip), self._st()))

    def ema_update(self, decay=0.9995):
        """Polyak averages (pixelvae.py:113-114, ExponentialMovingAverage(polyak_decay))."""
        if self.ema is None:
            self.ema = self.P.clone()
            return
        _ck(self.L.svae_pcnn_ema(_p(self.ema), _p(self.P), self.n_params, float(decay), self._st()))

    def train_step(self, x, h, lr=1e-3, clip=float("inf")):
        nll = self.loss(x, h, backward=True)
        self.adam(lr, clip=clip)
        return nll

    def sample(self, h, u_mix=None, u_log=None, seed=0, use_ema=False):
        """sample_from_model (pixelvae.py:170-194): x = 0, then for every position in raster order
        one network evaluation and one draw from the mixture at that position
        (sample_from_discretized_mix_logistic, nn.py:89-109).  u_mix [B,H,W,M] / u_log [B,H,W,3]
        may be injected (parity); otherwise drawn on the device per position."""
        s = self.s
        h = torch.as_tensor(h, dtype=torch.float32, device=self.dev).contiguous()
        B, H, W, M = h.shape[0], s["H"], s["W"], s["M"]
        gen = torch.Generator(device=self.dev)
        gen.manual_seed(seed)
        if u_mix is None:
            u_mix = torch.rand(B, H, W, M, device=self.dev, generator=gen) * (1 - 2e-5) + 1e-5
        if u_log is None:
            u_log = torch.rand(B, H, W, 3, device=self.dev, generator=gen) * (1 - 2e-5) + 1e-5
        u_mix = torch.as_tensor(u_mix, dtype=torch.float32, device=self.dev).contiguous()
        u_log = torch.as_tensor(u_log, dtype=torch.float32, device=self.dev).contiguous()
        saved = None
        if use_ema and self.ema is not None:
            saved = self.P.clone()
            self.P.copy_(self.ema)
        x = torch.zeros(B, H, W, 3, dtype=torch.float32, device=self.dev)
        try:
            for q in range(H * W):
                l = self._run(x, h, record=False)
                _ck(self.L.svae_pcnn_sample(l.ptr(), _p(u_mix), _p(u_log), B, H * W, M, _p(x), q, q + 1, 3,
                                            self._st()))
                self._drop()
        finally:
            if saved is not None:
                self.P.copy_(saved)
        return x

    def highway(self, sample, prev, latents, lo, hi):
        """pixelvae.py:135-137: per-image ratio r = lo + (hi - lo) sigmoid(latents . W + b),
        out = r sample + (1 - r) prev."""
        latents = torch.as_tensor(latents, dtype=torch.float32, device=self.dev).contiguous()
        B = latents.shape[0]
        z = torch.empty(B, dtype=torch.float32, device=self.dev)
        ow, _, _ = self.table["highway/W"]
        ob, _, _ = self.table["highway/b"]
        st = self._st()
        _ck(self.L.svae_pcnn_gemm_small(_p(latents), self.s["K"], 0, _p(self.P, ow), 1, 0, _p(z), 1, B, 1,
                                        self.s["K"], 0.0, st))
        sample = sample.contiguous()
        prev = prev.contiguous()
        out = torch.empty_like(sample)
        ratio = torch.empty(B, dtype=torch.float32, device=self.dev)
        _ck(self.L.svae_pcnn_highway(_p(sample), _p(prev), _p(z), _p(self.P, ob), B, sample[0].numel(), float(lo),
                                     float(hi), _p(out), _p(ratio), st))
        return out, ratio


def make_pixel_cnn(ground_images, prev_samples, latents, min_highway_connection, max_highway_connection,
                   net=None, u_mix=None, u_log=None):
    """pixelvae.make_pixel_cnn (pixelvae.py:68-158), repaired: the head conditioned on the latents,
    its training output the mixture sample of model(ground_images, latents) (:123-125) mixed per
    image with the previous chain sample (:135-137).  Returns (highway_train_out, 0, cache) like
    the reference; cache['net'] is the PixelCNNpp (its NLL via net.loss)."""
    B, H, W, C = ground_images.shape
    if net is None:
        net = PixelCNNpp(make_spec(H=H, W=W, K=latents.shape[1]))
    l = net.model(ground_images, latents)
    M = net.s["M"]
    dev = net.dev
    gen = torch.Generator(device=dev)
    gen.manual_seed(0)
    if u_mix is None:
        u_mix = torch.rand(B, H, W, M, device=dev, generator=gen) * (1 - 2e-5) + 1e-5
    if u_log is None:
        u_log = torch.rand(B, H, W, 3, device=dev, generator=gen) * (1 - 2e-5) + 1e-5
    x = torch.empty(B, H, W, 3, dtype=torch.float32, device=dev)
    # (device copies held in locals: a temporary's memory could be reused before the kernel runs)
    um = torch.as_tensor(u_mix, dtype=torch.float32, device=dev).contiguous()
    ul = torch.as_tensor(u_log, dtype=torch.float32, device=dev).contiguous()
    _ck(net.L.svae_pcnn_sample(_p(l), _p(um), _p(ul), B, H * W, M, _p(x), 0, H * W, 3, _lib.stream_ptr()))
    prev = torch.as_tensor(prev_samples, dtype=torch.float32, device=dev)
    out, ratio = net.highway(x, prev, latents, min_highway_connection, max_highway_connection)
    cache = {"net": net, "sample_op": x, "highway_test_ratio": ratio, "prev_samples": prev}
    return out, 0, cache
