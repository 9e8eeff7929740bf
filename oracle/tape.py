"""numpy float64 reverse-mode tape with TensorFlow-1.x op semantics — TEST INFRASTRUCTURE.

Each op stores its forward value and a hand-written backward closure.  The op
semantics restated here:

* conv2d, padding SAME: ``out = ceil(in/s)``, ``pad_total = max((out-1)*s + k - in, 0)``,
  ``pad_before = pad_total // 2`` (k=4: stride 2 -> 1/1, stride 1 -> 1/2);
  weights ``[kh, kw, Cin, Cout]``, cross-correlation (abstract_network.py:18).
* conv2d_transpose, padding SAME: the adjoint (input-gradient) of the SAME conv
  from an ``in*s`` image; weights ``[kh, kw, Cout, Cin]`` (abstract_network.py:37,56).
* batch_norm(training): ``center=True, scale=False, epsilon=1e-3``; batch mean
  and *biased* batch variance over every axis but the last (abstract_network.py:22).
* lrelu(x) = max(min(0.1x, 0), x) with TF's Maximum/Minimum gradient routing
  (ties go to the first operand) -> d/dx = 0.1 for x <= 0 (abstract_network.py:8-10).
* relu' (0) = 0, sigmoid' = y(1-y).
"""
import numpy as np


class Node:
    __slots__ = ("v", "g", "parents", "bw", "idx")

    def __init__(self, v, parents=(), bw=None):
        self.v, self.parents, self.bw, self.g = v, tuple(parents), bw, None


class Tape:
    def __init__(self):
        self.nodes = []

    def leaf(self, v):
        n = Node(np.asarray(v, dtype=np.float64))
        self.nodes.append(n)
        return n

    def op(self, v, parents, bw):
        n = Node(v, parents, bw)
        self.nodes.append(n)
        return n

    def backward(self, root, seed=1.0):
        root.g = np.asarray(seed, dtype=np.float64) * np.ones_like(root.v)
        for n in reversed(self.nodes):
            if n.g is None or n.bw is None:
                continue
            grads = n.bw(n.g)
            for p, g in zip(n.parents, grads):
                if g is None:
                    continue
                p.g = g if p.g is None else p.g + g


# ----------------------------------------------------------------- helpers
def same_pads(n_in, k, s):
    n_out = -(-n_in // s)
    total = max((n_out - 1) * s + k - n_in, 0)
    return n_out, total // 2, total - total // 2


def im2col(x, k, s, n_out, pb, pa):
    N, H, W, C = x.shape
    xp = np.pad(x, ((0, 0), (pb, pa), (pb, pa), (0, 0)))
    cols = np.empty((N, n_out, n_out, k, k, C), dtype=x.dtype)
    span = s * (n_out - 1) + 1
    for ky in range(k):
        for kx in range(k):
            cols[:, :, :, ky, kx, :] = xp[:, ky:ky + span:s, kx:kx + span:s, :]
    return cols


def col2im(cols, H, k, s, pb, pa):
    N, n_out, _, _, _, C = cols.shape
    xp = np.zeros((N, H + pb + pa, H + pb + pa, C), dtype=cols.dtype)
    span = s * (n_out - 1) + 1
    for ky in range(k):
        for kx in range(k):
            xp[:, ky:ky + span:s, kx:kx + span:s, :] += cols[:, :, :, ky, kx, :]
    return xp[:, pb:pb + H, pb:pb + H, :]


def conv2d_fwd(x, w, s):
    k = w.shape[0]
    n_out, pb, pa = same_pads(x.shape[1], k, s)
    cols = im2col(x, k, s, n_out, pb, pa)
    return cols.reshape(-1, k * k * w.shape[2]) @ w.reshape(-1, w.shape[3]), cols


def conv2d(tp, x, w, s):
    """tf.contrib.layers.convolution2d(..., padding='SAME', activation identity) minus bias."""
    k, cin, cout = w.v.shape[0], w.v.shape[2], w.v.shape[3]
    N, H = x.v.shape[0], x.v.shape[1]
    n_out, pb, pa = same_pads(H, k, s)
    y2, cols = conv2d_fwd(x.v, w.v, s)
    y = y2.reshape(N, n_out, n_out, cout)

    def bw(g):
        g2 = g.reshape(-1, cout)
        dw = cols.reshape(-1, k * k * cin).T @ g2
        dcols = (g2 @ w.v.reshape(-1, cout).T).reshape(cols.shape)
        return col2im(dcols, H, k, s, pb, pa), dw.reshape(w.v.shape)

    return tp.op(y, (x, w), bw)


def conv2d_transpose(tp, x, w, s):
    """tf.contrib.layers.convolution2d_transpose(padding='SAME'): out = in*s."""
    k, cout, cin = w.v.shape[0], w.v.shape[2], w.v.shape[3]
    N, H = x.v.shape[0], x.v.shape[1]
    Ho = H * s
    n_in_chk, pb, pa = same_pads(Ho, k, s)
    assert n_in_chk == H
    wm = w.v.reshape(k * k * cout, cin)
    dcols = (x.v.reshape(-1, cin) @ wm.T).reshape(N, H, H, k, k, cout)
    y = col2im(dcols, Ho, k, s, pb, pa)

    def bw(g):
        cols = im2col(g, k, s, H, pb, pa)  # [N,H,H,k,k,cout]
        c2 = cols.reshape(-1, k * k * cout)
        dx = (c2 @ wm).reshape(x.v.shape)
        dw = (c2.T @ x.v.reshape(-1, cin)).reshape(w.v.shape)
        return dx, dw

    return tp.op(y, (x, w), bw)


def matmul(tp, x, w):
    y = x.v @ w.v
    return tp.op(y, (x, w), lambda g: (g @ w.v.T, x.v.T @ g))


def bias_add(tp, x, b):
    axes = tuple(range(x.v.ndim - 1))
    return tp.op(x.v + b.v, (x, b), lambda g: (g, g.sum(axis=axes)))


def batch_norm(tp, x, beta, eps=1e-3):
    """tf.contrib.layers.batch_norm(is_training=True, center=True, scale=False)."""
    axes = tuple(range(x.v.ndim - 1))
    n = int(np.prod([x.v.shape[a] for a in axes]))
    mean = x.v.mean(axis=axes)
    var = ((x.v - mean) ** 2).mean(axis=axes)
    inv = 1.0 / np.sqrt(var + eps)
    xh = (x.v - mean) * inv
    y = xh + beta.v

    def bw(g):
        gs = g.sum(axis=axes)
        gx = (g * xh).sum(axis=axes)
        dx = inv * (g - gs / n - xh * gx / n)
        return dx, gs

    return tp.op(y, (x, beta), bw)


def lrelu(tp, x, rate=0.1):
    y = np.maximum(np.minimum(x.v * rate, 0.0), x.v)
    d = np.where(x.v > 0, 1.0, rate)
    return tp.op(y, (x,), lambda g: (g * d,))


def relu(tp, x):
    return tp.op(np.maximum(x.v, 0.0), (x,), lambda g: (g * (x.v > 0),))


def sigmoid(tp, x):
    y = 1.0 / (1.0 + np.exp(-x.v))
    return tp.op(y, (x,), lambda g: (g * y * (1.0 - y),))


def clip(tp, x, lo, hi):
    y = np.clip(x.v, lo, hi)
    m = (x.v >= lo) & (x.v <= hi)
    return tp.op(y, (x,), lambda g: (g * m,))


def reshape(tp, x, shape):
    return tp.op(x.v.reshape(shape), (x,), lambda g: (g.reshape(x.v.shape),))


def concat_last(tp, xs):
    sizes = [a.v.shape[-1] for a in xs]
    y = np.concatenate([a.v for a in xs], axis=-1)

    def bw(g):
        out, o = [], 0
        for s in sizes:
            out.append(g[..., o:o + s])
            o += s
        return tuple(out)

    return tp.op(y, tuple(xs), bw)


def split_last(tp, x, sizes):
    outs, o = [], 0
    for s in sizes:
        sl = slice(o, o + s)

        def bw(g, sl=sl):
            z = np.zeros_like(x.v)
            z[..., sl] = g
            return (z,)

        outs.append(tp.op(x.v[..., sl], (x,), bw))
        o += s
    return outs


def add(tp, a, b):
    return tp.op(a.v + b.v, (a, b), lambda g: (g, g))


def mul(tp, a, b):
    return tp.op(a.v * b.v, (a, b), lambda g: (g * b.v, g * a.v))


def affine(tp, x, scale, shift):
    return tp.op(scale * x.v + shift, (x,), lambda g: (scale * g,))


def tile_last(tp, x, reps):
    return tp.op(np.tile(x.v, (1,) * (x.v.ndim - 1) + (reps,)), (x,),
                 lambda g: (g.reshape(g.shape[:-1] + (reps, x.v.shape[-1])).sum(axis=-2),))


def scalar_sum(tp, xs, coeffs):
    v = sum(c * a.v for a, c in zip(xs, coeffs))
    return tp.op(np.asarray(v, dtype=np.float64), tuple(xs), lambda g: tuple(c * g for c in coeffs))


def mean_sq_err_per_row(tp, a, target):
    """reduce_mean(square(a - target), [1,2,3]) (sequential_vae.py:1146)."""
    d = a.v - target
    m = d[0].size
    y = (d ** 2).reshape(d.shape[0], -1).mean(axis=1)
    return tp.op(y, (a,), lambda g: (2.0 * d * g.reshape((-1,) + (1,) * (d.ndim - 1)) / m,))


def kl_per_row(tp, mu, sig, prior=1.0):
    """reduce_mean(-0.5 - log s + 0.5 s^2/p^2 + 0.5 mu^2/p^2, 1) (sequential_vae.py:1156-1158)."""
    D = mu.v.shape[1]
    p2 = prior ** 2
    y = (-0.5 - np.log(sig.v) + 0.5 * sig.v ** 2 / p2 + 0.5 * mu.v ** 2 / p2).mean(axis=1)

    def bw(g):
        g = g[:, None]
        return g * mu.v / p2 / D, g * (-1.0 / sig.v + sig.v / p2) / D

    return tp.op(y, (mu, sig), bw)


def mean_all(tp, x):
    n = x.v.size
    return tp.op(np.asarray(x.v.mean()), (x,), lambda g: (np.full(x.v.shape, g / n),))


# ---- chain-noise / predicted-noise / uniform-prior / improvement-maximisation variants ----
def zero_grads(tp):
    """Reset every node's gradient (a second backward on the same tape: the improvement-
    maximisation loss has its own compute_gradients, sequential_vae.py:1302-1303)."""
    for n in tp.nodes:
        n.g = None


def add_scaled_noise(tp, mle, sd, noise, scale):
    """training_sample = mle + reg * stddevs * N(0,1) (sequential_vae.py:1090): ``sd`` a node
    [B,H,W,1] broadcast over channels (predicted noise) or a python float (fixed noise_stddevs)."""
    if isinstance(sd, Node):
        y = mle.v + scale * sd.v * noise
        return tp.op(y, (mle, sd), lambda g: (g, scale * (g * noise).sum(axis=-1, keepdims=True)))
    return tp.op(mle.v + scale * float(sd) * noise, (mle,), lambda g: (g,))


def nll_per_row(tp, a, target, sd):
    """Per-image mean over H,W,C of log sd + 0.5 log 2pi + 0.5 ((a - target)/sd)^2
    (sequential_vae.py:1149-1150; its batch mean is the reference's reduce_mean over all axes).
    sd [B,H,W,1] broadcasts over the channels."""
    d = a.v - target
    s = sd.v
    m = d[0].size
    e = np.log(s) + 0.5 * np.log(2.0 * np.pi) + 0.5 * (d / s) ** 2
    y = e.reshape(e.shape[0], -1).mean(axis=1)

    def bw(g):
        gb = g.reshape((-1,) + (1,) * (d.ndim - 1)) / m
        da = gb * d / s ** 2
        ds = (gb * (1.0 / s - d ** 2 / s ** 3)).sum(axis=-1, keepdims=True)
        return da, ds

    return tp.op(y, (a, sd), bw)


def kl_uniform_per_row(tp, sig):
    """use_uniform_prior: reduce_mean(-log sigma, 1) (sequential_vae.py:1159-1160)."""
    D = sig.v.shape[1]
    y = (-np.log(sig.v)).mean(axis=1)
    return tp.op(y, (sig,), lambda g: (g[:, None] * (-1.0 / sig.v) / D,))


def sq_norm_diff_per_row(tp, a, b):
    """reduce_sum((a - b)^2, [1,2,3]) (sequential_vae.py:1190-1191)."""
    d = a.v - b.v
    y = (d ** 2).reshape(d.shape[0], -1).sum(axis=1)

    def bw(g):
        gd = 2.0 * d * g.reshape((-1,) + (1,) * (d.ndim - 1))
        return gd, -gd

    return tp.op(y, (a, b), bw)
