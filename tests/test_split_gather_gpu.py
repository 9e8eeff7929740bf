"""The split mode's gathers (dtype bf16x6) through svae_op_gather_bf16 with the split bits (path | 16 | 32):
the fp16-plane wave-split gather (csrc/halo_x3.hip; its stride-2 conv-T with one output-parity class
per wave), the fp16-plane halo_kw fallback (the 4x4-input stride-2 conv-T levels) and the bf16-plane
kernels of the other split shapes, against a float64 torch conv of the UNROUNDED fp32 operands.

The split mode claims fp32-grade products (opload.h split8_h16: 22-23 bits per operand, three MFMAs,
DESIGN §5), so the bound is the fp32 one: 2e-6 relative L2 and 2e-5 of max|ref| pointwise (measured
1.3e-7 .. 4.1e-7 on the CelebA B=128 shapes, profiles/r05_split_x3_microbench.txt).  The range cases
feed channel chunks of very different magnitude (the block's running exponent must shrink the
accumulators when a later chunk raises the maximum) and all-zero chunks."""
import numpy as np
import pytest
import torch

from conftest import pkg_mod

pytestmark = pytest.mark.gpu

# (n, h_in, cin, cout, stride, transpose)
SHAPES = [
    (16, 32, 64, 32, 1, 1), (8, 16, 128, 64, 1, 1), (8, 8, 256, 128, 1, 1),  # conv-T s1 (64-row tiles)
    (16, 32, 32, 32, 1, 0), (8, 16, 64, 64, 1, 0), (8, 8, 128, 128, 1, 0),   # conv s1
    (8, 32, 32, 64, 2, 0), (8, 16, 64, 128, 2, 0), (8, 8, 128, 128, 2, 0),   # conv s2 (32-row tiles)
    (128, 16, 64, 32, 2, 1), (128, 8, 128, 64, 2, 1),                        # conv-T s2: class per wave
    (128, 4, 384, 128, 2, 1), (16, 8, 128, 64, 2, 1),                        # conv-T s2: the halo_kw fallback
    (8, 16, 64, 32, 1, 0), (8, 32, 32, 64, 1, 0),                            # input-gradient shapes
    (128, 32, 32, 64, 2, 0), (128, 16, 64, 128, 2, 0),                       # conv s2: 64-row tiles, 8 items
    (128, 32, 64, 64, 1, 0), (128, 8, 256, 128, 1, 0), (32, 64, 32, 32, 1, 0),  # conv s1: 128-row tiles
    (128, 16, 128, 128, 1, 1),                                               # conv-T s1: 128-row tiles
]


def _split_planes(w):
    """csrc/common.h: three bf16 planes, then the scaled fp16 pair h16_pair(w) (raw 16-bit words)."""
    p0 = w.to(torch.bfloat16)
    r = w - p0.float()
    p1 = r.to(torch.bfloat16)
    p2 = (r - p1.float()).to(torch.bfloat16)
    s = w * 1024.0
    h0 = s.to(torch.float16)
    h1 = (s - h0.float()).to(torch.float16)
    return torch.stack([p0, p1, p2, h0.view(torch.bfloat16), h1.view(torch.bfloat16)]).contiguous()


def _ref(x, w_tnk, cin, cout, s, tr):
    import torch.nn.functional as F
    xd = x.double().permute(0, 3, 1, 2)
    wd = w_tnk.double().view(4, 4, cout, cin)
    h = xd.shape[2]
    if not tr:
        ho = h // s
        pad = max((ho - 1) * s + 4 - h, 0)
        pb = pad // 2
        y = F.conv2d(F.pad(xd, (pb, pad - pb, pb, pad - pb)), wd.permute(2, 3, 0, 1), stride=s)
    else:
        ho = h * s
        pb = max((h - 1) * s + 4 - ho, 0) // 2
        y = F.conv_transpose2d(xd, wd.permute(3, 2, 0, 1), stride=s)[:, :, pb:pb + ho, pb:pb + ho]
    return y.permute(0, 2, 3, 1)


def _run(x, w, n, h, cin, cout, s, tr):
    L = pkg_mod("_lib")
    ho = h * s if tr else h // s
    y = torch.full((n, ho, ho, cout), float("nan"), device="cuda")
    scratch = torch.empty(16 << 20, device="cuda")
    wp = _split_planes(w)
    L.check(L.lib().svae_op_gather_bf16(L.ptr(x), n, h, cin, L.ptr(wp), cout, s, tr, 2 | 16 | 32, L.ptr(y),
                                        L.ptr(scratch), scratch.numel() * 4, L.stream_ptr()))
    torch.cuda.synchronize()
    return y


def _check(y, r, tag):
    yd = y.double()
    assert torch.isfinite(yd).all(), tag
    rel = float((yd - r).norm() / r.norm())
    mx = float((yd - r).abs().max() / r.abs().max())
    print("%s rel %.2e max %.2e" % (tag, rel, mx))
    assert rel <= 2e-6 and mx <= 2e-5, (tag, rel, mx)


@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
def test_split_gather_matches_float64(shape):
    n, h, cin, cout, s, tr = shape
    g = torch.Generator(device="cuda").manual_seed(hash(shape) & 0xffff)
    x = torch.randn(n, h, h, cin, device="cuda", generator=g)
    w = torch.randn(16, cout, cin, device="cuda", generator=g) * 0.05
    _check(_run(x, w, *shape), _ref(x, w, cin, cout, s, tr), str(shape))


@pytest.mark.parametrize("shape", [(16, 32, 64, 32, 1, 1), (8, 8, 256, 128, 1, 1), (128, 16, 64, 32, 2, 1),
                                   (8, 16, 64, 128, 2, 0), (128, 8, 256, 128, 1, 0)])
def test_split_gather_chunk_ranges(shape):
    """Chunks of 32 channels at magnitudes 1e-3, 1e+3, 0 and 1 in turn: the running exponent rises and
    the accumulators are rescaled; an all-zero chunk leaves it; small chunks after a large one keep
    an absolute error of order 2^-40 of the maximum."""
    n, h, cin, cout, s, tr = shape
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(n, h, h, cin, device="cuda", generator=g)
    scale = torch.tensor([1e-3, 1e3, 0.0, 1.0], device="cuda").repeat(cin // 128 + 1)[:cin // 32]
    x = x * scale.repeat_interleave(32)
    w = torch.randn(16, cout, cin, device="cuda", generator=g) * 0.05
    _check(_run(x, w, *shape), _ref(x, w, cin, cout, s, tr), "ranges " + str(shape))
