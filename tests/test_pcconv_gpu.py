"""svae_pcnn_conv (the PixelCNN++ head's gather convolution, include/svae_pcnn.h) against a torch fp64
reference on the same bf16-rounded operands, over the geometries the head launches: the shifted
[2, 3] / [2, 2] / [1, 3] / [2, 1] convs (mode 0) and their input gradients (mode 1) at 64x64, 32x32,
16x16 and 8x8 (several images per block), the 1x1 nin / dense layers, shifted outputs (zero_edge),
accumulation, channel slices (ldx > cin), 1 - 10 column tiles, and shapes that take the fallback
kernel (stride 2, ragged rows).  Only bf16 products summed in fp32 differ from the reference."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import pkg_mod

pytestmark = pytest.mark.gpu


def _ref(x, w, n, hi, wi, cin, ho, wo, cout, kh, kw, s, pt, pl, mode, bias, zero_edge):
    """out(oy, ox) = sum_taps in(src(oy, ox, ky, kx)) . W[ky][kx] (svae_pcnn.h geometry), fp64."""
    xi = x.reshape(n, hi, wi, -1)[..., :cin].permute(0, 3, 1, 2).double()
    wt = w.double()  # [tap][cout][cin]
    W4 = wt.reshape(kh, kw, cout, cin).permute(2, 3, 0, 1)  # [cout][cin][kh][kw]
    if mode == 0:
        # iy = oy*s - pt + ky: cross-correlation over the input padded by pt / pl at the top / left
        pad_b = max(0, (ho - 1) * s - pt + kh - hi)
        pad_r = max(0, (wo - 1) * s - pl + kw - wi)
        xp = F.pad(xi, (pl, pad_r, pt, pad_b))
        y = F.conv2d(xp, W4, stride=s)[:, :, :ho, :wo]
    else:
        assert s == 1
        # iy = oy + pt - ky: the flipped kernel, origin oy + pt - kh + 1
        top, left = kh - 1 - pt, kw - 1 - pl
        pad_b = max(0, ho - 1 + pt - hi + 1)
        pad_r = max(0, wo - 1 + pl - wi + 1)
        xp = F.pad(xi, (max(left, 0), pad_r, max(top, 0), pad_b))
        xp = xp[:, :, max(-top, 0):, max(-left, 0):]
        y = F.conv2d(xp, W4.flip(2, 3))[:, :, :ho, :wo]
    y = y.permute(0, 2, 3, 1).reshape(n * ho * wo, cout)
    if bias is not None:
        y = y + bias.double()
    if zero_edge:
        m = torch.zeros(n, ho, wo, 1, dtype=torch.bool)
        if zero_edge == 1:
            m[:, 0] = True
        else:
            m[:, :, 0] = True
        y = torch.where(m.reshape(-1, 1), torch.zeros_like(y), y)
    return y


CASES = [
    # n, hi, ho, cin, ldx, cout, kh, kw, s, pt, pl, mode, acc, zero_edge
    (2, 64, 64, 160, 160, 160, 2, 3, 1, 1, 1, 0, 0, 0),    # u-stream resnet conv
    (2, 64, 64, 160, 160, 320, 2, 3, 1, 1, 1, 1, 0, 0),    # its input gradient, 2 column tiles
    (2, 32, 32, 64, 96, 96, 2, 2, 1, 1, 1, 0, 1, 0),       # ul-stream conv, channel slice, accumulate
    (2, 32, 32, 96, 96, 64, 2, 2, 1, 1, 1, 1, 1, 0),
    (2, 16, 16, 4, 4, 160, 2, 3, 1, 2, 1, 0, 0, 1),        # down_shift(ds_conv(x_pad)) of the input
    (8, 8, 8, 8, 8, 8, 2, 1, 1, 1, 1, 0, 1, 2),            # right_shift(drs_conv), 4 images per block
    (8, 8, 8, 8, 8, 8, 1, 3, 1, 1, 1, 1, 0, 0),
    (512, 1, 1, 320, 320, 100, 1, 1, 1, 0, 0, 0, 0, 0),    # nin / dense (10 M mixture logits)
    (2, 64, 64, 160, 160, 40, 2, 3, 1, 1, 1, 0, 0, 0),     # 2 column tiles of 32 (one partial)
    (2, 4, 4, 8, 8, 8, 2, 3, 1, 1, 1, 0, 0, 0),            # ragged rows: fallback kernel
    (2, 32, 16, 32, 32, 32, 2, 3, 2, 1, 1, 0, 0, 0),       # stride 2: fallback kernel
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "n%d_h%d_%dto%d_k%dx%d_s%d_m%d_a%d_z%d" % (
    c[0], c[2], c[3], c[5], c[6], c[7], c[8], c[11], c[12], c[13]))
def test_pcnn_conv_matches_reference(case):
    n, hi, ho, cin, ldx, cout, kh, kw, s, pt, pl, mode, acc, zero_edge = case
    wi, wo = hi, ho
    L = pkg_mod("_lib")
    rng = np.random.default_rng(hash(case) % 2 ** 32)
    kpad = (cin + 31) // 32 * 32
    taps = kh * kw
    x = torch.tensor(rng.uniform(-1, 1, (n * hi * wi, ldx)), dtype=torch.float32).to(torch.bfloat16).float()
    w = torch.tensor(rng.normal(0, 0.1, (taps, cout, cin)), dtype=torch.float32).to(torch.bfloat16)
    wk = torch.zeros(taps, cout, kpad, dtype=torch.bfloat16)
    wk[:, :, :cin] = w
    bias = torch.tensor(rng.normal(0, 0.1, cout), dtype=torch.float32)
    y0 = torch.tensor(rng.normal(0, 1, (n * ho * wo, cout)), dtype=torch.float32)
    xd, wkd, bd = x.cuda(), wk.cuda(), bias.cuda()
    yd = y0.clone().cuda() if acc else torch.full((n * ho * wo, cout), float("nan"), device="cuda")
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    L.check(L.lib().svae_pcnn_conv(p(xd), n, hi, wi, cin, ldx, 0, p(wkd), kpad, p(bd), p(yd), ho, wo, cout, cout, kh, kw,
                                   s, pt, pl, mode, acc, zero_edge, L.stream_ptr()))
    torch.cuda.synchronize()
    ref = _ref(x, w.float(), n, hi, wi, cin, ho, wo, cout, kh, kw, s, pt, pl, mode, bias, zero_edge)
    if acc:
        ref = ref + y0.double()
    got = yd.cpu().double()
    err = float((got - ref).abs().max() / ref.abs().max())
    print("\nconv %s: max rel err %.2e" % (case, err))
    assert torch.isfinite(got).all()
    assert err < 2e-5
    if cin % 8 == 0 and ldx % 8 == 0:  # the same operand stored as bf16 (x_bf16): bitwise the same result
        yb = y0.clone().cuda() if acc else torch.full((n * ho * wo, cout), float("nan"), device="cuda")
        xb = xd.to(torch.bfloat16)
        L.check(L.lib().svae_pcnn_conv(p(xb), n, hi, wi, cin, ldx, 1, p(wkd), kpad, p(bd), p(yb), ho, wo, cout, cout, kh,
                                       kw, s, pt, pl, mode, acc, zero_edge, L.stream_ptr()))
        torch.cuda.synchronize()
        assert torch.equal(yb.cpu(), yd.cpu())


def _gathered(x, n, hi, wi, cin, ho, wo, kh, kw, pt, pl, mode, ky, kx):
    """X[src(p, tap)] for every output pixel p of a stride-1 conv (zero outside the image), fp64."""
    xi = x.reshape(n, hi, wi, -1)[..., :cin].double()
    if mode == 0:
        top, left, oy, ox = pt, pl, ky, kx
    else:
        top, left, oy, ox = kh - 1 - pt, kw - 1 - pl, kh - 1 - ky, kw - 1 - kx
    big = torch.zeros(n, ho + kh + abs(top) + hi, wo + kw + abs(left) + wi, cin, dtype=torch.float64)
    big[:, kh + abs(top) + top - kh:, :][:, :hi, :][:, :, kw + abs(left) + left - kw:][:, :, :wi] = xi
    y0, x0 = kh + abs(top) - kh + oy, kw + abs(left) - kw + ox
    return big[:, y0:y0 + ho, x0:x0 + wo].reshape(n * ho * wo, cin)


WCASES = [
    # n, h, cin, ldx, cout, kh, kw, pt, pl, mode, x_bf16
    (2, 64, 160, 160, 160, 2, 3, 1, 1, 0, 1),     # resnet conv, bf16 input
    (2, 64, 160, 160, 320, 2, 2, 1, 1, 0, 1),
    (2, 32, 64, 96, 96, 2, 3, 1, 1, 1, 0),        # mode 1, fp32 input, channel slice
    (2, 16, 32, 32, 64, 2, 3, 2, 1, 0, 0),
    (512, 1, 320, 320, 160, 1, 1, 0, 0, 0, 1),    # nin
    (8, 8, 32, 32, 32, 2, 2, 1, 1, 0, 1),
    (2, 16, 4, 4, 32, 2, 3, 2, 1, 0, 0),          # 4 input channels (x_pad)
    (4, 16, 8, 8, 16, 2, 3, 1, 1, 0, 1),          # channel counts below one 32-wide sub-tile
    (4, 16, 16, 16, 8, 2, 3, 1, 1, 1, 0),
    (2, 32, 96, 96, 40, 2, 3, 1, 1, 0, 1),        # partial 64-wide tiles
]


@pytest.mark.parametrize("case", WCASES, ids=lambda c: "n%d_h%d_%dto%d_k%dx%d_m%d_xb%d" % (
    c[0], c[1], c[2], c[4], c[5], c[6], c[9], c[10]))
def test_pcnn_wgrad_matches_reference(case):
    n, h, cin, ldx, cout, kh, kw, pt, pl, mode, xb = case
    L = pkg_mod("_lib")
    rng = np.random.default_rng(hash(case) % 2 ** 32)
    x = torch.tensor(rng.uniform(-1, 1, (n * h * h, ldx)), dtype=torch.float32).to(torch.bfloat16).float()
    d = torch.tensor(rng.normal(0, 1, (n * h * h, cout)), dtype=torch.float32)
    db = d.to(torch.bfloat16).double()  # the kernels stage D as bf16
    ref = torch.stack([_gathered(x, n, h, h, cin, h, h, kh, kw, pt, pl, mode, t // kw, t % kw).T @ db
                       for t in range(kh * kw)])
    xd = x.cuda().to(torch.bfloat16) if xb else x.cuda()
    dd = d.cuda()
    dW = torch.full((kh * kw, cin, cout), float("nan"), device="cuda")
    sc = torch.empty(1 << 24, device="cuda")
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    db = torch.full((cout,), float("nan"), device="cuda")
    L.check(L.lib().svae_pcnn_conv_wgrad(p(xd), n, h, h, cin, ldx, xb, p(dd), cout, 0, h, h, cout, kh, kw, 1, pt, pl, mode,
                                         p(dW), p(db), p(sc), sc.numel(), L.stream_ptr()))
    torch.cuda.synchronize()
    got = dW.cpu().double()
    err = float((got - ref).abs().max() / ref.abs().max())
    dbref = d.double().sum(0)  # the bias gradient: fp32 dy summed (not bf16-rounded)
    eb = float((db.cpu().double() - dbref).abs().max() / dbref.abs().max())
    print("\nwgrad %s: max rel err %.2e, bias %.2e" % (case, err, eb))
    assert torch.isfinite(got).all()
    assert err < 1e-5 and eb < 1e-5


# ---------------- the split mode: operands as sums of 16-bit planes (include/svae_pcnn.h) ----------------
# fmt "bf16": 3 bf16 planes, 6 products; fmt "h16": two scaled fp16 planes, 3 products (16-bit storage only)
def _planes(L, t, fmt, bf=1):
    """svae_pcnn_split_planes of fp32 [rows][c] ``t`` (device): ([planes][rows][c] planes, scale or None)."""
    rows, c = t.shape
    h16 = fmt == "h16"
    P = 2 if h16 else 3
    out = torch.empty(P, rows, c, dtype=torch.bfloat16 if (bf or h16) else torch.float32, device="cuda")
    sc = torch.empty(2, device="cuda") if h16 else None
    L.check(L.lib().svae_pcnn_split_planes(ctypes.c_void_p(t.data_ptr()), rows, c, c, P,
                                           ctypes.c_void_p(out.data_ptr()), c, int(bf or h16),
                                           None if sc is None else ctypes.c_void_p(sc.data_ptr()), L.stream_ptr()))
    return out, sc


@pytest.mark.parametrize("rows,c,ld", [(4096, 160, 160), (1000, 12, 12), (777, 6, 6), (2048, 64, 80), (5, 4, 4)])
def test_pcnn_split_h16_is_exact(rows, c, ld):
    """The scaled fp16 pair of svae_pcnn_split_planes (the 4-channel vector kernels where c, ld % 4 == 0, the
    element loop else) bit for bit against torch: s = 15 - e (max|x| = f 2^e, f in [0.5, 1)), hi = fp16(x 2^s),
    lo = fp16(x 2^s - hi), scale[0] = 2^-s; a strided source (ld > c) and magnitudes over 2^-30 .. 2^20."""
    L = pkg_mod("_lib")
    g = torch.Generator(device="cuda").manual_seed(rows * 131 + c)
    src = torch.randn(rows, ld, device="cuda", generator=g) * torch.exp2(
        torch.randint(-30, 20, (rows, 1), device="cuda", generator=g).float())
    x = src[:, :c]
    out = torch.empty(2, rows, c, dtype=torch.bfloat16, device="cuda")
    sc = torch.empty(2, device="cuda")
    L.check(L.lib().svae_pcnn_split_planes(ctypes.c_void_p(src.data_ptr()), rows, c, ld, 2,
                                           ctypes.c_void_p(out.data_ptr()), c, 1, ctypes.c_void_p(sc.data_ptr()),
                                           L.stream_ptr()))
    torch.cuda.synchronize()
    e = int(torch.frexp(x.abs().max()).exponent)
    s = max(-60, min(60, 15 - e))
    t = torch.ldexp(x, torch.tensor(float(s), device="cuda"))
    hi = t.half()
    lo = (t - hi.float()).half()
    assert float(sc[0]) == 2.0 ** -s and float(sc[1]) == float(x.abs().max())
    assert torch.equal(out[0].view(torch.int16), hi.view(torch.int16))
    assert torch.equal(out[1].view(torch.int16), lo.view(torch.int16))


@pytest.mark.parametrize("n,ho,wo,c,ld,mask,acc", [(16, 32, 32, 160, 160, 0, 0), (16, 32, 32, 160, 160, 1, 1),
                                                   (8, 16, 16, 64, 96, 2, 0), (4, 8, 8, 6, 6, 1, 0),
                                                   (3, 7, 5, 12, 12, 2, 1), (128, 32, 32, 80, 80, 0, 0)])
def test_pcnn_colsum_matches_float64(n, ho, wo, c, ld, mask, acc):
    """svae_pcnn_colsum (the conv bias gradients: column sums over [rows][c], optionally without each image's first
    output row (mask 1) or column (mask 2), added to ``out`` with acc) against a float64 sum: the 4-column vector
    partials where c, ld % 4 == 0, the element ones else."""
    L = pkg_mod("_lib")
    g = torch.Generator(device="cuda").manual_seed(n * 1000 + c + mask)
    rows = n * ho * wo
    src = torch.randn(rows, ld, device="cuda", generator=g)
    out = torch.randn(c, device="cuda", generator=g)
    ref = src[:, :c].double().view(n, ho, wo, c)
    if mask == 1:
        ref = ref[:, 1:]
    elif mask == 2:
        ref = ref[:, :, 1:]
    ref = ref.sum((0, 1, 2)) + (out.double() if acc else 0)
    scratch = torch.empty(1 << 22, device="cuda")
    L.check(L.lib().svae_pcnn_colsum(ctypes.c_void_p(src.data_ptr()), rows, c, ld, ho, wo, mask,
                                     ctypes.c_void_p(out.data_ptr()), acc, ctypes.c_void_p(scratch.data_ptr()),
                                     L.stream_ptr()))
    torch.cuda.synchronize()
    err = float((out.double() - ref).abs().max() / (ref.abs().max() + 1.0))
    assert err < 1e-5, err


@pytest.mark.parametrize("kind,keep", [(2, 1.0), (1, 0.5), (0, 1.0)])
def test_pcnn_nonlin_absmax_then_premax_split_is_the_two_pass_split(kind, keep):
    """svae_pcnn_nonlin_absmax (the nonlinearity leaving max|y|) + svae_pcnn_split_h16_premax bit for bit the
    plain nonlinearity + svae_pcnn_split_planes' absmax and split passes (the split head's fused path)."""
    L = pkg_mod("_lib")
    rows, c = 3000, 40
    g = torch.Generator(device="cuda").manual_seed(kind)
    x = torch.randn(rows, c, device="cuda", generator=g) * 3
    cy = 2 * c if kind == 2 else c
    y0 = torch.empty(rows, cy, device="cuda")
    y1 = torch.empty(rows, cy, device="cuda")
    sc = torch.empty(2, device="cuda")
    vp = lambda t: ctypes.c_void_p(t.data_ptr())
    L.check(L.lib().svae_pcnn_nonlin(vp(x), rows, c, c, kind, None, keep, 99, vp(y0), cy, 0, L.stream_ptr()))
    L.check(L.lib().svae_pcnn_nonlin_absmax(vp(x), rows, c, c, kind, None, keep, 99, vp(y1), cy, vp(sc),
                                            L.stream_ptr()))
    p1 = torch.empty(2, rows, cy, dtype=torch.bfloat16, device="cuda")
    L.check(L.lib().svae_pcnn_split_h16_premax(vp(y1), rows, cy, cy, vp(p1), cy, vp(sc), L.stream_ptr()))
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)
    assert float(sc[1]) == float(y0.abs().max())
    p0, sc0 = _planes(L, y0, "h16")
    torch.cuda.synchronize()
    assert torch.equal(p0.view(torch.int16), p1.view(torch.int16)) and torch.equal(sc0, sc)


def _wn_planes(L, V, g, taps, cin, cout, fmt):
    """svae_pcnn_wnorm_planes: the forward copy's planes [planes][tap][cout][kf], its scale, the fp64 W [tap][cout][cin]."""
    h16 = fmt == "h16"
    P = 2 if h16 else 3
    kf, kd = (cin + 31) // 32 * 32, (cout + 31) // 32 * 32
    norm = torch.empty(cout, device="cuda")
    wkf = torch.empty(P * taps * cout * kf, dtype=torch.bfloat16, device="cuda")
    wkd = torch.empty(P * taps * cin * kd, dtype=torch.bfloat16, device="cuda")
    sc = torch.empty(2, device="cuda") if h16 else None
    Vd, gd = V.cuda(), g.cuda()
    p = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())
    L.check(L.lib().svae_pcnn_wnorm_planes(p(Vd), p(gd), taps, cin, cout, p(norm), p(wkf), kf, p(wkd), kd, P, p(sc),
                                           L.stream_ptr()))
    V64 = V.double().reshape(taps, cin, cout)
    W = V64 * (g.double() / V64.pow(2).sum((0, 1)).sqrt())
    return wkf, kf, sc, W.permute(0, 2, 1).contiguous()


def _fmts(c):
    return ["bf16", "h16"] if c % 8 == 0 else ["bf16"]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "n%d_h%d_%dto%d_k%dx%d_s%d_m%d_a%d_z%d" % (
    c[0], c[2], c[3], c[5], c[6], c[7], c[8], c[11], c[12], c[13]))
def test_pcnn_conv_planes_is_fp32_grade(case):
    """svae_pcnn_conv_planes over unrounded fp32 operands (x split by svae_pcnn_split_planes, W by
    svae_pcnn_wnorm_planes) in both plane formats -- 3 bf16 planes (fp32 and bf16 storage) and, where cin
    allows, two scaled fp16 planes -- against fp64: the fp32 bounds of tests/test_split_gather_gpu.py
    (2e-6 relative L2, 2e-5 of max|ref| pointwise).  The input is scaled by 1e-3 so the fp16 planes'
    scale is exercised away from 1."""
    n, hi, ho, cin, ldx, cout, kh, kw, s, pt, pl, mode, acc, zero_edge = case
    wi, wo = hi, ho
    L = pkg_mod("_lib")
    rng = np.random.default_rng(hash(case) % 2 ** 32 + 1)
    taps = kh * kw
    x = torch.tensor(rng.uniform(-1, 1, (n * hi * wi, cin)) * 1e-3, dtype=torch.float32)
    V = torch.tensor(rng.normal(0, 0.05, (taps, cin, cout)), dtype=torch.float32)
    g = torch.tensor(rng.uniform(0.5, 2.0, cout), dtype=torch.float32)
    bias = torch.tensor(rng.normal(0, 1e-4, cout), dtype=torch.float32)
    y0 = torch.tensor(rng.normal(0, 1e-3, (n * ho * wo, cout)), dtype=torch.float32)
    p = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())
    xd, bd = x.cuda(), bias.cuda()
    for fmt in _fmts(cin):
        wkf, kf, wsc, W = _wn_planes(L, V, g, taps, cin, cout, fmt)
        ref = _ref(x, W, n, hi, wi, cin, ho, wo, cout, kh, kw, s, pt, pl, mode, bias, zero_edge)
        if acc:
            ref = ref + y0.double()
        for bf in ([1] if fmt == "h16" else ([0, 1] if cin % 8 == 0 else [0])):
            xs, xsc = _planes(L, xd, fmt, bf)
            P = xs.shape[0]
            yd = y0.clone().cuda() if acc else torch.full((n * ho * wo, cout), float("nan"), device="cuda")
            L.check(L.lib().svae_pcnn_conv_planes(p(xs), n, hi, wi, cin, cin, bf, n * hi * wi * cin, p(wkf), kf, P,
                                                  p(xsc), p(wsc), p(bd), p(yd), ho, wo, cout, cout, kh, kw, s, pt, pl,
                                                  mode, acc, zero_edge, L.stream_ptr()))
            torch.cuda.synchronize()
            got = yd.cpu().double()
            rel = float((got - ref).norm() / ref.norm())
            mx = float((got - ref).abs().max() / ref.abs().max())
            print("\nconv planes %s %s bf%d: rel %.2e max %.2e" % (case, fmt, bf, rel, mx))
            assert torch.isfinite(got).all()
            assert rel <= 2e-6 and mx <= 2e-5


@pytest.mark.parametrize("case", WCASES, ids=lambda c: "n%d_h%d_%dto%d_k%dx%d_m%d_xb%d" % (
    c[0], c[1], c[2], c[4], c[5], c[6], c[9], c[10]))
def test_pcnn_wgrad_planes_is_fp32_grade(case):
    """svae_pcnn_conv_wgrad_planes: every product's slabs and one reduce, against fp64 on the unrounded
    operands, in both plane formats (fp16 where cin and cout allow; dy spans 6 decades to exercise the
    fp16 planes' floor)."""
    n, h, cin, ldx, cout, kh, kw, pt, pl, mode, xb = case
    L = pkg_mod("_lib")
    rng = np.random.default_rng(hash(case) % 2 ** 32 + 2)
    x = torch.tensor(rng.uniform(-1, 1, (n * h * h, cin)), dtype=torch.float32)
    d = torch.tensor(rng.normal(0, 1, (n * h * h, cout)) * 10.0 ** rng.uniform(-6, 0, (n * h * h, 1)),
                     dtype=torch.float32)
    ref = torch.stack([_gathered(x, n, h, h, cin, h, h, kh, kw, pt, pl, mode, t // kw, t % kw).T @ d.double()
                       for t in range(kh * kw)])
    p = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())
    rows = n * h * h
    for fmt in (["bf16", "h16"] if cin % 8 == 0 and cout % 8 == 0 else ["bf16"]):
        xbf = 1 if fmt == "h16" else (xb if cin % 8 == 0 else 0)
        xs, xsc = _planes(L, x.cuda(), fmt, xbf)
        ds, dsc = _planes(L, d.cuda(), fmt, 1 if fmt == "h16" else 0)
        dbf = 1 if fmt == "h16" else 0
        dW = torch.full((kh * kw, cin, cout), float("nan"), device="cuda")
        sc = torch.empty(1 << 24, device="cuda")
        L.check(L.lib().svae_pcnn_conv_wgrad_planes(p(xs), n, h, h, cin, cin, xbf, rows * cin, p(ds), cout, dbf,
                                                    rows * cout, xs.shape[0], p(xsc), p(dsc), h, h, cout, kh, kw, 1,
                                                    pt, pl, mode, p(dW), p(sc), sc.numel(), L.stream_ptr()))
        torch.cuda.synchronize()
        got = dW.cpu().double()
        rel = float((got - ref).norm() / ref.norm())
        mx = float((got - ref).abs().max() / ref.abs().max())
        print("\nwgrad planes %s %s: rel %.2e max %.2e" % (case, fmt, rel, mx))
        assert torch.isfinite(got).all()
        assert rel <= 2e-6 and mx <= 2e-5


@pytest.mark.parametrize("rows,c,ld,acc", [(131072, 160, 160, 0), (32768, 320, 320, 1), (3000, 40, 48, 0),
                                           (777, 6, 6, 1)])
def test_pcnn_colsum_absmax_is_colsum_plus_the_absmax_pass(rows, c, ld, acc):
    """svae_pcnn_colsum_absmax (the split head's gradient prologue: bias-gradient column sums and max|dy| in one
    pass) bit for bit svae_pcnn_colsum + the absmax pass of svae_pcnn_split_planes, and the premax split after it
    the planes of svae_pcnn_split_planes (the 4-column vector kernel where c, ld % 4 == 0, the two passes else)."""
    L = pkg_mod("_lib")
    g = torch.Generator(device="cuda").manual_seed(rows + c)
    src = torch.randn(rows, ld, device="cuda", generator=g) * 1e-3
    out0 = torch.randn(c, device="cuda", generator=g)
    out1 = out0.clone()
    scratch = torch.empty(1 << 22, device="cuda")
    sc = torch.empty(2, device="cuda")
    vp = lambda t: ctypes.c_void_p(t.data_ptr())
    L.check(L.lib().svae_pcnn_colsum(vp(src), rows, c, ld, 1, 1, 0, vp(out0), acc, vp(scratch), L.stream_ptr()))
    L.check(L.lib().svae_pcnn_colsum_absmax(vp(src), rows, c, ld, vp(out1), acc, vp(scratch), vp(sc), L.stream_ptr()))
    torch.cuda.synchronize()
    assert torch.equal(out0, out1)
    assert float(sc[1]) == float(src[:, :c].abs().max())
    if c % 4 == 0:
        dense = src[:, :c].contiguous()
        p1 = torch.empty(2, rows, c, dtype=torch.bfloat16, device="cuda")
        L.check(L.lib().svae_pcnn_colsum_absmax(vp(dense), rows, c, c, vp(out1), 0, vp(scratch), vp(sc), L.stream_ptr()))
        L.check(L.lib().svae_pcnn_split_h16_premax(vp(dense), rows, c, c, vp(p1), c, vp(sc), L.stream_ptr()))
        p0, sc0 = _planes(L, dense, "h16")
        torch.cuda.synchronize()
        assert torch.equal(p0.view(torch.int16), p1.view(torch.int16)) and torch.equal(sc0, sc)


@pytest.mark.parametrize("kind,keep,tensor_mask", [(0, 1.0, False), (0, 0.7, False), (0, 0.7, True), (1, 0.7, False),
                                                   (2, 1.0, False)])
def test_pcnn_nonlin_h16_planes_hold_the_nonlinearity(kind, keep, tensor_mask):
    """svae_pcnn_nonlin_h16 (the split head's conv input written straight as fp16 planes, the exponent from a bound
    on max|y| known before the pass): the planes sum to svae_pcnn_nonlin's fp32 output within 2^-21 of the bound
    (two fp16 planes: 22 bits of the scaled value) and the bound covers max|y| -- for the in-kernel seeded dropout
    and for a mask tensor."""
    L = pkg_mod("_lib")
    rows, c = 4096, 40
    g = torch.Generator(device="cuda").manual_seed(kind * 10 + int(keep * 10))
    x = torch.randn(rows, c, device="cuda", generator=g) * 3
    cy = 2 * c if kind == 2 else c
    vp = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())
    mask = None
    if tensor_mask:
        mask = (torch.rand(rows, cy, device="cuda", generator=g) < keep).float() / keep
    y = torch.empty(rows, cy, device="cuda")
    L.check(L.lib().svae_pcnn_nonlin(vp(x), rows, c, c, kind, vp(mask), 1.0 if tensor_mask else keep, 77, vp(y), cy, 0,
                                     L.stream_ptr()))
    xs = torch.tensor([0.0, float(x.abs().max())], device="cuda")
    pl = torch.empty(2, rows, cy, dtype=torch.float16, device="cuda")
    sc = torch.empty(2, device="cuda")
    mmax = float(mask.max()) if tensor_mask else 0.0
    L.check(L.lib().svae_pcnn_nonlin_h16(vp(x), rows, c, c, kind, vp(mask), mmax, 1.0 if tensor_mask else keep, 77,
                                         vp(xs), vp(pl), cy, vp(sc), L.stream_ptr()))
    torch.cuda.synchronize()
    bound = float(sc[1])
    assert bound >= float(y.abs().max())
    rec = (pl[0].double() + pl[1].double()) * float(sc[0])
    err = float((rec - y.double()).abs().max())
    assert err <= bound * 2.0 ** -21, (err, bound)
