"""Kernel-level parity: each HIP op (through the C ABI per-op entry points) vs a
float64 PyTorch-CPU reference of the same TF-SAME op (oracle/torch_twin.py helpers).
Tolerance: fp32 MFMA accumulation vs fp64 — max-abs error <= 2e-5 * (1 + max|ref|)."""
import numpy as np
import pytest
import torch

from conftest import pkg_mod
from oracle import torch_twin as TT

pytestmark = pytest.mark.gpu

CONV_CASES = [
    # n, h, cin, cout, stride, transpose
    (2, 16, 3, 32, 2, 0),     # layer-0 conv (small-C gather path)
    (2, 64, 3, 32, 2, 0),     # layer-0 conv at 64x64 (csrc/smallc.hip window kernel)
    (2, 32, 4, 64, 2, 0),     # 4 input channels, N = 64
    (2, 32, 32, 4, 2, 1),     # packed output conv-T [C | ratio]: its input gradient is the small-C gather
    (2, 8, 32, 32, 1, 0),     # stride-1 conv, N<=32 tile
    (2, 8, 64, 64, 1, 0),
    (2, 8, 128, 128, 2, 0),
    (2, 4, 128, 128, 1, 0),
    (2, 4, 384, 128, 2, 1),   # decoder conv-T s2 from the top fc
    (2, 4, 256, 128, 1, 1),   # decoder conv-T s1 over the concat
    (2, 8, 64, 32, 2, 1),
    (3, 8, 8, 8, 2, 0),       # tiny geometry (small-C, NK/KN small tiles)
    (3, 4, 16, 24, 1, 1),
    (3, 4, 48, 16, 2, 1),
]


def _lib():
    return pkg_mod("_lib")


def _rand(shape, seed):
    return torch.from_numpy(np.random.default_rng(seed).uniform(-1, 1, size=shape).astype(np.float32))


def _ref_conv(x, w, stride, tr):
    xn = x.double().permute(0, 3, 1, 2)
    y = (TT.conv2d_t_same if tr else TT.conv2d_same)(xn, w.double(), stride)
    return y.permute(0, 2, 3, 1)


def _close(got, ref, tol=2e-5):
    got = got.double().cpu()
    err = (got - ref).abs().max().item()
    assert err <= tol * (1 + ref.abs().max().item()), err


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd(case):
    n, h, cin, cout, s, tr = case
    L = _lib()
    x = _rand((n, h, h, cin), 1)
    w = _rand((4, 4, cout, cin) if tr else (4, 4, cin, cout), 2) * 0.2
    ho = h * s if tr else h // s
    y = torch.zeros(n, ho, ho, cout, device="cuda")
    xd, wd = x.cuda(), w.cuda()
    L.check(L.lib().svae_op_conv(L.ptr(xd), n, h, cin, L.ptr(wd), cout, s, tr, L.ptr(y), L.stream_ptr()))
    torch.cuda.synchronize()
    _close(y, _ref_conv(x, w, s, tr))


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_dgrad_wgrad(case):
    n, h, cin, cout, s, tr = case
    L = _lib()
    x = _rand((n, h, h, cin), 3).double().requires_grad_(True)
    w = (_rand((4, 4, cout, cin) if tr else (4, 4, cin, cout), 4) * 0.2).double().requires_grad_(True)
    y = _ref_conv(x, w, s, tr)
    dy = _rand(tuple(y.shape), 5).double()
    (y * dy).sum().backward()
    dyd = dy.float().cuda().contiguous()
    wd = w.detach().float().cuda().contiguous()
    xd = x.detach().float().cuda().contiguous()
    dx = torch.zeros(n, h, h, cin, device="cuda")
    L.check(L.lib().svae_op_conv_dgrad(L.ptr(dyd), n, h, cin, L.ptr(wd), cout, s, tr, L.ptr(dx), L.stream_ptr()))
    dw = torch.zeros(tuple(w.shape), device="cuda")
    scratch = torch.empty(16 << 20, device="cuda")
    L.check(L.lib().svae_op_conv_wgrad(L.ptr(xd), n, h, cin, L.ptr(dyd), cout, s, tr, L.ptr(dw), L.ptr(scratch),
                                       scratch.numel() * 4, L.stream_ptr()))
    torch.cuda.synchronize()
    _close(dx, x.grad)
    _close(dw, w.grad, tol=5e-5)


@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("rows,c", [(1000, 32), (128, 6144), (77, 24)])
def test_bn_act(act, rows, c):
    L = _lib()
    x = (_rand((rows, c), 6) * 3 + 0.5).double().requires_grad_(True)
    beta = (_rand((c,), 7) * 0.3).double().requires_grad_(True)
    m = x.mean(0)
    v = ((x - m) ** 2).mean(0)
    z = (x - m) / torch.sqrt(v + 1e-3) + beta
    y = {0: z, 1: torch.relu(z), 2: torch.maximum(torch.minimum(0.1 * z, torch.zeros_like(z)), z)}[act]
    dy = _rand((rows, c), 8).double()
    (y * dy).sum().backward()
    xd, bd = x.detach().float().cuda(), beta.detach().float().cuda()
    yd = torch.zeros(rows, c, device="cuda")
    mean = torch.zeros(c, device="cuda")
    inv = torch.zeros(c, device="cuda")
    scratch = torch.empty(4 << 20, device="cuda")
    L.check(L.lib().svae_op_bn_act(L.ptr(xd), rows, c, L.ptr(bd), act, L.ptr(yd), L.ptr(mean), L.ptr(inv),
                                   L.ptr(scratch), scratch.numel() * 4, L.stream_ptr()))
    dx = torch.zeros(rows, c, device="cuda")
    db = torch.zeros(c, device="cuda")
    dyd = dy.float().cuda()
    L.check(L.lib().svae_op_bn_act_bwd(L.ptr(dyd), L.ptr(yd), L.ptr(xd), rows, c, L.ptr(mean), L.ptr(inv), act,
                                       L.ptr(dx), L.ptr(db), L.ptr(scratch), scratch.numel() * 4, L.stream_ptr()))
    torch.cuda.synchronize()
    _close(yd, y.detach(), 1e-5)
    _close(mean, m.detach(), 1e-6)
    _close(dx, x.grad, 1e-4)
    _close(db, beta.grad, 1e-5)


@pytest.mark.parametrize("b,k,n", [(128, 896, 6144), (128, 2048, 384), (4, 40, 96), (256, 512, 6144)])
def test_fc(b, k, n):
    L = _lib()
    x, w = _rand((b, k), 9), _rand((k, n), 10) * 0.05
    y = torch.zeros(b, n, device="cuda")
    xd, wd = x.cuda(), w.cuda()
    L.check(L.lib().svae_op_fc(L.ptr(xd), b, k, L.ptr(wd), n, L.ptr(y), L.stream_ptr()))
    torch.cuda.synchronize()
    _close(y, x.double() @ w.double())
