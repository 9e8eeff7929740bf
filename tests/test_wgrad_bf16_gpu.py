"""bf16 weight-gradient kernels (csrc/gemm_bf16.hip) through svae_op_wgrad_bf16 on the conv /
conv-T layer shapes of the CelebA geometry (and wgrad_smallc.hip for the Cin <= 3 image convs).  Reference: float64 torch autograd of the TF-SAME
conv on the SAME bf16-rounded x and dy (oracle/torch_twin.py), so only fp32 accumulation order
differs: bound 2e-5 relative (L2), 1e-4 of max|ref| pointwise.  path 0 = tap-merged weight-GEMM,
path 2 = halo weight-GEMMs (transposed LDS reads; stride 1 on the compile-time-geometry kernel of
wgrad_halo2.hip), path 3 = the run-time-geometry halo weight-GEMM for stride 1 too."""
import pytest
import torch

from conftest import pkg_mod
from oracle import torch_twin

pytestmark = pytest.mark.gpu

# (n, h_in, cin, cout, stride, transpose)
SHAPES = [
    (4, 32, 32, 32, 1, 0), (4, 32, 32, 64, 2, 0), (4, 16, 64, 64, 1, 0), (4, 16, 64, 128, 2, 0),
    (4, 8, 128, 128, 1, 0), (8, 8, 128, 128, 2, 0),
    (4, 4, 384, 128, 2, 1), (4, 8, 256, 128, 1, 1), (4, 8, 128, 64, 2, 1), (4, 16, 128, 64, 1, 1),
    (4, 16, 64, 32, 2, 1), (4, 32, 64, 32, 1, 1),
]


def _bf(t):
    return t.to(torch.bfloat16).to(t.dtype)


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "n%d_h%d_%dto%d_s%d_%s" % (s[0], s[1], s[2], s[3], s[4],
                                                                                 "T" if s[5] else "C"))
@pytest.mark.parametrize("path", [0, 2, 3])
def test_wgrad_bf16(shape, path):
    L = pkg_mod("_lib")
    n, h, cin, cout, s, tr = shape
    g = torch.Generator().manual_seed(hash(shape) % 1000 + 7)
    ho = h * s if tr else h // s
    x = torch.randn(n, h, h, cin, generator=g)
    dy = torch.randn(n, ho, ho, cout, generator=g)
    wshape = (4, 4, cout, cin) if tr else (4, 4, cin, cout)
    dw = torch.full(wshape, float("nan"), device="cuda")
    scratch = torch.empty(32 << 20, device="cuda")
    xd, dyd = x.cuda(), dy.cuda()  # keep the device copies alive until the kernels ran
    rc = L.lib().svae_op_wgrad_bf16(L.ptr(xd), n, h, cin, L.ptr(dyd), cout, s, tr, path, L.ptr(dw),
                                    L.ptr(scratch), scratch.numel() * 4, L.stream_ptr())
    L.check(rc)
    torch.cuda.synchronize()
    xr = _bf(x).double().permute(0, 3, 1, 2)
    dyr = _bf(dy).double().permute(0, 3, 1, 2)
    w = torch.zeros(wshape, dtype=torch.float64, requires_grad=True)
    y = torch_twin.conv2d_t_same(xr, w, s) if tr else torch_twin.conv2d_same(xr, w, s)
    ref, = torch.autograd.grad(y, w, dyr)
    out = dw.cpu().double()
    assert torch.isfinite(out).all()
    rel = float((out - ref).norm() / ref.norm())
    mx = float((out - ref).abs().max() / ref.abs().max())
    assert rel <= 2e-5 and mx <= 1e-4, (rel, mx)


# image-space stride-2 convs with Cin <= 3 (the first conv of every recognition ladder / encoder):
# wgrad_smallc.hip, taken when dY is stored as bf16 (path bit 5), as the engine stores dpre
@pytest.mark.parametrize("shape", [(4, 64, 3, 32, 2, 0), (2, 64, 1, 32, 2, 0), (2, 64, 2, 64, 2, 0)],
                         ids=lambda s: "n%d_h%d_%dto%d" % (s[0], s[1], s[2], s[3]))
def test_wgrad_smallc(shape):
    L = pkg_mod("_lib")
    n, h, cin, cout, s, tr = shape
    g = torch.Generator().manual_seed(11 + cin)
    ho = h // s
    x = torch.randn(n, h, h, cin, generator=g)
    dy = torch.randn(n, ho, ho, cout, generator=g)
    dw = torch.full((4, 4, cin, cout), float("nan"), device="cuda")
    scratch = torch.empty(32 << 20, device="cuda")
    xd, dyd = x.cuda(), dy.to(torch.bfloat16).cuda()
    rc = L.lib().svae_op_wgrad_bf16(L.ptr(xd), n, h, cin, L.ptr(dyd), cout, s, tr, 2 | 32, L.ptr(dw),
                                    L.ptr(scratch), scratch.numel() * 4, L.stream_ptr())
    L.check(rc)
    torch.cuda.synchronize()
    xr = _bf(x).double().permute(0, 3, 1, 2)
    dyr = _bf(dy).double().permute(0, 3, 1, 2)
    w = torch.zeros((4, 4, cin, cout), dtype=torch.float64, requires_grad=True)
    ref, = torch.autograd.grad(torch_twin.conv2d_same(xr, w, s), w, dyr)
    out = dw.cpu().double()
    assert torch.isfinite(out).all()
    rel = float((out - ref).norm() / ref.norm())
    mx = float((out - ref).abs().max() / ref.abs().max())
    print("wgrad_smallc %s: rel L2 %.2e, max %.2e" % (shape, rel, mx))
    assert rel <= 2e-5 and mx <= 1e-4, (rel, mx)
