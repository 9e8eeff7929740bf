"""bf16 gather-GEMM kernels (csrc/gemm_bf16.hip) through svae_op_gather_bf16, on every
conv / conv-T layer shape of the CelebA geometry (forward shapes; the input-gradient
launches are the same two gather modes).  Reference: float64 torch conv of the SAME
bf16-rounded operands (oracle/torch_twin.py TF-SAME helpers), so the only difference left
is fp32 accumulation order: bound 2e-5 relative (L2) and 1e-4 of max|ref| pointwise.
Every kernel is checked: path 0 (per-tap gather), path 1 (halo-tile window) and path 2 (the
default dispatch, which adds the small-channel window kernels of csrc/smallc.hip: Cin <= 4 convs and
N <= 16 stride-2 conv-T gathers)."""
import numpy as np
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
    # input-gradient launches: conv dgrad = conv-T gather, conv-T dgrad = conv gather
    (4, 16, 64, 32, 2, 1), (4, 8, 128, 256, 1, 0), (4, 32, 32, 64, 1, 0),
    # image-space layers: output conv-T (N = C+1 = 4) and layer-0 input gradient (N = 3)
    (4, 32, 32, 4, 2, 1), (4, 32, 32, 3, 2, 1),
    # small-channel convs (csrc/smallc.hip on path 2): layer-0 conv of the image (Cin = 3) at the
    # CelebA / tiny geometries, 4 channels, N = 64 and 128 column tiles
    (4, 64, 3, 32, 2, 0), (2, 32, 3, 32, 2, 0), (2, 64, 4, 64, 2, 0), (2, 32, 1, 128, 2, 0),
    # small-N conv-T gathers (convt_smalln_kernel on path 2): 2 channel chunks, N = 16 / 1, Wi = 16 / 64
    (2, 16, 64, 16, 2, 1), (2, 32, 32, 1, 2, 1), (1, 64, 32, 4, 2, 1),
    # CelebA B=128 small-image layers: path 2 runs them on the wave-split kernel (csrc/halo_kw.hip)
    # with 64-row tiles instead of grid split-K
    (128, 8, 256, 128, 1, 1), (128, 4, 384, 128, 2, 1), (128, 8, 128, 128, 1, 0), (128, 8, 128, 64, 2, 1),
    # stride-2 convs at B = 128: halo_x3's 64-row tiles with 8 window items per thread
    (128, 32, 32, 64, 2, 0), (128, 16, 64, 128, 2, 0),
]




# shapes whose input window exceeds the halo kernel's LDS budget (csrc/gemm_bf16.hip halo_plan)
NOT_HALO = set()


def halo_eligible(shape):
    return shape[2] % 32 == 0 and shape not in NOT_HALO


def _bf(t):
    return t.to(torch.bfloat16).to(t.dtype)


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "n%d_h%d_%dto%d_s%d_%s" % (s[0], s[1], s[2], s[3], s[4],
                                                                                 "T" if s[5] else "C"))
@pytest.mark.parametrize("path", [0, 1, 2])
def test_gather_bf16(shape, path):
    L = pkg_mod("_lib")
    n, h, cin, cout, s, tr = shape
    g = torch.Generator().manual_seed(hash(shape) % 1000)
    x = torch.randn(n, h, h, cin, generator=g)
    w_tf = torch.randn(4, 4, cin, cout, generator=g) * 0.05 if not tr else torch.randn(4, 4, cout, cin, generator=g) * 0.05
    w_nk = (w_tf.permute(0, 1, 3, 2) if not tr else w_tf).reshape(16, cout, cin).contiguous()
    xd = x.cuda()
    wd = w_nk.to(torch.bfloat16).cuda()
    ho = h * s if tr else h // s
    y = torch.full((n, ho, ho, cout), float("nan"), device="cuda")
    scratch = torch.empty(8 << 20, device="cuda")
    rc = L.lib().svae_op_gather_bf16(L.ptr(xd), n, h, cin, L.ptr(wd), cout, s, tr, path, L.ptr(y), L.ptr(scratch),
                                     scratch.numel() * 4, L.stream_ptr())
    if path == 1 and not halo_eligible(shape):
        assert rc == -2  # SVAE_EBADARG: does not qualify
        return
    L.check(rc)
    torch.cuda.synchronize()
    xr = _bf(x).double().permute(0, 3, 1, 2)
    wr = _bf(w_tf).double()
    ref = (torch_twin.conv2d_t_same(xr, wr, s) if tr else torch_twin.conv2d_same(xr, wr, s)).permute(0, 2, 3, 1)
    out = y.cpu().double()
    assert torch.isfinite(out).all()
    rel = float((out - ref).norm() / ref.norm())
    mx = float((out - ref).abs().max() / ref.abs().max())
    assert rel <= 2e-5 and mx <= 1e-4, (rel, mx)
