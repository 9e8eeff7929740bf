"""bf16 gather-GEMM kernels checked in situ, inside the real bf16 training step.

For every inference-ladder conv of every chain step (the T steps run as one batched launch
per layer, grid.z = step), the stored pre-BatchNorm output is recomputed in float64 from the
stored bf16-rounded input activation and weights.  The kernels round exactly those operands
and accumulate in fp32, so the bound is accumulation-order only: 1e-6 relative (L2) and
1e-5 of max|ref| pointwise -- or, with the pre-BN output itself stored as bf16 (the default), within
half a bf16 ulp of the reference and equal to its bf16 rounding at all but <= 0.1 % of the elements.  At the CelebA geometry these launches run on the halo-tile
kernel (igemm_halo_kernel) except level-0 conv a (Cin = 3: conv_smallc_kernel, csrc/smallc.hip).

Why not compare halo against the per-tap kernel through the whole step: in bf16 mode a
1e-7 summation-order difference flips the bf16 rounding of a few downstream operands
(3.9e-3 each), which flips more in the next layer; within 2-3 layers any perturbation sits
at the bf16 noise floor (~1e-3 on activations), so step-level A/B differences say nothing
about kernel correctness.  tests/test_gather_bf16_gpu.py checks both kernels per op."""
import os

import numpy as np
import pytest
import torch

from conftest import pkg_mod
from oracle import spec, torch_twin

pytestmark = pytest.mark.gpu
# bf16 mode stores the conv layers' pre-BN outputs as bf16; SVAE_PRE_F32=1 keeps fp32
PRE_BF16 = os.environ.get("SVAE_PRE_F32", "0") != "1"


def _bf(a):
    return torch.as_tensor(a).to(torch.bfloat16).double()


def test_inference_convs_in_situ():
    B, T = 8, 2
    cfg = pkg_mod("config").preset("celeba", batch=B, mc_steps=T, dtype="bf16")
    net = pkg_mod("sequential_vae").SequentialVAE(cfg, seed=0)
    cd = spec.make_config("celeba", batch=B, mc_steps=T)
    x, tgt, eps = spec.make_inputs(cd, batch=B)
    net.forward(x, tgt, eps, 1.0)
    torch.cuda.synchronize()
    P = net.param_dict()
    F, S = cfg.filter_sizes, cfg.image_sizes
    prev = [torch.as_tensor(x).double()] * T
    worst = 0.0
    for lvl in range(cfg.levels - 1):
        shp = (T, B, S[lvl + 1], S[lvl + 1], F[lvl + 1])
        n = int(np.prod(shp))
        get = lambda code: net.copy_out(code, lvl, n).cpu().double().view(*shp)
        pre_a, act_a, pre_b, act_b = get(113), get(114), get(115), get(116)
        for t in range(T):
            wa = P["phi/inference_step_%d/%s/weights" % (t, "Conv" if lvl == 0 else "Conv_%d" % (2 * lvl))]
            wb = P["phi/inference_step_%d/Conv_%d/weights" % (t, 2 * lvl + 1)]
            for got, inp, w, s in ((pre_a[t], prev[t], wa, 2), (pre_b[t], act_a[t], wb, 1)):
                ref = torch_twin.conv2d_same(_bf(inp).permute(0, 3, 1, 2), _bf(w), s).permute(0, 2, 3, 1)
                if PRE_BF16:  # stored RNE-rounded: within half a bf16 ulp of the fp32 sum, equal to bf16(ref) but
                    # where the fp32 sum and the fp64 one straddle a rounding midpoint
                    err = (got - ref).abs()
                    assert bool((err <= 2.0 ** -8 * ref.abs() + 1e-5 * ref.abs().max()).all()), (lvl, t, s)
                    flips = float((got != _bf(ref)).double().mean())
                    assert flips <= 1e-3, (lvl, t, s, flips)
                    worst = max(worst, flips)
                    continue
                rel = float((got - ref).norm() / ref.norm())
                mx = float((got - ref).abs().max() / ref.abs().max())
                worst = max(worst, rel)
                assert rel <= 1e-6 and mx <= 1e-5, (lvl, t, s, rel, mx)
        prev = [act_b[t] for t in range(T)]
    print(("worst bf16 rounding-flip fraction %.2e" if PRE_BF16 else "worst rel %.2e") % worst)
