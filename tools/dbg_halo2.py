"""Per-layer check of the inference ladder convs inside the bf16 step: recompute each conv
(pre-BN output) in float64 from the stored bf16-rounded input activation and weights."""
import importlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
cfgmod = importlib.import_module("sequential-variational-autoencoder_amd.config")
SV = importlib.import_module("sequential-variational-autoencoder_amd.sequential_vae").SequentialVAE
from oracle import spec, torch_twin  # noqa: E402

B = 8
cfg = cfgmod.preset("celeba", batch=B, mc_steps=1, dtype="bf16")
net = SV(cfg, seed=0)
cd = spec.make_config("celeba", batch=B, mc_steps=1)
x, tgt, eps = spec.make_inputs(cd, batch=B)
net.forward(x, tgt, eps, 1.0)
torch.cuda.synchronize()
P = net.param_dict()
F, S = cfg.filter_sizes, cfg.image_sizes
bf = lambda a: torch.as_tensor(a).to(torch.bfloat16).double()
prev = torch.as_tensor(x).double()
for lvl in range(3):
    n_out = B * S[lvl + 1] ** 2 * F[lvl + 1]
    pre_a = net.copy_out(113, lvl, n_out).cpu().double().view(B, S[lvl + 1], S[lvl + 1], F[lvl + 1])
    act_a = net.copy_out(114, lvl, n_out).cpu().double().view(B, S[lvl + 1], S[lvl + 1], F[lvl + 1])
    pre_b = net.copy_out(115, lvl, n_out).cpu().double().view(B, S[lvl + 1], S[lvl + 1], F[lvl + 1])
    act_b = net.copy_out(116, lvl, n_out).cpu().double().view(B, S[lvl + 1], S[lvl + 1], F[lvl + 1])
    wa = P["phi/inference_step_0/%s/weights" % ("Conv" if lvl == 0 else "Conv_%d" % (2 * lvl))]
    wb = P["phi/inference_step_0/Conv_%d/weights" % (2 * lvl + 1)]
    ra = torch_twin.conv2d_same(bf(prev).permute(0, 3, 1, 2), bf(wa), 2).permute(0, 2, 3, 1)
    rb = torch_twin.conv2d_same(bf(act_a).permute(0, 3, 1, 2), bf(wb), 1).permute(0, 2, 3, 1)
    ea = float((pre_a - ra).norm() / ra.norm())
    eb = float((pre_b - rb).norm() / rb.norm())
    wa_b = float(((pre_a - ra).abs()).amax(dim=(0, 3)).max() / ra.abs().max())
    wb_b = float(((pre_b - rb).abs()).amax(dim=(0, 3)).max() / rb.abs().max())
    print("level %d: conv a rel %.2e (max %.2e) | conv b rel %.2e (max %.2e)" % (lvl, ea, wa_b, eb, wb_b))
    if eb > 1e-4:
        d = (pre_b - rb).abs().amax(dim=(0, 3))
        print("   conv b max-err map over (y,x):")
        print(np.array2string(d.numpy() / float(rb.abs().max()), precision=1, max_line_width=250))
    if ea > 1e-4:
        d = (pre_a - ra).abs().amax(dim=(0, 3))
        print("   conv a max-err map over (y,x):")
        print(np.array2string(d.numpy() / float(ra.abs().max()), precision=1, max_line_width=250))
    prev = act_b
