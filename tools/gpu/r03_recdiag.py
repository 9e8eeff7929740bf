"""Diagnostic: per-tensor gradient differences of one fwd+bwd between two engine settings."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from tests.conftest import pkg_mod  # noqa: E402


def run(env, preset="tiny", dtype="bf16"):
    for k in ("SVAE_REC_SPLIT", "SVAE_REC_GROUP"):
        os.environ.pop(k, None)
    os.environ.update(env)
    cfgmod, SV = pkg_mod("config"), pkg_mod("sequential_vae").SequentialVAE
    cfg = cfgmod.preset(preset, batch=4, dtype=dtype)
    net = SV(cfg, seed=0)
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    x = torch.rand(cfg.batch, cfg.height, cfg.width, cfg.channels, device="cuda", generator=g) * 2 - 1
    eps = torch.randn(cfg.mc_steps, cfg.batch, cfg.latent_dim, device="cuda", generator=g)
    net.forward(x, x, eps, 0.5)
    net.backward()
    torch.cuda.synchronize()
    out = (net.loss_value(), net.grad_dict())
    net.close()
    return out


for preset, dtype in (("tiny", "bf16"), ("tiny", "fp32")):
    l0, g0 = run({}, preset, dtype)
    for env in ({"SVAE_REC_SPLIT": "1"}, {"SVAE_REC_GROUP": "1"}, {}):
        l1, g1 = run(env, preset, dtype)
        bad = [(k, float(np.linalg.norm(g1[k] - g0[k]) / (np.linalg.norm(g0[k]) + 1e-30))) for k in g0]
        bad = [b for b in bad if b[1] > 1e-5]
        print(preset, dtype, env, "loss", l0, l1, "tensors differing:", len(bad), "of", len(g0))
        for k, v in sorted(bad, key=lambda b: -b[1])[:12]:
            print("   %-60s %.3e" % (k, v))
