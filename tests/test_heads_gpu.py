"""Recognition-heads backward with the batch rows split over thread groups (misc.hip heads_bwd_rg_kernel,
the default at B % 32 == 0) against the one-k-per-thread kernel (SVAE_HEADS_RG=0), inside the CelebA
B=128 training step: the input gradient of the heads is computed in the same order per row (the whole
step's gradient but the heads' own weights is bitwise equal); the heads' weight gradients sum the 128
rows in four row groups (fp32 re-association only)."""
import numpy as np
import pytest
import torch

from conftest import pkg_mod

pytestmark = pytest.mark.gpu


def _grads(monkeypatch, rg):
    monkeypatch.setenv("SVAE_HEADS_RG", rg)
    cfg = pkg_mod("config").preset("celeba", batch=128, dtype="bf16")
    net = pkg_mod("sequential_vae").SequentialVAE(cfg, seed=0)
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    x = torch.rand(cfg.batch, cfg.height, cfg.width, cfg.channels, device="cuda", generator=g) * 2 - 1
    eps = torch.randn(cfg.mc_steps, cfg.batch, cfg.latent_dim, device="cuda", generator=g)
    net.forward(x, x, eps, 1.0)
    net.backward()
    torch.cuda.synchronize()
    out = {k: v.copy() for k, v in net.grad_dict().items()}
    net.close()
    return out


def test_heads_row_groups_match(monkeypatch):
    g0 = _grads(monkeypatch, "0")
    g1 = _grads(monkeypatch, "1")
    differing = []
    for k, a in g0.items():
        b = g1[k]
        if np.array_equal(a, b):
            continue
        differing.append(k)
        rel = float(np.abs(a - b).max() / max(np.abs(a).max(), 1e-30))
        assert rel <= 1e-5, (k, rel)
    # only the heads' weights (mean / stddev per ladder level and step) may differ
    assert all(k.startswith("phi/") for k in differing), differing
    assert len(differing) <= 2 * 4 * 8, differing
    print("\n%d of %d gradient tensors re-associated (heads weights), all within 1e-5" % (len(differing), len(g0)))
