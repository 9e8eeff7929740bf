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


def test_heads_row_groups_match(monkeypatch, knob_lib):
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


def _lsun(monkeypatch, tile):
    monkeypatch.setenv("SVAE_HEADS_TILE", tile)
    cfg = pkg_mod("config").preset("lsun", dtype="fp32", mc_steps=1)
    net = pkg_mod("sequential_vae").SequentialVAE(cfg, seed=0)
    g = torch.Generator(device="cuda")
    g.manual_seed(9)
    x = torch.rand(cfg.batch, cfg.height, cfg.width, cfg.channels, device="cuda", generator=g) * 2 - 1
    eps = torch.randn(cfg.mc_steps, cfg.batch, cfg.latent_dim, device="cuda", generator=g)
    net.forward(x, x, eps, 1.0)
    lib = pkg_mod("_lib")
    mus = [net.latent(w, t).double().cpu() for t in range(cfg.mc_steps) for w in (lib.BUF_MU, lib.BUF_SIGMA)]
    net.backward()
    torch.cuda.synchronize()
    out = {k: v.copy() for k, v in net.grad_dict().items()}
    net.close()
    return mus, out


def test_wide_heads_tiles_match(monkeypatch, knob_lib):
    """LSUN (B = 256, 20-30 latents per level), one chain step, fp32: the tiled wide-heads forward
    (misc.hip heads_tile_fwd_kernel) against the skinny forward (SVAE_HEADS_TILE=2 vs 3): latent means /
    stddevs within 1e-5; the tiled backward (heads_tile_bwd_kernel) against the one-k-per-thread kernel
    with the same forward (SVAE_HEADS_TILE=1 vs 3, so no ReLU kink can flip between the runs): every
    gradient tensor within 1e-5 (L2) -- only the heads' summation order differs."""
    m_old, _ = _lsun(monkeypatch, "2")
    m_fb, g_old_bwd = _lsun(monkeypatch, "1")
    m_new, g_new = _lsun(monkeypatch, "3")
    worst_mu = max(float((a - b).norm() / a.norm()) for a, b in zip(m_old, m_new))
    assert worst_mu <= 1e-5, worst_mu
    assert all(bool((a == b).all()) for a, b in zip(m_fb, m_new))  # same forward kernel: bitwise
    worst, wk = 0.0, None
    for k, a in g_old_bwd.items():
        b = g_new[k]
        na = float(np.linalg.norm(a))
        if na == 0.0:
            assert float(np.abs(b).max()) == 0.0, k
            continue
        r = float(np.linalg.norm(a - b)) / na
        if r > worst:
            worst, wk = r, k
    assert worst <= 1e-5, (worst, wk)
    print("\nwide heads tiles: mu rel %.2e, worst gradient tensor rel %.2e (%s)" % (worst_mu, worst, wk))
