"""Backward with the optimizer step folded in (svae_backward_adam / SequentialVAE.backward_apply).

Each chain step's generator/encoder bucket gets its clip + Adam update (and, in bf16 mode, its
bf16 weight copies) on the engine's side stream as soon as the backward has finished it; the
recognition bucket follows the whole backward.  Adam is elementwise, so after several steps the
parameters must equal, bit for bit, those of svae_backward + svae_adam.  In bf16 mode the next
forward reuses the refreshed weight copies instead of rebuilding them, so equal losses on later
steps also check that every copy was refreshed."""
import numpy as np
import pytest
import torch

from conftest import pkg_mod

pytestmark = pytest.mark.gpu


def _run(preset, dtype, fused, over, steps=3, batch=4):
    cfgmod, SV = pkg_mod("config"), pkg_mod("sequential_vae").SequentialVAE
    cfg = cfgmod.preset(preset, batch=batch, dtype=dtype, **over)
    net = SV(cfg, seed=0)
    p0 = net.params.clone()
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    x = torch.rand(cfg.batch, cfg.height, cfg.width, cfg.channels, device="cuda", generator=g) * 2 - 1
    losses = []
    for it in range(1, steps + 1):
        eps = torch.randn(cfg.mc_steps, cfg.batch, cfg.latent_dim, device="cuda", generator=g)
        net.forward(x, x, eps, 0.5)
        if fused:
            net.backward_apply(1e-3, it)
        else:
            net.backward()
            net.apply_gradients(1e-3, it)
        losses.append(net.loss_value())
    torch.cuda.synchronize()
    changed = float((net.params - p0).abs().max())
    p = net.params.cpu().numpy().copy()
    net.close()
    return p, losses, changed


@pytest.mark.parametrize("preset,dtype,over", [
    ("tiny", "fp32", {}),
    ("tiny", "bf16", {}),
    ("tiny", "bf16", {"predict_latent_code": True}),
    ("tiny_homog", "bf16", {}),
    ("celeba", "bf16", {}),
])
def test_backward_apply_equals_backward_then_adam(preset, dtype, over):
    p0, l0, _ = _run(preset, dtype, False, over)
    p1, l1, changed = _run(preset, dtype, True, over)
    assert changed > 0
    assert np.isfinite(p1).all()
    assert l0 == l1, (l0, l1)
    np.testing.assert_array_equal(p0, p1)


def test_rebind_after_external_write_rebuilds_weight_copies():
    """Parameters written by the caller after an update are announced with svae_bind; the next
    forward then rebuilds the bf16 copies (same loss as a fresh network on those parameters)."""
    cfgmod, SV = pkg_mod("config"), pkg_mod("sequential_vae").SequentialVAE
    L = pkg_mod("_lib")
    cfg = cfgmod.preset("tiny", batch=4, dtype="bf16")
    a, b = SV(cfg, seed=0), SV(cfg, seed=5)
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    x = torch.rand(cfg.batch, cfg.height, cfg.width, cfg.channels, device="cuda", generator=g) * 2 - 1
    eps = torch.randn(cfg.mc_steps, cfg.batch, cfg.latent_dim, device="cuda", generator=g)
    a.forward(x, x, eps, 1.0)
    a.backward_apply(1e-3, 1)
    a.params.copy_(b.params)
    a.params_updated()
    a.forward(x, x, eps, 1.0)
    b.forward(x, x, eps, 1.0)
    torch.cuda.synchronize()
    assert a.loss_value() == b.loss_value()
    a.close()
    b.close()


@pytest.mark.parametrize("preset,dtype,over", [
    ("tiny", "bf16", {}),
    ("celeba", "bf16", {}),
    ("tiny", "bf16x6", {}),
    ("tiny_homog", "bf16", {}),
])
@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("rec_group", ["0", "1"])
def test_batched_side_handover_is_bitwise(preset, dtype, over, fused, rec_group, monkeypatch, knob_lib):
    """SVAE_SIDE_BATCH = k queues the weight-gradient work of k layers behind one main-stream
    event (engine.cpp on_side_q / side_flush): the same kernels on the same data, so losses and
    parameters after three steps equal the per-layer hand-over bit for bit (the per-bucket Adam
    of the fused path must still follow every weight gradient of its bucket).  With
    SVAE_REC_GROUP=1 the recognition backward of each step runs on a fourth stream and queues its
    weight gradients there: the queue must be flushed behind an event on THAT stream (ADVICE r03:
    flushed later from the main stream, the weight-GEMMs could read dpre st4 had not written)."""
    monkeypatch.setenv("SVAE_REC_GROUP", rec_group)
    monkeypatch.setenv("SVAE_SIDE_BATCH", "1")
    p0, l0, _ = _run(preset, dtype, fused, over)
    for k in ("3", "100"):
        monkeypatch.setenv("SVAE_SIDE_BATCH", k)
        p1, l1, changed = _run(preset, dtype, fused, over)
        assert changed > 0
        assert l0 == l1, (k, l0, l1)
        np.testing.assert_array_equal(p0, p1)


def _fwd_bwd(preset, dtype, over):
    cfgmod, SV = pkg_mod("config"), pkg_mod("sequential_vae").SequentialVAE
    cfg = cfgmod.preset(preset, batch=4, dtype=dtype, **over)
    net = SV(cfg, seed=0)
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    x = torch.rand(cfg.batch, cfg.height, cfg.width, cfg.channels, device="cuda", generator=g) * 2 - 1
    eps = torch.randn(cfg.mc_steps, cfg.batch, cfg.latent_dim, device="cuda", generator=g)
    net.forward(x, x, eps, 0.5)
    net.backward()
    torch.cuda.synchronize()
    loss, gr = net.loss_value(), net.grads.cpu().numpy().copy()
    net.close()
    return loss, gr


@pytest.mark.parametrize("preset,dtype,over", [
    ("tiny", "bf16", {}),
    ("tiny", "fp32", {}),
    ("tiny_homog", "bf16", {}),
])
@pytest.mark.parametrize("knob", ["SVAE_REC_SPLIT", "SVAE_REC_GROUP"])
def test_forward_recognition_split_matches(preset, dtype, over, knob, monkeypatch, knob_lib):
    """SVAE_REC_SPLIT=1 runs step 0's recognition ladder on the main stream and the batched ladders of
    steps 1..T-1 on a fourth stream beside the chain's step 0 (engine.cpp engine_forward).  The same
    per-step kernels run on the same data; only launch shapes that depend on the group count
    (split-K / tile choices of step 0's launches) may change a summation order, so the loss and the
    gradient of one step agree to fp32 rounding (reported when bitwise).  (Compared before any Adam
    step: Adam's first update is sign(g) * lr, which turns a rounding-level difference of a near-zero
    gradient into a full step.)  SVAE_REC_GROUP=1 is the backward counterpart: the recognition
    backward of each step on the fourth stream as soon as its dz is final.  Both read the bf16
    recognition activations at a step offset, which must count bf16 elements (engine.cpp elem_off:
    with float* arithmetic these gave steps >= 1 wrong conv weight gradients, 100-140 % off)."""
    monkeypatch.delenv("SVAE_REC_SPLIT", raising=False)
    monkeypatch.delenv("SVAE_REC_GROUP", raising=False)
    l0, g0 = _fwd_bwd(preset, dtype, over)
    monkeypatch.setenv(knob, "1")
    l1, g1 = _fwd_bwd(preset, dtype, over)
    gvec = float(np.linalg.norm(g1 - g0) / np.linalg.norm(g0))
    print("rec split %s %s/%s: bitwise %s, loss rel %.2e, gradient vector rel %.2e" % (
        knob, preset, dtype, l0 == l1 and np.array_equal(g0, g1), abs(l0 - l1) / abs(l0), gvec))
    # these geometries launch the same kernel shapes either way: bitwise.  (At the CelebA geometry a
    # one-group launch of step 0 may take a split-K form the batched one does not, and the chaotic
    # B=4 chain amplifies that rounding; there the knobs run the engine parity suite instead,
    # tools/gpu/r03_headsab.sh.)
    assert l0 == l1 and np.array_equal(g0, g1), (l0, l1, gvec)


@pytest.mark.parametrize("preset", ["tiny", "celeba"])
def test_fc_bn_backward_fusion_is_bitwise(preset, monkeypatch, knob_lib):
    """bf16 default: E.fc's BN-backward sums are formed in the top FC's split-K input gradient
    (engine.cpp fc_bn_bwd, splitk_reduce BwStat columns) instead of a bn_bwd_reduce pass.  The sums
    are fixed-point accumulated (order-free), so three training steps must equal the unfused path
    (SVAE_BWFUSE_FC=0) bit for bit."""
    monkeypatch.setenv("SVAE_BWFUSE_FC", "0")
    p0, l0, _ = _run(preset, "bf16", True, {})
    monkeypatch.setenv("SVAE_BWFUSE_FC", "1")
    p1, l1, changed = _run(preset, "bf16", True, {})
    assert changed > 0
    assert l0 == l1, (l0, l1)
    np.testing.assert_array_equal(p0, p1)


@pytest.mark.parametrize("preset,dtype", [("tiny", "bf16"), ("celeba", "bf16"), ("tiny", "bf16x6"), ("celeba", "bf16x6"),
                                          ("tiny_homog", "bf16")])
@pytest.mark.parametrize("fused", [False, True])
def test_second_side_stream_is_bitwise(preset, dtype, fused, monkeypatch, knob_lib):
    """SVAE_SIDE2=1 alternates the conv weight-GEMMs between two side streams (own split slab each;
    engine.cpp side_merge orders the per-bucket Adam, the DP hook and the final join after both):
    the same kernels on the same data, so three training steps equal the one-stream run bit for bit."""
    monkeypatch.setenv("SVAE_SIDE2", "0")
    p0, l0, _ = _run(preset, dtype, fused, {})
    monkeypatch.setenv("SVAE_SIDE2", "1")
    p1, l1, changed = _run(preset, dtype, fused, {})
    assert changed > 0
    assert l0 == l1, (l0, l1)
    np.testing.assert_array_equal(p0, p1)


@pytest.mark.parametrize("preset,dtype,over", [
    ("tiny", "bf16", {}), ("celeba", "bf16", {}),
    ("tiny_homog", "bf16", {}), ("tiny", "bf16", {"predict_latent_code": True}),
])
@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("pre_f32", ["0", "1"])
def test_forward_bn_fold_is_bitwise(preset, dtype, over, fused, pre_f32, monkeypatch, knob_lib):
    """(Knob-only, measured slower: DESIGN §9.)  SVAE_FOLD=1: the forward BN apply of the recognition / encoder conv-a and decoder s1 (level >= 1)
    outputs runs on the side stream, and the next layer's wave-split gather stages act(bn_y(pre)) from
    the pre-BN tensor itself with the statistics finalised as bn_apply does (engine.cpp
    conv_bn_act_fwd, halo_kw.hip ain): the same values, so three training steps are bitwise the
    unfolded run's.  In bf16 mode the pre-BN tensor is stored bf16 (widened, applied and rounded back
    while staging) or fp32 (SVAE_PRE_F32=1).  Not in the split mode (engine.cpp ain_ok): its gathers
    scale the staged window by a maximum taken before the consumer-side BN would apply."""
    if pre_f32 == "1" and dtype != "bf16":
        pytest.skip("fp32 / split modes store pre-BN tensors in fp32 either way")
    monkeypatch.setenv("SVAE_X3", "0")  # the fold runs on halo_kw: compare halo_kw with halo_kw
    monkeypatch.setenv("SVAE_PRE_F32", pre_f32)
    monkeypatch.setenv("SVAE_FOLD", "0")
    p0, l0, _ = _run(preset, dtype, fused, over)
    monkeypatch.setenv("SVAE_FOLD", "1")
    p1, l1, changed = _run(preset, dtype, fused, over)
    assert changed > 0
    assert l0 == l1, (l0, l1)
    np.testing.assert_array_equal(p0, p1)


@pytest.mark.parametrize("preset,dtype,batch", [
    ("tiny", "bf16", 4), ("celeba", "bf16", 128), ("celeba", "bf16x6", 128), ("tiny_homog", "bf16", 4),
])
@pytest.mark.parametrize("fused", [False, True])
def test_bn_last_arriver_finalisation_is_bitwise(preset, dtype, batch, fused, monkeypatch, knob_lib):
    """(Knob-only, measured slower: DESIGN §9.)  SVAE_BN_LAF: the last block of each halo_kw BN producer turns the fixed-point accumulators into
    mean / invstd (forward) or the backward sums a, b and dbeta (common.h bn_fin_arrive) with the apply
    passes' own expressions, ordered by device-scope atomics alone.  Three training steps at the headline
    batch (thousands of producer blocks on every XCD) are bitwise the per-block finalisation's: a block
    whose statistics the last arriver missed would move mean / invstd."""
    monkeypatch.setenv("SVAE_X3", "0")  # the finalisation runs on halo_kw: compare halo_kw with halo_kw
    monkeypatch.setenv("SVAE_BN_LAF", "0")
    p0, l0, _ = _run(preset, dtype, fused, {}, batch=batch)
    monkeypatch.setenv("SVAE_BN_LAF", "3")
    p1, l1, changed = _run(preset, dtype, fused, {}, batch=batch)
    assert changed > 0
    assert l0 == l1, (l0, l1)
    np.testing.assert_array_equal(p0, p1)


@pytest.mark.parametrize("preset,dtype,batch", [
    ("tiny", "fp32", 4), ("tiny", "bf16", 4), ("celeba", "bf16", 128), ("celeba", "bf16x6", 128),
    ("tiny_homog", "bf16x6", 4),
])
@pytest.mark.parametrize("fused", [False, True])
def test_bn_finalise_once_is_bitwise(preset, dtype, batch, fused, monkeypatch, knob_lib):
    """SVAE_BN_FIN: each conv BN layer's statistics (forward mean / invstd, backward a, b, dbeta) finalised by
    one small launch (bn.hip bn_fin_kernel) instead of by every apply block from the accumulator shards --
    the same fp64 expressions over the same integer sums, so three training steps are bitwise equal."""
    monkeypatch.setenv("SVAE_BN_FIN", "0")
    p0, l0, _ = _run(preset, dtype, fused, {}, batch=batch)
    monkeypatch.setenv("SVAE_BN_FIN", "1")
    p1, l1, changed = _run(preset, dtype, fused, {}, batch=batch)
    assert changed > 0
    assert l0 == l1, (l0, l1)
    np.testing.assert_array_equal(p0, p1)


@pytest.mark.parametrize("preset,dtype,batch,over", [
    ("tiny", "bf16", 4, {}), ("celeba", "bf16", 128, {}), ("tiny_homog", "bf16", 4, {}),
    ("tiny", "bf16", 4, {"predict_latent_code": True}),
])
@pytest.mark.parametrize("fused", [False, True])
def test_bf16_concat_storage_is_bitwise(preset, dtype, batch, over, fused, monkeypatch, knob_lib):
    """bf16 mode stores the decoder concat buffers [s2 output | split latent] as bf16 (engine.cpp cbf):
    their readers round them to bf16 anyway (the s1 gather and weight-GEMM) or use only the sign of the
    s2 output (act' in its BN backward), so three training steps are bitwise the fp32-stored ones
    (SVAE_CAT_F32=1)."""
    monkeypatch.setenv("SVAE_CAT_F32", "1")
    p0, l0, _ = _run(preset, dtype, fused, over, batch=batch)
    monkeypatch.setenv("SVAE_CAT_F32", "0")
    p1, l1, changed = _run(preset, dtype, fused, over, batch=batch)
    assert changed > 0
    assert l0 == l1, (l0, l1)
    np.testing.assert_array_equal(p0, p1)
