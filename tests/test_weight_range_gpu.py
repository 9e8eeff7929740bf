"""The split mode (bf16x6) with weights far outside their initial range.

The gathers' fp16 weight planes hold w * 2^e with a per-tensor exponent e (csrc/common.h h16_pair,
h16_wexp): a full shadow refresh (svae_bind, a checkpoint load) derives e from each tensor's max |w|,
and an Adam update (sequential_vae.py:1267-1276 moves weights without bound) that takes a weight past
2^15 in its tensor's units raises a device flag, on which the next forward re-derives every exponent
and re-makes the planes before any GEMM reads them (wexp_fixup).  Round 5's fixed 2^10 turned any
|w| >= 64 into an infinite plane and the step into NaN.

Both tests hold the bf16x6 engine to exactly the fp32 bounds of test_engine_gpu.py's CelebA-geometry
test against the float64 oracle (loss / per-step terms 1e-4, x_hat_t <= max(1e-4, 4 x the fp32 twin),
gradients by _check_grads), at B = 4, T = 2, so every split kernel runs: the wave-split gathers
(halo_x3), the 4x4-input conv-T fallback (halo_kw), the FC GEMMs (dense_kw) and the T-batched
recognition layers (a per-group exponent).
"""
import numpy as np
import pytest
import torch

from oracle import spec, torch_twin
from test_engine_gpu import _check_grads, _engine, _oracle_run, _rel

pytestmark = pytest.mark.gpu

# tensor -> factor; |w| of a N(0, 0.02) tensor reaches ~0.09, so x5000 and x1e4 put weights near 450 / 900
SCALES = {
    "theta/generative_step_1/Conv2d_transpose_1/weights": 300.0,   # decoder s1 conv-T at 8x8 (halo_x3)
    "theta/generative_encoder_step_1/Conv_3/weights": 1e-5,        # encoder conv at 16x16 (halo_x3)
    "theta/generative_step_1/fully_connected_4/weights": 5000.0,   # the top FC (dense_kw)
    "phi/inference_step_1/Conv_5/weights": 3000.0,                 # T-batched recognition, group 1 (halo_x3)
    "theta/generative_step_0/Conv2d_transpose/weights": 1e4,       # 4x4-input stride-2 conv-T (halo_kw)
}


def _check_against_oracle(net, cd, x, tgt, eps, reg=1.0):
    net.forward(x, tgt, eps, reg)
    net.backward()
    torch.cuda.synchronize()
    params = net.param_dict()
    o = _oracle_run(net, cd, x, tgt, eps, reg)
    _, struct = spec.build_params(cd)
    p32 = torch_twin.Twin(cd, struct, params, dtype=torch.float32).step(x, tgt, eps, reg)
    loss = net.loss_value(reg_coeff=reg)
    assert np.isfinite(loss)
    assert abs(loss - o["loss"]) <= 1e-4 * abs(o["loss"]), (loss, o["loss"])
    stats = net.step_stats().cpu().numpy()
    for t in range(cd["mc_steps"]):
        assert abs(stats[t, 0] - o["recon"][t]) <= 1e-4 * abs(o["recon"][t])
        assert abs(stats[t, 1] - o["kl"][t]) <= 1e-4 * abs(o["kl"][t])
        e_hip = _rel(net.xhat(t).cpu().numpy(), o["xhat"][t])
        e_32 = _rel(p32["xhat"][t], o["xhat"][t])
        print("x_hat_%d rel %.2e (fp32 twin %.2e)" % (t, e_hip, e_32))
        assert e_hip <= max(1e-4, 4 * e_32), (t, e_hip, e_32)
    g = net.grad_dict()
    assert all(np.isfinite(v).all() for v in g.values())
    _check_grads(g, o["grads"], p32["grads"], median_tol=1e-3)
    return o


def test_bound_weights_far_from_init():
    """Caller-bound weights x300 / x1e-5 / x3000 / x5000 / x1e4 (svae_bind): fp32-grade, finite."""
    net, _ = _engine("celeba", 4, mc_steps=2, dtype="bf16x6")
    cd = spec.make_config("celeba", batch=4, mc_steps=2)
    x, tgt, eps = spec.make_inputs(cd, batch=4)
    for name, f in SCALES.items():
        w = net.param(name).cpu().numpy()
        net.set_param(name, (w * f).astype(np.float32))
        assert np.abs(net.param(name).cpu().numpy()).max() > 0
    big = np.abs(net.param("theta/generative_step_0/Conv2d_transpose/weights").cpu().numpy()).max()
    assert big > 64.0  # past the former fixed scale's fp16 range
    _check_against_oracle(net, cd, x, tgt, eps)


def test_adam_update_past_the_planes_range():
    """An Adam update that moves each weight of four BN-followed GEMM tensors by ~lr = 5 (step 1:
    lr_t * m / sqrt(v) = lr * sign(g), svae_adam_range) takes them ~50x past their maxima, beyond the fp16
    planes' headroom at the exponents the update wrote them with: the next forward re-makes the planes
    (wexp_fixup) and the step stays fp32-grade; then a second forward with no update in between."""
    net, _ = _engine("celeba", 4, mc_steps=2, dtype="bf16x6")
    cd = spec.make_config("celeba", batch=4, mc_steps=2)
    x, tgt, eps = spec.make_inputs(cd, batch=4)
    names = ["theta/generative_step_1/Conv2d_transpose_1/weights", "theta/generative_step_1/fully_connected_4/weights",
             "phi/inference_step_1/Conv_5/weights", "theta/generative_step_0/Conv2d_transpose/weights"]
    before = {n: np.abs(net.param(n).cpu().numpy()).max() for n in names}
    net.forward(x, tgt, eps, 1.0)
    net.backward()
    for n in names:
        p = net._by_name[n]
        _lib = net.L
        rc = _lib.svae_adam_range(net.ctx, p["offset"], p["offset"] + p["size"], 5.0, 1, 10.0,
                                  torch.cuda.current_stream().cuda_stream)
        assert rc == 0
    torch.cuda.synchronize()
    for n in names:
        after = np.abs(net.param(n).cpu().numpy()).max()
        assert after > 30 * before[n], (n, before[n], after)
    _check_against_oracle(net, cd, x, tgt, eps[:, ::-1].copy())
    _check_against_oracle(net, cd, x, tgt, eps)
