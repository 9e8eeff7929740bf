"""Parity at the headline configuration itself (BASELINE.json configs[1]: CelebA 64x64, B=128,
T=8), in both precision modes, on the same inputs and the same injected eps.

* fp32 engine: loss within 1e-4 of the float64 restatement (north_star), and the first two
  decoder outputs x_hat_0, x_hat_1 within 1e-4 (relative L2) before the chain's amplification
  sets in (tests/test_chaos.py: ~3-4x per step at this geometry).
* bf16 engine (the mode bench.py measures): loss within the documented bf16 bound of the fp32
  engine (2e-2) and within 3x (+ floor) of the error of the bf16-emulating CPU
  restatement (oracle/torch_twin.py emulate_bf16, the same operands rounded); x_hat_t within 3x
  (+ floor) of that twin's own error; the gradient vector and per-tensor median vs float64 within 2x
  of that twin's own gradient error vs float64 (the twin's backward rounds the same legs).
* bf16x6 engine (split-bf16 MFMA, the fp32-accurate mode bench.py reports as `parity_value`): the
  fp32 bounds -- loss within 1e-4 of float64, x_hat_0 / x_hat_1 within 1e-4, x_hat_t within
  max(1e-4, 4x the fp32 twin's own error vs float64), and the gradient vector within 4x the fp32
  twin's own gradient error vs float64 of the fp32 engine's gradient.
Every measured error is printed (pytest -s / the GPU log)."""
import numpy as np
import pytest
import torch

from conftest import pkg_mod
from oracle import spec, torch_twin

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float(np.linalg.norm(np.ravel(a) - np.ravel(b)) / max(np.linalg.norm(np.ravel(b)), 1e-30))


def _engine(dtype):
    cfg = pkg_mod("config").preset("celeba", dtype=dtype)
    return pkg_mod("sequential_vae").SequentialVAE(cfg, seed=0), cfg


def test_headline_config_both_precisions():
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    cd = spec.make_config("celeba")            # B=128, T=8
    x, tgt, eps = spec.make_inputs(cd)
    res = {}
    for dt in ("fp32", "bf16", "bf16x6"):
        net, cfg = _engine(dt)
        net.forward(x, tgt, eps, 1.0)
        net.backward()
        torch.cuda.synchronize()
        res[dt] = dict(loss=net.loss_value(reg_coeff=1.0), elbo=net.elbo_per_image().cpu().numpy(),
                       xhat=[net.xhat(t).cpu().numpy() for t in range(cfg.mc_steps)],
                       grads=net.grads[:net.n_live].cpu().numpy().astype(np.float64), params=net.param_dict())
        net.close()
    params = res["fp32"]["params"]
    _, struct = spec.build_params(cd)
    # float64 and fp32 twins with their gradients (the fp32 twin's own gradient error vs float64 is
    # the chaos scale every fp32-class gradient is measured against)
    o64 = torch_twin.Twin(cd, struct, params, dtype=torch.float64).step(x, tgt, eps, 1.0)
    t32 = torch_twin.Twin(cd, struct, params, dtype=torch.float32).step(x, tgt, eps, 1.0)
    # the bf16-emulating twin WITH its backward: the same operands rounded in the same legs, fp32
    # accumulation -- its gradient error vs float64 is the scale the bf16 engine's gradient is held to
    emul = torch_twin.Twin(cd, struct, params, dtype=torch.float32, emulate_bf16=True).step(x, tgt, eps, 1.0)
    table = pkg_mod("weights").param_table(pkg_mod("config").preset("celeba"))[0]
    live = [p for p in table if p["offset"] + p["size"] <= len(res["fp32"]["grads"])]
    flat = lambda gd: np.concatenate([np.ravel(gd[p["name"]]).astype(np.float64) for p in live])
    g64, gt32, gem = flat(o64["grads"]), flat(t32["grads"]), flat(emul["grads"])
    e_twin = _rel(gt32, g64)
    e_emg = _rel(gem, g64)
    L64 = o64["loss"]
    e32 = abs(res["fp32"]["loss"] - L64) / abs(L64)
    e16 = abs(res["bf16"]["loss"] - L64) / abs(L64)
    eem = abs(emul["loss"] - L64) / abs(L64)
    e16_32 = abs(res["bf16"]["loss"] - res["fp32"]["loss"]) / abs(res["fp32"]["loss"])
    x32 = [_rel(res["fp32"]["xhat"][t], o64["xhat"][t]) for t in range(8)]
    x16 = [_rel(res["bf16"]["xhat"][t], o64["xhat"][t]) for t in range(8)]
    xem = [_rel(emul["xhat"][t], o64["xhat"][t]) for t in range(8)]
    g32, g16, gx6 = res["fp32"]["grads"], res["bf16"]["grads"], res["bf16x6"]["grads"]
    gflat = lambda g: np.concatenate([g[p["offset"]:p["offset"] + p["size"]] for p in live])
    g32f, g16f, gx6f = gflat(g32), gflat(g16), gflat(gx6)
    gvec = _rel(g16f, g32f)
    per = [_rel(g16[p["offset"]:p["offset"] + p["size"]], g32[p["offset"]:p["offset"] + p["size"]])
           for p in live if np.linalg.norm(g32[p["offset"]:p["offset"] + p["size"]]) > 1e-7]
    # bf16 engine and bf16-emulating twin, each vs float64: vector and per-tensor median
    g16_64 = _rel(g16f, g64)
    sl = lambda p: slice(p["offset"], p["offset"] + p["size"])
    big = [p for p in live if np.linalg.norm(np.ravel(o64["grads"][p["name"]])) > 1e-7]
    med16 = float(np.median([_rel(g16[sl(p)], o64["grads"][p["name"]]) for p in big]))
    medem = float(np.median([_rel(emul["grads"][p["name"]], o64["grads"][p["name"]]) for p in big]))
    ex6 = abs(res["bf16x6"]["loss"] - L64) / abs(L64)
    xx6 = [_rel(res["bf16x6"]["xhat"][t], o64["xhat"][t]) for t in range(8)]
    xt32 = [_rel(t32["xhat"][t], o64["xhat"][t]) for t in range(8)]
    gx6_32, gx6_64, g32_64 = _rel(gx6f, g32f), _rel(gx6f, g64), _rel(g32f, g64)
    print("\nheadline CelebA B=128 T=8: loss float64 %.6f  fp32 %.6f (rel %.2e)  bf16 %.6f (rel %.2e vs f64, "
          "%.2e vs fp32)  bf16-emulating twin %.6f (rel %.2e)" % (
              L64, res["fp32"]["loss"], e32, res["bf16"]["loss"], e16, e16_32, emul["loss"], eem))
    print("x_hat_t rel L2 vs float64: fp32 %s" % ["%.1e" % e for e in x32])
    print("                           bf16 %s" % ["%.1e" % e for e in x16])
    print("                 bf16-emul twin %s" % ["%.1e" % e for e in xem])
    x16e = [_rel(res["bf16"]["xhat"][t], emul["xhat"][t]) for t in range(8)]
    print("       bf16 engine vs emul twin %s" % ["%.1e" % e for e in x16e])
    print("gradients bf16 vs fp32 engine: vector %.3e, per-tensor median %.3e, p90 %.3e" % (
        gvec, float(np.median(per)), float(np.percentile(per, 90))))
    print("gradients vs float64: bf16 engine vector %.3e (median %.3e) | bf16-emulating twin vector %.3e "
          "(median %.3e) | bound 2 x the twin's" % (g16_64, med16, e_emg, medem))
    print("per-image ELBO bf16 vs fp32: max rel %.2e" % float(
        np.max(np.abs(res["bf16"]["elbo"] - res["fp32"]["elbo"]) / np.abs(res["fp32"]["elbo"]))))
    print("bf16x6: loss %.6f (rel %.2e vs f64); x_hat_t rel L2 vs float64 %s" % (
        res["bf16x6"]["loss"], ex6, ["%.1e" % e for e in xx6]))
    print("          fp32 twin x_hat_t rel L2 vs float64 %s" % ["%.1e" % e for e in xt32])
    print("gradient vectors: fp32 twin vs f64 %.3e | fp32 engine vs f64 %.3e | bf16x6 vs f64 %.3e, "
          "vs fp32 engine %.3e (bound 4 x %.3e)" % (e_twin, g32_64, gx6_64, gx6_32, e_twin))
    print("per-image ELBO bf16x6 vs fp32: max rel %.2e" % float(
        np.max(np.abs(res["bf16x6"]["elbo"] - res["fp32"]["elbo"]) / np.abs(res["fp32"]["elbo"]))))
    # bf16x6: the fp32 bounds
    assert ex6 <= 1e-4
    assert xx6[0] <= 1e-4 and xx6[1] <= 1e-4, xx6
    for t in range(8):
        assert xx6[t] <= max(1e-4, 4 * xt32[t]), (t, xx6[t], xt32[t])
    assert np.isfinite(gx6f).all() and gx6_32 <= 4 * e_twin, (gx6_32, e_twin)
    # fp32: north_star 1e-4 on the ELBO and on the decoder output before amplification
    assert e32 <= 1e-4
    assert x32[0] <= 1e-4 and x32[1] <= 1e-4
    assert np.abs(res["fp32"]["xhat"][0] - o64["xhat"][0]).max() <= 1e-3
    # bf16: the documented bound, and consistent with the emulated rounding
    assert e16_32 <= 2e-2
    assert e16 <= max(2e-3, 3 * eem)
    for t in range(8):
        assert x16[t] <= max(2e-3, 3 * xem[t]), (t, x16[t], xem[t])
    # bf16 gradients: bf16 rounding of the operands (~4e-3 relative) is
    # amplified ~3-4x per chain step (tests/test_chaos.py), so at T=8 the gradient of ANY bf16
    # evaluation of this graph is far from float64 -- the emulating twin's own error is that scale.
    # The engine's gradient must be within 2x of it (vector and per-tensor median), i.e. the engine
    # rounds no worse than the operand rounding it declares.
    assert np.isfinite(g16).all()
    assert g16_64 <= 2 * e_emg, (g16_64, e_emg)
    assert med16 <= 2 * max(medem, 1e-3), (med16, medem)
