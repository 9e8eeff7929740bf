"""PixelCNN++ head on the GPU against oracle/pcnn.py (fp64 torch, PARITY UNPINNED:
the reference's TF path cannot run, see the oracle's header).

The HIP path computes every conv in bf16 MFMA with fp32 accumulation; it is compared against the
oracle with the same bf16 rounding of the conv operands (``bf16=True``), where only fp32-vs-fp64
accumulation and the occasional flipped bf16 rounding of an input differ, and against the plain
fp64 oracle at a bf16 tolerance."""
import numpy as np
import pytest
import torch

from conftest import pkg_mod
from oracle import pcnn as opc

pytestmark = pytest.mark.gpu

SPEC = dict(H=8, W=8, K=5, nr_resnet=1, nr_filters=8, nr_mix=2)


def _setup(nl="relu", B=2, seed=0, **over):
    kw = dict(SPEC, nonlinearity=nl)
    kw.update(over)
    PC = pkg_mod("pixelcnn")
    spec = PC.make_spec(**kw)
    ospec = opc.make_spec(**kw)
    params = opc.init_params(ospec, seed)
    rng = np.random.default_rng(seed + 1)
    x = rng.uniform(-1, 1, (B, spec["H"], spec["W"], 3))
    x[0, 0, :2] = -1.0  # the discretized-logistic edge cases (nn.py:81)
    x[0, 1, :2] = 1.0
    h = rng.normal(size=(B, spec["K"]))
    return PC, spec, ospec, params, x, h


def _rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-12))


def test_param_table_matches_oracle():
    PC, spec, ospec, params, x, h = _setup()
    assert list(PC.param_shapes(spec).items()) == list(opc.param_shapes(ospec).items())


@pytest.mark.parametrize("nl", ["relu", "concat_elu"])
def test_model_loss_and_grads_match_oracle(nl):
    PC, spec, ospec, params, x, h = _setup(nl)
    net = PC.PixelCNNpp(spec, params=params)
    l = net.model(x, h).cpu().numpy().astype(np.float64)
    nll = net.loss(x, h, backward=True)
    g = net.grads()
    o_nll, o_l, o_g = opc.loss_and_grads(ospec, params, x, h, bf16=True)
    f_nll, f_l, _ = opc.loss_and_grads(ospec, params, x, h, bf16=False)
    el, en = _rel(l, o_l), abs(nll - o_nll) / abs(o_nll)
    print("\n%s: l rel err %.2e (vs fp64 %.2e), nll %.6f oracle-bf16 %.6f fp64 %.6f rel %.2e" % (
        nl, el, _rel(l, f_l), nll, o_nll, f_nll, en))
    assert el < 1e-2 and _rel(l, f_l) < 5e-2
    assert en < 1e-3 and abs(nll - f_nll) / abs(f_nll) < 1e-2
    worst = []
    for k, ref in o_g.items():
        if not ref.any():
            continue
        e = float(np.linalg.norm(g[k] - ref) / np.linalg.norm(ref))
        worst.append((e, k))
    worst.sort(reverse=True)
    print("  worst grad rel-norm errors:", ", ".join("%s %.2e" % (k, e) for e, k in worst[:5]))
    assert worst[0][0] < 3e-2, worst[:5]
    assert np.median([e for e, _ in worst]) < 5e-3


def test_mixture_loss_gradient_matches_autograd():
    """svae_pcnn_mixlogistic vs torch autograd of nn.py:46-87 on given l, all four branches."""
    PC = pkg_mod("pixelcnn")
    L = pkg_mod("_lib")
    rng = np.random.default_rng(3)
    B, H, W, M = 2, 4, 4, 3
    x = rng.uniform(-1, 1, (B, H, W, 3))
    x[0, 0, 0] = -1.0
    x[0, 0, 1] = 1.0
    l = rng.normal(size=(B, H, W, 10 * M))
    l[1, 0, 0, M + M:M + 2 * M] = -9.0  # log_scales clamped at -7, narrow bins: the cdf_delta < 1e-5 branch
    l[1, 0, 0, M:2 * M] = 0.9
    x[1, 0, 0] = -0.5
    lt = torch.tensor(l, dtype=torch.float64, requires_grad=True)
    ref = opc.mix_logistic_logprob(torch.tensor(x), lt)
    (-ref.sum()).backward()
    xd = torch.tensor(x, dtype=torch.float32, device="cuda").contiguous()
    ld = torch.tensor(l, dtype=torch.float32, device="cuda").contiguous()
    logp = torch.empty(B * H * W, device="cuda")
    dl = torch.empty_like(ld)
    L.check(L.lib().svae_pcnn_mixlogistic(PC._p(xd), PC._p(ld), B * H * W, M, PC._p(logp), PC._p(dl), 1.0,
                                          L.stream_ptr()))
    torch.cuda.synchronize()
    e1 = _rel(logp.cpu().numpy().reshape(ref.shape), ref.detach().numpy())
    e2 = _rel(dl.cpu().numpy(), lt.grad.numpy())
    print("\nmixture logp rel %.2e, dl rel %.2e" % (e1, e2))
    assert e1 < 1e-5 and e2 < 1e-4


def test_sample_and_highway_match_oracle():
    PC, spec, ospec, params, x, h = _setup()
    net = PC.PixelCNNpp(spec, params=params)
    B, H, W, M = x.shape[0], spec["H"], spec["W"], spec["M"]
    rng = np.random.default_rng(9)
    u_mix = rng.uniform(1e-5, 1 - 1e-5, (B, H, W, M))
    u_log = rng.uniform(1e-5, 1 - 1e-5, (B, H, W, 3))
    prev = rng.uniform(-1, 1, (B, H, W, 3))
    out, _, cache = PC.make_pixel_cnn(torch.tensor(x, dtype=torch.float32), torch.tensor(prev, dtype=torch.float32),
                                      torch.tensor(h, dtype=torch.float32), 0.2, 0.8, net=net,
                                      u_mix=torch.tensor(u_mix, dtype=torch.float32),
                                      u_log=torch.tensor(u_log, dtype=torch.float32))
    l = net.model(x, h).cpu().double()
    s_ref = opc.mix_logistic_sample(l, torch.tensor(u_mix), torch.tensor(u_log))
    s = cache["sample_op"].cpu().double()
    assert _rel(s.numpy(), s_ref.numpy()) < 1e-5
    P = opc.to_tensors(params, requires_grad=False)
    o_out, _ = opc.highway_mix(s_ref.permute(0, 3, 1, 2), torch.tensor(prev).permute(0, 3, 1, 2), torch.tensor(h),
                               P["highway/W"], P["highway/b"], 0.2, 0.8)
    assert _rel(out.cpu().double().numpy(), o_out.permute(0, 2, 3, 1).numpy()) < 1e-5


def test_autoregressive_sample_matches_oracle():
    """sample_from_model's raster loop (pixelvae.py:184-189) at 4x4: one network evaluation and one
    draw per position, the oracle repeating the same loop."""
    PC, spec, ospec, params, x, h = _setup(H=4, W=4)
    net = PC.PixelCNNpp(spec, params=params)
    B, H, W, M = 2, 4, 4, spec["M"]
    rng = np.random.default_rng(4)
    u_mix = rng.uniform(1e-5, 1 - 1e-5, (B, H, W, M))
    u_log = rng.uniform(1e-5, 1 - 1e-5, (B, H, W, 3))
    xs = net.sample(h, u_mix=torch.tensor(u_mix, dtype=torch.float32),
                    u_log=torch.tensor(u_log, dtype=torch.float32)).cpu().double().numpy()
    P = opc.to_tensors(params, requires_grad=False)
    xo = torch.zeros(B, H, W, 3, dtype=torch.float64)
    for q in range(H * W):
        yi, xi = divmod(q, W)
        l = opc.Net(ospec, P, bf16=True).model(xo, torch.tensor(h))
        sm = opc.mix_logistic_sample(l, torch.tensor(u_mix), torch.tensor(u_log))
        xo[:, yi, xi] = sm[:, yi, xi]
    err = np.abs(xs - xo.numpy()).max()
    print("\nautoregressive 4x4 sample max abs err %.2e" % err)
    assert err < 2e-2


def test_data_init_matches_oracle():
    PC, spec, ospec, params, x, h = _setup()
    net = PC.PixelCNNpp(spec, params=params)
    net.data_init(x, h)
    got = net.params()
    ref = opc.data_init(ospec, params, x, h)
    worst = max(_rel(got[k], ref[k]) for k in ref if k.endswith("/g") or k.endswith("/b"))
    print("\ndata-dependent init: worst g/b rel err %.2e" % worst)
    assert worst < 3e-2


def test_train_steps_reduce_nll():
    PC, spec, ospec, params, x, h = _setup()
    net = PC.PixelCNNpp(spec, params=params)
    losses = [net.train_step(x, h, lr=1e-3) for _ in range(6)]
    net.ema_update()
    net.ema_update()
    print("\nNLL over 6 Adam steps:", ["%.2f" % v for v in losses])
    assert all(np.isfinite(losses)) and losses[-1] < losses[0]


def test_autoregressive_property_hip():
    """The HIP model's output at raster position q is bit-for-bit unchanged by a perturbation of x
    at q or later (the shifted gathers never read it), and changes after it."""
    PC, spec, ospec, params, x, h = _setup(B=1)
    net = PC.PixelCNNpp(spec, params=params)
    base = net.model(x, h).cpu().numpy()
    for q in (0, 13, 40, 63):
        yi, xi = divmod(q, spec["W"])
        x2 = x.copy()
        x2[0, yi, xi] += 0.5
        d = np.abs(net.model(x2, h).cpu().numpy() - base).max(axis=-1)[0].reshape(-1)
        assert d[:q + 1].max() == 0.0, q
        if q < 63:
            assert d[q + 1:].max() > 0.0


def test_full_size_step_runs():
    """The pixelvae.py geometry (nr_resnet 3, 160 filters, 10 mixtures) at 64x64: one forward,
    backward and Adam update, finite."""
    PC = pkg_mod("pixelcnn")
    spec = PC.make_spec(H=64, W=64, K=48)
    net = PC.PixelCNNpp(spec, seed=0)
    rng = np.random.default_rng(0)
    x = rng.uniform(-1, 1, (2, 64, 64, 3)).astype(np.float32)
    h = rng.normal(size=(2, 48)).astype(np.float32)
    net.data_init(x, h)
    nll = net.train_step(x, h, lr=1e-4)
    bpd = nll / (2 * 64 * 64 * 3 * np.log(2))
    print("\nfull-size NLL %.1f (%.3f bits/dim at init), %d parameters" % (nll, bpd, net.n_params))
    assert np.isfinite(nll) and torch.isfinite(net.G).all() and torch.isfinite(net.P).all()


def test_seeded_dropout_matches_explicit_mask():
    """The training pass's dropout drawn inside the nonlinearity kernels (DropMask: seed, keep) gives
    bitwise the output and gradients of the same mask passed as a tensor, and keeps ~1 - p."""
    PC, spec, ospec, params, x, h = _setup(nr_filters=16)
    net = PC.PixelCNNpp(spec, params=params)
    torch.manual_seed(3)
    l1 = net.forward_train(x, h, dropout_p=0.3).clone()
    masks = list(net.last_masks)
    assert masks and all(isinstance(m, PC.DropMask) for m in masks)
    dl = torch.randn_like(l1)
    net.backward_from(dl.reshape(-1, l1.shape[-1]))
    g1 = net.G.clone()
    tens = [m.tensor(net) for m in masks]
    l2 = net.forward_train(x, h, masks=tens).clone()
    net.backward_from(dl.reshape(-1, l1.shape[-1]))
    torch.cuda.synchronize()
    assert torch.equal(l1, l2) and torch.equal(g1, net.G)
    kept = torch.cat([(t > 0).float().reshape(-1) for t in tens]).mean().item()
    scale = {float(v) for t in tens for v in t.unique().tolist()}
    print("\nseeded dropout: kept fraction %.4f, values %s" % (kept, sorted(scale)))
    assert abs(kept - 0.7) < 0.02 and len(scale) == 2 and abs(max(scale) - 1 / 0.7) < 1e-6


@pytest.mark.parametrize("nl", ["relu", "elu"])
def test_fused_activation_backward_is_bitwise(nl):
    """The relu / elu backward applied in the consuming conv's input-gradient epilogue
    (svae_pcnn_conv_act_bwd) gives bitwise the gradients of the separate nonlinearity pass, with
    seeded dropout on."""
    PC, spec, ospec, params, x, h = _setup(nl, nr_filters=16)
    net = PC.PixelCNNpp(spec, params=params)
    net.bf16_grads = False  # (the fused epilogue takes the fp32 output gradients)
    res = []
    for fuse in (True, False):
        net.fuse_act_bwd = fuse
        torch.manual_seed(5)
        l = net.forward_train(x, h, dropout_p=0.3).clone()
        dh = net.backward_from(torch.ones_like(l).reshape(-1, l.shape[-1]) * 0.01)
        torch.cuda.synchronize()
        res.append((l, net.G.clone(), dh.clone()))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1]) and torch.equal(res[0][2], res[1][2])


def test_bf16_gradient_buffers_match_fp32():
    """The resnet convs' output gradients stored bf16 (with their bias gradients summed in fp32 by the
    op that writes them) against fp32 storage: the same forward, the weight / input gradients equal up
    to fp32 summation order (the convs round dy to bf16 either way), the bias gradients to fp32 order."""
    PC, spec, ospec, params, x, h = _setup("relu", nr_filters=16)
    net = PC.PixelCNNpp(spec, params=params)
    res = []
    for b in (True, False):
        net.bf16_grads = b
        torch.manual_seed(9)
        l = net.forward_train(x, h, dropout_p=0.3).clone()
        dh = net.backward_from(torch.ones_like(l).reshape(-1, l.shape[-1]) * 0.01)
        torch.cuda.synchronize()
        res.append((l, net.grads(), dh.clone()))
    assert torch.equal(res[0][0], res[1][0])
    worst = max(float(np.abs(res[0][1][k] - res[1][1][k]).max() / max(np.abs(res[1][1][k]).max(), 1e-20))
                for k in res[1][1] if np.abs(res[1][1][k]).max() > 0)
    edh = float((res[0][2] - res[1][2]).abs().max() / res[1][2].abs().max())
    print("\nbf16 gradient buffers vs fp32: worst per-tensor rel max err %.2e, dh %.2e" % (worst, edh))
    assert worst < 1e-4 and edh < 1e-4
