"""PyTorch-CPU fp64 restatement of the c_pixelvae chain -- TEST INFRASTRUCTURE ONLY (imported by
tests/ and nothing in the product path).

PARITY UNPINNED: the reference's PixelCNN glue cannot run (pixel_cnn/pixelvae.py:108-112, :126,
:136; no TensorFlow here) and ships no vectors.  This composes the two restatements the product is
already checked against:

  * oracle/torch_twin.py for the sequential VAE part (sequential_vae.py:877-1212): the recognition
    network of every step (shared phi, :1573-1577) and step 0's generator_ladder
    (generator_first_step, :216, :1069);
  * oracle/pcnn.py for step e's generator_pixelcnn (:1943-1971 -> pixelvae.py:68-158, repaired):
    model_spec(target, z_e) with the training pass's dropout (nn.py:273-274; keep-masks injected),
    sample_from_discretized_mix_logistic with injected uniforms (nn.py:89-109), the per-image
    highway mix with x_hat_{e-1} (pixelvae.py:135-136);
  * the loss of compute_and_accumulate_loss (:1146-1176): step 0's 16 MSE + reg KL scaled by
    first_step_loss_coeff, step e's 16 MSE (its KL off: regularized_steps = [0]).

Gradients come from torch autograd in fp64; a variable shared by several steps gets the sum of its
copies' gradients (spec.sum_shared_grads), TF's gradient of a reused variable.
"""
import numpy as np
import torch

from . import pcnn, spec, torch_twin


def forward_backward(cd, pub, head_spec, head_params, x, tgt, eps, reg, u_mix, u_log, masks, bf16_head=True,
                     dtype=torch.float64):
    """cd: spec.make_config dict of the chain (mc_steps = e + 1, share_theta / share_phi, ...);
    pub: the engine's public parameters (name -> array); head_params: the head's (name -> array).
    dtype: float64 (the parity oracle) or float32 (bench.py's like-for-like CPU baseline of the fp32-grade
    step).  Returns dict(loss, xhat [per step], rec, kl, grads (public names), head_grads, l)."""
    DT = dtype
    T = cd["mc_steps"]
    e = T - 1
    sh_t, sh_p = cd.get("share_theta", True), cd.get("share_phi", True)
    table, struct = spec.build_params(cd)
    # per-step copies of the public tensors that the executed part uses (step e has no ladder generator)
    per = {}
    for p in table:
        k = spec.shared_name(p["name"], sh_t, sh_p, False)
        if k in pub:
            per[p["name"]] = np.asarray(pub[k], np.float64)
    tw = torch_twin.Twin(cd, struct, per, dtype=DT)
    Ph = {k: torch.tensor(np.asarray(v, np.float64), dtype=DT, requires_grad=True) for k, v in head_params.items()}
    xt = torch.as_tensor(np.asarray(x), dtype=DT).permute(0, 3, 1, 2)
    tg = torch.as_tensor(np.asarray(tgt), dtype=DT)
    tgc = tg.permute(0, 3, 1, 2)
    ep = torch.as_tensor(np.asarray(eps), dtype=DT)
    p2 = cd["latent_prior_stddev"] ** 2
    loss, xh, recs, kls = 0.0, [], [], []
    prev = None
    for t in range(T):
        st = struct[t]
        mu, sig = tw.inference(st["inference"], xt)
        z = mu + sig * ep[t]
        kl = (-0.5 - torch.log(sig) + 0.5 * sig ** 2 / p2 + 0.5 * mu ** 2 / p2).mean(1).mean()
        if t < e:
            out = tw.generator(st["generator"], prev, z, st.get("encoder"))   # NCHW
        else:
            net = pcnn.Net(head_spec, Ph, bf16=bf16_head)
            l = net.model(tg, z, masks=masks)
            smp = pcnn.mix_logistic_sample(l, torch.as_tensor(u_mix, dtype=DT), torch.as_tensor(u_log, dtype=DT))
            o, _ = pcnn.highway_mix(smp, prev.permute(0, 2, 3, 1), z, Ph["highway/W"], Ph["highway/b"],
                                    cd["min_highway"], cd["max_highway"])
            out = o.permute(0, 3, 1, 2)
            l_out = l
        rec = ((out - tgc) ** 2).mean()
        c = cd["first_step_loss_coeff"] if t == 0 else 1.0
        if cd["intermediate_reconstruction"] or t == T - 1:
            loss = loss + 16.0 * c * rec
        loss = loss + reg * c * spec.kl_on(cd, t) * kl
        xh.append(out.detach().permute(0, 2, 3, 1).numpy())
        recs.append(float(rec.detach()))
        kls.append(float(kl.detach()))
        prev = out
    names = list(tw.P.keys())
    hnames = list(Ph.keys())
    gs = torch.autograd.grad(loss, [tw.P[k] for k in names] + [Ph[k] for k in hnames], allow_unused=True)
    g_per = {k: (np.zeros(tw.P[k].shape) if g is None else g.numpy()) for k, g in zip(names, gs[:len(names)])}
    grads = spec.sum_shared_grads(g_per, sh_t, sh_p, False)
    head_grads = {k: (np.zeros(Ph[k].shape) if g is None else g.numpy()) for k, g in zip(hnames, gs[len(names):])}
    return dict(loss=float(loss.detach()), xhat=xh, rec=recs, kl=kls, grads=grads, head_grads=head_grads,
                l=l_out.detach().numpy())
