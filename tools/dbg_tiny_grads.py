import sys, numpy as np, torch, importlib
sys.path.insert(0, '.')
from oracle import spec, model
cfgmod = importlib.import_module("sequential-variational-autoencoder_amd.config")
SV = importlib.import_module("sequential-variational-autoencoder_amd.sequential_vae").SequentialVAE
L = importlib.import_module("sequential-variational-autoencoder_amd._lib")
def dbg(net, code, v):
    L.check(net.L.svae_copy_out(net.ctx, code, v, L.ptr(torch.empty(1, device="cuda")), 1, L.stream_ptr()), net.ctx)
rel=lambda a,b: np.linalg.norm(np.ravel(a)-np.ravel(b))/max(np.linalg.norm(np.ravel(b)),1e-30)
for B, T in ((8, 3), (8, 2)):
    cd = spec.make_config("tiny", batch=B, mc_steps=T)
    net = SV(cfgmod.preset("tiny", batch=B, mc_steps=T), seed=0)
    x,tgt,eps = spec.make_inputs(cd, batch=B)
    _, struct = spec.build_params(cd)
    o = model.forward_backward(cd, struct, {k:v.astype(np.float64) for k,v in net.param_dict().items()}, x, tgt, eps, 1.0)
    dg = o["dec_grads"][T-1]
    S = cd["image_sizes"]; F = cd["filter_sizes"]
    for lvl in (0, 1):
        net.grads.zero_()
        net.forward(x, tgt, eps, 1.0)
        dbg(net, 101, T-1); dbg(net, 111, lvl)
        net.backward(); torch.cuda.synchronize()
        C = F[lvl+1]; n = B*S[lvl+1]**2*C
        dy = net.copy_out(110, 0, n).cpu().numpy()
        y = net.copy_out(106, lvl, n).cpu().numpy()
        g = net.grad_dict()
        bn = "theta/generative_step_%d/BatchNorm_%d/beta" % (T-1, 10 if lvl == 0 else 8)
        print("B%d T%d lvl%d: dy rel %.2e  y rel %.2e  %s rel %.2e" % (B, T, lvl, rel(dy, dg["s1_act_%d" % lvl]),
              rel(y, o["dec_s1"][T-1][lvl] if "dec_s1" in o else y), bn, rel(g[bn], o["grads"][bn])))
        dbg(net, 111, -1); dbg(net, 101, -1)
