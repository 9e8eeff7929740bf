import sys, numpy as np, torch, importlib
sys.path.insert(0, '.')
from oracle import spec, model
cfgmod = importlib.import_module("sequential-variational-autoencoder_amd.config")
SV = importlib.import_module("sequential-variational-autoencoder_amd.sequential_vae").SequentialVAE
rel=lambda a,b: np.linalg.norm(np.ravel(a)-np.ravel(b))/max(np.linalg.norm(np.ravel(b)),1e-30)
B, T = 8, 2
cd = spec.make_config("tiny", batch=B, mc_steps=T)
net = SV(cfgmod.preset("tiny", batch=B, mc_steps=T, dtype="bf16"), seed=0)
x,tgt,eps = spec.make_inputs(cd, batch=B)
_, struct = spec.build_params(cd)
o = model.forward_backward(cd, struct, {k:v.astype(np.float64) for k,v in net.param_dict().items()}, x, tgt, eps, 1.0)
net.forward(x, tgt, eps, 1.0); net.backward(); torch.cuda.synchronize()
g = net.grad_dict()
for p in net.table:
    n = p["name"]
    if p["zero_grad"] or np.linalg.norm(o["grads"][n]) < 1e-7: continue
    if "step_1" in n and n.startswith("theta"):
        print("%.2e %s" % (rel(g[n], o["grads"][n]), n))
print("dz", [ "%.2e" % rel(net.latent(7,t).cpu().numpy(), o["dz"][t]) for t in range(T)])
