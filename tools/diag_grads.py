"""Per-tensor gradient errors of one engine step vs the float64 oracle (tiny geometry by default):
the worst tensors, for bisecting a kernel variant.   SVAE_...=... python tools/diag_grads.py [preset] [dtype]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import pkg_mod  # noqa: E402
from oracle import model, spec  # noqa: E402

preset = sys.argv[1] if len(sys.argv) > 1 else "tiny"
dtype = sys.argv[2] if len(sys.argv) > 2 else "bf16x6"
cfg = pkg_mod("config").preset(preset, batch=4, dtype=dtype)
net = pkg_mod("sequential_vae").SequentialVAE(cfg, seed=0)
cd = spec.make_config(preset, batch=4)
x, tgt, eps = spec.make_inputs(cd, batch=4)
net.forward(x, tgt, eps, 0.37)
net.backward()
import torch  # noqa: E402
torch.cuda.synchronize()
_, struct = spec.build_params(cd)
params = {k: v.astype(np.float64) for k, v in net.param_dict().items()}
o = model.forward_backward(cd, struct, params, x, tgt, eps, 0.37)
g = net.grad_dict()
errs = []
for k, v in o["grads"].items():
    n = np.linalg.norm(v)
    if n > 1e-7:
        errs.append((np.linalg.norm(g[k] - v) / n, k, g[k].shape))
errs.sort(reverse=True)
print("%s %s env %s: loss rel %.2e" % (preset, dtype, {k: v for k, v in os.environ.items() if k.startswith("SVAE_")},
                                       abs(net.loss_value(reg_coeff=0.37) - o["loss"]) / abs(o["loss"])))
for e, k, s in errs[:6]:
    print("   %.3e  %s %s" % (e, k, s))
