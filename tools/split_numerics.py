"""Numerics of the split (fp32-accurate, dtype bf16x6) mode's product schemes, emulated on the CPU twin.

    python tools/split_numerics.py [B] [schemes] [preset]     e.g. 16 fp32,x6,h3 celeba

Every conv / FC leg of oracle/torch_twin.py evaluated as the engine's kernels do it, against the float64 twin:
  fp32  plain fp32 (the reference precision)
  x6    3 bf16 planes, 6 products (the split gathers until round 5)
  x3    2 bf16 planes, 3 products (the split weight-GEMMs)
  h3    scaled fp16 hi/lo planes, 3 products (csrc/halo_x3.hip, opload.h split8_h16); per-tensor scale here,
        the kernel's per-block running scale is at least as fine
Gathers (forward / input gradient) take the scheme, weight gradients x3 (h3b: h3 for those too).
Prints the loss error, x_hat_t relative L2 error per chain step and the gradient-vector error."""
import sys, time, math, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle import spec, torch_twin as tt
torch.set_num_threads(8)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
schemes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["fp32", "x6", "h3"]

def bf(t): return t.to(torch.bfloat16).to(t.dtype)
def hf(t): return t.to(torch.float16).to(t.dtype)

def planes_bf(t, n):
    out = []
    r = t
    for i in range(n):
        p = bf(r); out.append(p); r = r - p
    return out

def planes_h(t, n=2, head=14):
    m = float(t.abs().max())
    if m == 0: return [t] + [torch.zeros_like(t)] * (n - 1)
    e = math.floor(math.log2(m))
    s = 2.0 ** (head - e)
    r = t * s
    out = []
    for i in range(n):
        p = hf(r); out.append(p / s); r = r - p
    return out

def prod(f, a, b, scheme):
    if scheme == "x6":
        p = planes_bf(a, 3); q = planes_bf(b, 3)
        return f(p[0], q[0]) + f(p[0], q[1]) + f(p[1], q[0]) + f(p[0], q[2]) + f(p[2], q[0]) + f(p[1], q[1])
    if scheme == "x3":
        p = planes_bf(a, 2); q = planes_bf(b, 2)
        return f(p[0], q[0]) + f(p[0], q[1]) + f(p[1], q[0])
    if scheme in ("h3", "h3b"):
        p = planes_h(a); q = planes_h(b)
        return f(p[0], q[0]) + f(p[0], q[1]) + f(p[1], q[0])
    if scheme == "h4":
        p = planes_h(a); q = planes_h(b)
        return f(p[0], q[0]) + f(p[0], q[1]) + f(p[1], q[0]) + f(p[1], q[1])
    raise ValueError(scheme)

MODE = {"g": "x6", "w": "x3"}
class Op(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, fn, rf, rd, rw, split=False):
        ctx.fn, ctx.rd, ctx.rw = fn, rd, rw
        ctx.save_for_backward(x, w)
        return prod(fn, x, w, MODE["g"]) if rf else fn(x, w)
    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        def vx(ww, g):
            with torch.enable_grad():
                xa = x.detach().requires_grad_(True)
                return torch.autograd.grad(ctx.fn(xa, ww), xa, g)[0]
        def vw(xx, g):
            with torch.enable_grad():
                wa = w.detach().requires_grad_(True)
                return torch.autograd.grad(ctx.fn(xx, wa), wa, g)[0]
        gx = prod(vx, w, gy, MODE["g"]) if ctx.rd else vx(w, gy)
        gw = prod(vw, x, gy, MODE["w"]) if ctx.rw else vw(x, gy)
        return gx, gw, None, None, None, None, None
tt._RoundedOp = Op

cd = spec.make_config(sys.argv[3] if len(sys.argv) > 3 else "celeba", batch=B)
_, struct, params = spec.init_params(cd, seed=0, dtype=np.float64)
x, tgt, eps = spec.make_inputs(cd, batch=B)
t0 = time.time()
ref = tt.Twin(cd, struct, params, dtype=torch.float64).step(x, tgt, eps, 1.0)
print("fp64 %.1fs" % (time.time() - t0), flush=True)
gref = np.concatenate([ref["grads"][k].ravel() for k in sorted(ref["grads"])])
for sc in schemes:
    t0 = time.time()
    if sc == "fp32":
        tw = tt.Twin(cd, struct, {k: v.astype(np.float32) for k, v in params.items()}, dtype=torch.float32)
    else:
        if sc == "h3b": MODE.update(g="h3", w="h3")
        else: MODE.update(g=sc, w="x3")
        tw = tt.Twin(cd, struct, {k: v.astype(np.float32) for k, v in params.items()}, dtype=torch.float32, emulate_split=True)
    o = tw.step(x, tgt, eps, 1.0)
    errs = [np.linalg.norm(a - b) / np.linalg.norm(b) for a, b in zip(o["xhat"], ref["xhat"])]
    g = np.concatenate([o["grads"][k].ravel() for k in sorted(o["grads"])])
    ge = np.linalg.norm(g - gref) / np.linalg.norm(gref)
    print("%-5s loss %.2e  xhat %s  grad %.3e  (%.0fs)" % (sc, abs(o["loss"] - ref["loss"]) / abs(ref["loss"]),
          " ".join("%.1e" % e for e in errs), ge, time.time() - t0), flush=True)
