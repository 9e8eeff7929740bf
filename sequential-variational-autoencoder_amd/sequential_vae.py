"""Drop-in mirror of the reference ``SequentialVAE`` training / test interface.

Reference interface (sequential_vae.py:1341-1391, abstract_network.py:155-160):

* ``train(input_batch, batch_target) -> float`` — one optimisation step: advances
  ``iteration``, decays the learning rate, feeds ``reg_coeff = 1 - exp(-it/5000)``,
  runs ``[train_op, loss, final_loss]`` and returns ``final_loss / H / W``.
* ``test(input_batch) -> ndarray[B,H,W,C]`` — the last training-branch MLE
  ``training_mles[-1]`` (BN in training mode, fresh eps).

Here the step runs on the HIP engine (libsvae_hip.so): the forward + backward of
the whole unrolled chain, then elementwise clip(+-10) + TF Adam on the flat
parameter buffer.  Parameters, gradients and inputs are torch device tensors whose
pointers are handed to the C ABI; no CPU fallback exists.
"""
import ctypes
import math

import numpy as np
import torch

from . import _lib
from .config import SVAEConfig, preset
from .weights import init_flat, param_table, unflatten


class SequentialVAE:
    def __init__(self, config="celeba", batch_size=None, device=None, seed=0, grad_hook=None):
        if not torch.cuda.is_available():
            raise RuntimeError("SequentialVAE (HIP engine) needs a GPU; no CPU fallback exists")
        cfg = preset(config) if isinstance(config, str) else config
        if batch_size is not None:
            cfg = preset_copy(cfg, batch=batch_size)
        self.cfg = cfg
        self.name = config if isinstance(config, str) else "custom"
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        self.batch_size = cfg.batch
        self.data_dims = [cfg.height, cfg.width, cfg.channels]
        self.iteration = 0                                 # abstract_network.py:103
        self.learning_rate = cfg.learning_rate             # sequential_vae.py:253
        self.grad_hook = grad_hook                         # e.g. data-parallel all-reduce
        self.overlap = None                                # bucketed all-reduce during backward
        self.L = _lib.lib()
        self.table, self.n_total, self.n_live = param_table(cfg)
        self._by_name = {p["name"]: p for p in self.table}
        with torch.cuda.device(self.device):
            self.params = torch.from_numpy(init_flat(cfg, seed)).to(self.device)
            self.grads = torch.zeros(self.n_total, dtype=torch.float32, device=self.device)
            h = ctypes.c_void_p()
            c = cfg.to_c()
            _lib.check(self.L.svae_create(ctypes.byref(c), self.device.index, ctypes.byref(h)))
        self.ctx = h
        _lib.check(self.L.svae_bind(self.ctx, _lib.ptr(self.params), _lib.ptr(self.grads)), self.ctx)
        self._last_reg = 1.0
        # Adam updates applied so far (the AdamOptimizer's step count behind beta1_power); with the
        # improvement-maximisation loss two apply_gradients run per iteration (:1267, :1306)
        self.adam_updates = 0
        self.grads_imp = None
        if cfg.add_improvement_maximization_loss:
            with torch.cuda.device(self.device):
                self.grads_imp = torch.zeros(self.n_total, dtype=torch.float32, device=self.device)
            _lib.check(self.L.svae_bind_imp(self.ctx, _lib.ptr(self.grads_imp)), self.ctx)
            pe = ctypes.c_int64()
            _lib.check(self.L.svae_imp_range(self.ctx, ctypes.byref(pe)), self.ctx)
            self.phi_end = int(pe.value)

    # ------------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "ctx", None):
            self.L.svae_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ low level
    def _dev(self, a):
        if isinstance(a, torch.Tensor):
            t = a.to(self.device, dtype=torch.float32)
        else:
            t = torch.as_tensor(np.asarray(a, dtype=np.float32), device=self.device)
        return t.contiguous()

    def forward(self, x, target, eps=None, reg_coeff=1.0, stream=None, noise=None):
        """Forward of the unrolled chain.  eps [T,B,Dz] or None (device Philox).  With
        add_noise_to_chain, noise [T,B,H,W,C] is the N(0,1) of training_sample = mle + reg*sd*noise
        (sequential_vae.py:1090), or None (device Philox)."""
        x, target = self._dev(x), self._dev(target)
        nz = None
        if self.cfg.add_noise_to_chain:
            if noise is not None:
                nz = self._dev(noise)
                c = self.cfg
                if tuple(nz.shape) != (c.mc_steps, c.batch, c.height, c.width, c.channels):
                    raise ValueError("noise must be [T,B,H,W,C]")
            _lib.check(self.L.svae_set_chain_noise(self.ctx, _lib.ptr(nz)), self.ctx)
        elif noise is not None:
            raise ValueError("noise given but add_noise_to_chain is off")
        exp = (self.cfg.batch, self.cfg.height, self.cfg.width, self.cfg.channels)
        if tuple(x.shape) != exp or tuple(target.shape) != exp:
            raise ValueError("input must be %s, got %s / %s" % (exp, tuple(x.shape), tuple(target.shape)))
        e = None
        if eps is not None:
            e = self._dev(eps)
            if tuple(e.shape) != (self.cfg.mc_steps, self.cfg.batch, self.cfg.latent_dim):
                raise ValueError("eps must be [T,B,Dz]")
        self._keep = (x, target, e, nz)  # keep device inputs alive until backward
        self._last_reg = float(reg_coeff)
        _lib.check(self.L.svae_forward(self.ctx, _lib.ptr(x), _lib.ptr(target), _lib.ptr(e), float(reg_coeff),
                                       _lib.stream_ptr(stream)), self.ctx)

    def backward(self, stream=None):
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        with torch.cuda.stream(s):  # overlapped DP hooks enqueue on the caller's stream
            _lib.check(self.L.svae_backward(self.ctx, _lib.stream_ptr(s)), self.ctx)
        if self.overlap is not None:
            self.overlap.check()
        if self.grad_hook is not None:
            self.grad_hook(self.grads[:self.n_live])

    def enable_overlapped_allreduce(self, dist, group=None, force=False):
        """Data parallel: all-reduce the gradient in per-step buckets during the backward
        (parallel.OverlappedAllReduce) instead of one call after it."""
        from .parallel import OverlappedAllReduce
        self.overlap = OverlappedAllReduce(self, dist, group, force=force)
        return self.overlap

    def backward_apply(self, lr=None, step=None, stream=None):
        """backward() then apply_gradients() as one engine call (svae_backward_adam): every chain
        step's generator/encoder bucket gets its clip + Adam update on the engine's side stream as
        soon as the backward has finished it (after that bucket's overlapped all-reduce), the
        recognition bucket last.  Bit for bit the parameters of the two separate calls."""
        lr = self.learning_rate if lr is None else lr
        step = self._adam_step(step)
        if self.grad_hook is not None:  # the exchange follows the whole backward: Adam after it
            self.backward(stream)
            self.apply_gradients(lr, step, stream)
            return
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        if self.overlap is not None:
            self.overlap.eager = True
        try:
            with torch.cuda.stream(s):
                _lib.check(self.L.svae_backward_adam(self.ctx, float(lr), int(step), float(self.cfg.clip_grad_value),
                                                     _lib.stream_ptr(s)), self.ctx)
        finally:
            if self.overlap is not None:
                self.overlap.eager = False
        if self.overlap is not None:
            self.overlap.check()

    def backward_imp(self, stream=None):
        """d improvement_maximization_loss / d every variable into ``grads_imp``
        (sequential_vae.py:1302-1303; the optimiser reads only the recognition part)."""
        if self.grads_imp is None:
            raise RuntimeError("add_improvement_maximization_loss is off")
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _lib.check(self.L.svae_backward_imp(self.ctx, _lib.stream_ptr(s)), self.ctx)
        if self.grad_hook is not None:
            self.grad_hook(self.grads_imp[:self.phi_end])

    def apply_imp_gradients(self, lr=None, step=None, stream=None):
        """clip + Adam of the recognition variables with ``grads_imp`` (:1304-1306)."""
        lr = self.learning_rate if lr is None else lr
        step = self._adam_step(step)
        _lib.check(self.L.svae_adam_imp(self.ctx, float(lr), int(step), float(self.cfg.clip_grad_value),
                                        _lib.stream_ptr(stream)), self.ctx)

    def imp_loss_value(self, reg_coeff=None):
        """``self.improvement_maximization_loss`` (:1189-1199) = sum_{t>=1} reg * coeff * -mean_b
        ||mle_t - mle_{t-1}||^2."""
        reg = self._last_reg if reg_coeff is None else reg_coeff
        tot = 0.0
        for t in range(1, self.cfg.mc_steps):
            tot += float(self.copy_out(_lib.BUF_IMP_IMG, t, self.cfg.batch).double().mean())
        return -reg * self.cfg.latent_pred_loss_coeff * tot

    def _adam_step(self, step):
        """The Adam step an update runs as (TF's beta1_power = 0.9^step): the next one by default.
        Every update path records it, so save_checkpoint's beta powers match the updates taken
        whichever API (train, backward_apply, apply_gradients, apply_imp_gradients) drove them."""
        step = self.adam_updates + 1 if step is None else int(step)
        self.adam_updates = step
        return step

    def apply_gradients(self, lr=None, step=None, stream=None):
        lr = self.learning_rate if lr is None else lr
        step = self._adam_step(step)
        _lib.check(self.L.svae_adam(self.ctx, float(lr), int(step), float(self.cfg.clip_grad_value),
                                    _lib.stream_ptr(stream)), self.ctx)

    def copy_out(self, which, step, n):
        out = torch.empty(n, dtype=torch.float32, device=self.device)
        _lib.check(self.L.svae_copy_out(self.ctx, which, step, _lib.ptr(out), n, _lib.stream_ptr()), self.ctx)
        return out

    def step_stats(self):
        """[T,2] tensor of (mean recon_t, mean KL_t)  (sequential_vae.py:1163-1164)."""
        return torch.stack([self.copy_out(_lib.BUF_STEP_STATS, t, 2) for t in range(self.cfg.mc_steps)])

    def loss_value(self, stats=None, reg_coeff=None):
        """``self.loss`` (sequential_vae.py:1166-1176) = mean over the batch of the per-image ELBO."""
        st = self.step_stats() if stats is None else stats
        st = st.double().cpu().numpy() if isinstance(st, torch.Tensor) else np.asarray(st, np.float64)
        reg = self._last_reg if reg_coeff is None else reg_coeff
        T = self.cfg.mc_steps
        tot = 0.0
        for t in range(T):
            c = self.cfg.first_step_loss_coeff if t == 0 else 1.0
            if self.cfg.intermediate_reconstruction or t == T - 1:
                tot += 16.0 * c * st[t, 0]
            tot += reg * c * self.cfg.kl_on(t) * st[t, 1]
        return tot

    def elbo_per_image(self):
        T, B = self.cfg.mc_steps, self.cfg.batch
        out = torch.zeros(B, dtype=torch.float64, device=self.device)
        for t in range(T):
            c = self.cfg.first_step_loss_coeff if t == 0 else 1.0
            if self.cfg.intermediate_reconstruction or t == T - 1:
                out += 16.0 * c * self.copy_out(_lib.BUF_REC_IMG, t, B).double()
            out += self._last_reg * c * self.cfg.kl_on(t) * self.copy_out(_lib.BUF_KL_IMG, t, B).double()
        return out

    def sample(self, t=-1):
        """training_samples[t] (:963): the MLE plus reg * stddevs * noise under add_noise_to_chain."""
        t = t % self.cfg.mc_steps
        c = self.cfg
        return self.copy_out(_lib.BUF_SAMPLE, t, c.batch * c.height * c.width * c.channels).view(
            c.batch, c.height, c.width, c.channels)

    def stddevs(self, t=-1):
        """Predicted stddevs [B,H,W,1] of step t (stddevs_prediction, :1866-1875)."""
        t = t % self.cfg.mc_steps
        c = self.cfg
        return self.copy_out(_lib.BUF_STDDEV, t, c.batch * c.height * c.width).view(c.batch, c.height, c.width, 1)

    def xhat(self, t=-1):
        t = t % self.cfg.mc_steps
        c = self.cfg
        return self.copy_out(_lib.BUF_XHAT, t, c.batch * c.height * c.width * c.channels).view(
            c.batch, c.height, c.width, c.channels)

    def latent(self, which, t):
        return self.copy_out(which, t, self.cfg.batch * self.cfg.latent_dim).view(self.cfg.batch, self.cfg.latent_dim)

    def param_dict(self):
        return unflatten(self.params.cpu().numpy(), self.table)

    def grad_dict(self):
        return unflatten(self.grads.cpu().numpy(), self.table)

    def param(self, name):
        """Read-only copy of one variable (write through set_param, or write ``params`` and call
        params_updated(): in bf16 mode the engine keeps bf16 copies of the weights that an
        unannounced write would leave stale)."""
        p = self._by_name[name]
        return self.params[p["offset"]:p["offset"] + p["size"]].view(p["shape"]).clone()

    def set_param(self, name, value):
        p = self._by_name[name]
        self.params[p["offset"]:p["offset"] + p["size"]] = self._dev(value).reshape(-1)
        self.params_updated()

    def params_updated(self):
        """Announce a direct write to ``params`` (copy_, dist.broadcast, a checkpoint load): the
        next forward rebuilds the engine's bf16 weight copies from the fp32 master.  Gradients
        are zeroed as by svae_bind."""
        _lib.check(self.L.svae_bind(self.ctx, _lib.ptr(self.params), _lib.ptr(self.grads)), self.ctx)

    # ------------------------------------------------------------------ reference API
    def train(self, input_batch, batch_target, eps=None, noise=None):
        """One training update; returns the final-step reconstruction loss per pixel
        (sequential_vae.py:1341-1375).  ``eps`` [T,B,Dz] and ``noise`` [T,B,H,W,C] (extensions for
        parity tests) replace the on-device N(0,1) draws of tf.random_normal (:1022, :1090).

        With the improvement-maximisation loss, train_op = tf.group(elbo_train_op,
        pred_latent_train_op) (:1316): two apply_gradients of one AdamOptimizer, both on gradients of
        the same forward.  TF leaves their order open; here the ELBO update (all variables, Adam step
        2k-1) runs first and the improvement update (recognition variables, step 2k) second, sharing
        the Adam moments, so beta1_power advances twice per iteration as in TF."""
        self.iteration += 1
        self.learning_rate *= self.cfg.learning_rate_decay
        reg = 1.0 - math.exp(-self.iteration / self.cfg.reg_coeff_rate)
        self.forward(input_batch, batch_target, eps, reg, noise=noise)
        if self.grads_imp is None:
            self.backward_apply(self.learning_rate)
        else:
            self.backward()
            self.backward_imp()
            self.apply_gradients(self.learning_rate)
            self.apply_imp_gradients(self.learning_rate)
        final = float(self.copy_out(_lib.BUF_STEP_STATS, self.cfg.mc_steps - 1, 2)[0])
        return final / self.data_dims[0] / self.data_dims[1]

    # ------------------------------------------------------------------ checkpoint / resume
    def _adam_state(self, m=None, v=None):
        load = m is not None
        if not load:
            m = torch.empty(self.n_live, dtype=torch.float32, device=self.device)
            v = torch.empty_like(m)
        _lib.check(self.L.svae_adam_state(self.ctx, 1 if load else 0, _lib.ptr(m), _lib.ptr(v), self.n_live,
                                          _lib.stream_ptr(torch.cuda.current_stream(self.device))), self.ctx)
        return m, v

    def save_checkpoint(self, path):
        """Training state under the reference's names (tf.train.Saver, abstract_network.py:124-135):
        every variable, the Adam slots "<name>/Adam" and "<name>/Adam_1" of the tensors on the
        executed path, "beta1_power" / "beta2_power", and iteration / learning_rate as metadata
        (which the reference does not restore).  safetensors file."""
        from safetensors.torch import save_file
        m, v = self._adam_state()
        torch.cuda.synchronize(self.device)
        P, M, V = self.params.cpu(), m.cpu(), v.cpu()
        out = {}
        for p in self.table:
            a, b = p["offset"], p["offset"] + p["size"]
            out[p["name"]] = P[a:b].reshape(p["shape"]).clone()
            if b <= self.n_live:
                out[p["name"] + "/Adam"] = M[a:b].reshape(p["shape"]).clone()
                out[p["name"] + "/Adam_1"] = V[a:b].reshape(p["shape"]).clone()
        # TF's AdamOptimizer starts beta{1,2}_power at beta{1,2} and multiplies after every update,
        # so after N updates it holds beta^(N+1) (tf.train.AdamOptimizer._create_slots / _finish)
        out["beta1_power"] = torch.tensor(0.9 ** (self.adam_updates + 1), dtype=torch.float32)
        out["beta2_power"] = torch.tensor(0.999 ** (self.adam_updates + 1), dtype=torch.float32)
        save_file(out, path, metadata={"iteration": str(self.iteration), "learning_rate": repr(self.learning_rate),
                                       "adam_updates": str(self.adam_updates), "config": self.name})

    def load_checkpoint(self, path):
        """Restore save_checkpoint's state (init_network's restore, abstract_network.py:139-152);
        every variable must be present with its shape."""
        from safetensors import safe_open
        P = self.params.cpu()
        M = torch.zeros(self.n_live, dtype=torch.float32)
        V = torch.zeros(self.n_live, dtype=torch.float32)
        with safe_open(path, framework="pt") as f:
            meta = f.metadata() or {}
            keys = set(f.keys())
            for p in self.table:
                a, b = p["offset"], p["offset"] + p["size"]
                if p["name"] not in keys:
                    raise KeyError("checkpoint lacks %s" % p["name"])
                t = f.get_tensor(p["name"])
                if tuple(t.shape) != tuple(p["shape"]):
                    raise ValueError("%s: shape %s, expected %s" % (p["name"], tuple(t.shape), tuple(p["shape"])))
                P[a:b] = t.reshape(-1)
                if b <= self.n_live and p["name"] + "/Adam" in keys:
                    M[a:b] = f.get_tensor(p["name"] + "/Adam").reshape(-1)
                    V[a:b] = f.get_tensor(p["name"] + "/Adam_1").reshape(-1)
        self.params.copy_(P.to(self.device))
        self._adam_state(M.to(self.device), V.to(self.device))
        self.params_updated()  # caller-written parameters: rebuild the engine's bf16 copies
        torch.cuda.synchronize(self.device)
        per_it = 2 if self.grads_imp is not None else 1  # Adam updates per iteration
        if "iteration" in meta:
            self.iteration = int(meta["iteration"])
            self.adam_updates = int(meta.get("adam_updates", per_it * self.iteration))
        elif "beta1_power" in keys:  # a TF-converted checkpoint: recover the Adam step from beta1^(N+1)
            with safe_open(path, framework="pt") as f:
                b1p = float(f.get_tensor("beta1_power"))
            self.adam_updates = max(0, int(round(math.log(b1p) / math.log(0.9))) - 1)
            self.iteration = self.adam_updates // per_it
        else:
            self.iteration = 0
            self.adam_updates = 0
        self.learning_rate = float(meta.get("learning_rate", self.learning_rate))

    def generate(self, z=None, stream=None, noise=None):
        """Generator chain on latents z [T,B,Dz] (None: N(0,1) on device), no recognition network
        (sequential_vae.py:947-952, :1025).  With add_noise_to_chain, ``noise`` [T,B,H,W,C] injects
        the chain noise (None: drawn on device, never the last forward's).  Returns [x_hat_t]
        device tensors [B,H,W,C]."""
        e = None
        if z is not None:
            e = self._dev(z)
            if tuple(e.shape) != (self.cfg.mc_steps, self.cfg.batch, self.cfg.latent_dim):
                raise ValueError("z must be [T,B,Dz]")
        nz = None
        if noise is not None:
            if not self.cfg.add_noise_to_chain:
                raise ValueError("noise given but add_noise_to_chain is off")
            nz = self._dev(noise)
            _lib.check(self.L.svae_set_chain_noise(self.ctx, _lib.ptr(nz)), self.ctx)
        self._keep = (e, nz)
        _lib.check(self.L.svae_generate(self.ctx, _lib.ptr(e), _lib.stream_ptr(stream)), self.ctx)
        return [self.xhat(t) for t in range(self.cfg.mc_steps)]

    def generate_mc_samples(self, input_batch=None, batch_size=None):
        """Reference generate_mc_samples (sequential_vae.py:1393-1428, add_noise_to_chain=False):
        [x_0 ~ U[0,1) (the chain's unused initial sample, :947-949), x_hat_0, ..., x_hat_{T-1}]
        as numpy arrays; latents N(0,1).  Only the batch size the context was built for is valid."""
        bs = self.cfg.batch if batch_size is None else batch_size
        if bs != self.cfg.batch:
            raise ValueError("batch_size must equal the context batch (%d)" % self.cfg.batch)
        x0 = torch.rand(bs, self.cfg.height, self.cfg.width, self.cfg.channels, device=self.device)
        return [x0.cpu().numpy()] + [x.cpu().numpy() for x in self.generate()]

    def test(self, input_batch):
        """training_mles[-1] for the batch (sequential_vae.py:1381-1391; reg_coeff default 1.0)."""
        self.forward(input_batch, input_batch, None, 1.0)
        return self.xhat(-1).cpu().numpy()


def preset_copy(cfg, **over):
    from dataclasses import replace
    return replace(cfg, **over)
