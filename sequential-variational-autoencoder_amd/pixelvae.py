"""The c_pixelvae chain: a sequential VAE whose step-1 generator is the PixelCNN++ head.

Reference wiring (BASELINE.json configs[4]):
  * netname ``c_pixelvae`` (sequential_vae.py:529-543): shared theta / phi, T = 2, latents
    [12, 12, 12, 12], filters [3, 16, 32, 64, 128, 384], ``regularized_steps = [0]``,
    ``first_step_loss_coeff = 2``, ``latent_mean_clip = 4``, highway ratio in [0.2, 0.8], lr decay
    0.99999, ``generator = generator_pixelcnn``.
  * step 0: ``generator_first_step`` stays ``generator_ladder`` (:216, :1069) -- the HIP engine's
    ladder decoder; the recognition network of both steps is the engine's as well.
  * step t >= 1: ``generator_pixelcnn`` (:1943-1971) -> ``make_pixel_cnn`` (pixel_cnn/pixelvae.py:
    68-158): PixelCNN++ ``model_spec`` on the ground-truth images (``true_samples`` =
    ``target_placeholder``, :958-959) conditioned on h = z_t, dropout 0.3 in the training pass
    (:62, :123; nn.py:273-274), one draw of ``sample_from_discretized_mix_logistic`` (nn.py:89-109),
    mixed per IMAGE with the previous chain sample by r = min + (max - min) sigmoid(fc(z_t))
    (:135-136).  The chain's MSE (compute_and_accumulate_loss :1146, :1166-1168) is taken on that
    mixed output, so the head trains through the reparameterised logistic draw.
  * train(): the init pass (:1360-1362) before the step, one Adam over every variable, and the
    Polyak EMA of the head grouped with the train op (:1318-1320; pixelvae.py:113-114).
  * generation: ``sample_from_model`` (pixelvae.py:170-194) on the EMA weights.

The glue is broken as written (pixelvae.py:108-112, :126, :136); this is the
repaired restatement of DESIGN.md §12, checked against oracle/pixelvae.py (parity unpinned).  One
deliberate reading: the reference re-runs the data-dependent init pass before EVERY train step
(:1360-1362), which would reset every weight-normed g, b each iteration; ``init_every_step=False``
(default) runs it before the first step only, as the OpenAI head intends; True follows :1360-1362.

Everything numeric runs in libsvae_hip.so: the engine (recognition, step 0, their backward, given
d loss / d x_hat_0 and d loss / d z_1 through svae_set_external_grads) and the head's kernels
(include/svae_pcnn.h).  torch allocates device memory and draws the uniforms / dropout masks.
"""
import ctypes
import math
from dataclasses import replace

import torch

from . import _lib
from .config import preset
from .pixelcnn import PixelCNNpp, _ck, _p, make_spec
from .sequential_vae import SequentialVAE


class PixelVAE:
    def __init__(self, config="c_pixelvae", batch_size=None, seed=0, head=None, dropout_p=0.3, polyak_decay=0.9995,
                 init_every_step=False, head_planes=None, **over):
        cfg = preset(config, **over) if isinstance(config, str) else config
        if batch_size is not None:
            cfg = replace(cfg, batch=batch_size)
        e = cfg.external_generator_from
        if e < 1 or cfg.mc_steps - e != 1:
            raise ValueError("PixelVAE needs external_generator_from = mc_steps - 1 (c_pixelvae: one head step)")
        if cfg.channels != 3:
            raise ValueError("the PixelCNN++ head models RGB images (nn.py:58-87)")
        self.cfg = cfg
        self.vae = SequentialVAE(cfg, seed=seed)
        hs = dict(nr_resnet=3, nr_filters=160, nr_mix=10, nonlinearity="relu")  # pixelvae.py:54-63
        hs.update(head or {})
        # the head's GEMM operands: bf16 (1 plane), or the split mode's 3 bf16 planes (fp32-grade) -- by default
        # the split mode with the engine's split dtype, so dtype "bf16x6" is an fp32-accurate step end to end
        if head_planes is None:
            head_planes = 3 if cfg.dtype == "bf16x6" else 1
        self.head = PixelCNNpp(make_spec(H=cfg.height, W=cfg.width, C=3, K=cfg.latent_dim, **hs), seed=seed + 1,
                               planes=head_planes)
        self.L = self.vae.L
        self.dev = self.vae.device
        self.e = e
        self.dropout_p = float(dropout_p)
        self.polyak_decay = float(polyak_decay)
        self.init_every_step = bool(init_every_step)
        self.initialized = False
        self.iteration = 0
        self.learning_rate = cfg.learning_rate
        self._fw = None

    def close(self):
        self.vae.close()

    # ------------------------------------------------------------------ forward / backward
    def _uniforms(self, u_mix, u_log):
        B, H, W, M = self.cfg.batch, self.cfg.height, self.cfg.width, self.head.s["M"]
        if u_mix is None:  # tf.random_uniform(minval=1e-5, maxval=1-1e-5) (nn.py:96, :103)
            u_mix = torch.rand(B, H, W, M, device=self.dev) * (1 - 2e-5) + 1e-5
        if u_log is None:
            u_log = torch.rand(B, H, W, 3, device=self.dev) * (1 - 2e-5) + 1e-5
        return (torch.as_tensor(u_mix, dtype=torch.float32, device=self.dev).contiguous(),
                torch.as_tensor(u_log, dtype=torch.float32, device=self.dev).contiguous())

    def forward(self, x, target, eps=None, reg_coeff=1.0, u_mix=None, u_log=None, masks=None):
        """Both steps of the chain.  eps [T,B,Dz] / u_mix [B,H,W,M] / u_log [B,H,W,3] / masks (the
        head's dropout keep-masks in gated-resnet order) may be injected (parity); otherwise drawn on
        the device."""
        c, st = self.cfg, _lib.stream_ptr()
        self.vae.forward(x, target, eps, reg_coeff)
        tgt = self.vae._keep[1]
        B, D = c.batch, c.latent_dim
        z = self.vae.latent(_lib.BUF_Z, self.e)           # h = z_e  [B, Dz]
        prev = self.vae.xhat(self.e - 1).contiguous()     # the previous chain sample (no chain noise)
        um, ul = self._uniforms(u_mix, u_log)
        l = self.head.forward_train(tgt, z, dropout_p=self.dropout_p, masks=masks)
        M, HW = self.head.s["M"], c.height * c.width
        sample = torch.empty(B, c.height, c.width, 3, dtype=torch.float32, device=self.dev)
        _ck(self.L.svae_pcnn_sample(_p(l), _p(um), _p(ul), B, HW, M, _p(sample), 0, HW, 3, st))
        # highway (pixelvae.py:135-136): the 1-unit FC's pre-sigmoid output zl, then the mix
        ow, _, _ = self.head.table["highway/W"]
        ob, _, _ = self.head.table["highway/b"]
        zl = torch.empty(B, dtype=torch.float32, device=self.dev)
        _ck(self.L.svae_pcnn_gemm_small(_p(z), D, 0, _p(self.head.P, ow), 1, 0, _p(zl), 1, B, 1, D, 0.0, st))
        out = torch.empty_like(sample)
        ratio = torch.empty(B, dtype=torch.float32, device=self.dev)
        _ck(self.L.svae_pcnn_highway(_p(sample), _p(prev), _p(zl), _p(self.head.P, ob), B, 3 * HW, float(c.min_highway),
                                     float(c.max_highway), _p(out), _p(ratio), st))
        rec = torch.empty(B, dtype=torch.float32, device=self.dev)
        _ck(self.L.svae_pcnn_sqerr(_p(out), _p(tgt), B, 3 * HW, 0.0, _p(rec), None, st))
        self._fw = dict(tgt=tgt, z=z, prev=prev, um=um, ul=ul, l=l, sample=sample, zl=zl, out=out, ratio=ratio, rec=rec,
                        reg=float(reg_coeff))
        return out

    def _rec_coef(self):
        """The head step's MSE weight in self.loss: 16 (intermediate_reconstruction or the last step)."""
        return 16.0 if (self.cfg.intermediate_reconstruction or self.e == self.cfg.mc_steps - 1) else 0.0

    def loss_value(self):
        """self.loss (:1166-1176): the engine's steps (step 0 scaled by first_step_loss_coeff, KL only
        at the regularized steps) plus 16 * the head step's mean MSE."""
        return self.vae.loss_value() + self._rec_coef() * float(self._fw["rec"].double().mean())

    def recon(self, t):
        """mean_b recon_t (training_mles' MSE of step t)."""
        if t == self.e:
            return float(self._fw["rec"].double().mean())
        return float(self.vae.step_stats()[t, 0])

    def xhat(self, t):
        return self._fw["out"] if t == self.e else self.vae.xhat(t)

    def backward(self):
        """d self.loss / d every variable: the head's gradients in ``head.G``, the engine's in
        ``vae.grads``."""
        f, c, st = self._fw, self.cfg, _lib.stream_ptr()
        B, D, HW, M = c.batch, c.latent_dim, c.height * c.width, self.head.s["M"]
        dout = torch.empty_like(f["out"])
        _ck(self.L.svae_pcnn_sqerr(_p(f["out"]), _p(f["tgt"]), B, 3 * HW, self._rec_coef() / B, None, _p(dout), st))
        ds = torch.empty_like(dout)
        dprev = torch.empty_like(dout)
        dzl = torch.empty(B, dtype=torch.float32, device=self.dev)
        ob, _, _ = self.head.table["highway/b"]
        _ck(self.L.svae_pcnn_highway_bwd(_p(f["sample"]), _p(f["prev"]), _p(f["zl"]), _p(self.head.P, ob), B, 3 * HW,
                                         float(c.min_highway), float(c.max_highway), _p(dout), _p(ds), _p(dprev), 0,
                                         _p(dzl), st))
        dl = torch.empty(B * HW, 10 * M, dtype=torch.float32, device=self.dev)
        _ck(self.L.svae_pcnn_sample_bwd(_p(f["l"]), _p(f["um"]), _p(f["ul"]), B, HW, M, _p(ds), 3, _p(dl), st))
        dh = self.head.backward_from(dl)                  # head.G written; d / d h = d / d z_e
        ow, _, _ = self.head.table["highway/W"]
        # highway FC: dW [D][1] = z^T dzl, db = sum dzl, dz += dzl W^T
        _ck(self.L.svae_pcnn_gemm_small(_p(f["z"]), D, 1, _p(dzl), 1, 0, _p(self.head.G, ow), 1, D, 1, B, 0.0, st))
        _ck(self.L.svae_pcnn_sum(_p(dzl), B, _p(self.head.G, ob), None, st))
        _ck(self.L.svae_pcnn_gemm_small(_p(dzl), 1, 0, _p(self.head.P, ow), 1, 1, _p(dh), D, B, D, 1, 1.0, st))
        dz = torch.zeros(c.mc_steps, B, D, dtype=torch.float32, device=self.dev)
        dz[self.e].copy_(dh)
        self._ext = (dprev, dz)  # alive until the engine's backward has run
        _lib.check(self.L.svae_set_external_grads(self.vae.ctx, _p(dprev), _p(dz)), self.vae.ctx)
        self.vae.backward()

    def apply_gradients(self, lr=None, step=None):
        """One TF AdamOptimizer over every trainable variable (:1246-1276: clip +-10, the same step
        count), then the head's Polyak EMA (maintain_averages_op grouped with train_op, :1318-1320)."""
        lr = self.learning_rate if lr is None else lr
        step = self.vae._adam_step(step)
        self.vae.apply_gradients(lr, step)
        self.head.adam(lr, step=step, clip=self.cfg.clip_grad_value)
        self.head.ema_update(self.polyak_decay)

    # ------------------------------------------------------------------ reference API
    def init_pass(self, target, masks=None):
        """pixelcnn_cache['init_pass'] (:1360-1362): the head's data-dependent init on the ground
        truth and the current z_e (pixelvae.py:103-105: model(x_init, h_init, init=True, dropout_p))."""
        tgt = torch.as_tensor(target, dtype=torch.float32, device=self.dev).contiguous()
        z = self.vae.latent(_lib.BUF_Z, self.e)
        self.head.data_init(tgt, z, dropout_p=self.dropout_p, masks=masks)

    def train(self, input_batch, batch_target, eps=None, u_mix=None, u_log=None, masks=None, init_masks=None):
        """One iteration of SequentialVAE.train (:1341-1375) for c_pixelvae; returns final_loss / H / W
        (the head step's mean MSE per pixel)."""
        self.iteration += 1
        self.learning_rate *= self.cfg.learning_rate_decay
        self.vae.iteration = self.iteration
        reg = 1.0 - math.exp(-self.iteration / self.cfg.reg_coeff_rate)
        if self.init_every_step or not self.initialized:
            self.vae.forward(input_batch, batch_target, eps, reg)
            self.init_pass(batch_target, init_masks)
            self.initialized = True
        self.forward(input_batch, batch_target, eps, reg, u_mix, u_log, masks)
        self.backward()
        self.apply_gradients(self.learning_rate)
        return self.recon(self.e) / self.cfg.height / self.cfg.width

    def test(self, input_batch, u_mix=None, u_log=None):
        """training_mles[-1] for the batch (:1381-1391): the training branch, dropout included."""
        self.forward(input_batch, input_batch, None, 1.0, u_mix, u_log)
        return self._fw["out"].cpu().numpy()

    def generate_mc_samples(self, z=None, use_ema=True, seed=0):
        """generate_mc_samples (:1397-1428) with two_step_pixelvae (:1420-1422): the engine's
        generative chain for the steps before e, then sample_from_model (pixelvae.py:170-194) --
        the head's autoregressive raster loop on the EMA weights, conditioned on z_e -- mixed with
        the previous sample by the highway ratio.  z [T,B,Dz] or None (N(0,1))."""
        c = self.cfg
        if z is None:
            z = torch.randn(c.mc_steps, c.batch, c.latent_dim, device=self.dev)
        z = torch.as_tensor(z, dtype=torch.float32, device=self.dev).contiguous()
        xs = self.vae.generate(z)[:self.e]
        prev = xs[-1].contiguous()
        P0 = self.head.P.clone()
        if use_ema and self.head.ema is not None:
            self.head.P.copy_(self.head.ema)
        try:
            samp = self.head.sample(z[self.e], seed=seed)
            out, _ = self.head.highway(samp, prev, z[self.e], c.min_highway, c.max_highway)
        finally:
            self.head.P.copy_(P0)
        return [x.cpu().numpy() for x in xs] + [out.cpu().numpy()]
