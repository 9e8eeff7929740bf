"""Typed configuration of the Sequential-VAE path (replaces the netname if/elif chain).

Only the geometry / loss knobs of the executed path of the BASELINE configs are
modelled: sequential_vae.py:201-258 defaults plus the netname
overrides for ``c_inhomog`` (:727) / ``sequential_vae_celebA_inhomog`` (:671),
``sequential_vae_lsun`` (:712-714) and the MNIST ``m_*`` geometry (:842-848).
Unknown presets raise ``KeyError`` instead of ``exit(-1)`` (:860-862).
"""
import math
from dataclasses import dataclass, field, replace
from typing import List, Tuple

from . import _lib


@dataclass
class SVAEConfig:
    batch: int = 128
    height: int = 64
    width: int = 64
    channels: int = 3
    levels: int = 4                                   # vlae_levels (:204)
    filter_sizes: List[int] = field(default_factory=lambda: [3, 32, 64, 128, 384, 512])  # :209
    latent_dims: List[int] = field(default_factory=lambda: [3, 3, 3, 3])                 # :205
    mc_steps: int = 8                                 # :219
    intermediate_reconstruction: bool = True          # :221
    first_step_loss_coeff: float = 1.0                # :227
    latent_prior_stddev: float = 1.0                  # :232
    latent_mean_clip: float = math.inf                # :230
    range: Tuple[float, float] = (-1.0, 1.0)          # dataset.range (dataset_celeba.py:29)
    min_highway: float = 0.0                          # :244
    max_highway: float = 1.0                          # :243
    learning_rate: float = 2e-4                       # :253
    learning_rate_decay: float = 1.0                  # :252
    reg_coeff_rate: float = 5000.0                    # :254
    clip_grad_value: float = 10.0                     # :259
    # "fp32" (parity, fp32 MFMA) | "bf16" (bf16 MFMA, fp32 accumulate) | "bf16x6" (fp32-accurate on bf16
    # MFMA: operands split into bf16 planes, 6 plane products per gather-GEMM, 3 per weight-GEMM)
    dtype: str = "fp32"
    share_theta_weights: bool = False                 # :213 (homogeneous generator / encoder)
    share_phi_weights: bool = False                   # :214 (homogeneous recognition)
    predict_latent_code: bool = False                 # :225 (Latent InfoMax: q(z_t | x_{t-1}))
    predict_latent_code_with_regularization: bool = False  # :230
    regularized_steps: Tuple[int, ...] = None         # :220 (None = every step)
    # chain variants
    use_uniform_prior: bool = False                   # :232, KL = mean(-log sigma) (:1159-1160)
    add_noise_to_chain: bool = False                  # :233, sample = mle + reg*sd*N(0,1) (:1090)
    noise_stddevs: Tuple[float, ...] = None           # :239 (None = the reference's list)
    predict_generator_noise: bool = False             # :234, stddevs_prediction + NLL (:1147-1150)
    predict_generator_stddev_max: float = 1.0         # :236
    predict_generator_stddev_filter_sizes: Tuple[int, ...] = (5, 5, 5, 5, 5)  # :237-238
    add_improvement_maximization_loss: bool = False   # :227, own optimiser over phi (:1299-1316)
    latent_pred_loss_coeff: float = 0.001             # :253
    # c_pixelvae (generator = generator_pixelcnn, :535): steps t >= this run the PixelCNN++ head
    # (pixelvae.PixelVAE); the engine runs their recognition only.  0 = off
    external_generator_from: int = 0

    def noise_list(self):
        """noise_stddevs[t] per step (sequential_vae.py:239; the reference indexes noise_stddevs[step])."""
        if not self.add_noise_to_chain or self.predict_generator_noise:
            return [0.0] * self.mc_steps
        nd = self.noise_stddevs
        if nd is None:
            nd = [0.5 ** 1, 0.5 ** 2, 0.5 ** 3, 0.5 ** 4, 0.5 ** 5, 0.5 ** 6, 0.5 ** 7, 0.0]
        if len(nd) < self.mc_steps:
            raise ValueError("noise_stddevs needs mc_steps = %d entries" % self.mc_steps)
        return [float(v) for v in nd[:self.mc_steps]]

    @property
    def latent_dim(self):
        return int(sum(self.latent_dims))

    @property
    def image_sizes(self):
        return [self.height >> i for i in range(self.levels + 1)]

    def to_c(self):
        c = _lib.SvaeConfig()
        c.batch, c.height, c.width, c.channels = self.batch, self.height, self.width, self.channels
        c.levels, c.mc_steps = self.levels, self.mc_steps
        for i, f in enumerate(self.filter_sizes):
            c.filter_sizes[i] = f
        for i, d in enumerate(self.latent_dims):
            c.latent_dims[i] = d
        c.intermediate_reconstruction = int(self.intermediate_reconstruction)
        c.first_step_loss_coeff = self.first_step_loss_coeff
        c.latent_prior_stddev = self.latent_prior_stddev
        c.latent_mean_clip = self.latent_mean_clip
        c.range_lo, c.range_hi = self.range
        c.min_highway, c.max_highway = self.min_highway, self.max_highway
        c.dtype = {"fp32": 0, "bf16": 1, "bf16x6": 2}[self.dtype]
        c.share_theta, c.share_phi = int(self.share_theta_weights), int(self.share_phi_weights)
        c.predict_latent_code = int(self.predict_latent_code)
        c.predict_latent_code_with_regularization = int(self.predict_latent_code_with_regularization)
        unreg = 0
        if self.regularized_steps is not None:
            for t in range(self.mc_steps):
                if t not in self.regularized_steps:
                    unreg |= 1 << t
        c.unregularized_steps_mask[0], c.unregularized_steps_mask[1] = unreg & 0xFFFFFFFF, unreg >> 32
        c.use_uniform_prior = int(self.use_uniform_prior)
        c.add_noise_to_chain = int(self.add_noise_to_chain)
        for t, v in enumerate(self.noise_list()):
            c.noise_stddevs[t] = v
        c.predict_generator_noise = int(self.predict_generator_noise)
        c.predict_generator_stddev_max = self.predict_generator_stddev_max
        fs = list(self.predict_generator_stddev_filter_sizes)
        c.stddev_layers = len(fs)
        for i, f in enumerate(fs[:8]):
            c.stddev_filter_sizes[i] = f
        c.add_improvement_maximization_loss = int(self.add_improvement_maximization_loss)
        c.latent_pred_loss_coeff = self.latent_pred_loss_coeff
        c.external_generator_from = int(self.external_generator_from)
        return c

    def as_dict(self):
        """Plain-dict view (the layout the oracle's make_config produces)."""
        return dict(H=self.height, W=self.width, C=self.channels, levels=self.levels,
                    filter_sizes=list(self.filter_sizes), latent_dims=list(self.latent_dims),
                    mc_steps=self.mc_steps, batch=self.batch, range=tuple(self.range),
                    intermediate_reconstruction=self.intermediate_reconstruction,
                    first_step_loss_coeff=self.first_step_loss_coeff,
                    latent_prior_stddev=self.latent_prior_stddev, latent_mean_clip=self.latent_mean_clip,
                    min_highway=self.min_highway, max_highway=self.max_highway,
                    image_sizes=self.image_sizes, latent_dim=self.latent_dim,
                    share_theta=self.share_theta_weights, share_phi=self.share_phi_weights,
                    predict_latent_code=self.predict_latent_code,
                    predict_latent_code_with_regularization=self.predict_latent_code_with_regularization,
                    regularized_steps=self.regularized_steps,
                    use_uniform_prior=self.use_uniform_prior, add_noise_to_chain=self.add_noise_to_chain,
                    noise_stddevs=(self.noise_list() if self.add_noise_to_chain and not self.predict_generator_noise
                                   else None),
                    predict_generator_noise=self.predict_generator_noise,
                    predict_generator_stddev_max=self.predict_generator_stddev_max,
                    stddev_filter_sizes=tuple(self.predict_generator_stddev_filter_sizes),
                    add_improvement_maximization_loss=self.add_improvement_maximization_loss,
                    latent_pred_loss_coeff=self.latent_pred_loss_coeff,
                    external_generator_from=self.external_generator_from)

    def kl_on(self, t):
        """1 if step t's KL term enters self.loss (sequential_vae.py:1154, :1170-1172), else 0."""
        if self.regularized_steps is not None and t not in self.regularized_steps:
            return 0.0
        return 1.0 if (not self.predict_latent_code or self.predict_latent_code_with_regularization or t == 0) else 0.0


PRESETS = {
    "celeba": SVAEConfig(),
    "lsun": SVAEConfig(batch=256, latent_dims=[20, 30, 30, 30]),
    "mnist_1step": SVAEConfig(batch=64, height=32, width=32, channels=1, levels=3,
                              filter_sizes=[1, 64, 128, 192, 256], latent_dims=[8, 8, 8], mc_steps=1,
                              range=(0.0, 1.0)),
    "tiny": SVAEConfig(batch=4, height=32, width=32, channels=3, levels=4, filter_sizes=[3, 8, 8, 16, 24, 16],
                       latent_dims=[2, 2, 3, 2], mc_steps=3),
    # homogeneous chains (shared phi / theta across steps)
    "c_homog_v1": SVAEConfig(latent_dims=[12, 12, 12, 12], filter_sizes=[3, 16, 32, 64, 128, 384],
                             share_theta_weights=True, share_phi_weights=True),         # :316-321
    "c_homog_one_step": SVAEConfig(latent_dims=[12, 12, 12, 12], filter_sizes=[3, 16, 32, 64, 128, 384],
                                   share_theta_weights=True, share_phi_weights=True, mc_steps=1),  # :281-288
    # Latent InfoMax chains (:369-405)
    "c_homog_reg_pred_latent": SVAEConfig(latent_dims=[12, 12, 12, 12], filter_sizes=[3, 16, 32, 64, 128, 384],
                                          share_theta_weights=True, share_phi_weights=True, predict_latent_code=True,
                                          latent_mean_clip=32.0, predict_latent_code_with_regularization=True),
    "c_homog_no_reg_pred_latent": SVAEConfig(latent_dims=[12, 12, 12, 12], filter_sizes=[3, 16, 32, 64, 128, 384],
                                             share_theta_weights=True, share_phi_weights=True,
                                             predict_latent_code=True, regularized_steps=(0,), latent_mean_clip=32.0),
    "c_v2_coeff_change_abl": SVAEConfig(latent_dims=[12, 12, 12, 12], filter_sizes=[3, 16, 32, 64, 128, 384],
                                        share_theta_weights=True, share_phi_weights=True, predict_latent_code=True,
                                        regularized_steps=(0,), latent_mean_clip=32.0, first_step_loss_coeff=2.0),
    # chain variants
    "sequential_vae_celebA_inhomog_inf_max_uniform": SVAEConfig(predict_latent_code=True,
                                                                use_uniform_prior=True),          # :700-702
    "c_homog_no_reg_imp_max": SVAEConfig(latent_dims=[12, 12, 12, 12], filter_sizes=[3, 16, 32, 64, 128, 384],
                                         share_theta_weights=True, share_phi_weights=True, predict_latent_code=True,
                                         regularized_steps=(0,), add_improvement_maximization_loss=True,
                                         latent_mean_clip=32.0),                                    # :408-418
    "c_v2_diag_noise_abl": SVAEConfig(latent_dims=[12, 12, 12, 12], filter_sizes=[3, 16, 32, 64, 128, 384],
                                      share_theta_weights=True, share_phi_weights=True, predict_latent_code=True,
                                      regularized_steps=(0,), latent_mean_clip=32.0, add_noise_to_chain=True,
                                      predict_generator_noise=True),                                # :469-482
    "c_homog_imp_max_var_pred": SVAEConfig(latent_dims=[12, 12, 12, 12], filter_sizes=[3, 16, 32, 64, 128, 384],
                                           share_theta_weights=True, share_phi_weights=True,
                                           predict_latent_code=True, add_improvement_maximization_loss=True,
                                           latent_mean_clip=32.0, predict_latent_code_with_regularization=True,
                                           add_noise_to_chain=True, predict_generator_noise=True),  # :568-582
    # c_pixelvae (:529-543): shared theta / phi, T=2, step 1's generator is the PixelCNN++ head
    # (generator_pixelcnn :1943-1971 via pixelvae.make_pixel_cnn): the engine runs the recognition of
    # both steps and step 0's ladder generator (generator_first_step is still generator_ladder, :216)
    "c_pixelvae": SVAEConfig(latent_mean_clip=4.0, max_highway=0.8, min_highway=0.2, mc_steps=2,
                             learning_rate_decay=0.99999, latent_dims=[12, 12, 12, 12],
                             filter_sizes=[3, 16, 32, 64, 128, 384], share_theta_weights=True,
                             share_phi_weights=True, regularized_steps=(0,), first_step_loss_coeff=2.0,
                             external_generator_from=1),
    "tiny_homog": SVAEConfig(batch=4, height=32, width=32, channels=3, levels=4, filter_sizes=[3, 8, 8, 16, 24, 16],
                             latent_dims=[2, 2, 3, 2], mc_steps=3, share_theta_weights=True,
                             share_phi_weights=True),
}
# reference netnames that map onto the presets (sequential_vae.py:671, :712, :727)
NETNAMES = {"c_inhomog": "celeba", "sequential_vae_celebA_inhomog": "celeba", "sequential_vae_lsun": "lsun"}


def preset(name, **over):
    name = NETNAMES.get(name, name)
    return replace(PRESETS[name], **over)
