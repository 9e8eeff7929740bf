/* libsvae_hip.so — C ABI of the MI355X Sequential-VAE training-step engine.
 *
 * Drop-in boundary.  The reference has no FFI: its path sits
 * behind the Python methods
 *     SequentialVAE.train(input_batch, batch_target) -> float   sequential_vae.py:1341-1375
 *     SequentialVAE.test(input_batch) -> ndarray[B,H,W,C]        sequential_vae.py:1381-1391
 * which run  sess.run([train_op, loss, final_loss])  (sequential_vae.py:1365) over the
 * graph built by construct_network (sequential_vae.py:877-984).  The Python mirror of that
 * interface (sequential-variational-autoencoder_amd/sequential_vae.py) binds the entry points
 * below through ctypes; the binding a maintainer would add is shown in INTEGRATION.md.
 *
 * Conventions: every function returns 0 on success or a negative svae_status; the
 * message is available from svae_last_error(ctx) (ctx may be NULL for create/layout
 * errors).  No function calls exit().  All device work is enqueued on the caller's
 * stream (hipStream_t passed as void*); no call allocates or synchronises on the hot
 * path.  Tensors are NHWC fp32, row-major.
 */
#ifndef SVAE_HIP_H
#define SVAE_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum svae_status {
  SVAE_OK = 0,
  SVAE_EBADCONFIG = -1, /* config rejected (sequential_vae.py:861-862, :1617-1627 analogue) */
  SVAE_EBADARG = -2,    /* null pointer / unbound buffers / bad index */
  SVAE_EHIP = -3,       /* HIP runtime error */
  SVAE_ENOMEM = -4      /* device allocation failed */
};

/* Geometry + hyper-parameters of one SequentialVAE (sequential_vae.py:201-258, netname
 * overrides :281-862).  Only the executed-path knobs of the BASELINE configs. */
typedef struct svae_config {
  int32_t batch;            /* per-GPU batch B (BN statistics are per shard) */
  int32_t height, width, channels;   /* dataset.data_dims */
  int32_t levels;           /* vlae_levels L */
  int32_t mc_steps;         /* T */
  int32_t filter_sizes[10]; /* L+2 entries */
  int32_t latent_dims[8];   /* L entries */
  int32_t intermediate_reconstruction;
  float first_step_loss_coeff;
  float latent_prior_stddev;
  float latent_mean_clip;   /* +inf = no clip */
  float range_lo, range_hi; /* dataset.range */
  float min_highway, max_highway;
  int32_t dtype;            /* 0 = fp32 (parity, fp32 MFMA); 1 = bf16 MFMA, fp32 accumulate (throughput);
                             * 2 = bf16x6: fp32-accurate on bf16 MFMA (operands split into bf16 planes,
                             * 6 plane products in the forward / input-gradient GEMMs, 3 in the
                             * weight-gradient GEMMs; fp32 storage) */
  /* homogeneous chain (sequential_vae.py:107-113, scopes :1573-1577, :1683-1687, :1757-1761):
   * share_phi: one "phi/inference_network" for every step; share_theta: one
   * "theta/generative_encoder_network" and one "theta/generative_network" for steps >= 1
   * ("theta/generative_step_0" stays its own).  The parameter table then lists each shared
   * tensor once and its gradient is the sum over the steps that use it. */
  int32_t share_theta, share_phi;
  /* Latent InfoMax (predict_latent_code :129-131, create_recognition_network :1013-1020):
   * q(z_t | x_{t-1}) for t >= 1 (gradient flows into x_{t-1}); the KL term only at step 0
   * unless predict_latent_code_with_regularization (:1170-1172).  Under share_phi step 0 keeps
   * its own "phi/inference_step_0" (:1573). */
  int32_t predict_latent_code, predict_latent_code_with_regularization;
  /* regularized_steps (:220, :1154): bit t set = step t carries NO KL term (0 = every step) */
  uint32_t unregularized_steps_mask[2];
  /* ---- chain variants ---- */
  int32_t use_uniform_prior;          /* KL_b = mean_d(-log sigma) (:1159-1160) */
  /* add_noise_to_chain (:1088-1090): the sample fed to step t+1 is mle_t + reg * sd_t * N(0,1);
   * sd_t = noise_stddevs[t] (:1665-1666), or predicted (below).  The loss keeps the MLE. */
  int32_t add_noise_to_chain;
  float noise_stddevs[64];            /* mc_steps entries (:239) */
  /* predict_generator_noise (:1667, stddevs_prediction :1866-1875): sd_t = max * sigmoid(1x1 conv of
   * stddev_layers x conv2d_bn_lrelu(4x4, s1) of the output conv-T's sigmoid); the reconstruction
   * term becomes the Gaussian NLL mean(log sd + 0.5 log 2pi + 0.5 ((mle - target)/sd)^2) (:1149-1150).
   * Requires add_noise_to_chain.  Filter sizes <= 8 (reference default 5 x 5). */
  int32_t predict_generator_noise;
  float predict_generator_stddev_max;
  int32_t stddev_layers;
  int32_t stddev_filter_sizes[8];
  /* add_improvement_maximization_loss (:1182-1201): imp = reg * latent_pred_loss_coeff *
   * -mean_b sum_{t>=1} ||mle_t - mle_{t-1}||^2, minimised over the recognition variables only by its
   * own clip + Adam update (:1299-1316): svae_backward_imp / svae_adam_imp. */
  int32_t add_improvement_maximization_loss;
  float latent_pred_loss_coeff;
  /* External generator (c_pixelvae, :529-543; generator_pixelcnn :1943-1971): steps t >= this run
   * the caller's generator (the PixelCNN++ head of svae_pcnn.h); the engine runs only their
   * recognition (z_t, KL_t) and creates no encoder / generator variables for them.  The caller hands
   * d loss / d x_hat_{e-1} and d loss / d z_t back with svae_set_external_grads.  0 = off. */
  int32_t external_generator_from;
} svae_config;

typedef struct svae_param_desc {
  char name[96];            /* TF variable name, e.g. "phi/inference_step_0/Conv/weights" */
  int32_t ndim;
  int32_t shape[4];         /* TF shape: conv [kh,kw,Cin,Cout], conv-T [kh,kw,Cout,Cin], FC [in,out] */
  int64_t offset;           /* element offset in the flat parameter / gradient buffers */
  int32_t init;             /* 0 zeros, 1 normal(0,0.02), 2 glorot-uniform */
  int32_t flags;            /* bit0: dead (never on the executed path), bit1: gradient identically 0 */
} svae_param_desc;

typedef struct svae_ctx svae_ctx;

/* Buffers readable through svae_copy_out. */
enum svae_buffer {
  SVAE_BUF_XHAT = 0,     /* training_mles[t]  [B,H,W,C] (sequential_vae.py:962) */
  SVAE_BUF_MU = 1,       /* latent mean (pre-clip) [B,Dz] */
  SVAE_BUF_SIGMA = 2,    /* latent stddev [B,Dz] */
  SVAE_BUF_Z = 3,        /* latent sample [B,Dz] */
  SVAE_BUF_STEP_STATS = 4, /* [T][2] = (mean_b recon_t, mean_b KL_t)   (:1163-1164) */
  SVAE_BUF_REC_IMG = 5,  /* [B] per-image recon of step t */
  SVAE_BUF_KL_IMG = 6,   /* [B] per-image KL of step t */
  SVAE_BUF_DZ = 7,       /* [B,Dz] d loss / d z_t (after svae_backward) */
  SVAE_BUF_SAMPLE = 8,   /* training_samples[t] [B,H,W,C] (= the MLE without chain noise, :963) */
  SVAE_BUF_STDDEV = 9,   /* predicted stddevs [B,H,W,1] of step t (predict_generator_noise) */
  SVAE_BUF_IMP_IMG = 10  /* [B] ||mle_t - mle_{t-1}||^2 per image (improvement loss, t >= 1) */
};

/* Hash (16 hex digits) of the sources this library was compiled from (build.py src_hash); the
 * Python mirror refuses a library whose hash differs from its tree's.  No reference counterpart. */
const char* svae_build_hash(void);

/* Parameter table (pure host; callable without a GPU).  Live (trainable, non-zero-grad)
 * tensors occupy [0, n_live); dead / pre-BN-bias tensors the tail [n_live, n_total). */
int svae_param_count(const svae_config* cfg, int64_t* n_total, int64_t* n_live, int32_t* n_tensors);
int svae_param_layout(const svae_config* cfg, svae_param_desc* out, int32_t cap);

/* Context: owns the activation arena (sized for cfg->batch) and Adam state. */
int svae_create(const svae_config* cfg, int device, svae_ctx** out);
int svae_destroy(svae_ctx* ctx);
const char* svae_last_error(const svae_ctx* ctx);
/* Borrow caller-owned flat fp32 buffers (n_total elements each). */
int svae_bind(svae_ctx* ctx, float* params, float* grads);
int64_t svae_workspace_bytes(const svae_ctx* ctx);

/* Forward of the whole chain: x, target [B,H,W,C]; eps [T,B,Dz] or NULL (device Philox).
 * reg_coeff as fed at sequential_vae.py:1357. */
int svae_forward(svae_ctx* ctx, const float* x, const float* target, const float* eps, float reg_coeff,
                 void* stream);
/* d self.loss / d every variable (sequential_vae.py:1273) into the bound gradient buffer. */
/* Generative mode (sequential_vae.py:947-952 / :1025 / generate_mc_samples :1393-1428): run the
 * unrolled generator chain on latents z [T,B,Dz] fp32 (device; NULL = N(0,1) drawn on device),
 * without the recognition networks: x_0 = generator_first_step(z_0), x_t = generator(x_{t-1}, z_t),
 * BatchNorm on the generated batch's statistics (training mode, as the reference's shared
 * variables).  Outputs via svae_copy_out(SVAE_BUF_XHAT, t).  Invalidates the training forward
 * state (svae_backward needs a new svae_forward). */
int svae_generate(svae_ctx* ctx, const float* z, void* stream);
int svae_backward(svae_ctx* ctx, void* stream);
/* external_generator_from = e: gradients from the caller's generator steps for the NEXT backward
 * (device pointers, one-shot): dxhat [B,H,W,C] = d loss / d x_hat_{e-1} (the chain sample the
 * external step reads, e.g. the PixelVAE highway's previous sample, pixelvae.py:136), dz [T,B,Dz]
 * whose rows t >= e are d loss / d z_t (the head's conditioning and highway ratio, :123-136); the
 * KL terms' gradients are the engine's own.  NULL = zero. */
int svae_set_external_grads(svae_ctx* ctx, const float* dxhat, const float* dz);
/* Chain noise N(0,1) [T,B,H,W,C] for the NEXT svae_forward or svae_generate only (device pointer,
 * kept by reference until that call's backward; NULL or not set = drawn on device, as
 * tf.random_normal :1090-1091).  One-shot: every forward / generate call clears it, so a generative
 * chain never reuses the noise injected for an earlier training forward. */
int svae_set_chain_noise(svae_ctx* ctx, const float* noise);
/* Improvement-maximisation loss (add_improvement_maximization_loss): bind a caller-owned gradient
 * buffer (n_total elements, public layout), then after svae_forward, svae_backward_imp writes
 * d imp / d every variable into it (the optimiser uses only the recognition part, :1302).
 * svae_adam_imp applies clip + Adam to the recognition variables [0, phi_end) with that gradient and
 * the same Adam moments (one AdamOptimizer, :1267); *phi_end from svae_imp_range. */
int svae_bind_imp(svae_ctx* ctx, float* grads_imp);
int svae_backward_imp(svae_ctx* ctx, void* stream);
int svae_adam_imp(svae_ctx* ctx, float lr, int64_t step, float clip, void* stream);
int svae_imp_range(svae_ctx* ctx, int64_t* phi_end);
/* Data-parallel hook (no reference counterpart; the reference has no collective).  During
 * svae_backward, hook(user, t) is called on the host after the backward of chain step t is
 * enqueued (t = T-1 .. 0): at that point svae_hook_stream(ctx) is ordered after every kernel of
 * that step, so a collective enqueued on it reduces the step's complete generator/encoder
 * gradients while the earlier steps' backward still runs.  hook(user, -1) follows the whole
 * backward (recognition gradients complete, on the caller's stream).  NULL hook: off. */
typedef void (*svae_step_hook)(void* user, int t);
int svae_set_backward_hook(svae_ctx* ctx, svae_step_hook hook, void* user);
void* svae_hook_stream(svae_ctx* ctx);
/* clip(+-clip) + TF Adam on the live region (sequential_vae.py:1274-1276); step >= 1.  In bf16
 * mode (no weight sharing) the update also refreshes the engine's bf16 weight copies, and the next
 * svae_forward reuses them when the updates since the last forward covered the whole live region.
 * Parameters the caller writes itself must be announced with svae_bind before the next forward. */
int svae_adam(svae_ctx* ctx, float lr, int64_t step, float clip, void* stream);
/* The same update on the live sub-range [lo, hi) (lo a multiple of 4; tensor-aligned ranges). */
int svae_adam_range(svae_ctx* ctx, int64_t lo, int64_t hi, float lr, int64_t step, float clip, void* stream);
/* svae_backward then svae_adam as one call (sess.run(train_op), sequential_vae.py:1365), bit for bit
 * the same parameters: each chain step's generator/encoder bucket is updated on the engine's side
 * stream as soon as its gradient is final, right after hook(user, t) -- a hook that exchanges
 * gradients must have made svae_hook_stream(ctx) wait for the exchange of that bucket before it
 * returns -- and the recognition bucket after hook(user, -1).  Shared weights: the two calls in
 * sequence. */
int svae_backward_adam(svae_ctx* ctx, float lr, int64_t step, float clip, void* stream);
/* Adam moments of the live region [0, n_live) (tf.train.Saver's "<var>/Adam", "<var>/Adam_1" slots,
 * abstract_network.py:124-152): dir 0 copies them out to m, v; dir 1 in.  Device pointers. */
int svae_adam_state(svae_ctx* ctx, int dir, float* m, float* v, int64_t n, void* stream);
/* Copy an internal buffer (device -> caller device pointer). */
int svae_copy_out(svae_ctx* ctx, int which, int step, float* dst, int64_t n, void* stream);

/* Launch probe (instrumentation, no reference counterpart): between begin and end, every
 * launch of the bf16 GEMM instance `kernel_id` (see svae_kernel_name) issued by forward /
 * backward is bracketed by an event pair on the launch stream.  end() synchronises those
 * events and returns the launch count, the number timed (<= max_launches), their summed
 * algorithmic FLOPs and summed duration in ms.  Used by bench.py for roofline.achieved. */
int svae_probe_begin(svae_ctx* ctx, int kernel_id, int max_launches);
int svae_probe_end(svae_ctx* ctx, int64_t* launches, int64_t* timed, double* flops, double* total_ms);
const char* svae_kernel_name(int kernel_id);

/* ---- per-op entry points (kernel-level parity tests) ---- */
/* TF-SAME conv2d (transpose=0, W [4,4,Cin,Cout]) or conv2d_transpose (transpose=1,
 * W [4,4,Cout,Cin]) forward on x [N,H,H,Cin]; stride 1|2. */
int svae_op_conv(const float* x, int n, int h, int cin, const float* w, int cout, int stride, int transpose,
                 float* y, void* stream);
/* input gradient and weight gradient of the same op */
/* bf16 gather-GEMM (throughput mode kernels): y = conv2d (transpose=0) or conv2d_transpose
 * (transpose=1) of fp32 NHWC x with bf16 weights already in the engine's NK shadow layout
 * w_nk[tap][cout][cin] (tap = ky*4+kx); x is rounded to bf16 while staged, fp32 accumulate.
 * path: 0 per-tap gather kernel, 1 halo-tile kernel (SVAE_EBADARG if the shape does not
 * qualify), 2 automatic.  scratch (optional) enables split-K.  path | 16: the split-bf16 mode
 * (dtype bf16x6): w_nk holds three planes of 16*cin*cout elements each (x = p0 + p1 + p2); path | 48:
 * two more planes follow, the scaled fp16 pair fp16(w * 2^10), fp16(w * 2^10 - h0) that the
 * wave-split gathers use in that mode. */
int svae_op_gather_bf16(const float* x, int n, int h, int cin, const void* w_nk, int cout, int stride, int transpose,
                        int path, float* y, void* scratch, int64_t scratch_bytes, void* stream);
/* bf16 weight gradient of a conv (transpose=0) / conv-T (transpose=1) layer: dw in TF layout
 * ([4,4,cin,cout] / [4,4,cout,cin]) from fp32 NHWC x and dy, operands rounded to bf16, fp32
 * accumulation.  path: 0 tap-merged weight-GEMM kernel, 2 halo weight-GEMM where it qualifies;
 * + 16: x is a bf16 tensor, + 32: dy is a bf16 tensor (the engine's bf16 activation / BN-backward
 * storage, opload.h).  scratch: split slab (required). */
int svae_op_wgrad_bf16(const float* x, int n, int h, int cin, const float* dy, int cout, int stride, int transpose,
                       int path, float* dw, void* scratch, int64_t scratch_bytes, void* stream);
int svae_op_conv_dgrad(const float* dy, int n, int h, int cin, const float* w, int cout, int stride, int transpose,
                       float* dx, void* stream);
int svae_op_conv_wgrad(const float* x, int n, int h, int cin, const float* dy, int cout, int stride, int transpose,
                       float* dw, void* scratch, int64_t scratch_bytes, void* stream);
/* training BN (+act 0 none,1 relu,2 lrelu) over rows of x [rows,C].
 * scratch: >= 1032*c bytes (sharded fixed-point column accumulators + constants); bwd: >= 1024*c bytes */
int svae_op_bn_act(const float* x, int64_t rows, int c, const float* beta, int act, float* y, float* mean,
                   float* invstd, void* scratch, int64_t scratch_bytes, void* stream);
int svae_op_bn_act_bwd(const float* dy, const float* y, const float* x, int64_t rows, int c, const float* mean,
                       const float* invstd, int act, float* dx, float* dbeta, void* scratch, int64_t scratch_bytes,
                       void* stream);
/* y[B,N] = x[B,K] @ w[K,N]  (fully_connected, no bias) */
int svae_op_fc(const float* x, int b, int k, const float* w, int nout, float* y, void* stream);

#ifdef __cplusplus
}
#endif
#endif
