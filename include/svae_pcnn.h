/* PixelCNN++ decoder head: C ABI of the MI355X kernels.
 *
 * Replaces the TF graph that pixel_cnn/pixelvae.py:68-158 builds over
 * pixel_cnn/pixel_cnn_pp/model.py:11-117 and nn.py:46-320 (every op below cites the reference
 * function it computes).  Plain pointers (device memory), sizes and a hipStream_t passed as
 * void*; every tensor is NHWC fp32 with an explicit pixel stride (ld, in elements).
 *
 * Convolution geometry (one gather rule for every conv / deconv and their input gradients):
 *   mode 0 (conv):       out(oy, ox) += in(oy*s - pt + ky, ox*s - pl + kx) . W[ky][kx]
 *   mode 1 (transposed): out(oy, ox) += in(iy, ix) . W[ky][kx]  where  iy*s + ky = oy + pt,
 *                                                                      ix*s + kx = ox + pl
 * Out-of-image sources read zero.  nn.down_shifted_conv2d = mode 0, pt = kh-1, pl = (kw-1)/2;
 * nn.down_right_shifted_conv2d: pt = kh-1, pl = kw-1; nn.down_shifted_deconv2d (stride 2, VALID,
 * cropped): mode 1, pt = 0, pl = (kw-1)/2.  The input gradient of a mode-m op is the mode-(1-m)
 * op with the same s, pt, pl over the output gradient and the transposed weight copy.
 *
 * Weights: canonical V [kh][kw][Cin][Cout] fp32 (nn.py's weight norm W = g V / ||V||, the norm
 * over all axes but Cout).  svae_pcnn_wnorm writes the two bf16 copies the bf16-MFMA kernels read:
 *   wk_f [tap][Cout][kf]  (forward: K = Cin contiguous, zero-padded to kf = roundup(Cin, 16))
 *   wk_d [tap][Cin][kd]   (input gradient: K = Cout contiguous, kd = roundup(Cout, 16))
 * Returns 0 on success, a negative SVAE_E* code on bad arguments (message: svae_last_error of a NULL context).
 */
#ifndef SVAE_PCNN_H
#define SVAE_PCNN_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* nn.conv2d / deconv2d / dense weight norm (nn.py:173, :201, :236): norm[co] = ||V[..,co]||,
 * W = g / norm * V into both bf16 copies (either may be NULL). */
int svae_pcnn_wnorm(const float* V, const float* g, int taps, int cin, int cout, float* norm, void* wk_f, int kf,
                    void* wk_d, int kd, void* stream);
/* weight-norm backward: dW [tap][Cin][Cout] -> dg[co] = sum dW . V / norm,
 * dV = g / norm (dW - dg V / norm)  (written, not accumulated). */
int svae_pcnn_wnorm_bwd(const float* V, const float* g, const float* norm, const float* dW, int taps, int cin,
                        int cout, float* dV, float* dg, void* stream);

/* gather conv (bf16 MFMA, fp32 accumulate): y[rows][ldy] (rows = n*ho*wo) = gather(x) . wk
 * (+ bias); wk [tap][cout][kpad]; accumulate: y += result; zero_edge 1 / 2: output row oy == 0 /
 * column ox == 0 written as 0 (nn.down_shift / right_shift folded in: pass pt + 1 / pl + 1).
 * x is fp32, or bf16 with x_bf16 = 1 (cin, ldx multiples of 8): the MFMA operand precision, so a
 * bf16 x gives bitwise the result of its fp32 source.  Stride-1 launches whose rows fill 256-row
 * blocks of whole image rows (or whole images) run the halo-window kernel, the rest pc_conv2. */
int svae_pcnn_conv(const void* x, int n, int hi, int wi, int cin, int ldx, int x_bf16, const void* wk, int kpad,
                   const float* bias, float* y, int ho, int wo, int cout, int ldy, int kh, int kw, int s, int pt,
                   int pl, int mode, int accumulate, int zero_edge, void* stream);
/* the input gradient of a conv whose input is a resnet nonlinearity's output t = f(src) . mask
 * (kind 0 relu, 1 elu; mask as svae_pcnn_nonlin: given, or drawn from keep / seed): the mode-(1-m)
 * gather of dy (fp32, the transposed weight copy wk) with dsrc (+)= result . mask . f'(src) written
 * in the epilogue -- d t and the nonlinearity's backward pass are never materialised.  src [rows][lds],
 * rows = n*ho*wo of the gather's output space (= t's pixels). */
int svae_pcnn_conv_act_bwd(const float* dy, int n, int hi, int wi, int cin, int lddy, const void* wk, int kpad,
                           float* dsrc, int ho, int wo, int cout, int ldd, int kh, int kw, int s, int pt, int pl, int mode,
                           int accumulate, const float* src, int lds, int kind, const float* mask, float keep,
                           uint64_t seed, void* stream);
/* weight gradient of that conv: dW[tap][cin][cout] = sum_rows gather(x)[row][ci] . dy[row][co]
 * (split over rows into `scratch` slabs, then a fixed-order reduce: deterministic); x fp32 or bf16
 * (x_bf16 = 1), dy fp32 or bf16 (dy_bf16 = 1).  dbias (may be NULL, fp32 dy only): the bias gradient
 * sum_rows dy[row][co], written, from the same pass over dy (fp32 sums). */
int svae_pcnn_conv_wgrad(const void* x, int n, int hi, int wi, int cin, int ldx, int x_bf16, const void* dy, int ldd,
                         int dy_bf16, int ho, int wo, int cout, int kh, int kw, int s, int pt, int pl, int mode, float* dW,
                         float* dbias, float* scratch, int64_t scratch_elems, void* stream);
/* ---- split mode (fp32-grade head, pixelvae dtype "bf16x6"): operands as sums of 16-bit planes ----
 * Two plane formats replace the fp32 tf.nn.conv2d / conv2d_transpose / matmul of nn.py:189-252:
 *  - fp16 (h16_scale / x_scale / w_scale given, planes = 2): a tensor scaled by 2^s (s: max|v| 2^s in
 *    [2^14, 2^15), computed on the device) as h0 = fp16(v 2^s), h1 = fp16(v 2^s - h0): 22 significant
 *    bits; a product is h0.h0' + h0.h1' + h1.h0' (3 fp16-MFMA launches) times 2^-(s + s').  A scale
 *    buffer is 2 floats: [0] <- 2^-s, [1] scratch (max|v|).  Needs 16-bit storage (channels % 8 == 0).
 *  - bf16 (no scales, planes 1..3): p_k = bf16 of what p_0..p_{k-1} left of v (8 bits per plane); a
 *    product is the sum over i + j < planes of x_i . w_j (3 planes: 6 launches, fp32-grade).  Any shape.
 * Every launch is one of the bf16 / fp16-MFMA kernels above (fp32 accumulate), largest product first.
 * svae_pcnn_wnorm_planes: svae_pcnn_wnorm writing `planes` planes per copy (plane p of wk_f at
 *   p * taps*cout*kf, of wk_d at p * taps*cin*kd); h16_scale: the fp16 format (planes = 2). */
int svae_pcnn_wnorm_planes(const float* V, const float* g, int taps, int cin, int cout, float* norm, void* wk_f,
                           int kf, void* wk_d, int kd, int planes, float* h16_scale, void* stream);
/* x [rows][ldx] fp32 -> planes [rows][ldo] at plane stride rows*ldo: bf16 (out_bf16 = 1) or fp32 (the last
 * fp32 plane keeps the exact remainder, which the consuming kernel rounds to bf16); h16_scale: the two
 * scaled fp16 planes (planes = 2, out_bf16 = 1: 16-bit storage). */
int svae_pcnn_split_planes(const float* x, int64_t rows, int c, int ldx, int planes, void* out, int ldo, int out_bf16,
                           float* h16_scale, void* stream);
/* the fp16 format's split with max|x| already in h16_scale[1] (svae_pcnn_nonlin_absmax wrote it). */
int svae_pcnn_split_h16_premax(const float* x, int64_t rows, int c, int ldx, void* out, int ldo, float* h16_scale,
                               void* stream);
/* svae_pcnn_conv over plane operands: x planes at x_pstride elements apart (fp32, or 16-bit with x_bf16),
 * wk `planes` planes of [tap][cout][kpad]; x_scale / w_scale (both or neither): the fp16 format. */
int svae_pcnn_conv_planes(const void* x, int n, int hi, int wi, int cin, int ldx, int x_bf16, int64_t x_pstride,
                          const void* wk, int kpad, int planes, const float* x_scale, const float* w_scale,
                          const float* bias, float* y, int ho, int wo, int cout, int ldy, int kh, int kw, int s, int pt,
                          int pl, int mode, int accumulate, int zero_edge, void* stream);
/* svae_pcnn_conv_wgrad over plane operands (x planes x_pstride apart, dy planes dy_pstride apart; x_scale /
 * dy_scale: the fp16 format): every product's partial slabs go to scratch and one fixed-order reduce
 * writes dW.  No bias gradient (its column sum is svae_pcnn_colsum of the fp32 dy). */
int svae_pcnn_conv_wgrad_planes(const void* x, int n, int hi, int wi, int cin, int ldx, int x_bf16, int64_t x_pstride,
                                const void* dy, int ldd, int dy_bf16, int64_t dy_pstride, int planes,
                                const float* x_scale, const float* dy_scale, int ho, int wo, int cout, int kh, int kw,
                                int s, int pt, int pl, int mode, float* dW, float* scratch, int64_t scratch_elems,
                                void* stream);
/* column sums over rows (bias gradients): out[c] (+)= sum_r x[r][c]; mask_edge 1 / 2 skips
 * rows with oy == 0 / ox == 0 of a [n][ho][wo] row space (the zeroed shifted outputs). */
int svae_pcnn_colsum(const float* x, int64_t rows, int c, int ldx, int ho, int wo, int mask_edge, float* out,
                     int accumulate, float* scratch, void* stream);
/* The split mode's gradient operand prologue in one pass over x (fp32 [rows][c], ld ldx): its column sums into
 * out (as svae_pcnn_colsum, mask_edge 0: bitwise) and max|x| into h16_scale[1] (as the absmax pass of
 * svae_pcnn_split_planes), after which svae_pcnn_split_h16_premax writes the two fp16 planes. */
int svae_pcnn_colsum_absmax(const float* x, int64_t rows, int c, int ldx, float* out, int accumulate, float* scratch,
                            float* h16_scale, void* stream);
/* im2col of a stride-1 mode-0 conv input x ([n][hi][wi][cin], ld ldx, fp32) as the two scaled fp16 planes of a
 * [n*ho*wo][kc] operand (planes kc * rows elements apart; h16_scale as svae_pcnn_split_planes: [2^-s, max|x|]):
 * column (ky * kw + kx) * cin + ci holds x at (oy - pt + ky, ox - pl + kx), 0 outside the image and for columns
 * >= kh * kw * cin.  The conv is then the 1x1 svae_pcnn_conv_planes over it with the [1][cout][kc] weight copy
 * of V viewed as [kh * kw * cin][cout] (svae_pcnn_wnorm_planes with taps 1). */
int svae_pcnn_im2col_h16(const float* x, int n, int hi, int wi, int cin, int ldx, int ho, int wo, int kh, int kw, int pt,
                         int pl, void* out, int kc, float* h16_scale, void* stream);
/* svae_pcnn_conv_planes that also leaves max |y| (after the accumulate) in y_scale[1]: the bound the consuming
 * svae_pcnn_nonlin_h16 takes. */
int svae_pcnn_conv_planes_amax(const void* x, int n, int hi, int wi, int cin, int ldx, int x_bf16, int64_t x_pstride,
                               const void* wk, int kpad, int planes, const float* x_scale, const float* w_scale,
                               const float* bias, float* y, int ho, int wo, int cout, int ldy, int kh, int kw, int s,
                               int pt, int pl, int mode, int accumulate, int zero_edge, float* y_scale, void* stream);
/* svae_pcnn_nonlin with the dropout (a mask tensor [rows][cy] whose largest value is mask_max, or, mask NULL,
 * the in-kernel one of keep, seed; keep 1: none) writing y only as the two scaled fp16 planes [2][rows][ldo] of
 * the consuming conv (planes rows * ldo elements apart), at the exponent of a bound on max |y| known before the
 * pass: x_scale[1] (= max |x|, from x's producer; at least 1 for elu / concat_elu) times the dropout's largest
 * factor.  h16_scale <- [2^-s, the bound].  Needs c, ldx, ldo % 4 == 0, 16-B x and mask, 8-B out. */
int svae_pcnn_nonlin_h16(const float* x, int64_t rows, int c, int ldx, int kind, const float* mask, float mask_max,
                         float keep, uint64_t seed, const float* x_scale, void* out, int ldo, float* h16_scale,
                         void* stream);
/* zero the rows / columns a zero_edge conv wrote as 0 (its output gradient there is dead). */
int svae_pcnn_mask_edge(float* x, int n, int ho, int wo, int c, int ldx, int mask_edge, void* stream);

/* resnet nonlinearity (model.py:24-31): kind 0 relu, 1 elu, 2 concat_elu (y has 2c channels
 * [elu(x), elu(-x)], nn.py:12-15), times the training pass's dropout keep-mask (nn.py:273-274):
 * mask [rows][cy] holding 1 / keep_prob or 0 (cy = y's channels), or, with mask NULL and keep < 1,
 * the mask svae_pcnn_dropout_mask(rows * cy, keep, seed) writes, drawn inside the kernel; keep >= 1
 * and no mask: none.  y fp32 or bf16 (y_bf16 = 1: for a consumer that reads it as a bf16 MFMA
 * operand).  Dropout or a bf16 y needs c, ldx, ldy multiples of 4 and 16-B aligned rows. */
int svae_pcnn_nonlin(const float* x, int64_t rows, int c, int ldx, int kind, const float* mask, float keep,
                     uint64_t seed, void* y, int ldy, int y_bf16, void* stream);
/* svae_pcnn_nonlin with fp32 y that also leaves max|y| in h16_scale[1] (the split mode's scale of the
 * conv input y, for svae_pcnn_split_h16_premax).  Needs the aligned 4-channel rows of dropout. */
int svae_pcnn_nonlin_absmax(const float* x, int64_t rows, int c, int ldx, int kind, const float* mask, float keep,
                            uint64_t seed, float* y, int ldy, float* h16_scale, void* stream);
/* its backward: dx (+)= f'(x) . (dy . mask), the mask given or drawn as in the forward.  dx fp32, or
 * bf16 (dx_bf16 = 1: a gradient read only as a bf16 MFMA operand); dsum (may be NULL): the column
 * sums of the written gradient over all rows, fp32 (a conv's bias gradient), from the same pass
 * (scratch: ceil(rows / 64) * c floats).  bf16 / dsum: kinds 0 / 1, accumulate = 0, aligned rows. */
int svae_pcnn_nonlin_bwd(const float* x, int64_t rows, int c, int ldx, int kind, const float* mask, float keep,
                         uint64_t seed, const float* dy, int ldy, void* dx, int lddx, int dx_bf16, int accumulate,
                         float* dsum, float* scratch, void* stream);
/* the seeded dropout keep-mask: out[i] = 1 / keep with probability keep, else 0 (splitmix64 of
 * seed + i, 24-bit uniform), i < n -- what the two calls above draw for a NULL mask. */
int svae_pcnn_dropout_mask(int64_t n, float keep, uint64_t seed, float* out, void* stream);

/* gated_resnet tail (nn.py:283-288): with c2 = [a | b] (2f channels) + hp[img] (h . hw):
 * out = x + a . sigmoid(b). */
int svae_pcnn_gate(const float* x, int ldx, const float* c2, const float* hp, int64_t rows, int pix_per_img, int f,
                   float* out, int ldo, void* stream);
/* svae_pcnn_gate leaving max |out| in out_scale[1] (the bound svae_pcnn_nonlin_h16 takes for out's planes). */
int svae_pcnn_gate_amax(const float* x, int ldx, const float* c2, const float* hp, int64_t rows, int pix_per_img, int f,
                        float* out, int ldo, float* out_scale, void* stream);
/* its backward from the saved c2 and hp: dc2 [rows][2f] = [dout . sig(b), dout . a . sig'(b)]
 * (the residual's gradient dx is dout itself), fp32 or bf16 (dc2_bf16 = 1); dhp (may be NULL): the
 * per-image sums of dc2, [nimg][2f] (d loss / d (h . hw)); dsum (may be NULL): its sums over all rows
 * (the producing conv's bias gradient); both fp32 from the same pass (scratch: rows / 64 * 2f floats). */
int svae_pcnn_gate_bwd(const float* c2, const float* hp, const float* dout, int lddo, int64_t rows, int pix_per_img,
                       int f, void* dc2, int dc2_bf16, float* dhp, float* dsum, float* scratch, void* stream);

/* small fp32 GEMM (conditioning projections, highway FC): C[m][n] = beta C + sum_k A(m,k) B(k,n),
 * A(m,k) = ta ? A[k*lda + m] : A[m*lda + k], B(k,n) = tb ? B[n*ldb + k] : B[k*ldb + n]. */
int svae_pcnn_gemm_small(const float* A, int lda, int ta, const float* B, int ldb, int tb, float* C, int ldc, int m,
                         int n, int k, float beta, void* stream);
/* per-image channel sums: out[img][c] = sum_{p < pix_per_img} x[img*pix + p][c] (fixed order over
 * 256-pixel partials in `scratch`, nimg * c * ceil(pix_per_img / 256) floats). */
int svae_pcnn_imgsum(const float* x, int ldx, int nimg, int pix_per_img, int c, float* out, float* scratch,
                     void* stream);

/* strided channel copy: y[r][0..c) = x[r][0..c) (concat / split of channel slices). */
int svae_pcnn_copy(const float* x, int ldx, int64_t rows, int c, float* y, int ldy, int accumulate, void* stream);
/* x_pad (model.py:37): y[r] = [x[r][0..c), 1, 0 ...] with ldy channels. */
int svae_pcnn_pad_ones(const float* x, int64_t rows, int c, float* y, int ldy, void* stream);

/* discretized_mix_logistic_loss (nn.py:46-87) per pixel and its gradient: logp[p] = log p(x_p)
 * (the negated loss summand), dl[p][10m] = coef * d(-logp_p)/dl (skipped if dl == NULL).
 * x [pixels][3] in [-1, 1], l [pixels][10 m]. */
int svae_pcnn_mixlogistic(const float* x, const float* l, int64_t pixels, int m, float* logp, float* dl, float coef,
                          void* stream);
/* fixed-order sum of n floats into out[0] (fp64 accumulation, written as fp32 and fp64). */
int svae_pcnn_sum(const float* x, int64_t n, float* out, double* out64, void* stream);
/* sample_from_discretized_mix_logistic (nn.py:89-109) with its uniforms given:
 * u_mix [pixels][m], u_log [pixels][3] (pixels = nimg * per_img); only the positions q in [q0, q1)
 * of every image are written (x [pixels][pix_stride]): one autoregressive step writes one q. */
int svae_pcnn_sample(const float* l, const float* u_mix, const float* u_log, int nimg, int per_img, int m, float* x,
                     int q0, int q1, int pix_stride, void* stream);
/* highway mix (pixelvae.py:135-137): out = r . s + (1 - r) . prev,
 * r = lo + (hi - lo) sigmoid(z[img] + zb[0]) (z = latents . W of the 1-unit FC; zb its bias or NULL). */
int svae_pcnn_highway(const float* s, const float* prev, const float* z, const float* zb, int nimg, int64_t per_img,
                      float lo, float hi, float* out, float* ratio, void* stream);

/* backward of svae_pcnn_sample over every position: dl [pixels][10 m] = d x / d l . dx (dx [pixels]
 * [dx_stride], first 3 used): the selected component's mean, log-scale (not where clamped at -7)
 * and tanh coefficients, through the [-1, 1] clips (inclusive) and the channel coupling; zero
 * elsewhere (the mixture indicator carries no gradient). */
int svae_pcnn_sample_bwd(const float* l, const float* u_mix, const float* u_log, int nimg, int per_img, int m,
                         const float* dx, int dx_stride, float* dl, void* stream);
/* backward of svae_pcnn_highway: ds = r dout (NULL: skipped), dprev (+)= (1 - r) dout (prev_acc),
 * dz[img] = d loss / d z[img] (the 1-unit FC's output, before the sigmoid). */
int svae_pcnn_highway_bwd(const float* s, const float* prev, const float* z, const float* zb, int nimg, int64_t per_img,
                          float lo, float hi, const float* dout, float* ds, float* dprev, int prev_acc, float* dz,
                          void* stream);
/* dropout with a given mask (nn.py:273-274, tf.nn.dropout): y = x * mask elementwise, mask
 * [rows][c] holding 1 / keep_prob (kept) or 0; in place allowed; the backward is the same call on
 * the gradient. */
int svae_pcnn_dropout(const float* x, int64_t rows, int c, int ldx, const float* mask, float* y, int ldy, void* stream);

/* per-image mean squared error (compute_and_accumulate_loss :1146 on the head's chain output):
 * rec[img] = mean (a - t)^2 over per_img elements; da = coef * 2 (a - t) / per_img (either may be NULL). */
int svae_pcnn_sqerr(const float* a, const float* t, int nimg, int64_t per_img, float coef, float* rec, float* da,
                    void* stream);

/* data-dependent init (nn.py:176-180, :206-210): column moments of y [rows][c] (fp64, two passes over
 * row blocks, fixed order), then g *= scale / sqrt(v + 1e-10), b -= m * scale / sqrt(v + 1e-10).
 * scratch: 1024 * c doubles. */
int svae_pcnn_wn_init(const float* y, int64_t rows, int c, int ldy, float init_scale, float* g, float* b,
                      double* scratch, void* stream);
/* TF Adam (tf.train.AdamOptimizer semantics as sequential_vae.py's optimiser, with the gradient
 * clipped to +-clip) on a flat buffer; and the Polyak EMA (pixelvae.py:113-114). */
int svae_pcnn_adam(float* p, const float* g, float* m, float* v, int64_t n, float lr, int64_t step, float clip,
                   void* stream);
int svae_pcnn_ema(float* avg, const float* p, int64_t n, float decay, void* stream);

#ifdef __cplusplus
}
#endif
#endif
