// Chain-variant kernels: chain noise, the predicted-stddev network with its
// Gaussian NLL, and the improvement-maximisation loss.
//
//   training_sample = training_mle + reg * stddevs * N(0,1)        sequential_vae.py:1088-1090
//   stddevs = max * sigmoid(conv1x1(5 x conv2d_bn_lrelu(conv_output)))  :1866-1875 (:1734-1735)
//   recon   = mean(log sd + 0.5 log 2pi + 0.5 ((mle - target)/sd)^2)   :1149-1150
//   imp     = reg * coeff * -mean_b ||mle_t - mle_{t-1}||^2            :1189-1199
//
// The stddev network works on the image itself: 4x4 stride-1 TF-SAME convs (pad 1 before, 2
// after) with <= 8 channels at full resolution, BN over B*H*W rows.  At 5 channels a layer is
// 0.4 GFLOP and ~20 MB of fp32 traffic, so these are plain fp32 direct-convolution kernels (one
// output pixel per thread), not MFMA tiles.  Every reduction (BN statistics, weight gradients,
// per-image losses) writes per-block partials that a second kernel sums in a fixed order, so
// results are bit-deterministic.
#include "kernels.h"

#define SD_TPB 256
#define SD_MAXC 8
#define SD_ROWS 4  // weight-gradient block: SD_ROWS image rows of one image

namespace {

__device__ __forceinline__ float sd_in(const float* in, long long p, int ldi, int ci, int in_sig) {
  const float v = in[p * ldi + ci];
  return in_sig ? sigmoid_f(v) : v;
}

// y[p][co] = sum_{tap, ci} x[src(p, tap)][ci] * W[ky][kx][ci][co]; per-block (sum, sum^2) partials
__global__ __launch_bounds__(SD_TPB) void sd_conv_fwd_kernel(const float* in, int ldi, int in_sig, int Ci,
                                                             const float* W, int Co, int H, int Wd, long long P,
                                                             float* pre, double* part) {
  __shared__ float w_s[16 * SD_MAXC * SD_MAXC];
  __shared__ float red[SD_TPB][SD_MAXC];
  for (int i = threadIdx.x; i < 16 * Ci * Co; i += SD_TPB) w_s[i] = W[i];
  __syncthreads();
  const long long p = (long long)blockIdx.x * SD_TPB + threadIdx.x;
  float acc[SD_MAXC];
#pragma unroll
  for (int o = 0; o < SD_MAXC; ++o) acc[o] = 0.f;
  if (p < P) {
    const int hw = H * Wd;
    const int n = (int)(p / hw), r = (int)(p % hw);
    const int oy = r / Wd, ox = r % Wd;
    for (int ky = 0; ky < 4; ++ky) {
      const int iy = oy - 1 + ky;
      if (iy < 0 || iy >= H) continue;
      for (int kx = 0; kx < 4; ++kx) {
        const int ix = ox - 1 + kx;
        if (ix < 0 || ix >= Wd) continue;
        const long long q = (long long)n * hw + iy * Wd + ix;
        const float* wt = w_s + (ky * 4 + kx) * Ci * Co;
        for (int ci = 0; ci < Ci; ++ci) {
          const float x = sd_in(in, q, ldi, ci, in_sig);
#pragma unroll
          for (int o = 0; o < SD_MAXC; ++o)
            if (o < Co) acc[o] = fmaf(x, wt[ci * Co + o], acc[o]);
        }
      }
    }
    for (int o = 0; o < Co; ++o) pre[p * Co + o] = acc[o];
  }
#pragma unroll
  for (int o = 0; o < SD_MAXC; ++o) red[threadIdx.x][o] = acc[o];
  __syncthreads();
  if (threadIdx.x < 2 * Co) {  // fixed-order block sums in fp64
    const int o = threadIdx.x >> 1, sq = threadIdx.x & 1;
    double s = 0.0;
    for (int i = 0; i < SD_TPB; ++i) {
      const double v = red[i][o];
      s += sq ? v * v : v;
    }
    part[(long long)blockIdx.x * 2 * Co + threadIdx.x] = s;
  }
}

// per channel: (S, Q) = fixed-order sums of the block partials; mode 0 (forward) mean / invstd
// (biased variance, eps); mode 1 (backward) out0 = S (dbeta, optional), sums[2c..] = (S, Q)
__global__ void sd_stat_fin_kernel(const double* part, int nblk, int Co, double n, float eps, int mode, float* mean,
                                   float* invstd, float* sums, float* dbeta) {
  __shared__ double red[SD_TPB];
  const int k = threadIdx.x >> 5, lane = threadIdx.x & 31;  // 8 (channel, moment) slots x 32 lanes
  for (int base = 0; base < 2 * Co; base += SD_TPB / 32) {
    const int col = base + k;
    double s = 0.0;
    if (col < 2 * Co)
      for (int b = lane; b < nblk; b += 32) s += part[(long long)b * 2 * Co + col];
    red[threadIdx.x] = s;
    __syncthreads();
    if (lane == 0 && col < 2 * Co) {
      double t = 0.0;
      for (int i = 0; i < 32; ++i) t += red[threadIdx.x + i];
      red[threadIdx.x] = t;
    }
    __syncthreads();
    if (lane == 0 && col < 2 * Co && (col & 1) == 0) {
      const double S = red[threadIdx.x], Q = red[threadIdx.x + 32];
      const int c = col >> 1;
      if (mode == 0) {
        const double m = S / n;
        const double var = fmax(Q / n - m * m, 0.0);
        mean[c] = (float)m;
        invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
      } else {
        sums[2 * c] = (float)S;
        sums[2 * c + 1] = (float)Q;
        if (dbeta) dbeta[c] = (float)S;
      }
    }
    __syncthreads();
  }
}

__global__ void sd_bn_apply_kernel(const float* pre, int Co, long long P, const float* mean, const float* invstd,
                                   const float* beta, float* act) {
  const long long i = (long long)blockIdx.x * SD_TPB + threadIdx.x;
  if (i >= P * Co) return;
  const int c = (int)(i % Co);
  act[i] = lrelu_f(bn_y1(pre[i], mean[c], invstd[c], beta[c]));
}

// backward BN + lrelu: per-block partials of sum dz and sum dz*xhat, dz = dact * lrelu'(y)
__global__ __launch_bounds__(SD_TPB) void sd_bn_bwd_reduce_kernel(const float* dact, const float* pre, int Co,
                                                                  long long P, const float* mean,
                                                                  const float* invstd, const float* beta,
                                                                  double* part) {
  __shared__ float red[SD_TPB][2 * SD_MAXC];
  const long long p = (long long)blockIdx.x * SD_TPB + threadIdx.x;
  for (int c = 0; c < Co; ++c) {
    float dz = 0.f, dx = 0.f;
    if (p < P) {
      const float x = pre[p * Co + c];
      const float y = bn_y1(x, mean[c], invstd[c], beta[c]);
      dz = dact[p * Co + c] * dact_from_y(y, ACT_LRELU);
      dx = dz * ((x - mean[c]) * invstd[c]);
    }
    red[threadIdx.x][2 * c] = dz;
    red[threadIdx.x][2 * c + 1] = dx;
  }
  __syncthreads();
  if (threadIdx.x < 2 * Co) {
    double s = 0.0;
    for (int i = 0; i < SD_TPB; ++i) s += red[i][threadIdx.x];
    part[(long long)blockIdx.x * 2 * Co + threadIdx.x] = s;
  }
}

// dpre = invstd * (dz - S/n - xhat * Q/n)   (training BN, scale = False)
__global__ void sd_bn_bwd_apply_kernel(const float* dact, const float* pre, int Co, long long P, const float* mean,
                                       const float* invstd, const float* beta, const float* sums, float* dpre) {
  const long long i = (long long)blockIdx.x * SD_TPB + threadIdx.x;
  if (i >= P * Co) return;
  const int c = (int)(i % Co);
  const float x = pre[i];
  const float y = bn_y1(x, mean[c], invstd[c], beta[c]);
  const float dz = dact[i] * dact_from_y(y, ACT_LRELU);
  const float xh = (x - mean[c]) * invstd[c];
  const float inv_n = 1.f / (float)P;
  dpre[i] = invstd[c] * (dz - sums[2 * c] * inv_n - xh * (sums[2 * c + 1] * inv_n));
}

// din[q][ci] = sum_{tap, co} dpre[q + 1 - k][co] * W[ky][kx][ci][co]  (adjoint of the stride-1
// SAME conv).  mode 0: din[q*ldd + ci] = v; mode 1 (layer 0, input = sigmoid(a_out)): the
// output conv-T pre-activation gradient da[q*ldd + ci] += v * s (1 - s), s = sigmoid(src)
__global__ __launch_bounds__(SD_TPB) void sd_conv_dgrad_kernel(const float* dpre, int Co, const float* W, int Ci,
                                                               int H, int Wd, long long P, float* din, int ldd,
                                                               const float* src, int lds, int mode) {
  __shared__ float w_s[16 * SD_MAXC * SD_MAXC];
  for (int i = threadIdx.x; i < 16 * Ci * Co; i += SD_TPB) w_s[i] = W[i];
  __syncthreads();
  const long long q = (long long)blockIdx.x * SD_TPB + threadIdx.x;
  if (q >= P) return;
  const int hw = H * Wd;
  const int n = (int)(q / hw), r = (int)(q % hw);
  const int iy = r / Wd, ix = r % Wd;
  float acc[SD_MAXC];
#pragma unroll
  for (int i = 0; i < SD_MAXC; ++i) acc[i] = 0.f;
  for (int ky = 0; ky < 4; ++ky) {
    const int oy = iy + 1 - ky;
    if (oy < 0 || oy >= H) continue;
    for (int kx = 0; kx < 4; ++kx) {
      const int ox = ix + 1 - kx;
      if (ox < 0 || ox >= Wd) continue;
      const float* d = dpre + ((long long)n * hw + oy * Wd + ox) * Co;
      const float* wt = w_s + (ky * 4 + kx) * Ci * Co;
      for (int co = 0; co < Co; ++co) {
        const float g = d[co];
#pragma unroll
        for (int ci = 0; ci < SD_MAXC; ++ci)
          if (ci < Ci) acc[ci] = fmaf(g, wt[ci * Co + co], acc[ci]);
      }
    }
  }
  for (int ci = 0; ci < Ci; ++ci) {
    if (mode == 0) {
      din[q * ldd + ci] = acc[ci];
    } else {
      const float s = sigmoid_f(src[q * lds + ci]);
      din[q * ldd + ci] += acc[ci] * s * (1.f - s);
    }
  }
}

// weight-gradient partials of one block (SD_ROWS output rows of one image):
// part[blk][(tap*Ci + ci)*Co + co] = sum_p x[src(p, tap)][ci] * dpre[p][co]
__global__ __launch_bounds__(SD_TPB) void sd_conv_wgrad_kernel(const float* in, int ldi, int in_sig, int Ci,
                                                               const float* dpre, int Co, int H, int Wd,
                                                               float* part) {
  extern __shared__ float sm[];
  const int WP = Wd + 3;                 // padded window row (1 before, 2 after)
  const int RW = SD_ROWS + 3;            // window rows
  float* win = sm;                       // [RW][WP][Ci]
  float* dp = sm + RW * WP * Ci;         // [SD_ROWS*Wd][Co]
  const int blocks_per_img = H / SD_ROWS;
  const int n = blockIdx.x / blocks_per_img;
  const int oy0 = (blockIdx.x % blocks_per_img) * SD_ROWS;
  const long long img = (long long)n * H * Wd;
  for (int i = threadIdx.x; i < RW * WP * Ci; i += SD_TPB) {
    const int ci = i % Ci, c = (i / Ci) % WP, rr = i / (Ci * WP);
    const int iy = oy0 - 1 + rr, ix = c - 1;
    float v = 0.f;
    if (iy >= 0 && iy < H && ix >= 0 && ix < Wd) v = sd_in(in, img + iy * Wd + ix, ldi, ci, in_sig);
    win[i] = v;
  }
  const int npix = SD_ROWS * Wd;
  for (int i = threadIdx.x; i < npix * Co; i += SD_TPB) dp[i] = dpre[(img + (long long)oy0 * Wd) * Co + i];
  __syncthreads();
  const int nw = 16 * Ci * Co;
  for (int j = threadIdx.x; j < nw; j += SD_TPB) {
    const int co = j % Co, ci = (j / Co) % Ci, tap = j / (Co * Ci);
    const int ky = tap >> 2, kx = tap & 3;
    float acc = 0.f;
    for (int pix = 0; pix < npix; ++pix) {
      const int y = pix / Wd, x = pix % Wd;
      acc = fmaf(win[((y + ky) * WP + (x + kx)) * Ci + ci], dp[pix * Co + co], acc);
    }
    part[(long long)blockIdx.x * nw + j] = acc;
  }
}

// out0[j] (j < n0) / out1[j - n0] = fixed-order fp64 sum over the block partials part[blk][j]
__global__ void sd_wsum_kernel(const float* part, int nblk, int nw, float* out0, int n0, float* out1) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nw) return;
  double s = 0.0;
  for (int b = 0; b < nblk; ++b) s += part[(long long)b * nw + j];
  if (j < n0) out0[j] = (float)s;
  else out1[j - n0] = (float)s;
}

// stddev head + noisy sample + NLL partials.  Per pixel: sd = max * sigmoid(act . W5 + b5);
// sample[c] = mle[c] + reg * sd * noise[c]; per-image partial of sum_c log sd + 0.5 log 2pi +
// 0.5 ((mle - target) / sd)^2 into rec_part[n * nblk + blk] (output_fwd's layout)
__global__ __launch_bounds__(SD_TPB) void sd_head_fwd_kernel(const float* act, int Ci, const float* W5,
                                                             const float* b5, float smax, const float* mle,
                                                             const float* target, const float* noise, float reg,
                                                             int C, int HW, float* sd, float* sample,
                                                             float* rec_part, int nblk) {
  __shared__ float red[SD_TPB / 64];
  const int n = blockIdx.y;
  const int pix = blockIdx.x * SD_TPB + threadIdx.x;
  float e = 0.f;
  if (pix < HW) {
    const long long p = (long long)n * HW + pix;
    float a = b5[0];
    for (int ci = 0; ci < Ci; ++ci) a = fmaf(act[p * Ci + ci], W5[ci], a);
    const float s = smax * sigmoid_f(a);
    sd[p] = s;
    const float ls = logf(s), is = 1.f / s;
    for (int c = 0; c < C; ++c) {
      const long long i = p * C + c;
      sample[i] = mle[i] + reg * s * noise[i];
      const float d = (mle[i] - target[i]) * is;
      e += ls + 0.91893853320467274f + 0.5f * d * d;
    }
  }
  e = wave_sum(e);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = e;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < SD_TPB / 64; ++w) t += red[w];
    rec_part[n * nblk + blockIdx.x] = t;
  }
}

// backward of sd_head_fwd.  dsample = d loss / d sample (chain, may be null), nll_coef = d loss /
// d e per element.  dmle = dsample + nll_coef (mle - target) / sd^2;
// dsd = sum_c reg * noise * dsample + nll_coef (1/sd - (mle - target)^2 / sd^3);
// da5 = dsd * max * s (1 - s); dact[p][ci] = W5[ci] * da5; part[blk][ci] = sum act*da5, [Ci] = sum da5
__global__ __launch_bounds__(SD_TPB) void sd_head_bwd_kernel(const float* act, int Ci, const float* W5,
                                                             const float* b5, float smax, const float* mle,
                                                             const float* target, const float* noise, float reg,
                                                             float nll_coef, const float* dsample, int C,
                                                             long long P, float* dmle, float* dact, float* part) {
  __shared__ float red[SD_TPB][SD_MAXC + 1];
  const long long p = (long long)blockIdx.x * SD_TPB + threadIdx.x;
  float da5 = 0.f;
  float av[SD_MAXC];
#pragma unroll
  for (int ci = 0; ci < SD_MAXC; ++ci) av[ci] = 0.f;
  if (p < P) {
    float a = b5[0];
    for (int ci = 0; ci < Ci; ++ci) {
      av[ci] = act[p * Ci + ci];
      a = fmaf(av[ci], W5[ci], a);
    }
    const float sg = sigmoid_f(a);
    const float s = smax * sg, is = 1.f / s;
    float dsd = 0.f;
    for (int c = 0; c < C; ++c) {
      const long long i = p * C + c;
      const float g = dsample ? dsample[i] : 0.f;
      const float d = mle[i] - target[i];
      dmle[i] = g + nll_coef * d * is * is;
      dsd += reg * noise[i] * g + nll_coef * (is - d * d * is * is * is);
    }
    da5 = dsd * smax * sg * (1.f - sg);
    for (int ci = 0; ci < Ci; ++ci) dact[p * Ci + ci] = W5[ci] * da5;
  }
#pragma unroll
  for (int ci = 0; ci < SD_MAXC; ++ci) red[threadIdx.x][ci] = av[ci] * da5;
  red[threadIdx.x][SD_MAXC] = da5;
  __syncthreads();
  if (threadIdx.x <= Ci) {
    const int col = threadIdx.x < Ci ? threadIdx.x : SD_MAXC;
    double s = 0.0;
    for (int i = 0; i < SD_TPB; ++i) s += red[i][col];
    part[(long long)blockIdx.x * (Ci + 1) + threadIdx.x] = (float)s;
  }
}

__global__ void chain_noise_kernel(const float* mle, const float* noise, float scale, long long n, float* sample) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) sample[i] = mle[i] + scale * noise[i];
}

// out = (dxin ? dxin : 0) + 2 coef ((x - xp) [xp] - (xn - x) [xn])
__global__ void imp_seed_kernel(const float* dxin, const float* xp, const float* x, const float* xn, float coef,
                                long long n, float* out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float g = 0.f;
  if (xp) g += x[i] - xp[i];
  if (xn) g -= xn[i] - x[i];
  out[i] = (dxin ? dxin[i] : 0.f) + 2.f * coef * g;
}

// out[n] = sum over the image of (a - b)^2, one block per image, fixed-order reduction
__global__ __launch_bounds__(SD_TPB) void sqdiff_img_kernel(const float* a, const float* b, long long per_img,
                                                            float* out) {
  __shared__ double red[SD_TPB];
  const long long base = (long long)blockIdx.x * per_img;
  double s = 0.0;
  for (long long i = threadIdx.x; i < per_img; i += SD_TPB) {
    const double d = (double)a[base + i] - (double)b[base + i];
    s += d * d;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < SD_TPB; ++i) t += red[i];
    out[blockIdx.x] = (float)t;
  }
}

inline unsigned nb(long long n) { return (unsigned)((n + SD_TPB - 1) / SD_TPB); }

}  // namespace

int sd_pixel_blocks(long long P) { return (int)nb(P); }
int sd_wgrad_blocks(int B, int H) { return B * (H / SD_ROWS); }

void sd_conv_fwd(const float* in, int ldi, int in_sig, int Ci, const float* W, int Co, int H, int Wd, long long P,
                 float* pre, double* part, hipStream_t s) {
  hipLaunchKernelGGL(sd_conv_fwd_kernel, dim3(nb(P)), dim3(SD_TPB), 0, s, in, ldi, in_sig, Ci, W, Co, H, Wd, P, pre,
                     part);
}

void sd_stat_fin(const double* part, int nblk, int Co, long long n, float eps, int mode, float* mean, float* invstd,
                 float* sums, float* dbeta, hipStream_t s) {
  hipLaunchKernelGGL(sd_stat_fin_kernel, dim3(1), dim3(SD_TPB), 0, s, part, nblk, Co, (double)n, eps, mode, mean,
                     invstd, sums, dbeta);
}

void sd_bn_apply(const float* pre, int Co, long long P, const float* mean, const float* invstd, const float* beta,
                 float* act, hipStream_t s) {
  hipLaunchKernelGGL(sd_bn_apply_kernel, dim3(nb(P * Co)), dim3(SD_TPB), 0, s, pre, Co, P, mean, invstd, beta, act);
}

void sd_bn_bwd_reduce(const float* dact, const float* pre, int Co, long long P, const float* mean, const float* invstd,
                      const float* beta, double* part, hipStream_t s) {
  hipLaunchKernelGGL(sd_bn_bwd_reduce_kernel, dim3(nb(P)), dim3(SD_TPB), 0, s, dact, pre, Co, P, mean, invstd, beta,
                     part);
}

void sd_bn_bwd_apply(const float* dact, const float* pre, int Co, long long P, const float* mean, const float* invstd,
                     const float* beta, const float* sums, float* dpre, hipStream_t s) {
  hipLaunchKernelGGL(sd_bn_bwd_apply_kernel, dim3(nb(P * Co)), dim3(SD_TPB), 0, s, dact, pre, Co, P, mean, invstd,
                     beta, sums, dpre);
}

void sd_conv_dgrad(const float* dpre, int Co, const float* W, int Ci, int H, int Wd, long long P, float* din, int ldd,
                   const float* src, int lds, int mode, hipStream_t s) {
  hipLaunchKernelGGL(sd_conv_dgrad_kernel, dim3(nb(P)), dim3(SD_TPB), 0, s, dpre, Co, W, Ci, H, Wd, P, din, ldd, src,
                     lds, mode);
}

void sd_conv_wgrad(const float* in, int ldi, int in_sig, int Ci, const float* dpre, int Co, int B, int H, int Wd,
                   float* part, float* dW, hipStream_t s) {
  const int nblk = sd_wgrad_blocks(B, H);
  const size_t lds = (size_t)((SD_ROWS + 3) * (Wd + 3) * Ci + SD_ROWS * Wd * Co) * sizeof(float);
  hipLaunchKernelGGL(sd_conv_wgrad_kernel, dim3(nblk), dim3(SD_TPB), lds, s, in, ldi, in_sig, Ci, dpre, Co, H, Wd,
                     part);
  const int nw = 16 * Ci * Co;
  hipLaunchKernelGGL(sd_wsum_kernel, dim3((nw + 255) / 256), dim3(256), 0, s, part, nblk, nw, dW, nw, nullptr);
}

void sd_head_fwd(const float* act, int Ci, const float* W5, const float* b5, float smax, const float* mle,
                 const float* target, const float* noise, float reg, int B, int C, int HW, float* sd, float* sample,
                 float* rec_part, int nblk, hipStream_t s) {
  hipLaunchKernelGGL(sd_head_fwd_kernel, dim3(nblk, B), dim3(SD_TPB), 0, s, act, Ci, W5, b5, smax, mle, target, noise,
                     reg, C, HW, sd, sample, rec_part, nblk);
}

void sd_head_bwd(const float* act, int Ci, const float* W5, const float* b5, float smax, const float* mle,
                 const float* target, const float* noise, float reg, float nll_coef, const float* dsample, int C,
                 long long P, float* dmle, float* dact, float* part, float* dW5, float* db5, hipStream_t s) {
  const int nblk = (int)nb(P);
  hipLaunchKernelGGL(sd_head_bwd_kernel, dim3(nblk), dim3(SD_TPB), 0, s, act, Ci, W5, b5, smax, mle, target, noise,
                     reg, nll_coef, dsample, C, P, dmle, dact, part);
  hipLaunchKernelGGL(sd_wsum_kernel, dim3(1), dim3(64), 0, s, part, nblk, Ci + 1, dW5, Ci, db5);
}

void chain_noise(const float* mle, const float* noise, float scale, long long n, float* sample, hipStream_t s) {
  hipLaunchKernelGGL(chain_noise_kernel, dim3(nb(n)), dim3(SD_TPB), 0, s, mle, noise, scale, n, sample);
}

void imp_seed(const float* dxin, const float* xp, const float* x, const float* xn, float coef, long long n, float* out,
              hipStream_t s) {
  hipLaunchKernelGGL(imp_seed_kernel, dim3(nb(n)), dim3(SD_TPB), 0, s, dxin, xp, x, xn, coef, n, out);
}

void sqdiff_img(const float* a, const float* b, int B, long long per_img, float* out, hipStream_t s) {
  hipLaunchKernelGGL(sqdiff_img_kernel, dim3(B), dim3(SD_TPB), 0, s, a, b, per_img, out);
}
