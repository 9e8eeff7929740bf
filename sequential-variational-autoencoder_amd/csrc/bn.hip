// Training-mode BatchNorm (center=True, scale=False, eps=1e-3; abstract_network.py:22) + activation.
//
// Forward statistics come from the producing GEMM's epilogue (per-row-block
// partial sum / sum^2); bn_finalize reduces them in fp64.  The normalise +
// beta + shortcut + activation pass writes straight into the consumer's view
// (e.g. the channel half of a concat buffer, combine_noise sequential_vae.py:1833).
// Backward: dz = dy*act'(y) (act' from the stored output, TF tie rules),
// dpre = invstd*(dz - mean(dz) - xhat*mean(dz*xhat)), dbeta = sum(dz).
#include "common.h"
#include "kernels.h"

// BN output before the activation, per element through common.h bn_y1 (one expression shared
// by every kernel that needs it, so the backward's act' sign is bitwise the forward's)
__device__ __forceinline__ f32x4 bn_y(f32x4 x, f32x4 m, f32x4 is, f32x4 b) {
  f32x4 r;
#pragma unroll
  for (int e = 0; e < 4; ++e) r[e] = bn_y1(x[e], m[e], is[e], b[e]);
  return r;
}

// partial rows are reduced by FIN_L lanes per channel quad (4 quads = 16 channels per block),
// each lane summing its share in fp64, then a fixed-order LDS tree: deterministic, and short
// serial chains (the kernel is latency-bound at these sizes)
#define FIN_Q 4
#define FIN_L 64
__global__ __launch_bounds__(256) void bn_finalize_kernel(const float* part, long long part_gs, int nrb, int C,
                                                          double count, float eps, float* mean, float* invstd,
                                                          long long ms_gs, int mode, float* dbeta,
                                                          long long dbeta_gs) {
  // mode 0: stats -> mean/invstd ; mode 1: bwd sums -> ab (mean slots), dbeta
  __shared__ double red[2][FIN_L][FIN_Q * 4];
  const int group = blockIdx.y;
  const int qi = threadIdx.x % FIN_Q, li = threadIdx.x / FIN_Q;
  const int c0 = (blockIdx.x * FIN_Q + qi) * 4;
  const float* P = part + group * part_gs;
  double s[4] = {0.0, 0.0, 0.0, 0.0}, q[4] = {0.0, 0.0, 0.0, 0.0};
  if (c0 < C) {
    for (int rb = li; rb < nrb; rb += FIN_L) {
      const f32x4 a = *(const f32x4*)(P + (long long)rb * 2 * C + c0);
      const f32x4 b2 = *(const f32x4*)(P + (long long)rb * 2 * C + C + c0);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s[e] += (double)a[e];
        q[e] += (double)b2[e];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    red[0][li][qi * 4 + e] = s[e];
    red[1][li][qi * 4 + e] = q[e];
  }
  __syncthreads();
  for (int w = FIN_L / 2; w > 0; w >>= 1) {
    if (li < w) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        red[0][li][qi * 4 + e] += red[0][li + w][qi * 4 + e];
        red[1][li][qi * 4 + e] += red[1][li + w][qi * 4 + e];
      }
    }
    __syncthreads();
  }
  if (li == 0 && c0 < C) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int cc = c0 + e;
      const double ss = red[0][0][qi * 4 + e], qq = red[1][0][qi * 4 + e];
      if (mode == 0) {
        const double m = ss / count;
        double var = qq / count - m * m;
        if (var < 0.0) var = 0.0;
        mean[group * ms_gs + cc] = (float)m;
        invstd[group * ms_gs + cc] = (float)(1.0 / sqrt(var + (double)eps));
      } else {
        mean[group * ms_gs + cc] = (float)(ss / count);        // a = mean(dz)
        mean[group * ms_gs + C + cc] = (float)(qq / count);    // b = mean(dz*xhat)
        if (dbeta) dbeta[group * dbeta_gs + cc] = (float)ss;
      }
    }
  }
}

void bn_finalize(const float* part, long long part_gs, int nrb, int C, long long count, float eps, float* mean,
                 float* invstd, long long ms_gs, int groups, hipStream_t s) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 4 * FIN_Q - 1) / (4 * FIN_Q), groups), dim3(256), 0, s, part,
                     part_gs, nrb, C, (double)count, eps, mean, invstd, ms_gs, 0, (float*)nullptr, 0LL);
}

void bn_bwd_finalize(const float* part, long long part_gs, int nrb, int C, long long count, float* ab, long long ab_gs,
                     float* dbeta, long long dbeta_gs, int groups, hipStream_t s) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 4 * FIN_Q - 1) / (4 * FIN_Q), groups), dim3(256), 0, s, part,
                     part_gs, nrb, C, (double)count, 0.f, ab, (float*)nullptr, ab_gs, 1, dbeta, dbeta_gs);
}

__global__ void bn_apply_kernel(const float* pre, int ldp, long long pre_gs, long long rows, int C,
                                const float* mean, const float* invstd, long long ms_gs, const float* beta,
                                long long beta_gs, const float* res, int ldr, long long res_gs, int act, float* out,
                                int ldo, long long out_gs) {
  const int group = blockIdx.y;
  const int Q = C >> 2;
  const long long total = rows * Q;
  pre += group * pre_gs;
  out += group * out_gs;
  mean += group * ms_gs;
  invstd += group * ms_gs;
  beta += group * beta_gs;
  if (res) res += group * res_gs;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / Q;
    const int c = (int)(i - r * Q) * 4;
    f32x4 x = *(const f32x4*)(pre + r * ldp + c);
    f32x4 m = *(const f32x4*)(mean + c), is = *(const f32x4*)(invstd + c), b = *(const f32x4*)(beta + c);
    f32x4 y = bn_y(x, m, is, b);
    if (res) y += *(const f32x4*)(res + r * ldr + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) y[e] = act_f(y[e], act);
    *(f32x4*)(out + r * ldo + c) = y;
  }
}

static int ew_blocks(long long work) {
  long long b = (work + 255) / 256;
  return (int)(b < 2048 ? (b < 1 ? 1 : b) : 2048);
}

void bn_apply(const float* pre, int ldp, long long pre_gs, long long rows, int C, const float* mean,
              const float* invstd, long long ms_gs, const float* beta, long long beta_gs, const float* res, int ldr,
              long long res_gs, int act, float* out, int ldo, long long out_gs, int groups, hipStream_t s) {
  hipLaunchKernelGGL(bn_apply_kernel, dim3(ew_blocks(rows * (C / 4)), groups), dim3(256), 0, s, pre, ldp, pre_gs,
                     rows, C, mean, invstd, ms_gs, beta, beta_gs, res, ldr, res_gs, act, out, ldo, out_gs);
}

#define BWD_RPB 256  // rows per row-block of the backward reduction

int bn_bwd_rowblocks(long long rows, int C) {
  (void)C;
  return (int)((rows + BWD_RPB - 1) / BWD_RPB);
}

// y == nullptr: act' from the recomputed pre-activation bn_y(pre) (layers without a shortcut add)
__global__ void bn_bwd_reduce_kernel(const float* dy, int lddy, long long dy_gs, const float* y, int ldy,
                                     long long y_gs, const float* pre, int ldp, long long pre_gs, long long rows,
                                     int C, const float* mean, const float* invstd, long long ms_gs, const float* beta,
                                     long long beta_gs, int act, float* part, long long part_gs) {
  __shared__ f32x4 red[2][256];
  const int group = blockIdx.z;
  const int Q = C >> 2;
  const int QB = Q < 16 ? Q : 16;   // quads per block
  const int RL = 256 / QB;          // row lanes
  const int tid = threadIdx.x;
  const int qi = tid % QB, rl = tid / QB;
  const int q = blockIdx.x * QB + qi;
  const bool active = rl < RL && q < Q;
  dy += group * dy_gs;
  if (y) y += group * y_gs;
  pre += group * pre_gs;
  mean += group * ms_gs;
  invstd += group * ms_gs;
  f32x4 sd = {0.f, 0.f, 0.f, 0.f}, sx = {0.f, 0.f, 0.f, 0.f};
  if (active) {
    const int c = q * 4;
    const f32x4 m = *(const f32x4*)(mean + c), is = *(const f32x4*)(invstd + c);
    const f32x4 bb = y ? f32x4{0.f, 0.f, 0.f, 0.f} : *(const f32x4*)(beta + group * beta_gs + c);
    const long long r0 = (long long)blockIdx.y * BWD_RPB;
    const long long r1 = r0 + BWD_RPB < rows ? r0 + BWD_RPB : rows;
#pragma unroll 4
    for (long long r = r0 + rl; r < r1; r += RL) {
      f32x4 g = *(const f32x4*)(dy + r * lddy + c);
      const f32x4 xp = *(const f32x4*)(pre + r * ldp + c);
      f32x4 yy = y ? *(const f32x4*)(y + r * ldy + c) : bn_y(xp, m, is, bb);
      f32x4 xh = (xp - m) * is;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float dz = g[e] * dact_from_y(yy[e], act);
        sd[e] += dz;
        sx[e] += dz * xh[e];
      }
    }
  }
  red[0][tid] = sd;
  red[1][tid] = sx;
  __syncthreads();
  if (active && rl == 0) {
    for (int j = 1; j < RL; ++j) {
      sd += red[0][j * QB + qi];
      sx += red[1][j * QB + qi];
    }
    float* P = part + group * part_gs + (long long)blockIdx.y * 2 * C;
    *(f32x4*)(P + q * 4) = sd;
    *(f32x4*)(P + C + q * 4) = sx;
  }
}

void bn_bwd_reduce(const float* dy, int lddy, long long dy_gs, const float* y, int ldy, long long y_gs,
                   const float* pre, int ldp, long long pre_gs, long long rows, int C, const float* mean,
                   const float* invstd, long long ms_gs, const float* beta, long long beta_gs, int act, float* part,
                   long long part_gs, int groups, hipStream_t s) {
  const int Q = C / 4;
  const int QB = Q < 16 ? Q : 16;
  dim3 grid((Q + QB - 1) / QB, bn_bwd_rowblocks(rows, C), groups);
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, grid, dim3(256), 0, s, dy, lddy, dy_gs, y, ldy, y_gs, pre, ldp, pre_gs,
                     rows, C, mean, invstd, ms_gs, beta, beta_gs, act, part, part_gs);
}

__global__ void bn_bwd_apply_kernel(const float* dy, int lddy, long long dy_gs, const float* y, int ldy,
                                    long long y_gs, const float* pre, int ldp, long long pre_gs, long long rows,
                                    int C, const float* mean, const float* invstd, long long ms_gs, const float* beta,
                                    long long beta_gs, const float* ab, long long ab_gs, int act, float* dpre, int lddp,
                                    long long dpre_gs, float* dres, int ldres, long long dres_gs, int res_acc) {
  const int group = blockIdx.y;
  const int Q = C >> 2;
  const long long total = rows * Q;
  dy += group * dy_gs;
  if (y) y += group * y_gs;
  else beta += group * beta_gs;
  pre += group * pre_gs;
  mean += group * ms_gs;
  invstd += group * ms_gs;
  ab += group * ab_gs;
  dpre += group * dpre_gs;
  if (dres) dres += group * dres_gs;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / Q;
    const int c = (int)(i - r * Q) * 4;
    f32x4 g = *(const f32x4*)(dy + r * lddy + c);
    f32x4 is = *(const f32x4*)(invstd + c);
    const f32x4 m = *(const f32x4*)(mean + c);
    const f32x4 xp = *(const f32x4*)(pre + r * ldp + c);
    f32x4 yy = y ? *(const f32x4*)(y + r * ldy + c) : bn_y(xp, m, is, *(const f32x4*)(beta + c));
    f32x4 xh = (xp - m) * is;
    f32x4 a = *(const f32x4*)(ab + c), b = *(const f32x4*)(ab + C + c);
    f32x4 dz;
#pragma unroll
    for (int e = 0; e < 4; ++e) dz[e] = g[e] * dact_from_y(yy[e], act);
    *(f32x4*)(dpre + r * lddp + c) = is * (dz - a - xh * b);
    if (dres) {
      f32x4* d = (f32x4*)(dres + r * ldres + c);
      *d = res_acc ? *d + dz : dz;
    }
  }
}

void bn_bwd_apply(const float* dy, int lddy, long long dy_gs, const float* y, int ldy, long long y_gs,
                  const float* pre, int ldp, long long pre_gs, long long rows, int C, const float* mean,
                  const float* invstd, long long ms_gs, const float* beta, long long beta_gs, const float* ab,
                  long long ab_gs, int act, float* dpre, int lddp, long long dpre_gs, float* dres, int ldres,
                  long long dres_gs, int res_acc, int groups, hipStream_t s) {
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(ew_blocks(rows * (C / 4)), groups), dim3(256), 0, s, dy, lddy, dy_gs,
                     y, ldy, y_gs, pre, ldp, pre_gs, rows, C, mean, invstd, ms_gs, beta, beta_gs, ab, ab_gs, act, dpre,
                     lddp, dpre_gs, dres, ldres, dres_gs, res_acc);
}
