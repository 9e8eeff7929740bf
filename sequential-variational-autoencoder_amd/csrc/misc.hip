// Bandwidth-bound kernels of the hot path: split_latent FC+BN, recognition heads,
// reparameterised latent + KL, small-N conv (output / layer-0 dgrad), output +
// highway + reconstruction loss, loss reduction, clip+Adam, Philox normals.
#include <algorithm>
#include <cstdint>

#include "common.h"
#include "knobs.h"
#include "kernels.h"

#define KMAX 32  // max latent dims per level handled in registers (LSUN: 30)

static int ew_blocks(long long work, int per = 256, int cap = 4096) {
  long long b = (work + per - 1) / per;
  return (int)(b < cap ? (b < 1 ? 1 : b) : cap);
}

// ---------------------------------------------------------------------------
// split_latent: ladder_i = lrelu(BN_batch(z_i @ W_i + b_i))   (sequential_vae.py:1801-1806)
// block = 64 output features x 4 row groups (wave w owns rows n = w mod 4); the batch
// column of each feature is recomputed from z (K <= 32 FMAs) instead of stored.
// ---------------------------------------------------------------------------
#define SFC_COLS 64
#define SFC_RG 4

template <int KM>
__device__ __forceinline__ void splitfc_fwd_body(const float* z, int ldz, int zoff, int B, int K, const float* W,
                                                 const float* beta, int J, float* mean, float* invstd, float* out,
                                                 long long o_n, int F, int ldo, int out_bf16, float* zs) {
  __shared__ float red[SFC_RG][SFC_COLS];
  for (int i = threadIdx.x; i < B * KM; i += blockDim.x) {
    const int d = i % KM;
    zs[i] = d < K ? z[(i / KM) * ldz + zoff + d] : 0.f;
  }
  __syncthreads();
  const int c = threadIdx.x & (SFC_COLS - 1), rg = threadIdx.x / SFC_COLS;
  const int j = blockIdx.x * SFC_COLS + c;
  const bool ok = j < J;
  float w[KM];
#pragma unroll
  for (int d = 0; d < KM; ++d) w[d] = (ok && d < K) ? W[(long long)d * J + j] : 0.f;
  auto pre = [&](int n) {  // (16-byte LDS reads of the z row, the same fma order)
    float s = 0.f;
#pragma unroll
    for (int d4 = 0; d4 < KM; d4 += 4) {
      const f32x4 zv = *(const f32x4*)&zs[n * KM + d4];
#pragma unroll
      for (int e = 0; e < 4; ++e) s = fmaf(zv[e], w[d4 + e], s);
    }
    return s;
  };
  float s = 0.f;
  for (int n = rg; n < B; n += SFC_RG) s += pre(n);
  red[rg][c] = s;
  __syncthreads();
  const float m = (red[0][c] + red[1][c] + red[2][c] + red[3][c]) / B;
  __syncthreads();
  float q = 0.f;
  for (int n = rg; n < B; n += SFC_RG) {
    const float dd = pre(n) - m;
    q += dd * dd;
  }
  red[rg][c] = q;
  __syncthreads();
  const float is = 1.f / sqrtf((red[0][c] + red[1][c] + red[2][c] + red[3][c]) / B + 1e-3f);
  if (!ok) return;
  if (rg == 0) {
    mean[j] = m;
    invstd[j] = is;
  }
  const float b = beta[j];
  const long long o0 = (long long)(j / F) * ldo + (j % F);
  if (out_bf16) {  // read only by bf16 GEMMs (the s1 gather and weight gradient round it the same way)
    __bf16* dh = (__bf16*)out + o0;
    for (int n = rg; n < B; n += SFC_RG) dh[n * o_n] = (__bf16)lrelu_f((pre(n) - m) * is + b);
    return;
  }
  float* dst = out + o0;
  for (int n = rg; n < B; n += SFC_RG) dst[n * o_n] = lrelu_f((pre(n) - m) * is + b);
}

template <int KM>
__global__ __launch_bounds__(256) void splitfc_fwd_kernel(const float* z, int ldz, int zoff, int B, int K,
                                                          const float* W, const float* beta, int J, float* mean,
                                                          float* invstd, float* out, long long o_n, int F, int ldo,
                                                          int out_bf16) {
  extern __shared__ __attribute__((aligned(16))) float zs[];  // [B][KM], zero padded past K
  splitfc_fwd_body<KM>(z, ldz, zoff, B, K, W, beta, J, mean, invstd, out, o_n, F, ldo, out_bf16, zs);
}

// one level of split_latent for the chain steps t0 .. t0 + nt - 1 in one launch (grid.y = step): every
// z_t is known after the T-batched recognition, so the forward of all steps is one launch per level
// instead of one per (level, step) -- the same block body, bitwise the per-step launches
template <int KM>
__global__ __launch_bounds__(256) void splitfc_fwd_steps_kernel(const float* z, long long z_ts, int ldz, int zoff,
                                                                int B, int K, int J, int F, int ldo, int out_bf16,
                                                                SfcSteps a) {
  extern __shared__ __attribute__((aligned(16))) float zs[];
  const int i = blockIdx.y;
  splitfc_fwd_body<KM>(z + i * z_ts, ldz, zoff, B, K, a.W[i], a.beta[i], J, a.mean[i], a.invstd[i], a.out[i], a.o_n[i], F,
                       ldo, out_bf16, zs);
}

static int sfc_km(int K) { return K <= 4 ? 4 : (K <= 8 ? 8 : 32); }

void splitfc_fwd(const float* z, int ldz, int zoff, int B, int K, const float* W, const float* beta, int J,
                 float* mean, float* invstd, float* out, long long o_n, int F, int ldo, hipStream_t s, int out_bf16) {
  const int km = sfc_km(K);
  dim3 g((J + SFC_COLS - 1) / SFC_COLS);
  const size_t lds = (size_t)B * km * sizeof(float);
  if (km == 4)
    hipLaunchKernelGGL(splitfc_fwd_kernel<4>, g, dim3(256), lds, s, z, ldz, zoff, B, K, W, beta, J, mean, invstd, out,
                       o_n, F, ldo, out_bf16);
  else if (km == 8)
    hipLaunchKernelGGL(splitfc_fwd_kernel<8>, g, dim3(256), lds, s, z, ldz, zoff, B, K, W, beta, J, mean, invstd, out,
                       o_n, F, ldo, out_bf16);
  else
    hipLaunchKernelGGL(splitfc_fwd_kernel<32>, g, dim3(256), lds, s, z, ldz, zoff, B, K, W, beta, J, mean, invstd,
                       out, o_n, F, ldo, out_bf16);
}

int splitfc_blocks(int J) { return (J + SFC_COLS - 1) / SFC_COLS; }

void splitfc_fwd_steps(const float* z, long long z_ts, int ldz, int zoff, int B, int K, int J, int F, int ldo,
                       int out_bf16, const SfcSteps& a, int nt, hipStream_t s) {
  const int km = sfc_km(K);
  dim3 g((J + SFC_COLS - 1) / SFC_COLS, nt);
  const size_t lds = (size_t)B * km * sizeof(float);
  if (km == 4)
    hipLaunchKernelGGL(splitfc_fwd_steps_kernel<4>, g, dim3(256), lds, s, z, z_ts, ldz, zoff, B, K, J, F, ldo, out_bf16, a);
  else if (km == 8)
    hipLaunchKernelGGL(splitfc_fwd_steps_kernel<8>, g, dim3(256), lds, s, z, z_ts, ldz, zoff, B, K, J, F, ldo, out_bf16, a);
  else
    hipLaunchKernelGGL(splitfc_fwd_steps_kernel<32>, g, dim3(256), lds, s, z, z_ts, ldz, zoff, B, K, J, F, ldo, out_bf16, a);
}


// backward: dW [K][J], dbeta [J], and per-block partial dz: dz_part[blk][n][d] = sum_{j in blk} dpre[n][j] W[d][j].
// dpre rows are staged in LDS (pitch 65: conflict-free column reads) and the dz partials are then
// formed by plain per-thread dot products over the block's 64 features.
#define SFC_PITCH (SFC_COLS + 4)  // (a multiple of 4: 16-byte row reads in the dz pass; column accesses are per wave)
template <int KM>
__global__ __launch_bounds__(256) void splitfc_bwd_kernel(const float* z, int ldz, int zoff, int B, int K,
                                                          const float* W, const float* beta, int J,
                                                          const float* mean, const float* invstd, const float* dout,
                                                          long long o_n, int F, int ldo, float* dW, float* dbeta,
                                                          float* dz_part) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* zs = sm;                 // [B][KM]
  float* dps = sm + B * KM;       // [B][SFC_PITCH]
  __shared__ float red[2][SFC_RG][SFC_COLS];
  __shared__ __attribute__((aligned(16))) float ws[KM][SFC_COLS];
  for (int i = threadIdx.x; i < B * KM; i += blockDim.x) {
    const int d = i % KM;
    zs[i] = d < K ? z[(i / KM) * ldz + zoff + d] : 0.f;
  }
  const int c = threadIdx.x & (SFC_COLS - 1), rg = threadIdx.x / SFC_COLS;
  const int j = blockIdx.x * SFC_COLS + c;
  const bool ok = j < J;
  float w[KM];
#pragma unroll
  for (int d = 0; d < KM; ++d) w[d] = (ok && d < K) ? W[(long long)d * J + j] : 0.f;
  if (rg == 0) {
#pragma unroll
    for (int d = 0; d < KM; ++d) ws[d][c] = w[d];
  }
  const float m = ok ? mean[j] : 0.f, is = ok ? invstd[j] : 0.f, b = ok ? beta[j] : 0.f;
  const float* src = dout + (long long)(j / F) * ldo + (j % F);
  // dout rows are staged into this column of the LDS tile (independent loads, all in flight)
#pragma unroll 32
  for (int n = rg; n < B; n += SFC_RG) dps[n * SFC_PITCH + c] = ok ? src[n * o_n] : 0.f;
  __syncthreads();
  auto xhat = [&](int n) {  // (16-byte LDS reads of the z row: a quarter of the LDS instructions, same fma order)
    float s = 0.f;
#pragma unroll
    for (int d4 = 0; d4 < KM; d4 += 4) {
      const f32x4 zv = *(const f32x4*)&zs[n * KM + d4];
#pragma unroll
      for (int e = 0; e < 4; ++e) s = fmaf(zv[e], w[d4 + e], s);
    }
    return (s - m) * is;
  };
  float sd = 0.f, sx = 0.f;
  for (int n = rg; n < B; n += SFC_RG) {
    const float xh = xhat(n);
    const float dzv = dps[n * SFC_PITCH + c] * ((xh + b) > 0.f ? 1.f : 0.1f);
    dps[n * SFC_PITCH + c] = dzv;
    sd += dzv;
    sx += dzv * xh;
  }
  red[0][rg][c] = sd;
  red[1][rg][c] = sx;
  __syncthreads();
  sd = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
  sx = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
  const float a = sd / B, cc = sx / B;
  float gw[KM];
#pragma unroll
  for (int d = 0; d < KM; ++d) gw[d] = 0.f;
  for (int n = rg; n < B; n += SFC_RG) {
    const float dp = ok ? is * (dps[n * SFC_PITCH + c] - a - xhat(n) * cc) : 0.f;
    dps[n * SFC_PITCH + c] = dp;
#pragma unroll
    for (int d4 = 0; d4 < KM; d4 += 4) {
      const f32x4 zv = *(const f32x4*)&zs[n * KM + d4];
#pragma unroll
      for (int e = 0; e < 4; ++e) gw[d4 + e] = fmaf(zv[e], dp, gw[d4 + e]);
    }
  }
  __syncthreads();
  float* P = dz_part + (long long)blockIdx.x * B * K;
  for (int p = threadIdx.x; p < B * K; p += blockDim.x) {
    const int n = p / K, d = p - n * K;
    const float* row = dps + n * SFC_PITCH;
    float s = 0.f;
#pragma unroll 4
    for (int q = 0; q < SFC_COLS; q += 4) {
      const f32x4 rv = *(const f32x4*)&row[q], wv = *(const f32x4*)&ws[d][q];
#pragma unroll
      for (int e = 0; e < 4; ++e) s = fmaf(rv[e], wv[e], s);
    }
    P[p] = s;
  }
  __syncthreads();  // dps reused below as the dW reduction buffer
  float* gwr = dps;  // [SFC_RG][KM][SFC_COLS] fits in B*SFC_PITCH floats when B >= 4*KM
#pragma unroll
  for (int d = 0; d < KM; ++d) gwr[(rg * KM + d) * SFC_COLS + c] = gw[d];
  __syncthreads();
  if (ok && rg == 0) {
    for (int d = 0; d < K; ++d)
      dW[(long long)d * J + j] = gwr[(0 * KM + d) * SFC_COLS + c] + gwr[(1 * KM + d) * SFC_COLS + c] +
                                 gwr[(2 * KM + d) * SFC_COLS + c] + gwr[(3 * KM + d) * SFC_COLS + c];
    dbeta[j] = sd;
  }
}

void splitfc_bwd(const float* z, int ldz, int zoff, int B, int K, const float* W, const float* beta, int J,
                 const float* mean, const float* invstd, const float* dout, long long o_n, int F, int ldo, float* dW,
                 float* dbeta, float* dz_part, hipStream_t s) {
  const int km = sfc_km(K);
  dim3 g((J + SFC_COLS - 1) / SFC_COLS);
  const int rows = B > 4 * km ? B : 4 * km;  // dps doubles as the [4][KM][64] dW reduction buffer
  const size_t lds = ((size_t)B * km + (size_t)rows * SFC_PITCH) * sizeof(float);
  static bool attr = false;
  if (!attr) {  // B=256, K=30 needs ~100 KB of the 160 KB LDS
    hipFuncSetAttribute((const void*)splitfc_bwd_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    hipFuncSetAttribute((const void*)splitfc_bwd_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    hipFuncSetAttribute((const void*)splitfc_bwd_kernel<32>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
    attr = true;
  }
  if (km == 4)
    hipLaunchKernelGGL(splitfc_bwd_kernel<4>, g, dim3(256), lds, s, z, ldz, zoff, B, K, W, beta, J, mean, invstd,
                       dout, o_n, F, ldo, dW, dbeta, dz_part);
  else if (km == 8)
    hipLaunchKernelGGL(splitfc_bwd_kernel<8>, g, dim3(256), lds, s, z, ldz, zoff, B, K, W, beta, J, mean, invstd,
                       dout, o_n, F, ldo, dW, dbeta, dz_part);
  else
    hipLaunchKernelGGL(splitfc_bwd_kernel<32>, g, dim3(256), lds, s, z, ldz, zoff, B, K, W, beta, J, mean, invstd,
                       dout, o_n, F, ldo, dW, dbeta, dz_part);
}

// ---------------------------------------------------------------------------
// skinny GEMM over a long reduction: part[split][n][coff+o] = sum_{k in split} X[n][k] * W[k*sk + o*so]
// (recognition heads K=32768 -> D=3, and dz = dpre @ W^T of split_latent)
// ---------------------------------------------------------------------------
#define SK_ROWS 4
#define SK_CHUNK 2048  // = HF_CHUNK: both fill heads_splits(K) partial rows

template <int DM>
// D outputs from W, and (W2 != nullptr) D more from W2 into columns coff2.. of part: the mean and
// stddev heads read the shared input X once (per-output arithmetic unchanged)
__global__ __launch_bounds__(256) void skinny_kernel(const float* __restrict__ X, int ldx, long long x_gs, int B,
                                                     int K, const float* __restrict__ W, long long sk, long long so,
                                                     long long w_gs, int D, float* __restrict__ part, long long p_gs,
                                                     int pcols, int coff, const float* __restrict__ W2, int coff2) {
  __shared__ float red[4][SK_ROWS][DM];
  const int group = blockIdx.z;
  const int split = blockIdx.y;
  const int r0 = blockIdx.x * SK_ROWS;
  X += group * x_gs;
  W += group * w_gs;
  if (W2) W2 += group * w_gs;
  const int DT = W2 ? 2 * D : D;  // outputs of this launch
  float acc[SK_ROWS][DM];
#pragma unroll
  for (int r = 0; r < SK_ROWS; ++r)
#pragma unroll
    for (int o = 0; o < DM; ++o) acc[r][o] = 0.f;
  const int k0 = split * SK_CHUNK, k1 = min(K, k0 + SK_CHUNK);
  for (int k = k0 + threadIdx.x; k < k1; k += 256) {
    float w[DM];
#pragma unroll
    for (int o = 0; o < DM; ++o) w[o] = o < D ? W[k * sk + o * so] : (o < DT ? W2[k * sk + (o - D) * so] : 0.f);
#pragma unroll
    for (int r = 0; r < SK_ROWS; ++r) {
      if (r0 + r < B) {
        const float x = X[(long long)(r0 + r) * ldx + k];
#pragma unroll
        for (int o = 0; o < DM; ++o) acc[r][o] = fmaf(x, w[o], acc[r][o]);
      }
    }
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int r = 0; r < SK_ROWS; ++r)
#pragma unroll
    for (int o = 0; o < DM; ++o) {
      if (o < DT) {
        float v = wave_sum(acc[r][o]);
        if (lane == 0) red[wave][r][o] = v;
      }
    }
  __syncthreads();
  if (threadIdx.x < SK_ROWS * DM) {
    const int r = threadIdx.x / DM, o = threadIdx.x % DM;
    if (o < DT && r0 + r < B) {
      float v = red[0][r][o] + red[1][r][o] + red[2][r][o] + red[3][r][o];
      part[group * p_gs + ((long long)split * B + r0 + r) * pcols + (o < D ? coff + o : coff2 + o - D)] = v;
    }
  }
}

static void skinny(const float* X, int ldx, long long x_gs, int B, int K, const float* W, long long sk, long long so,
                   long long w_gs, int D, float* part, long long p_gs, int pcols, int coff, int groups,
                   hipStream_t s, const float* W2 = nullptr, int coff2 = 0) {
  dim3 grid((B + SK_ROWS - 1) / SK_ROWS, (K + SK_CHUNK - 1) / SK_CHUNK, groups);
  const int DT = W2 ? 2 * D : D;
  if (DT <= 4) hipLaunchKernelGGL(skinny_kernel<4>, grid, dim3(256), 0, s, X, ldx, x_gs, B, K, W, sk, so, w_gs, D,
                                  part, p_gs, pcols, coff, W2, coff2);
  else if (DT <= 8) hipLaunchKernelGGL(skinny_kernel<8>, grid, dim3(256), 0, s, X, ldx, x_gs, B, K, W, sk, so, w_gs,
                                       D, part, p_gs, pcols, coff, W2, coff2);
  else if (DT <= 32) hipLaunchKernelGGL(skinny_kernel<32>, grid, dim3(256), 0, s, X, ldx, x_gs, B, K, W, sk, so, w_gs,
                                        D, part, p_gs, pcols, coff, W2, coff2);
  else {  // wide heads: the two passes
    skinny(X, ldx, x_gs, B, K, W, sk, so, w_gs, D, part, p_gs, pcols, coff, groups, s);
    skinny(X, ldx, x_gs, B, K, W2, sk, so, w_gs, D, part, p_gs, pcols, coff2, groups, s);
  }
}

// Narrow heads (D <= 4, the CelebA latents): both heads over 8 rows and a 2048-wide K chunk per block.
// Each thread takes 4 consecutive k per step as one 16-byte X load per row and the matching 4*D
// contiguous weights of each head as D 16-byte loads (reused by the block's 8 rows: W is read B/8
// times, not B/4), then the per-thread sums go through the wave and the block in a fixed order.
#define HF_ROWS 8
#define HF_CHUNK 2048
template <int D>
__global__ __launch_bounds__(256) void heads_fwd_kernel(const float* __restrict__ X, long long x_gs, int B, int K,
                                                        const float* __restrict__ Wm, const float* __restrict__ Ws,
                                                        long long w_gs, float* __restrict__ part, long long p_gs,
                                                        int pcols, int coff, int coff2) {
  __shared__ float red[4][HF_ROWS][2 * D];
  const int group = blockIdx.z, split = blockIdx.y, r0 = blockIdx.x * HF_ROWS;
  X += group * x_gs;
  Wm += group * w_gs;
  Ws += group * w_gs;
  float acc[HF_ROWS][2 * D];
#pragma unroll
  for (int r = 0; r < HF_ROWS; ++r)
#pragma unroll
    for (int o = 0; o < 2 * D; ++o) acc[r][o] = 0.f;
  const int k1 = min(K, (split + 1) * HF_CHUNK);
  for (int k = split * HF_CHUNK + 4 * threadIdx.x; k < k1; k += 1024) {
    float wm[4 * D], ws[4 * D];  // [j][o] of k + j
#pragma unroll
    for (int i = 0; i < D; ++i) {
      const f32x4 a = *(const f32x4*)(Wm + (long long)k * D + 4 * i), b = *(const f32x4*)(Ws + (long long)k * D + 4 * i);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        wm[4 * i + e] = a[e];
        ws[4 * i + e] = b[e];
      }
    }
    f32x4 x[HF_ROWS];
#pragma unroll
    for (int r = 0; r < HF_ROWS; ++r)
      x[r] = r0 + r < B ? *(const f32x4*)(X + (long long)(r0 + r) * K + k) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < HF_ROWS; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int o = 0; o < D; ++o) {
          acc[r][o] = fmaf(x[r][j], wm[j * D + o], acc[r][o]);
          acc[r][D + o] = fmaf(x[r][j], ws[j * D + o], acc[r][D + o]);
        }
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int r = 0; r < HF_ROWS; ++r)
#pragma unroll
    for (int o = 0; o < 2 * D; ++o) {
      const float v = wave_sum(acc[r][o]);
      if (lane == 0) red[wave][r][o] = v;
    }
  __syncthreads();
  if (threadIdx.x < HF_ROWS * 2 * D) {
    const int r = threadIdx.x / (2 * D), o = threadIdx.x % (2 * D);
    if (r0 + r < B) {
      const float v = red[0][r][o] + red[1][r][o] + red[2][r][o] + red[3][r][o];
      part[group * p_gs + ((long long)split * B + r0 + r) * pcols + (o < D ? coff + o : coff2 + o - D)] = v;
    }
  }
}

int heads_splits(int K) { return (K + HF_CHUNK - 1) / HF_CHUNK; }

static bool heads_narrow_off() {  // SVAE_HEADS_SKINNY=1: the former 4-row skinny pass (A/B)
  static const bool v = svae_knob("SVAE_HEADS_SKINNY", 0) == 1;
  return v;
}

// Wide heads (4 < D <= 32, e.g. LSUN's 20-30 latents per level): a block owns 64 batch rows x both heads'
// 2D outputs (padded to 64) over one HF_CHUNK split of K, staged through LDS 32 k at a time; each thread
// keeps a 4 x 4 output tile.  The weights of a split are read once per 64 rows (skinny_kernel<32> read
// them once per 4 rows and spilled: 3.9 GB of L2 traffic and 630 us per LSUN level-0 launch).
#define HT_KS 32
__global__ __launch_bounds__(256) void heads_tile_fwd_kernel(const float* __restrict__ X, long long x_gs, int B, int K,
                                                             const float* __restrict__ Wm, const float* __restrict__ Ws,
                                                             long long w_gs, int D, float* __restrict__ part,
                                                             long long p_gs, int pcols, int coff, int coff2) {
  __shared__ __attribute__((aligned(16))) float xs[64][HT_KS + 4];  // pitch 36: 16-byte row reads, 4 rows per wave in 4 banks
  __shared__ __attribute__((aligned(16))) float ws[HT_KS][64];
  const int group = blockIdx.z, split = blockIdx.y, r0 = blockIdx.x * 64;
  X += group * x_gs;
  Wm += group * w_gs;
  Ws += group * w_gs;
  const int tid = threadIdx.x, tr = tid >> 4, tc = tid & 15;
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
  const int k0 = split * HF_CHUNK, k1 = min(K, k0 + HF_CHUNK);
  for (int kb = k0; kb < k1; kb += HT_KS) {
    {  // X: 64 rows x 32 k, 8 consecutive k per thread
      const int row = tid >> 2, kp = (tid & 3) * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = kb + kp + e;
        xs[row][kp + e] = (r0 + row < B && k < k1) ? X[(long long)(r0 + row) * K + k] : 0.f;
      }
    }
    {  // W: 32 k x [mean D | std D | 0 ...], 8 columns per thread
      const int kk = tid >> 3, c0 = (tid & 7) * 8;
      const int k = kb + kk;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = c0 + e;
        float w = 0.f;
        if (k < k1) {
          if (c < D) w = Wm[(long long)k * D + c];
          else if (c < 2 * D) w = Ws[(long long)k * D + c - D];
        }
        ws[kk][c] = w;
      }
    }
    __syncthreads();
#pragma unroll 2
    for (int kk = 0; kk < HT_KS; kk += 4) {  // 4 k per step: 8 16-byte LDS reads for 64 fma (same order per output)
      f32x4 x[4], w[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) x[i] = *(const f32x4*)&xs[4 * tr + i][kk];
#pragma unroll
      for (int q = 0; q < 4; ++q) w[q] = *(const f32x4*)&ws[kk + q][4 * tc];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(x[i][q], w[q][j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = r0 + 4 * tr + i;
    if (r >= B) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int o = 4 * tc + j;
      if (o < 2 * D)
        part[group * p_gs + ((long long)split * B + r) * pcols + (o < D ? coff + o : coff2 + o - D)] = acc[i][j];
    }
  }
}

void heads_fwd(const float* X, long long x_gs, int B, int K, const float* Wm, const float* Ws, long long w_gs, int D,
               float* part, long long part_gs, int pcols, int coff, int groups, hipStream_t s) {
  // mean and stddev heads in one pass over X (the shared recognition features)
  const bool al = ((uintptr_t)X % 16 == 0) && ((uintptr_t)Wm % 16 == 0) && ((uintptr_t)Ws % 16 == 0) &&
                  (x_gs % 4 == 0) && (w_gs % 4 == 0);
  if (D <= 4 && K % 4 == 0 && al && !heads_narrow_off()) {
    dim3 grid((B + HF_ROWS - 1) / HF_ROWS, heads_splits(K), groups);
    const int c2 = pcols / 2 + coff;
#define HF_L(DD) hipLaunchKernelGGL(heads_fwd_kernel<DD>, grid, dim3(256), 0, s, X, x_gs, B, K, Wm, Ws, w_gs, part, \
                                    part_gs, pcols, coff, c2)
    if (D == 1) HF_L(1);
    else if (D == 2) HF_L(2);
    else if (D == 3) HF_L(3);
    else HF_L(4);
#undef HF_L
    return;
  }
  // SVAE_HEADS_TILE bit 0 off: the skinny pass for the wide heads (knob builds read it per call: the A/B tests)
  const bool tile_off = !(svae_knob("SVAE_HEADS_TILE", 3) & 1);
  if (D > 4 && D <= 32 && !tile_off) {
    dim3 grid((B + 63) / 64, heads_splits(K), groups);
    hipLaunchKernelGGL(heads_tile_fwd_kernel, grid, dim3(256), 0, s, X, x_gs, B, K, Wm, Ws, w_gs, D, part, part_gs, pcols,
                       coff, pcols / 2 + coff);
    return;
  }
  // the splits follow HF_CHUNK (heads_splits); skinny's chunk must match
  skinny(X, K, x_gs, B, K, Wm, D, 1, w_gs, D, part, part_gs, pcols, coff, groups, s, Ws, pcols / 2 + coff);
}

// dz[n][zoff+d] += sum_split part   where part = skinny(dpre [B][J], W^T)
// dz[n][zoff+d] += sum over blocks of part[blk][n][d]: one wave per (n, d)
__global__ void splitfc_dz_kernel(const float* part, int nsplit, int B, int K, float* dz, int ldz, int zoff) {
  const int wv = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  if (wv >= B * K) return;
  const int n = wv / K, d = wv % K;
  float s = 0.f;
  for (int sp = lane; sp < nsplit; sp += 64) s += part[((long long)sp * B + n) * K + d];
  s = wave_sum(s);
  if (lane == 0) dz[n * ldz + zoff + d] += s;
}

void splitfc_dz_reduce(const float* dz_part, int nblk, int B, int K, float* dz, int ldz, int zoff, hipStream_t s) {
  hipLaunchKernelGGL(splitfc_dz_kernel, dim3((B * K * 64 + 255) / 256), dim3(256), 0, s, dz_part, nblk, B, K, dz, ldz,
                     zoff);
}

// ---------------------------------------------------------------------------
// latent: mu = clip(sum + bm), sig = sigmoid(sum + bs), z = mu + sig*eps, KL per image
// (sequential_vae.py:1592-1594, :1023, :1156-1158)
// ---------------------------------------------------------------------------
// one thread per (image, latent dimension): the 2 x nsplit head partials of a dimension load
// together, 32 splits at a time (summed in split order for any nsplit), and each image's KL terms
// are added in dimension order from LDS (the order of the former one-thread-per-image loop: bitwise
// the same mu, sigma, z and KL).  Blocks of 256 threads hold 256 / Dz images (Dz <= 256: make_geo caps
// the latent at 8 levels x 32 dimensions and svae_create rejects more).
__global__ __launch_bounds__(256) void latent_fwd_kernel(const float* __restrict__ part, long long part_gs,
                                                          int nsplit, int B, int Dz, LatentLvls lv, long long bias_gs,
                                                          float clipv, float prior, int uniform,
                                                          const float* __restrict__ eps, long long eps_gs,
                                                          float* __restrict__ mu, float* __restrict__ sig,
                                                          float* __restrict__ z, long long ms_gs,
                                                          float* __restrict__ kl_img, long long kl_gs) {
  __shared__ float klt[1024];
  const int group = blockIdx.y;
  const int ipb = (int)blockDim.x / Dz;  // images per block
  const int il = threadIdx.x / Dz, c = threadIdx.x - il * Dz;
  const int n = blockIdx.x * ipb + il;
  const bool act = il < ipb && n < B;
  float term = 0.f;
  if (act) {
    int l = 0;
    while (l + 1 < lv.L && c >= lv.off[l + 1]) ++l;
    const int d = c - lv.off[l];
    const float* P = part + group * part_gs;
    float sm = 0.f, ss = 0.f;
    for (int s0 = 0; s0 < nsplit; s0 += 32) {
      float pm[32], ps[32];
#pragma unroll
      for (int sp = 0; sp < 32; ++sp) {
        pm[sp] = s0 + sp < nsplit ? P[((long long)(s0 + sp) * B + n) * 2 * Dz + c] : 0.f;
        ps[sp] = s0 + sp < nsplit ? P[((long long)(s0 + sp) * B + n) * 2 * Dz + Dz + c] : 0.f;
      }
#pragma unroll
      for (int sp = 0; sp < 32; ++sp)
        if (s0 + sp < nsplit) {
          sm += pm[sp];
          ss += ps[sp];
        }
    }
    const float p2 = prior * prior;
    const float m = sm + lv.bm[l][group * bias_gs + d];
    const float mc = fminf(fmaxf(m, -clipv), clipv);
    const float sg = sigmoid_f(ss + lv.bs[l][group * bias_gs + d]);
    const long long o = group * ms_gs + (long long)n * Dz + c;
    mu[o] = m;  // raw (pre-clip) mean; the clip mask is re-derived in latent_bwd
    sig[o] = sg;
    z[o] = mc + sg * eps[group * eps_gs + (long long)n * Dz + c];
    // use_uniform_prior: reduce_mean(-log sigma) (sequential_vae.py:1159-1160)
    term = uniform ? -__logf(sg) : -0.5f - __logf(sg) + 0.5f * sg * sg / p2 + 0.5f * mc * mc / p2;
  }
  klt[threadIdx.x] = term;
  __syncthreads();
  if (act && c == 0) {
    float kl = 0.f;
    for (int j = 0; j < Dz; ++j) kl += klt[threadIdx.x + j];
    kl_img[group * kl_gs + n] = kl / Dz;
  }
}

void latent_fwd(const float* part, long long part_gs, int nsplit, int B, int Dz, const LatentLvls& lv,
                long long bias_gs, float clipv, float prior, int uniform, const float* eps, long long eps_gs, float* mu,
                float* sig, float* z, long long ms_gs, float* kl_img, long long kl_gs, int groups, hipStream_t s) {
  const int bs = 256;  // (svae_create rejects Dz > 256)
  const int ipb = bs / Dz;
  hipLaunchKernelGGL(latent_fwd_kernel, dim3((B + ipb - 1) / ipb, groups), dim3(bs), 0, s, part, part_gs, nsplit, B, Dz,
                     lv, bias_gs, clipv, prior, uniform, eps, eps_gs, mu, sig, z, ms_gs, kl_img, kl_gs);
}

// dhead[n][d] = d(mu_raw), dhead[n][Dz+d] = d(sig pre-sigmoid); kl_coef = reg*c_first/B
__global__ void latent_bwd_kernel(const float* mu, const float* sig, const float* eps, const float* dz, long long gs,
                                  long long eps_gs, int B, int Dz, const float* kl_coef, long long kc_gs, float prior,
                                  int uniform, float clipv, float* dhead, long long dh_gs) {
  const int group = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * Dz) return;
  const int n = i / Dz, c = i % Dz;
  const long long o = group * gs + i;
  const float p2 = prior * prior;
  const float kc = kl_coef[group * kc_gs] / Dz;
  const float m = mu[o], sg = sig[o], g = dz[o];
  const bool pass = m >= -clipv && m <= clipv;
  const float mc = fminf(fmaxf(m, -clipv), clipv);
  const float dmu = pass ? (uniform ? g : g + kc * mc / p2) : 0.f;
  const float dsig = g * eps[group * eps_gs + i] + kc * (uniform ? -1.f / sg : -1.f / sg + sg / p2);
  dhead[group * dh_gs + (long long)n * 2 * Dz + c] = dmu;
  dhead[group * dh_gs + (long long)n * 2 * Dz + Dz + c] = dsig * sg * (1.f - sg);
}

void latent_bwd(const float* mu, const float* sig, const float* eps, const float* dz, long long gs, long long eps_gs,
                int B, int Dz, const float* kl_coef, long long kc_gs, float prior, int uniform, float clipv, float* dhead,
                long long dh_gs, int groups, hipStream_t s) {
  hipLaunchKernelGGL(latent_bwd_kernel, dim3((B * Dz + 255) / 256, groups), dim3(256), 0, s, mu, sig, eps, dz, gs,
                     eps_gs, B, Dz, kl_coef, kc_gs, prior, uniform, clipv, dhead, dh_gs);
}

// heads backward for one level: dX (+)= dhead_l @ W^T ; dW = X^T dhead_l ; db = sum_n dhead_l
template <int DM>
__global__ __launch_bounds__(256) void heads_bwd_kernel(const float* __restrict__ X, long long x_gs,
                                                        float* __restrict__ dX, long long dx_gs, int B, int K,
                                                        const float* __restrict__ Wm, const float* __restrict__ Ws,
                                                        long long w_gs, int D, const float* __restrict__ dhead,
                                                        long long dh_gs, int dcols, int coff, float* __restrict__ dWm,
                                                        float* __restrict__ dWs, float* __restrict__ dbm,
                                                        float* __restrict__ dbs, int accumulate) {
  extern __shared__ float dh[];  // [B][2*D]
  const int group = blockIdx.y;
  X += group * x_gs;
  dX += group * dx_gs;
  Wm += group * w_gs;
  Ws += group * w_gs;
  dhead += group * dh_gs;
  for (int i = threadIdx.x; i < B * 2 * D; i += blockDim.x) {
    const int n = i / (2 * D), o = i % (2 * D);
    dh[i] = dhead[(long long)n * dcols + (o < D ? coff + o : dcols / 2 + coff + o - D)];
  }
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x < 2 * D) {
    float s = 0.f;
    for (int n = 0; n < B; ++n) s += dh[n * 2 * D + threadIdx.x];
    if (threadIdx.x < D) dbm[group * w_gs + threadIdx.x] = s;
    else dbs[group * w_gs + threadIdx.x - D] = s;
  }
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  float wm[DM], ws[DM], gm[DM], gs[DM];
#pragma unroll
  for (int o = 0; o < DM; ++o) {
    wm[o] = o < D ? Wm[(long long)k * D + o] : 0.f;
    ws[o] = o < D ? Ws[(long long)k * D + o] : 0.f;
    gm[o] = gs[o] = 0.f;
  }
  // rows in groups of 8: the 8 independent loads (and accumulate reads) issue together
  // (same per-thread operation order as one row at a time: bitwise the same result)
  constexpr int RB = 8;
  for (int n0 = 0; n0 < B; n0 += RB) {
    float xs[RB], old[RB];
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const int n = n0 + j;
      xs[j] = n < B ? X[(long long)n * K + k] : 0.f;
      old[j] = (accumulate && n < B) ? dX[(long long)n * K + k] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const int n = n0 + j;
      if (n >= B) break;
      float dx = 0.f;
#pragma unroll
      for (int o = 0; o < DM; ++o) {
        if (o < D) {
          const float a = dh[n * 2 * D + o], b = dh[n * 2 * D + D + o];
          dx = fmaf(a, wm[o], fmaf(b, ws[o], dx));
          gm[o] = fmaf(xs[j], a, gm[o]);
          gs[o] = fmaf(xs[j], b, gs[o]);
        }
      }
      dX[(long long)n * K + k] = accumulate ? old[j] + dx : dx;
    }
  }
#pragma unroll
  for (int o = 0; o < DM; ++o)
    if (o < D) {
      dWm[group * w_gs + (long long)k * D + o] = gm[o];
      dWs[group * w_gs + (long long)k * D + o] = gs[o];
    }
}

// The same with the batch rows split over HR_RG thread groups of a block (64 k per block): a thread walks
// B / HR_RG rows instead of all B (4 dependent load batches instead of 16 at B = 128: the one-k-per-thread
// form is latency-bound at ~1.7 TB/s), and the RG partial weight-gradient sums of a k are added in LDS
// in row-group order (deterministic; a different summation order from heads_bwd_kernel)
#define HR_RG 4
template <int DM>
__global__ __launch_bounds__(256) void heads_bwd_rg_kernel(const float* __restrict__ X, long long x_gs,
                                                           float* __restrict__ dX, long long dx_gs, int B, int K,
                                                           const float* __restrict__ Wm, const float* __restrict__ Ws,
                                                           long long w_gs, int D, const float* __restrict__ dhead,
                                                           long long dh_gs, int dcols, int coff, float* __restrict__ dWm,
                                                           float* __restrict__ dWs, float* __restrict__ dbm,
                                                           float* __restrict__ dbs, int accumulate) {
  extern __shared__ float dh[];  // [B][2*D], then the partial sums [2 * DM][HR_RG][64]
  float* red = dh + B * 2 * D;
  const int group = blockIdx.y;
  X += group * x_gs;
  dX += group * dx_gs;
  Wm += group * w_gs;
  Ws += group * w_gs;
  dhead += group * dh_gs;
  for (int i = threadIdx.x; i < B * 2 * D; i += blockDim.x) {
    const int n = i / (2 * D), o = i % (2 * D);
    dh[i] = dhead[(long long)n * dcols + (o < D ? coff + o : dcols / 2 + coff + o - D)];
  }
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x < 2 * D) {
    float s = 0.f;
    for (int n = 0; n < B; ++n) s += dh[n * 2 * D + threadIdx.x];
    if (threadIdx.x < D) dbm[group * w_gs + threadIdx.x] = s;
    else dbs[group * w_gs + threadIdx.x - D] = s;
  }
  const int kl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int k = blockIdx.x * 64 + kl;
  const bool kv = k < K;
  float wm[DM], ws[DM], gm[DM], gs[DM];
#pragma unroll
  for (int o = 0; o < DM; ++o) {
    wm[o] = (kv && o < D) ? Wm[(long long)k * D + o] : 0.f;
    ws[o] = (kv && o < D) ? Ws[(long long)k * D + o] : 0.f;
    gm[o] = gs[o] = 0.f;
  }
  const int rows = B / HR_RG, r0 = rg * rows;
  constexpr int RB = 8;
  if (kv) {
    for (int n0 = r0; n0 < r0 + rows; n0 += RB) {
      float xs[RB], old[RB];
#pragma unroll
      for (int j = 0; j < RB; ++j) {
        const int n = n0 + j;
        const bool ok = n < r0 + rows;
        xs[j] = ok ? X[(long long)n * K + k] : 0.f;
        old[j] = (accumulate && ok) ? dX[(long long)n * K + k] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < RB; ++j) {
        const int n = n0 + j;
        if (n >= r0 + rows) break;
        float dx = 0.f;
#pragma unroll
        for (int o = 0; o < DM; ++o) {
          if (o < D) {
            const float a = dh[n * 2 * D + o], b = dh[n * 2 * D + D + o];
            dx = fmaf(a, wm[o], fmaf(b, ws[o], dx));
            gm[o] = fmaf(xs[j], a, gm[o]);
            gs[o] = fmaf(xs[j], b, gs[o]);
          }
        }
        dX[(long long)n * K + k] = accumulate ? old[j] + dx : dx;
      }
    }
  }
#pragma unroll
  for (int o = 0; o < DM; ++o) {
    red[((2 * o) * HR_RG + rg) * 64 + kl] = gm[o];
    red[((2 * o + 1) * HR_RG + rg) * 64 + kl] = gs[o];
  }
  __syncthreads();
  if (rg == 0 && kv) {
#pragma unroll
    for (int o = 0; o < DM; ++o)
      if (o < D) {
        float sm = 0.f, ss = 0.f;
#pragma unroll
        for (int g = 0; g < HR_RG; ++g) {
          sm += red[((2 * o) * HR_RG + g) * 64 + kl];
          ss += red[((2 * o + 1) * HR_RG + g) * 64 + kl];
        }
        dWm[group * w_gs + (long long)k * D + o] = sm;
        dWs[group * w_gs + (long long)k * D + o] = ss;
      }
  }
}

// Wide heads backward (8 < D <= 32): a block owns 64 k columns over all B rows, 32 rows at a time through
// LDS: dW[k][o] = sum_n X[n][k] dh[n][o] (a 4 k x 4 o tile per thread, accumulated over the row steps in
// row order) and dX[n][k] (+)= sum_o dh[n][o] W[k][o] (2 rows x 4 k per thread) with the block's weights
// held in LDS transposed [o][k].  heads_bwd_kernel<32> (one k per thread over every row, 188 VGPRs) took
// 1.2 ms per LSUN level-0 launch.
__global__ __launch_bounds__(256) void heads_tile_bwd_kernel(const float* __restrict__ X, long long x_gs,
                                                             float* __restrict__ dX, long long dx_gs, int B, int K,
                                                             const float* __restrict__ Wm, const float* __restrict__ Ws,
                                                             long long w_gs, int D, const float* __restrict__ dhead,
                                                             long long dh_gs, int dcols, int coff, float* __restrict__ dWm,
                                                             float* __restrict__ dWs, float* __restrict__ dbm,
                                                             float* __restrict__ dbs, int accumulate) {
  __shared__ __attribute__((aligned(16))) float wt[64][64];   // [o][k]
  __shared__ __attribute__((aligned(16))) float xs[32][64];   // [n][k]
  __shared__ __attribute__((aligned(16))) float dhs[32][68];  // [n][o] (pitch 68: the dX loop's 4 rows per wave in 4 banks)
  const int group = blockIdx.y, k0 = blockIdx.x * 64, tid = threadIdx.x;
  X += group * x_gs;
  dX += group * dx_gs;
  Wm += group * w_gs;
  Ws += group * w_gs;
  dhead += group * dh_gs;
  auto dh_at = [&](int n, int o) -> float {
    return o < D ? dhead[(long long)n * dcols + coff + o] : (o < 2 * D ? dhead[(long long)n * dcols + dcols / 2 + coff + o - D] : 0.f);
  };
  if (blockIdx.x == 0 && tid < 2 * D) {  // bias gradients (row order)
    float sb = 0.f;
    for (int n = 0; n < B; ++n) sb += dh_at(n, tid);
    if (tid < D) dbm[group * w_gs + tid] = sb;
    else dbs[group * w_gs + tid - D] = sb;
  }
  for (int i = tid; i < 64 * 64; i += 256) {
    const int kk = i >> 6, o = i & 63, k = k0 + kk;
    float w = 0.f;
    if (k < K) {
      if (o < D) w = Wm[(long long)k * D + o];
      else if (o < 2 * D) w = Ws[(long long)k * D + o - D];
    }
    wt[o][kk] = w;
  }
  const int tk = tid >> 4, tq = tid & 15;  // dW: k = 4 tk .. + 3, o = 4 tq .. + 3;  dX: rows 2 tk, 2 tk + 1, k = 4 tq ..
  float gw[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) gw[i][j] = 0.f;
  for (int n0 = 0; n0 < B; n0 += 32) {
    __syncthreads();  // (wt written; the previous step's xs / dhs read)
    for (int i = tid; i < 32 * 64; i += 256) {
      const int r = i >> 6, c = i & 63, n = n0 + r, k = k0 + c;
      xs[r][c] = (n < B && k < K) ? X[(long long)n * K + k] : 0.f;
      dhs[r][c] = n < B ? dh_at(n, c) : 0.f;
    }
    __syncthreads();
#pragma unroll 4
    for (int r = 0; r < 32; ++r) {
      const f32x4 x = *(const f32x4*)&xs[r][4 * tk];
      const f32x4 g = *(const f32x4*)&dhs[r][4 * tq];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) gw[i][j] = fmaf(x[i], g[j], gw[i][j]);
    }
    f32x4 dx[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll 2
    for (int o = 0; o < 64; o += 4) {  // 4 o per step: 6 16-byte LDS reads for 32 fma (same order per output)
      f32x4 w[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) w[q] = *(const f32x4*)&wt[o + q][4 * tq];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 d = *(const f32x4*)&dhs[2 * tk + h][o];
#pragma unroll
        for (int q = 0; q < 4; ++q) dx[h] += d[q] * w[q];
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int n = n0 + 2 * tk + h;
      if (n >= B) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = k0 + 4 * tq + e;
        if (k >= K) continue;
        float* d = dX + (long long)n * K + k;
        *d = accumulate ? *d + dx[h][e] : dx[h][e];
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = k0 + 4 * tk + i;
    if (k >= K) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int o = 4 * tq + j;
      if (o < D) dWm[group * w_gs + (long long)k * D + o] = gw[i][j];
      else if (o < 2 * D) dWs[group * w_gs + (long long)k * D + o - D] = gw[i][j];
    }
  }
}

void heads_bwd(const float* X, long long x_gs, float* dX, long long dx_gs, int B, int K, const float* Wm,
               const float* Ws, long long w_gs, int D, const float* dhead, long long dh_gs, int dcols, int coff,
               float* dWm, float* dWs, float* dbm, float* dbs, int accumulate, int groups, hipStream_t s) {
  // SVAE_HEADS_TILE bit 1 off: heads_bwd_kernel<32> for the wide heads (knob builds: per call)
  const bool tile_off = !(svae_knob("SVAE_HEADS_TILE", 3) & 2);
  if (D > 8 && D <= 32 && !tile_off) {
    dim3 grid((K + 63) / 64, groups);
    hipLaunchKernelGGL(heads_tile_bwd_kernel, grid, dim3(256), 0, s, X, x_gs, dX, dx_gs, B, K, Wm, Ws, w_gs, D, dhead,
                       dh_gs, dcols, coff, dWm, dWs, dbm, dbs, accumulate);
    return;
  }
  // SVAE_HEADS_RG=0: one thread per k over all rows (round 3; knob builds: per call)
  const bool rg_on = svae_knob("SVAE_HEADS_RG", 1) != 0;
  if (rg_on && B % (HR_RG * 8) == 0 && D <= 8) {
    dim3 grid((K + 63) / 64, groups);
    size_t lds = (size_t)B * 2 * D * sizeof(float) + (size_t)2 * 8 * HR_RG * 64 * sizeof(float);
    if (D <= 4)
      hipLaunchKernelGGL(heads_bwd_rg_kernel<4>, grid, dim3(256), lds, s, X, x_gs, dX, dx_gs, B, K, Wm, Ws, w_gs, D,
                         dhead, dh_gs, dcols, coff, dWm, dWs, dbm, dbs, accumulate);
    else
      hipLaunchKernelGGL(heads_bwd_rg_kernel<8>, grid, dim3(256), lds, s, X, x_gs, dX, dx_gs, B, K, Wm, Ws, w_gs, D,
                         dhead, dh_gs, dcols, coff, dWm, dWs, dbm, dbs, accumulate);
    return;
  }
  dim3 grid((K + 255) / 256, groups);
  size_t lds = (size_t)B * 2 * D * sizeof(float);
  if (D <= 4)
    hipLaunchKernelGGL(heads_bwd_kernel<4>, grid, dim3(256), lds, s, X, x_gs, dX, dx_gs, B, K, Wm, Ws, w_gs, D, dhead,
                       dh_gs, dcols, coff, dWm, dWs, dbm, dbs, accumulate);
  else if (D <= 8)
    hipLaunchKernelGGL(heads_bwd_kernel<8>, grid, dim3(256), lds, s, X, x_gs, dX, dx_gs, B, K, Wm, Ws, w_gs, D, dhead,
                       dh_gs, dcols, coff, dWm, dWs, dbm, dbs, accumulate);
  else
    hipLaunchKernelGGL(heads_bwd_kernel<32>, grid, dim3(256), lds, s, X, x_gs, dX, dx_gs, B, K, Wm, Ws, w_gs, D,
                       dhead, dh_gs, dcols, coff, dWm, dWs, dbm, dbs, accumulate);
}

// ---------------------------------------------------------------------------
// small-N gather conv (N <= 4): C[p][o] (+)= bias + sum_tap sum_k A[src(p,tap)][k] * W(tap,o,k)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void gconv_smalln_kernel(const float* A, int lda, int K, const float* W0, int n0,
                                                           const float* W1, int n1, long long w_tap,
                                                           long long w1_tap, const float* bias0, const float* bias1,
                                                           ConvGeom g, long long rows, float* C, int ldc,
                                                           int accumulate) {
  extern __shared__ float ws[];  // [16 taps][4][K]
  const int taps = g.ksz * g.ksz;
  const int N = n0 + n1;
  for (int i = threadIdx.x; i < taps * 4 * K; i += blockDim.x) {
    const int t = i / (4 * K), r = i % (4 * K), o = r / K, k = r % K;
    float v = 0.f;
    if (o < n0) v = W0[t * w_tap + (long long)o * K + k];
    else if (o < N) v = W1[t * w1_tap + (long long)(o - n0) * K + k];
    ws[i] = v;
  }
  __syncthreads();
  const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= rows) return;
  const int HWo = g.Ho * g.Wo;
  const int n = (int)(p / HWo);
  const int rem = (int)(p - (long long)n * HWo);
  const int oy = rem / g.Wo, ox = rem % g.Wo;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int ky = 0; ky < g.ksz; ++ky) {
    int iy;
    if (g.mode == GM_CONV) iy = oy * g.stride - g.pad + ky;
    else {
      int t = oy + g.pad - ky;
      if (t < 0 || (t % g.stride) != 0) continue;
      iy = t / g.stride;
    }
    if (iy < 0 || iy >= g.Hi) continue;
    for (int kx = 0; kx < g.ksz; ++kx) {
      int ix;
      if (g.mode == GM_CONV) ix = ox * g.stride - g.pad + kx;
      else {
        int t = ox + g.pad - kx;
        if (t < 0 || (t % g.stride) != 0) continue;
        ix = t / g.stride;
      }
      if (ix < 0 || ix >= g.Wi) continue;
      const float* a = A + ((long long)(n * g.Hi + iy) * g.Wi + ix) * lda;
      const float* w = ws + (ky * g.ksz + kx) * 4 * K;
      if ((K & 3) == 0 && (lda & 3) == 0) {
        for (int k = 0; k < K; k += 4) {
          f32x4 av = *(const f32x4*)(a + k);
#pragma unroll
          for (int o = 0; o < 4; ++o)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[o] = fmaf(av[e], w[o * K + k + e], acc[o]);
        }
      } else {
        for (int k = 0; k < K; ++k) {
          const float av = a[k];
#pragma unroll
          for (int o = 0; o < 4; ++o) acc[o] = fmaf(av, w[o * K + k], acc[o]);
        }
      }
    }
  }
  for (int o = 0; o < N; ++o) {
    float v = acc[o];
    if (o < n0 && bias0) v += bias0[o];
    if (o >= n0 && bias1) v += bias1[o - n0];
    float* d = C + p * ldc + o;
    *d = accumulate ? *d + v : v;
  }
}

// Lane-parallel variant for K % 4 == 0, K/4 a power of two <= 64 (the CelebA output layer and
// layer-0 input gradient: K = 32): LP = K/4 lanes share one output pixel, each owning a channel
// quad, so a pixel's gather is one coalesced 16*LP-byte read; the 4 partial outputs are
// summed across the LP lanes with xor shuffles.  stride is 1 or 2 (shift / mask, no division).
template <int LP>
__global__ __launch_bounds__(256) void gconv_smalln_lp_kernel(const float* A, int lda, int K, const float* W0, int n0,
                                                              const float* W1, int n1, long long w_tap,
                                                              long long w1_tap, const float* bias0, const float* bias1,
                                                              ConvGeom g, long long rows, float* C, int ldc,
                                                              int accumulate) {
  extern __shared__ float ws[];  // [16 taps][K][4] (output fastest: one f32x4 per channel)
  const int taps = g.ksz * g.ksz;
  const int N = n0 + n1;
  for (int i = threadIdx.x; i < taps * 4 * K; i += blockDim.x) {
    const int t = i / (4 * K), r = i - t * 4 * K, k = r >> 2, o = r & 3;
    float v = 0.f;
    if (o < n0) v = W0[t * w_tap + (long long)o * K + k];
    else if (o < N) v = W1[t * w1_tap + (long long)(o - n0) * K + k];
    ws[i] = v;
  }
  __syncthreads();
  const int HWo = g.Ho * g.Wo;
  const int sm = g.stride - 1, sh = g.stride == 2 ? 1 : 0;
  const int cq = threadIdx.x % LP;
  // grid-stride over pixels: the weight table above is staged once per block
  for (long long p0 = (long long)blockIdx.x * (blockDim.x / LP); p0 < rows; p0 += (long long)gridDim.x * (blockDim.x / LP)) {
    const long long p = p0 + threadIdx.x / LP;
    const bool live = p < rows;
    const long long pp = live ? p : 0;
    const int n = (int)(pp / HWo);
    const int rem = (int)(pp - (long long)n * HWo);
    const int oy = rem / g.Wo, ox = rem - (rem / g.Wo) * g.Wo;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int ky = 0; ky < g.ksz; ++ky) {
      int iy;
      if (g.mode == GM_CONV) iy = oy * g.stride - g.pad + ky;
      else {
        const int t = oy + g.pad - ky;
        if (t < 0 || (t & sm)) continue;
        iy = t >> sh;
      }
      if (iy < 0 || iy >= g.Hi) continue;
      for (int kx = 0; kx < g.ksz; ++kx) {
        int ix;
        if (g.mode == GM_CONV) ix = ox * g.stride - g.pad + kx;
        else {
          const int t = ox + g.pad - kx;
          if (t < 0 || (t & sm)) continue;
          ix = t >> sh;
        }
        if (ix < 0 || ix >= g.Wi) continue;
        const f32x4* w = (const f32x4*)(ws + (ky * g.ksz + kx) * 4 * K) + cq * 4;
        for (int kk = cq * 4; kk < K; kk += 4 * LP) {
          const f32x4 av = *(const f32x4*)(A + ((long long)(n * g.Hi + iy) * g.Wi + ix) * lda + kk);
          const f32x4* wk = w + (kk - cq * 4);
          acc += av[0] * wk[0] + av[1] * wk[1] + av[2] * wk[2] + av[3] * wk[3];
        }
      }
    }
#pragma unroll
    for (int o = LP / 2; o > 0; o >>= 1) {
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] += __shfl_xor(acc[e], o, 64);
    }
    if (live && cq < N) {
      float v = acc[cq];
      if (cq < n0 && bias0) v += bias0[cq];
      if (cq >= n0 && bias1) v += bias1[cq - n0];
      float* d = C + p * ldc + cq;
      *d = accumulate ? *d + v : v;
    }
  }
}

// Stride-2 conv-T gather with <= 4 outputs and K = 4*LP channels (output / ratio conv-T and the
// layer-0 input gradient): grid.y = output parity class (cy, cx), whose 2x2 taps are fixed, so
// each lane keeps its 4 channels x 4 taps x 4 outputs of weights in registers; LP lanes share a
// pixel (one coalesced 16*LP-byte read per tap) and are summed with xor shuffles.
template <int LP>
__global__ __launch_bounds__(256) void gconv_s2t_kernel(const float* A, int lda, int K, const float* W0, int n0,
                                                        const float* W1, int n1, long long w_tap, long long w1_tap,
                                                        const float* bias0, const float* bias1, ConvGeom g,
                                                        float* C, int ldc, int accumulate) {
  const int cls = blockIdx.y, cy = cls >> 1, cx = cls & 1;
  const int ky0 = (cy + g.pad) & 1, kx0 = (cx + g.pad) & 1;
  const int N = n0 + n1;
  const int cq = threadIdx.x % LP;
  f32x4 w[4][4];  // [tap][channel e] -> 4 outputs
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int tap = (ky0 + 2 * (t >> 1)) * g.ksz + kx0 + 2 * (t & 1);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = cq * 4 + e;
#pragma unroll
      for (int o = 0; o < 4; ++o) {
        float v = 0.f;
        if (o < n0) v = W0[tap * w_tap + (long long)o * K + k];
        else if (o < N) v = W1[tap * w1_tap + (long long)(o - n0) * K + k];
        w[t][e][o] = v;
      }
    }
  }
  const int qh = g.Ho >> 1, qw = g.Wo >> 1;
  const long long rows = (long long)g.nimg * qh * qw;
  for (long long q0 = (long long)blockIdx.x * (blockDim.x / LP); q0 < rows; q0 += (long long)gridDim.x * (blockDim.x / LP)) {
    const long long q = q0 + threadIdx.x / LP;
    const bool live = q < rows;
    const long long qq = live ? q : 0;
    const int n = (int)(qq / (qh * qw));
    const int r = (int)(qq - (long long)n * qh * qw);
    const int qy = r / qw, qx = r - (r / qw) * qw;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int iy = qy + (cy + g.pad - ky0) / 2 - (t >> 1);
      const int ix = qx + (cx + g.pad - kx0) / 2 - (t & 1);
      if (iy >= 0 && iy < g.Hi && ix >= 0 && ix < g.Wi) {
        const f32x4 av = *(const f32x4*)(A + ((long long)(n * g.Hi + iy) * g.Wi + ix) * lda + cq * 4);
        acc += av[0] * w[t][0] + av[1] * w[t][1] + av[2] * w[t][2] + av[3] * w[t][3];
      }
    }
#pragma unroll
    for (int o = LP / 2; o > 0; o >>= 1) {
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[e] += __shfl_xor(acc[e], o, 64);
    }
    if (live && cq < N) {
      float v = acc[cq];
      if (cq < n0 && bias0) v += bias0[cq];
      if (cq >= n0 && bias1) v += bias1[cq - n0];
      const long long orow = ((long long)n * g.Ho + 2 * qy + cy) * g.Wo + 2 * qx + cx;
      float* d = C + orow * ldc + cq;
      *d = accumulate ? *d + v : v;
    }
  }
}

void gconv_smalln(const float* A, int lda, int K, const float* W0, int n0, const float* W1, int n1, long long w_tap,
                  long long w1_tap, const float* bias0, const float* bias1, ConvGeom g, long long rows_total,
                  float* C, int ldc, int accumulate, hipStream_t s) {
  size_t lds = (size_t)g.ksz * g.ksz * 4 * K * sizeof(float);
  if (g.mode == GM_CONVT && g.stride == 2 && g.ksz == 4 && (lda & 3) == 0 && n0 + n1 <= 4 &&
      (K == 16 || K == 32 || K == 64) && g.Ho % 2 == 0 && g.Wo % 2 == 0) {
    const long long pix = (long long)g.nimg * (g.Ho / 2) * (g.Wo / 2);
    const int lp = K / 4;
    dim3 grid((unsigned)std::min<long long>((pix * lp + 255) / 256, 1024), 4);
    if (lp == 4)
      hipLaunchKernelGGL(gconv_s2t_kernel<4>, grid, dim3(256), 0, s, A, lda, K, W0, n0, W1, n1, w_tap, w1_tap, bias0,
                         bias1, g, C, ldc, accumulate);
    else if (lp == 8)
      hipLaunchKernelGGL(gconv_s2t_kernel<8>, grid, dim3(256), 0, s, A, lda, K, W0, n0, W1, n1, w_tap, w1_tap, bias0,
                         bias1, g, C, ldc, accumulate);
    else
      hipLaunchKernelGGL(gconv_s2t_kernel<16>, grid, dim3(256), 0, s, A, lda, K, W0, n0, W1, n1, w_tap, w1_tap, bias0,
                         bias1, g, C, ldc, accumulate);
    return;
  }
  if ((K & 3) == 0 && (lda & 3) == 0 && K >= 16 && K <= 256 && (K & (K - 1)) == 0 && g.ksz <= 4 && n0 + n1 <= 4) {
    const int lp = K / 4 > 64 ? 64 : K / 4;  // lanes per pixel (power of two)
    const long long threads = rows_total * lp;
    dim3 grid((unsigned)std::min<long long>((threads + 255) / 256, 2048));
    if (lp == 4)
      hipLaunchKernelGGL(gconv_smalln_lp_kernel<4>, grid, dim3(256), lds, s, A, lda, K, W0, n0, W1, n1, w_tap, w1_tap,
                         bias0, bias1, g, rows_total, C, ldc, accumulate);
    else if (lp == 8)
      hipLaunchKernelGGL(gconv_smalln_lp_kernel<8>, grid, dim3(256), lds, s, A, lda, K, W0, n0, W1, n1, w_tap, w1_tap,
                         bias0, bias1, g, rows_total, C, ldc, accumulate);
    else if (lp == 16)
      hipLaunchKernelGGL(gconv_smalln_lp_kernel<16>, grid, dim3(256), lds, s, A, lda, K, W0, n0, W1, n1, w_tap, w1_tap,
                         bias0, bias1, g, rows_total, C, ldc, accumulate);
    else if (lp == 32)
      hipLaunchKernelGGL(gconv_smalln_lp_kernel<32>, grid, dim3(256), lds, s, A, lda, K, W0, n0, W1, n1, w_tap, w1_tap,
                         bias0, bias1, g, rows_total, C, ldc, accumulate);
    else
      hipLaunchKernelGGL(gconv_smalln_lp_kernel<64>, grid, dim3(256), lds, s, A, lda, K, W0, n0, W1, n1, w_tap, w1_tap,
                         bias0, bias1, g, rows_total, C, ldc, accumulate);
    return;
  }
  hipLaunchKernelGGL(gconv_smalln_kernel, dim3((unsigned)((rows_total + 255) / 256)), dim3(256), lds, s, A, lda, K, W0,
                     n0, W1, n1, w_tap, w1_tap, bias0, bias1, g, rows_total, C, ldc, accumulate);
}

// ---------------------------------------------------------------------------
// output layer + highway + reconstruction partials (sequential_vae.py:1720-1729, :1146)
// a[p][0..C) = output deconv pre-act, a[p][C] = ratio deconv pre-act (ld = C+1)
// ---------------------------------------------------------------------------
#define OUT_TPB 256
int output_blocks_per_img(int HW) { return (HW + OUT_TPB - 1) / OUT_TPB; }

__global__ void output_fwd_kernel(const float* __restrict__ a, int HW, int C, const float* __restrict__ xprev,
                                  const float* __restrict__ target, float lo, float hi, float minh, float maxh,
                                  float* __restrict__ xhat, float* __restrict__ rec_part, int nblk) {
  __shared__ float red[OUT_TPB / 64];
  const int n = blockIdx.y;
  const int pix = blockIdx.x * OUT_TPB + threadIdx.x;
  float s = 0.f;
  if (pix < HW) {
    const long long p = (long long)n * HW + pix;
    const float* ap = a + p * (C + 1);
    f32x4 av = {0.f, 0.f, 0.f, 0.f};
    if (C == 3) av = *(const f32x4*)ap;  // RGB: the packed [C | ratio] row as one 16-byte load
    float rr = 1.f;
    if (xprev) rr = minh + (maxh - minh) * sigmoid_f(C == 3 ? av[3] : ap[C]);
    for (int c = 0; c < C; ++c) {
      float out = (hi - lo) * sigmoid_f(C == 3 ? av[c] : ap[c]) + lo;
      float x = xprev ? rr * out + (1.f - rr) * xprev[p * C + c] : out;
      xhat[p * C + c] = x;
      float d = x - target[p * C + c];
      s += d * d;
    }
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < OUT_TPB / 64; ++w) t += red[w];
    rec_part[n * nblk + blockIdx.x] = t;
  }
}

void output_fwd(const float* a, int B, int HW, int C, const float* xprev, const float* target, float lo, float hi,
                float minh, float maxh, float* xhat, float* rec_part, int nblk, hipStream_t s) {
  hipLaunchKernelGGL(output_fwd_kernel, dim3(nblk, B), dim3(OUT_TPB), 0, s, a, HW, C, xprev, target, lo, hi, minh, maxh,
                     xhat, rec_part, nblk);
}

// g = dxhat_in + rec_coef*2*(xhat - target); da (pre-sigmoid), dxprev = (1-r)*g
__global__ void output_bwd_kernel(const float* __restrict__ a, long long P, int C, const float* __restrict__ xprev,
                                  const float* __restrict__ xhat, const float* __restrict__ target, float lo, float hi,
                                  float minh, float maxh, float rec_coef, const float* __restrict__ dxhat_in,
                                  float* __restrict__ da, float* __restrict__ dxprev) {
  const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  if (C == 3) {  // RGB: the packed [C | ratio] row is one 16-byte vector in and out (same arithmetic)
    const f32x4 av = *(const f32x4*)(a + p * 4);
    float rr = 1.f, sr = 0.f;
    if (xprev) {
      sr = sigmoid_f(av[3]);
      rr = minh + (maxh - minh) * sr;
    }
    float drr = 0.f;
    f32x4 dv;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const long long i = p * 3 + c;
      float g = rec_coef * 2.f * (xhat[i] - target[i]);
      if (dxhat_in) g += dxhat_in[i];
      const float o = sigmoid_f(av[c]);
      const float out = (hi - lo) * o + lo;
      const float dout = xprev ? rr * g : g;
      dv[c] = dout * (hi - lo) * o * (1.f - o);
      if (xprev) {
        drr += g * (out - xprev[i]);
        dxprev[i] = (1.f - rr) * g;
      }
    }
    dv[3] = xprev ? drr * (maxh - minh) * sr * (1.f - sr) : 0.f;
    *(f32x4*)(da + p * 4) = dv;
    return;
  }
  const float* ap = a + p * (C + 1);
  float* dap = da + p * (C + 1);
  float rr = 1.f, sr = 0.f;
  if (xprev) {
    sr = sigmoid_f(ap[C]);
    rr = minh + (maxh - minh) * sr;
  }
  float drr = 0.f;
  for (int c = 0; c < C; ++c) {
    const long long i = p * C + c;
    float g = rec_coef * 2.f * (xhat[i] - target[i]);
    if (dxhat_in) g += dxhat_in[i];
    const float o = sigmoid_f(ap[c]);
    const float out = (hi - lo) * o + lo;
    const float dout = xprev ? rr * g : g;
    dap[c] = dout * (hi - lo) * o * (1.f - o);
    if (xprev) {
      drr += g * (out - xprev[i]);
      dxprev[i] = (1.f - rr) * g;
    }
  }
  dap[C] = xprev ? drr * (maxh - minh) * sr * (1.f - sr) : 0.f;
}

void output_bwd(const float* a, int B, int HW, int C, const float* xprev, const float* xhat, const float* target,
                float lo, float hi, float minh, float maxh, float rec_coef, const float* dxhat_in, float* da,
                float* dxprev, hipStream_t s) {
  long long P = (long long)B * HW;
  hipLaunchKernelGGL(output_bwd_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, a, P, C, xprev, xhat,
                     target, lo, hi, minh, maxh, rec_coef, dxhat_in, da, dxprev);
}

// step scalars: stats_out[0] = mean_b recon_b, stats_out[1] = mean_b kl_b; rec_img_out[b] = recon_b
__global__ void loss_reduce_kernel(const float* rec_part, int nblk, const float* kl_img, int B, int HWC,
                                   float* stats_out, float* rec_img_out) {
  __shared__ float red[2][4];
  float sr = 0.f, sk = 0.f;
  for (int n = threadIdx.x; n < B; n += blockDim.x) {
    float r = 0.f;
    for (int b = 0; b < nblk; ++b) r += rec_part[n * nblk + b];
    r /= HWC;
    rec_img_out[n] = r;
    sr += r;
    sk += kl_img[n];
  }
  sr = wave_sum(sr);
  sk = wave_sum(sk);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = sr;
    red[1][threadIdx.x >> 6] = sk;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f, b = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
      a += red[0][w];
      b += red[1][w];
    }
    stats_out[0] = a / B;
    stats_out[1] = b / B;
  }
}

void loss_reduce(const float* rec_part, int nblk, const float* kl_img, int B, int HWC, float* stats_out,
                 float* rec_img_out, hipStream_t s) {
  hipLaunchKernelGGL(loss_reduce_kernel, dim3(1), dim3(256), 0, s, rec_part, nblk, kl_img, B, HWC, stats_out,
                     rec_img_out);
}

// ---------------------------------------------------------------------------
// clip_by_value(+-clip) + tf.train.AdamOptimizer (sequential_vae.py:1267,1274-1276)
// ---------------------------------------------------------------------------
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void adam1(float& w, float g, float& m, float& v, float lr_t, float b1, float b2, float eps,
                                      float clipv) {
  const float gg = fminf(fmaxf(g, -clipv), clipv);
  m = b1 * m + (1.f - b1) * gg;
  v = b2 * v + (1.f - b2) * gg * gg;
  w -= lr_t * m / (sqrtf(v) + eps);
}

// 16-B vectors (w/g/m/v 16-B aligned: ranges start on a multiple of 4 elements); wn != nullptr
// also writes the bf16 copy of the updated weights (the GEMMs' N-layout shadow, shadow_n_kernel's
// rounding), which saves the next forward's separate conversion pass over the live region
typedef _Float16 ol4h __attribute__((ext_vector_type(4)));
// split mode: the fp16 planes at the tensor's exponent wtab[(wbase + i) / 64] (H16_WS without a table); a
// weight at or past 2^15 in those units raises *ovf, and the next forward re-makes every tensor's planes
// (wexp_fixup) before a GEMM reads them
__device__ __forceinline__ void adam_h16(float w, int e, _Float16& h0, _Float16& h1, bool& ovf) {
  h16_pair(w, e, h0, h1);
  ovf |= !(fabsf(w * __uint_as_float((unsigned)(e + 127) << 23)) < H16_WOVF);
}
__global__ void adam_kernel(float* w, const float* g, float* m, float* v, __bf16* wn, long long n, float lr_t, float b1,
                            float b2, float eps, float clipv, int nsp, long long plane, const int* wtab, long long wbase,
                            int* ovf_flag) {
  bool ovf = false;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long nq = n >> 2;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += stride) {
    const f32x4 gg = ((const f32x4*)g)[q];
    f32x4 mm = ((f32x4*)m)[q], vv = ((f32x4*)v)[q], ww = ((f32x4*)w)[q];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float w1 = ww[e], m1 = mm[e], v1 = vv[e];
      adam1(w1, gg[e], m1, v1, lr_t, b1, b2, eps, clipv);
      ww[e] = w1;
      mm[e] = m1;
      vv[e] = v1;
    }
    ((f32x4*)m)[q] = mm;
    ((f32x4*)v)[q] = vv;
    ((f32x4*)w)[q] = ww;
    if (wn) {  // the bf16 N-layout copy (split mode: nsp planes, opload.h split4; and the fp16 planes)
      bool bfp = true;  // the bf16 planes (split mode: only the tensors flagged in the table)
      if (nsp == 3) {
        _Float16 h0[4], h1[4];
        const int tv = wtab ? wtab[(wbase + 4 * q) >> 6] : (H16_WS | WTAB_BF16);
        bfp = wtab_bf16(tv);
        for (int e = 0; e < 4; ++e) adam_h16(ww[e], wtab_exp(tv), h0[e], h1[e], ovf);
        *(ol4h*)((_Float16*)wn + H16_PLANE * plane + 4 * q) = ol4h{h0[0], h0[1], h0[2], h0[3]};
        *(ol4h*)((_Float16*)wn + (H16_PLANE + 1) * plane + 4 * q) = ol4h{h1[0], h1[1], h1[2], h1[3]};
      }
      if (bfp)
      for (int p = 0; p < nsp; ++p) {
        const bf16x4_t h = __builtin_convertvector(ww, bf16x4_t);
        *(bf16x4_t*)(wn + p * plane + 4 * q) = h;
        ww = ww - __builtin_convertvector(h, f32x4);
      }
    }
  }
  for (long long i = 4 * nq + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    adam1(w[i], g[i], m[i], v[i], lr_t, b1, b2, eps, clipv);
    if (wn) {
      float x = w[i];
      const int tv = wtab ? wtab[(wbase + i) >> 6] : (H16_WS | WTAB_BF16);
      if (nsp == 3)
        adam_h16(x, wtab_exp(tv), ((_Float16*)wn)[H16_PLANE * plane + i], ((_Float16*)wn)[(H16_PLANE + 1) * plane + i], ovf);
      if (nsp != 3 || wtab_bf16(tv))
      for (int p = 0; p < nsp; ++p) {
        const __bf16 h = (__bf16)x;
        wn[p * plane + i] = h;
        x -= (float)h;
      }
    }
  }
  if (ovf && ovf_flag) *ovf_flag = 1;  // (a plain store: every writer stores the same value)
}

void adam_step(float* w, const float* g, float* m, float* v, void* wn, long long n, float lr_t, float b1, float b2,
               float eps, float clipv, int nsp, long long plane, hipStream_t s, const int* wtab, long long wbase,
               int* ovf) {
  if (n <= 0) return;
  hipLaunchKernelGGL(adam_kernel, dim3(ew_blocks((n + 3) / 4, 256, 8192)), dim3(256), 0, s, w, g, m, v, (__bf16*)wn,
                     n, lr_t, b1, b2, eps, clipv, nsp, plane, wtab, wbase, ovf);
}

__global__ void bf16_to_f32_kernel(const __bf16* src, float* dst, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    dst[i] = (float)src[i];
}
void bf16_to_f32(const void* src, float* dst, long long n, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(bf16_to_f32_kernel, dim3(ew_blocks(n)), dim3(256), 0, s, (const __bf16*)src, dst, n);
}

__global__ void fill_kernel(float* p, long long n, float v) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    p[i] = v;
}
void fill_f32(float* p, long long n, float v, hipStream_t s) {
  hipLaunchKernelGGL(fill_kernel, dim3(ew_blocks(n)), dim3(256), 0, s, p, n, v);
}

// Philox4x32-10 -> Box-Muller normals (throughput-mode eps; parity mode injects eps)
__device__ __forceinline__ void philox(unsigned& c0, unsigned& c1, unsigned& c2, unsigned& c3, unsigned k0,
                                       unsigned k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    unsigned long long p0 = (unsigned long long)0xD2511F53u * c0;
    unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c2;
    unsigned h0 = (unsigned)(p0 >> 32), l0 = (unsigned)p0;
    unsigned h1 = (unsigned)(p1 >> 32), l1 = (unsigned)p1;
    unsigned n0 = h1 ^ c1 ^ k0, n2 = h0 ^ c3 ^ k1;
    c0 = n0; c1 = l1; c2 = n2; c3 = l0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

__global__ void philox_normal_kernel(float* out, long long n, unsigned long long seed, unsigned long long offset) {
  const long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (q * 4 >= n) return;
  unsigned long long ctr = offset + q;
  unsigned c0 = (unsigned)ctr, c1 = (unsigned)(ctr >> 32), c2 = 0, c3 = 0;
  philox(c0, c1, c2, c3, (unsigned)seed, (unsigned)(seed >> 32));
  const float inv = 2.3283064365386963e-10f;
  float u0 = (c0 + 0.5f) * inv, u1 = (c1 + 0.5f) * inv, u2 = (c2 + 0.5f) * inv, u3 = (c3 + 0.5f) * inv;
  float r0 = sqrtf(-2.f * __logf(u0)), r1 = sqrtf(-2.f * __logf(u2));
  float v[4] = {r0 * __cosf(6.2831853f * u1), r0 * __sinf(6.2831853f * u1), r1 * __cosf(6.2831853f * u3),
                r1 * __sinf(6.2831853f * u3)};
  for (int e = 0; e < 4; ++e)
    if (q * 4 + e < n) out[q * 4 + e] = v[e];
}

void philox_normal(float* out, long long n, unsigned long long seed, unsigned long long offset, hipStream_t s) {
  long long q = (n + 3) / 4;
  hipLaunchKernelGGL(philox_normal_kernel, dim3((unsigned)((q + 255) / 256)), dim3(256), 0, s, out, n, seed, offset);
}

// column sums of a narrow matrix (C <= 4): output conv-T bias gradients (sum over pixels)
#define CS_BLOCKS 256
__global__ void colsum_part_kernel(const float* __restrict__ X, int ld, long long rows, int C, float* __restrict__ part) {
  __shared__ float red[4][4];
  float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += (long long)gridDim.x * blockDim.x)
    for (int c = 0; c < C; ++c) s[c] += X[r * ld + c];
  for (int c = 0; c < 4; ++c) {
    float v = wave_sum(s[c]);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][c] = v;
  }
  __syncthreads();
  if (threadIdx.x < 4) part[blockIdx.x * 4 + threadIdx.x] = red[0][threadIdx.x] + red[1][threadIdx.x] +
                                                            red[2][threadIdx.x] + red[3][threadIdx.x];
}
__global__ void colsum_fin_kernel(const float* part, int nblk, int C, float* out0, int n0, float* out1) {
  const int c = threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
#pragma unroll 16
  for (int b = 0; b < nblk; ++b) s += part[b * 4 + c];  // loads batched, adds in the same order
  if (c < n0) out0[c] = s;
  else if (out1) out1[c - n0] = s;
}
void colsum_small(const float* X, int ld, long long rows, int C, float* part, float* out0, int n0, float* out1,
                  hipStream_t s) {
  hipLaunchKernelGGL(colsum_part_kernel, dim3(CS_BLOCKS), dim3(256), 0, s, X, ld, rows, C, part);
  hipLaunchKernelGGL(colsum_fin_kernel, dim3(1), dim3(64), 0, s, part, CS_BLOCKS, C, out0, n0, out1);
}

// ---- weight sharing: broadcast the public tensors into the per-step copies, and sum the
// copies' gradients into the public gradient (sequential_vae.py:1573-1577,1683-1687,1757-1761:
// a TF variable used by several steps receives the sum of their gradients) ----
__global__ void share_bcast_kernel(const float* P, float* Pv, const long long* seg) {
  const long long* sg = seg + 3LL * blockIdx.y;
  const long long v = sg[0], p = sg[1], n = sg[2];
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    Pv[v + i] = P[p + i];
}

__global__ void share_gather_kernel(const float* Gv, float* G, const long long* tab, const long long* cp) {
  const long long* t = tab + 4LL * blockIdx.y;
  const long long p = t[0], n = t[1], first = t[2], nc = t[3];
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float acc = 0.f;
    for (long long k = 0; k < nc; ++k) acc += Gv[cp[first + k] + i];
    G[p + i] = acc;
  }
}

void share_broadcast(const float* P, float* Pv, const long long* seg, int nseg, hipStream_t s) {
  if (nseg > 0) hipLaunchKernelGGL(share_bcast_kernel, dim3(64, nseg), dim3(256), 0, s, P, Pv, seg);
}

void share_gather(const float* Gv, float* G, const long long* tab, const long long* cp, int ntab, hipStream_t s) {
  if (ntab > 0) hipLaunchKernelGGL(share_gather_kernel, dim3(64, ntab), dim3(256), 0, s, Gv, G, tab, cp);
}

struct Small64 {
  float v[64];
};
__global__ void set_small_kernel(float* dst, Small64 a, int n) {
  if ((int)threadIdx.x < n) dst[threadIdx.x] = a.v[threadIdx.x];
}
void set_small(float* dst, const float* vals, int n, hipStream_t s) {
  Small64 a{};
  for (int i = 0; i < n && i < 64; ++i) a.v[i] = vals[i];
  hipLaunchKernelGGL(set_small_kernel, dim3(1), dim3(64), 0, s, dst, a, n);
}

// ---------------------------------------------------------------------------
// packed output / ratio conv-T operands of up to PACK_MAXT chain steps in one launch
// (sequential_vae.py:1720 `conv2d_t` out, :1727 ratio): wpack[t] = [tap][C+1][F1] with the
// ratio row zero at t = 0, then 4 bias floats [b_out | b_ratio | 0...]; wpack_h[t] its bf16
// copy (shadow_n_kernel's rounding).  Replaces per step a memset, two copies, two 2-D copies and
// a conversion pass on the main stream (6 dependent launches -> one per forward).
// ---------------------------------------------------------------------------
__global__ void pack_out_kernel(PackOutArgs a) {
  const int t = blockIdx.y;
  const int C = a.C, C1 = C + 1, F1 = a.F1;
  const int nw = 16 * C1 * F1;
  const float* wout = a.P + a.owout[t];
  const float* wratio = a.owratio[t] >= 0 ? a.P + a.owratio[t] : nullptr;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nw + 4; i += gridDim.x * blockDim.x) {
    float v;
    if (i < nw) {
      const int tap = i / (C1 * F1);
      const int rem = i - tap * C1 * F1;
      const int co = rem / F1, ci = rem - co * F1;
      v = co < C ? wout[((long long)tap * C + co) * F1 + ci] : (wratio ? wratio[tap * F1 + ci] : 0.f);
      if (a.wpack_h[t]) {  // bf16 copy; split mode: plane q = bf16(v - the earlier planes)
        float r = v;
        for (int q = 0; q < a.nsp; ++q) {
          const __bf16 b = (__bf16)r;
          a.wpack_h[t][(long long)q * nw + i] = b;
          r -= (float)b;
        }
      }
    } else {
      const int j = i - nw;
      v = j < C ? a.P[a.obout[t] + j] : ((j == C && a.obratio[t] >= 0) ? a.P[a.obratio[t]] : 0.f);
    }
    a.wpack[t][i] = v;
  }
}

void pack_out(const PackOutArgs& a, int nt, hipStream_t s) {
  const int n = 16 * (a.C + 1) * a.F1 + 4;
  hipLaunchKernelGGL(pack_out_kernel, dim3((n + 255) / 256, nt), dim3(256), 0, s, a);
}
