// PixelCNN++ decoder head on gfx950: weight-normed shifted convolutions as
// bf16-MFMA gather GEMMs, their weight gradients, the gated-resnet / nonlinearity elementwise
// ops, the discretized logistic mixture loss (forward + analytic gradient in one pass) and its
// sampler.  C ABI: include/svae_pcnn.h.  Reference: pixel_cnn/pixel_cnn_pp/{model,nn}.py,
// pixel_cnn/pixelvae.py (cited per function).
#include <math.h>
#include <cstdint>
#include <cstdlib>
#include <string>

#include "common.h"
#include "knobs.h"
#include "kernels.h"
#include "svae_hip.h"
#include "svae_pcnn.h"

void svae_tls_error(const std::string& msg);  // engine.cpp: svae_last_error(NULL)

namespace {

typedef __bf16 pc_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 pc_bf16x4 __attribute__((ext_vector_type(4)));
typedef float pc_f32x8 __attribute__((ext_vector_type(8)));
typedef _Float16 pc_f16x8 __attribute__((ext_vector_type(8)));

// H: the 16-bit operand lanes hold fp16 bits (the split mode's scaled hi / lo planes), else bf16
template <bool H>
__device__ __forceinline__ f32x16 pc_mfma(pc_bf16x8 a, pc_bf16x8 b, f32x16 c) {
  if constexpr (H)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(pc_f16x8, a), __builtin_bit_cast(pc_f16x8, b), c,
                                                  0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// the fp16 planes' inverse scales (svae_pcnn.h: a[0] of the x planes, b[0] of the weight / dy planes):
// a product of two scaled fp16 operands is multiplied by a[0] * b[0] (exact powers of two)
struct PcScale {
  const float* a;
  const float* b;
};
__device__ __forceinline__ float pc_alpha(const PcScale& sc) { return sc.a ? sc.a[0] * sc.b[0] : 1.f; }

int bad(const char* msg) {
  svae_tls_error(msg);
  return SVAE_EBADARG;
}
int hipchk() {
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess) return 0;
  svae_tls_error(std::string("HIP: ") + hipGetErrorString(e));
  return SVAE_EHIP;
}
#define PC_MAXPLANES 3  // operand planes of the split mode (svae_pcnn_*_planes)

int blocks_for(long long n, int per = 256, int cap = 16384) {
  long long b = (n + per - 1) / per;
  if (b < 1) b = 1;
  return (int)(b < cap ? b : cap);
}

// ---------------------------------------------------------------------------------------------
// gather geometry (svae_pcnn.h): source pixel of output pixel (oy, ox) for tap (ky, kx)
// ---------------------------------------------------------------------------------------------
struct PcGeom {
  int n, hi, wi, cin, ldx;  // gathered operand
  int ho, wo, cout;         // row space (output pixels) and output channels
  int kh, kw, s, pt, pl, mode;
};

__device__ __forceinline__ bool pc_src(const PcGeom& g, int oy, int ox, int ky, int kx, int& iy, int& ix) {
  if (g.mode == 0) {
    iy = oy * g.s - g.pt + ky;
    ix = ox * g.s - g.pl + kx;
  } else {
    const int ty = oy + g.pt - ky, tx = ox + g.pl - kx;
    if (ty < 0 || tx < 0) return false;
    if (g.s == 2) {
      if ((ty | tx) & 1) return false;
      iy = ty >> 1;
      ix = tx >> 1;
    } else {
      iy = ty;
      ix = tx;
    }
  }
  return iy >= 0 && iy < g.hi && ix >= 0 && ix < g.wi;
}

// The input-gradient epilogue of a conv whose input is a resnet nonlinearity's output t = f(src) *
// mask (relu / elu, nn.py:270-274): the conv writes d src = d t * mask * f'(src) instead of d t,
// so the nonlinearity's backward pass (and d t's buffer) disappear.  on = 0: a plain epilogue.
struct NlbArgs {
  const float* src; int lds;  // the nonlinearity's input, [rows][lds]
  int kind;                    // 0 relu, 1 elu
  const float* mask;           // keep-mask [rows][cols], or NULL: hashed (keep, seed) / none (keep >= 1)
  float keep; unsigned long long seed;
  int on;
};
__device__ __forceinline__ float drop_scale(unsigned long long seed, unsigned long long idx, float keep, float inv);
__device__ __forceinline__ float nlb_apply(const NlbArgs& e, long long row, int col, int cols, float g) {
  if (e.mask) g *= e.mask[row * cols + col];
  else if (e.keep < 1.f) g *= drop_scale(e.seed, (unsigned long long)(row * cols + col), e.keep, 1.f / e.keep);
  const float v = e.src[row * e.lds + col];
  return e.kind == 0 ? (v > 0.f ? g : 0.f) : g * (v > 0.f ? 1.f : expf(v));  // (relu'(0) = 0, elu' as delu_f)
}

// ---------------------------------------------------------------------------------------------
// weight norm (nn.py:173, :201, :236)
// ---------------------------------------------------------------------------------------------
// fixed-order block sum (256 threads, fp64)
__device__ __forceinline__ double block_sum256(double v, double* red) {
  red[threadIdx.x] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  return red[0];
}

// norm[co] = sqrt(sum_{tap, ci} V^2): one block per output channel, fixed-order sums
__global__ __launch_bounds__(256) void wn_norm_kernel(const float* __restrict__ V, int K, int cout,
                                                      float* __restrict__ norm) {
  __shared__ double red[256];
  const int c = blockIdx.x;
  double s = 0.0;
  for (int k = threadIdx.x; k < K; k += 256) {
    const double v = V[(long long)k * cout + c];
    s += v * v;
  }
  s = block_sum256(s, red);
  if (threadIdx.x == 0) norm[c] = (float)sqrt(s);
}

// W = g / norm * V -> wk_f [tap][co][kf] (K = ci) and wk_d [tap][ci][kd] (K = co), zero padded.
// planes > 1 (the head's split mode): `planes` bf16 planes per copy, plane p at p * (copy size), with
// W = sum_p plane_p up to the last plane's rounding (plane p = bf16 of what planes 0..p-1 left)
// The split mode's fp16 planes: a tensor scaled by 2^s, s such that max|v| * 2^s is in [2^14, 2^15) (fp16's
// top binade: 11 significant bits per plane, no overflow), held as h0 = fp16(v 2^s), h1 = fp16(v 2^s - h0):
// 22 significant bits down to fp16's subnormal floor, 2^-24 * 2^-s, i.e. 2^-39 of the tensor's maximum.
// `mx` holds the bits of max|v| (non-negative floats order as unsigned ints).
__device__ __forceinline__ int h16_shift(unsigned mx) {
  const float m = __uint_as_float(mx);
  if (!(m > 0.f)) return 0;
  int e;
  (void)frexpf(m, &e);  // m = f 2^e, f in [0.5, 1)
  const int sh = 15 - e;
  return sh < -60 ? -60 : (sh > 60 ? 60 : sh);  // (two inverse scales multiply: keep their product normal)
}
__device__ __forceinline__ void h16_put(__bf16* w, long long i, long long pstride, float v, int sh) {
  const float x = ldexpf(v, sh);
  const _Float16 h0 = (_Float16)x;
  const _Float16 h1 = (_Float16)(x - (float)h0);
  w[i] = __builtin_bit_cast(__bf16, h0);
  w[i + pstride] = __builtin_bit_cast(__bf16, h1);
}
// max |v| over a block into *mx (one device-scope atomic per block, integer max of the float bits)
__device__ __forceinline__ void block_absmax_put(float v, unsigned* mx) {
  __shared__ unsigned red[8];
  unsigned b = __float_as_uint(fabsf(v));
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned t = __shfl_xor(b, o);
    b = t > b ? t : b;
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = b;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned m = 0;
    for (int w = 0; w < (int)(blockDim.x + 63) / 64; ++w) m = red[w] > m ? red[w] : m;
    // (one contended address for thousands of blocks: most find the maximum already at least theirs, and a
    // plain read of it spares them the serialised atomic -- 70 us of a 25 us pass, r05_hpv)
    if (m > __hip_atomic_load(mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(mx, m);
  }
}
// max |W| = max_co max_k |V[k][co]| * |g[co] / norm[co]| (the product apply forms: monotone in |V|) into *mx
__global__ __launch_bounds__(256) void wn_absmax_kernel(const float* __restrict__ V, const float* __restrict__ g,
                                                        const float* __restrict__ norm, int K, int cout,
                                                        unsigned* __restrict__ mx) {
  const int c = blockIdx.x;
  float m = 0.f;
  for (int k = threadIdx.x; k < K; k += 256) m = fmaxf(m, fabsf(V[(long long)k * cout + c]));
  block_absmax_put(m * fabsf(g[c] / norm[c]), mx);
}

__device__ __forceinline__ void wn_put(__bf16* w, long long i, long long pstride, int planes, float v) {
  for (int p = 0; p < planes; ++p) {
    const __bf16 b = (__bf16)v;
    w[i + p * pstride] = b;
    v -= (float)b;
  }
}
// h16 != NULL: the two scaled fp16 planes (h16[1] = the bits of max|W|, h16[0] <- the inverse scale)
__global__ void wn_apply_kernel(const float* __restrict__ V, const float* __restrict__ g,
                                const float* __restrict__ norm, int taps, int cin, int cout, __bf16* wk_f, int kf,
                                __bf16* wk_d, int kd, int planes, float* h16) {
  const long long nf = wk_f ? (long long)taps * cout * kf : 0, nd = wk_d ? (long long)taps * cin * kd : 0;
  const int sh = h16 ? h16_shift(__float_as_uint(h16[1])) : 0;
  if (h16 && blockIdx.x == 0 && threadIdx.x == 0) h16[0] = ldexpf(1.f, -sh);
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nf + nd; i += stride) {
    if (i < nf) {
      const int ci = (int)(i % kf);
      const long long r = i / kf;
      const int co = (int)(r % cout), tap = (int)(r / cout);
      float w = 0.f;
      if (ci < cin) w = V[((long long)tap * cin + ci) * cout + co] * (g[co] / norm[co]);
      if (h16) h16_put(wk_f, i, nf, w, sh);
      else wn_put(wk_f, i, nf, planes, w);
    } else {
      const long long j = i - nf;
      const int co = (int)(j % kd);
      const long long r = j / kd;
      const int ci = (int)(r % cin), tap = (int)(r / cin);
      float w = 0.f;
      if (co < cout) w = V[((long long)tap * cin + ci) * cout + co] * (g[co] / norm[co]);
      if (h16) h16_put(wk_d, j, nd, w, sh);
      else wn_put(wk_d, j, nd, planes, w);
    }
  }
}

// dg[co] = sum_k dW V / norm  (one block per output channel, fixed order, fp64)
__global__ __launch_bounds__(256) void wn_dg_kernel(const float* __restrict__ V, const float* __restrict__ dW,
                                                    const float* __restrict__ norm, int K, int cout,
                                                    float* __restrict__ dg) {
  __shared__ double red[256];
  const int c = blockIdx.x;
  double s = 0.0;
  for (int k = threadIdx.x; k < K; k += 256) s += (double)dW[(long long)k * cout + c] * V[(long long)k * cout + c];
  s = block_sum256(s, red);
  if (threadIdx.x == 0) dg[c] = (float)(s / norm[c]);
}

__global__ void wn_dv_kernel(const float* __restrict__ V, const float* __restrict__ g, const float* __restrict__ norm,
                             const float* __restrict__ dW, const float* __restrict__ dg, long long n, int cout,
                             float* __restrict__ dV) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int c = (int)(i % cout);
    const float in = 1.f / norm[c];
    dV[i] = g[c] * in * (dW[i] - dg[c] * in * V[i]);
  }
}

// ---------------------------------------------------------------------------------------------
// gather conv: one wave = 32 output pixels x 32*NT output channels, fragments straight from
// HBM/L2 (no LDS: each lane's A row is its own gathered pixel, 8 consecutive channels = two 16-B
// loads; B rows are 16-B bf16 runs of the K-contiguous weight copy).  4 waves per block stacked
// along the pixels, so the block's B fragments are shared through L1.
// ---------------------------------------------------------------------------------------------
template <int NT>
__global__ __launch_bounds__(256) void pc_conv_kernel(PcGeom g, const float* __restrict__ X,
                                                      const __bf16* __restrict__ Wk, int kpad,
                                                      const float* __restrict__ bias, float* __restrict__ Y, int ldy,
                                                      int accumulate, int zero_edge) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l32 = lane & 31, h = lane >> 5;
  const int per_img = g.ho * g.wo;
  const long long rows = (long long)g.n * per_img;
  const long long m0 = ((long long)blockIdx.x * 4 + wave) * 32;
  if (m0 >= rows) return;
  const int n0 = blockIdx.y * 32 * NT;
  const long long m = m0 + l32;
  const bool mv = m < rows;
  int img = 0, oy = 0, ox = 0;
  if (mv) {
    img = (int)(m / per_img);
    const int r = (int)(m - (long long)img * per_img);
    oy = r / g.wo;
    ox = r - oy * g.wo;
  }
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  const int ntap = g.kh * g.kw;
  for (int tap = 0; tap < ntap; ++tap) {
    const int ky = tap / g.kw, kx = tap - ky * g.kw;
    int iy = 0, ix = 0;
    const bool v = mv && pc_src(g, oy, ox, ky, kx, iy, ix);
    const float* xp = X + ((long long)(img * g.hi + iy) * g.wi + ix) * g.ldx;
    const __bf16* wp = Wk + (long long)tap * g.cout * kpad;
#pragma unroll 2
    for (int k0 = 0; k0 < kpad; k0 += 16) {
      const int ci = k0 + 8 * h;
      f32x4 lo = {0.f, 0.f, 0.f, 0.f}, hi = {0.f, 0.f, 0.f, 0.f};
      if (v) {
        if (ci < g.cin) lo = *(const f32x4*)(xp + ci);
        if (ci + 4 < g.cin) hi = *(const f32x4*)(xp + ci + 4);
      }
      const pc_f32x8 a8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      const pc_bf16x8 af = __builtin_convertvector(a8, pc_bf16x8);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int n = n0 + t * 32 + l32;
        pc_bf16x8 bf = {};
        if (n < g.cout) bf = *(const pc_bf16x8*)(wp + (long long)n * kpad + ci);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf, acc[t], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const long long mm = m0 + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (mm >= rows) continue;
    bool zero = false;
    if (zero_edge) {
      const int rr = (int)(mm % per_img);
      zero = zero_edge == 1 ? (rr / g.wo == 0) : (rr % g.wo == 0);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n = n0 + t * 32 + l32;
      if (n >= g.cout) continue;
      float val = zero ? 0.f : acc[t][r] + (bias ? bias[n] : 0.f);
      float* p = Y + mm * ldy + n;
      if (accumulate) val += *p;
      *p = val;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// LDS-staged gather conv: block = 128 output pixels x 32*NT output channels, K in chunks of one tap
// x 32 channels.  Per chunk the block stages the 128 gathered pixel rows (fp32 -> bf16, 16-B
// stores) and the 32*NT weight rows once in LDS (80-B pitch: conflict-free 16-B fragment reads);
// each wave then runs 2*NT MFMAs on its 32 rows.  The next chunk's rows are loaded into registers
// while the current chunk's MFMAs run (double-buffered LDS, one barrier per chunk).  Needs kpad
// % 32 == 0.
// ---------------------------------------------------------------------------------------------
#define PC2_P 40  // LDS row pitch (bf16)
template <int NT, bool XB, bool H = false>
__global__ __launch_bounds__(256) void pc_conv2_kernel(PcGeom g, const void* __restrict__ Xv,
                                                       const __bf16* __restrict__ Wk, int kpad,
                                                       const float* __restrict__ bias, float* __restrict__ Y,
                                                       int ldy, int accumulate, int zero_edge, NlbArgs nlb,
                                                       PcScale sc) {
  static_assert(XB || !H, "fp16 planes are stored 16-bit");
  constexpr int BR = 32 * NT;  // weight rows (output channels) per block
  __shared__ __attribute__((aligned(16))) __bf16 As[2][128 * PC2_P];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[2][BR * PC2_P];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int per_img = g.ho * g.wo;
  const long long rows = (long long)g.n * per_img;
  const long long m0 = (long long)blockIdx.x * 128;
  const int n0 = blockIdx.y * BR;
  // staging roles: A row ar = tid >> 1, channel half ah (16 channels); B items tid + 256 i
  const int ar = tid >> 1, ah = tid & 1;
  const long long am = m0 + ar;
  int aimg = 0, aoy = 0, aox = 0;
  const bool amv = am < rows;
  if (amv) {
    aimg = (int)(am / per_img);
    const int r = (int)(am - (long long)aimg * per_img);
    aoy = r / g.wo;
    aox = r - aoy * g.wo;
  }
  constexpr int BI = (BR * 4 + 255) / 256;  // 16-B weight items per thread (4 per row of 32 k)
  const int nk = kpad / 32, ntap = g.kh * g.kw, nchunk = ntap * nk;
  f32x4 ra[4];
  pc_bf16x8 rh[2];
  pc_bf16x8 rb[BI];
  auto load = [&](int c) {
    const int tap = c / nk, k0 = (c - tap * nk) * 32;
    const int ky = tap / g.kw, kx = tap - ky * g.kw;
    int iy = 0, ix = 0;
    const bool v = amv && pc_src(g, aoy, aox, ky, kx, iy, ix);
    const long long xo = ((long long)(aimg * g.hi + iy) * g.wi + ix) * g.ldx + k0 + 16 * ah;
    if constexpr (XB) {  // bf16 X: 8 channels per 16-B load (cin % 8 == 0)
      const __bf16* xp = (const __bf16*)Xv + xo;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int ci = k0 + 16 * ah + 8 * j;
        pc_bf16x8 z = {};
        rh[j] = (v && ci < g.cin) ? *(const pc_bf16x8*)(xp + 8 * j) : z;
      }
    } else {
      const float* xp = (const float*)Xv + xo;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ci = k0 + 16 * ah + 4 * j;
        ra[j] = (v && ci < g.cin) ? *(const f32x4*)(xp + 4 * j) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    const __bf16* wp = Wk + (long long)tap * g.cout * kpad + k0;
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int it = tid + 256 * i, row = it >> 2, q = it & 3;
      pc_bf16x8 z = {};
      rb[i] = (row < BR && n0 + row < g.cout) ? *(const pc_bf16x8*)(wp + (long long)(n0 + row) * kpad + q * 8) : z;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if constexpr (XB) {
        *(pc_bf16x8*)&As[buf][ar * PC2_P + 16 * ah + 8 * j] = rh[j];
      } else {
        const pc_f32x8 v8 = {ra[2 * j][0], ra[2 * j][1], ra[2 * j][2], ra[2 * j][3],
                             ra[2 * j + 1][0], ra[2 * j + 1][1], ra[2 * j + 1][2], ra[2 * j + 1][3]};
        *(pc_bf16x8*)&As[buf][ar * PC2_P + 16 * ah + 8 * j] = __builtin_convertvector(v8, pc_bf16x8);
      }
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int it = tid + 256 * i, row = it >> 2, q = it & 3;
      if (row < BR) *(pc_bf16x8*)&Bs[buf][row * PC2_P + q * 8] = rb[i];
    }
  };
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  load(0);
  store(0);
  __syncthreads();
  for (int c = 0; c < nchunk; ++c) {
    const int buf = c & 1;
    if (c + 1 < nchunk) load(c + 1);
#pragma unroll
    for (int kq = 0; kq < 2; ++kq) {
      const pc_bf16x8 af = *(const pc_bf16x8*)&As[buf][(wave * 32 + l32) * PC2_P + kq * 16 + 8 * h];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const pc_bf16x8 bf = *(const pc_bf16x8*)&Bs[buf][(t * 32 + l32) * PC2_P + kq * 16 + 8 * h];
        acc[t] = pc_mfma<H>(af, bf, acc[t]);
      }
    }
    if (c + 1 < nchunk) store(buf ^ 1);
    __syncthreads();
  }
  const long long mw = m0 + wave * 32;
  const float al = H ? pc_alpha(sc) : 1.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const long long mm = mw + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (mm >= rows) continue;
    bool zero = false;
    if (zero_edge) {
      const int rr = (int)(mm % per_img);
      zero = zero_edge == 1 ? (rr / g.wo == 0) : (rr % g.wo == 0);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n = n0 + t * 32 + l32;
      if (n >= g.cout) continue;
      float val = zero ? 0.f : (H ? acc[t][r] * al : acc[t][r]) + (bias ? bias[n] : 0.f);
      if (nlb.on) val = nlb_apply(nlb, mm, n, g.cout, val);
      float* p = Y + mm * ldy + n;
      if (accumulate) val += *p;
      *p = val;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Halo-window gather conv (stride 1, both modes; every shifted conv of the resnets and its input
// gradient, and the 1x1 nin / dense layers): block = BM = 256 * TM output pixels (whole image rows,
// or whole images) x 32*NT output channels, eight waves of 32 * TM rows x all NT column tiles.  K
// runs in chunks of 32 input channels; per chunk the block stages ONE input window -- its rows plus
// the kernel's halo, nimg x (R + kh - 1) x (wo + kw - 1) pixels, ~1.3x the block's pixels instead of
// taps x as pc_conv2 gathers them -- and the chunk's weight rows of every tap, then each wave runs
// taps x 2 x NT x TM MFMAs (60 - 120 for the [2, 3] convs) between two barriers.  The next chunk's
// window and weights are loaded into registers under the current chunk's MFMAs.
//   mode 0: iy = oy - pt + ky -> window row ry + ky          (origin oy0 - pt, column origin -pl)
//   mode 1: iy = oy + pt - ky -> window row ry + kh - 1 - ky (origin oy0 + pt - kh + 1, pl - kw + 1)
// ---------------------------------------------------------------------------------------------
struct Pc3 {
  int R, nimg, PR, PC, npix;  // image rows per block (per image), images per block, window dims
  int oy_off, ox_off;         // window origin relative to the block's first output row / column 0
};
#define PC3_MAXPIX 640
#define PC3_MAXTAPS 6
// XB: X stored as bf16 (a nonlinearity output the head writes in the conv's operand precision)
// HP (with H): both fp16 planes of x (xpst elements apart) and of the weights (wpst apart) staged per chunk, the
// three plane products h0 h0' + h0 h1' + h1 h0' per fragment pair in ONE launch (svae_pcnn_conv_planes)
template <int NT, int TM, bool XB, bool H = false, bool HP = false>
__global__ __launch_bounds__(512) void pc_conv3_kernel(PcGeom g, Pc3 h, const void* __restrict__ Xv,
                                                       const __bf16* __restrict__ Wk, int kpad,
                                                       const float* __restrict__ bias, float* __restrict__ Y,
                                                       int ldy, int accumulate, int zero_edge, NlbArgs nlb,
                                                       PcScale sc, long long xpst, long long wpst) {
  static_assert(XB || !H, "fp16 planes are stored 16-bit");
  static_assert(H || !HP, "fused planes are the fp16 ones");
  constexpr int NPL = HP ? 2 : 1;
  constexpr int BM = 256 * TM;
  constexpr int BR = 32 * NT;                                  // weight rows (output channels) per tap
  constexpr int AI = (PC3_MAXPIX * 4 + 511) / 512;             // window items (8 channels) per thread
  constexpr int BI = (PC3_MAXTAPS * BR * 4 + 511) / 512;       // 16-B weight items per thread
  extern __shared__ __attribute__((aligned(16))) __bf16 pc3s[];
  __bf16* As = pc3s;                          // [plane][npix][PC2_P]
  __bf16* Bs = pc3s + NPL * h.npix * PC2_P;   // [plane][tap][BR][PC2_P]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, hh = lane >> 5;
  const int taps = g.kh * g.kw;
  const int per_img = g.ho * g.wo;
  const long long m0 = (long long)blockIdx.x * BM;
  const int n0 = blockIdx.y * BR;
  const int img0 = (int)(m0 / per_img);
  const int oy0 = (int)(m0 - (long long)img0 * per_img) / g.wo;
  const int iy0 = oy0 + h.oy_off, ix0 = h.ox_off;

  // window items: pixel it >> 2, channels (it & 3) * 8 .. + 8 of the chunk; -1 zero, -2 no item
  long long aoff[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int it = tid + 512 * i;
    aoff[i] = -2;
    if (it < h.npix * 4) {
      const int pix = it >> 2, part = it & 3;
      const int il = pix / (h.PR * h.PC);
      const int r2 = pix - il * h.PR * h.PC;
      const int pr = r2 / h.PC, pc = r2 - pr * h.PC;
      const int iy = iy0 + pr, ix = ix0 + pc;
      aoff[i] = (iy >= 0 && iy < g.hi && ix >= 0 && ix < g.wi)
                    ? ((long long)((img0 + il) * g.hi + iy) * g.wi + ix) * g.ldx + part * 8
                    : -1;
    }
  }
  const float* X = (const float*)Xv;
  const __bf16* Xh = (const __bf16*)Xv;
  f32x4 ra[XB ? 1 : AI][2];
  pc_bf16x8 rh[XB ? AI : 1], rh1[HP ? AI : 1];
  pc_bf16x8 rb[BI], rb1[HP ? BI : 1];
  const int nb = taps * BR;  // staged weight rows
  auto load = [&](int c) {
    const int k0 = c * 32;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int ci = k0 + ((tid + 512 * i) & 3) * 8;
      if constexpr (XB) {  // 8 channels = one 16-B load (cin % 8 == 0)
        pc_bf16x8 z = {};
        const bool ok = aoff[i] >= 0 && ci < g.cin;
        rh[i] = ok ? *(const pc_bf16x8*)(Xh + aoff[i] + k0) : z;
        if constexpr (HP) rh1[i] = ok ? *(const pc_bf16x8*)(Xh + xpst + aoff[i] + k0) : z;
      } else {
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        ra[i][0] = z;
        ra[i][1] = z;
        if (aoff[i] >= 0) {
          const float* xp = X + aoff[i] + k0;
          if (ci < g.cin) ra[i][0] = *(const f32x4*)xp;
          if (ci + 4 < g.cin) ra[i][1] = *(const f32x4*)(xp + 4);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int it = tid + 512 * i, row = it >> 2, q = it & 3;
      const int t = row / BR, n = row - t * BR;
      pc_bf16x8 z = {};
      const bool ok = row < nb && n0 + n < g.cout;
      const long long wo = ((long long)t * g.cout + n0 + n) * kpad + k0 + q * 8;
      rb[i] = ok ? *(const pc_bf16x8*)(Wk + wo) : z;
      if constexpr (HP) rb1[i] = ok ? *(const pc_bf16x8*)(Wk + wpst + wo) : z;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      if (aoff[i] < -1) continue;
      const int it = tid + 512 * i;
      if constexpr (XB) {
        *(pc_bf16x8*)&As[(it >> 2) * PC2_P + (it & 3) * 8] = rh[i];
        if constexpr (HP) *(pc_bf16x8*)&As[(h.npix + (it >> 2)) * PC2_P + (it & 3) * 8] = rh1[i];
      } else {
        const pc_f32x8 v8 = {ra[i][0][0], ra[i][0][1], ra[i][0][2], ra[i][0][3],
                             ra[i][1][0], ra[i][1][1], ra[i][1][2], ra[i][1][3]};
        *(pc_bf16x8*)&As[(it >> 2) * PC2_P + (it & 3) * 8] = __builtin_convertvector(v8, pc_bf16x8);
      }
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int it = tid + 512 * i, row = it >> 2, q = it & 3;
      if (row < nb) {
        *(pc_bf16x8*)&Bs[row * PC2_P + q * 8] = rb[i];
        if constexpr (HP) *(pc_bf16x8*)&Bs[(nb + row) * PC2_P + q * 8] = rb1[i];
      }
    }
  };

  // this lane's A rows: block row ml -> window pixel (il * PR + ry) * PC + rx
  int abase[TM];
  const int rows_img = h.R * g.wo;
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int ml = wave * 32 * TM + tm * 32 + l32;
    const int il = ml / rows_img;
    const int rem = ml - il * rows_img;
    const int ry = rem / g.wo, rx = rem - ry * g.wo;
    abase[tm] = ((il * h.PR + ry) * h.PC + rx) * PC2_P + 8 * hh;
  }
  f32x16 acc[TM][NT];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[tm][t][r] = 0.f;

  const int nchunk = kpad / 32;
  load(0);
  store();
  __syncthreads();
  for (int c = 0; c < nchunk; ++c) {
    if (c + 1 < nchunk) load(c + 1);
    for (int t = 0; t < taps; ++t) {
      const int ky = t / g.kw, kx = t - ky * g.kw;
      const int toff = (g.mode == 0 ? ky * h.PC + kx : (g.kh - 1 - ky) * h.PC + (g.kw - 1 - kx)) * PC2_P;
      const __bf16* bt = Bs + (t * BR + l32) * PC2_P + 8 * hh;
#pragma unroll
      for (int kq = 0; kq < 2; ++kq) {
        pc_bf16x8 af[TM], af1[HP ? TM : 1];
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          af[tm] = *(const pc_bf16x8*)&As[abase[tm] + toff + kq * 16];
          if constexpr (HP) af1[tm] = *(const pc_bf16x8*)&As[h.npix * PC2_P + abase[tm] + toff + kq * 16];
        }
#pragma unroll
        for (int tn = 0; tn < NT; ++tn) {
          const pc_bf16x8 bf = *(const pc_bf16x8*)(bt + tn * 32 * PC2_P + kq * 16);
          if constexpr (HP) {  // h0 h0' + h0 h1' + h1 h0'
            const pc_bf16x8 bf1 = *(const pc_bf16x8*)(bt + (nb + tn * 32) * PC2_P + kq * 16);
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) {
              acc[tm][tn] = pc_mfma<true>(af[tm], bf, acc[tm][tn]);
              acc[tm][tn] = pc_mfma<true>(af[tm], bf1, acc[tm][tn]);
              acc[tm][tn] = pc_mfma<true>(af1[tm], bf, acc[tm][tn]);
            }
          } else {
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) acc[tm][tn] = pc_mfma<H>(af[tm], bf, acc[tm][tn]);
          }
        }
      }
    }
    __syncthreads();  // every wave is done with this chunk's window and weights
    if (c + 1 < nchunk) {
      store();
      __syncthreads();
    }
  }
  if constexpr (H) {  // the fp16 planes' scales, once (the activation epilogue below then sees true values)
    const float al = pc_alpha(sc);
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int tn = 0; tn < NT; ++tn)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[tm][tn][r] *= al;
  }
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const long long mw = m0 + wave * 32 * TM + tm * 32;
    if (nlb.on) {  // activation-backward epilogue: per column tile, every load of the 16 rows before the stores
      const float* __restrict__ srcp = nlb.src;
      const float* __restrict__ mskp = nlb.mask;
      const float inv = 1.f / nlb.keep;
#pragma unroll
      for (int tn = 0; tn < NT; ++tn) {
        const int n = n0 + tn * 32 + l32;
        if (n >= g.cout) continue;
        float sv[16], mv[16], cv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const long long mm = mw + (r & 3) + 8 * (r >> 2) + 4 * hh;
          sv[r] = srcp[mm * nlb.lds + n];
          mv[r] = mskp ? mskp[mm * g.cout + n]
                       : (nlb.keep < 1.f ? drop_scale(nlb.seed, (unsigned long long)(mm * g.cout + n), nlb.keep, inv) : 1.f);
          cv[r] = accumulate ? Y[mm * ldy + n] : 0.f;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const long long mm = mw + (r & 3) + 8 * (r >> 2) + 4 * hh;
          const float gm = acc[tm][tn][r] * mv[r];
          const float d = nlb.kind == 0 ? (sv[r] > 0.f ? gm : 0.f) : gm * (sv[r] > 0.f ? 1.f : expf(sv[r]));
          Y[mm * ldy + n] = accumulate ? d + cv[r] : d;
        }
      }
      continue;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const long long mm = mw + (r & 3) + 8 * (r >> 2) + 4 * hh;
      bool zero = false;
      if (zero_edge) {
        const int rr = (int)(mm % per_img);
        zero = zero_edge == 1 ? (rr / g.wo == 0) : (rr % g.wo == 0);
      }
#pragma unroll
      for (int tn = 0; tn < NT; ++tn) {
        const int n = n0 + tn * 32 + l32;
        if (n >= g.cout) continue;
        float val = zero ? 0.f : acc[tm][tn][r] + (bias ? bias[n] : 0.f);
        float* p = Y + mm * ldy + n;
        if (accumulate) val += *p;
        *p = val;
      }
    }
  }
}

// plan of the halo kernel for a launch (false: not eligible -> pc_conv2)
bool pc3_plan(const PcGeom& g, int kpad, int TM, Pc3* out, size_t* lds) {
  const int BM = 256 * TM;
  const int taps = g.kh * g.kw;
  if (g.s != 1 || kpad % 32 || taps > PC3_MAXTAPS) return false;
  const long long rows = (long long)g.n * g.ho * g.wo;
  const int per_img = g.ho * g.wo;
  if (rows % BM) return false;
  Pc3 h;
  if (per_img % BM == 0 && BM % g.wo == 0) {
    h.R = BM / g.wo;
    h.nimg = 1;
  } else if (BM % per_img == 0) {
    h.R = g.ho;
    h.nimg = BM / per_img;
  } else {
    return false;
  }
  h.PR = h.R + g.kh - 1;
  h.PC = g.wo + g.kw - 1;
  h.npix = h.nimg * h.PR * h.PC;
  if (h.npix > PC3_MAXPIX) return false;
  if (g.mode == 0) {
    h.oy_off = -g.pt;
    h.ox_off = -g.pl;
  } else {
    h.oy_off = g.pt - (g.kh - 1);
    h.ox_off = g.pl - (g.kw - 1);
  }
  *out = h;
  return true;
}

template <int NT, int TM, bool XB, bool H = false, bool HP = false>
void pc3_launch(const PcGeom& g, const Pc3& h, const void* x, const __bf16* w, int kpad, const float* bias, float* y,
                int ldy, int accumulate, int zero_edge, const NlbArgs& nlb, const PcScale& sc, hipStream_t st,
                long long xpst = 0, long long wpst = 0) {
  const size_t lds = (size_t)(h.npix + g.kh * g.kw * 32 * NT) * PC2_P * 2 * (HP ? 2 : 1);
  static bool attr = false;
  if (!attr) {  // the largest window + weight stage: 640 pixels + 6 taps x 160 rows (128 KB); HP: the 160 KB cap
    const int mx = (PC3_MAXPIX + PC3_MAXTAPS * 32 * NT) * PC2_P * 2 * (HP ? 2 : 1);
    (void)hipFuncSetAttribute((const void*)pc_conv3_kernel<NT, TM, XB, H, HP>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, mx < 160 * 1024 ? mx : 160 * 1024);
    attr = true;
  }
  const long long rows = (long long)g.n * g.ho * g.wo;
  const dim3 grid((unsigned)(rows / (256 * TM)), (unsigned)((g.cout + 32 * NT - 1) / (32 * NT)));
  hipLaunchKernelGGL((pc_conv3_kernel<NT, TM, XB, H, HP>), grid, dim3(512), lds, st, g, h, x, w, kpad, bias, y, ldy,
                     accumulate, zero_edge, nlb, sc, xpst, wpst);
}

// ---------------------------------------------------------------------------------------------
// Row-staged halo conv of the split mode (both fp16 planes, three products per fragment pair): the
// block covers up to 160 output channels (NT = 5 column tiles) so the input window -- 4 B per element
// in two planes -- is staged ONCE per chunk for all of them (pc_conv3 HP holds every tap's weight rows
// in LDS, which caps it at 64 columns: the window was re-read by 3 / 5 column blocks of the 160 / 320-
// channel convs and the 160-channel ones computed 192).  Per 32-channel chunk the window stays in LDS
// while the weight rows of ONE kernel row (kw taps x 32 NT rows, both planes) at a time pass through
// it: per row phase each wave runs kw x 2 x NT x 3 MFMAs (90 for the [2, 3] convs at NT = 5) and the
// next phase's operands (the next row's weights, or the next chunk's window and row 0) load into
// registers meanwhile.  Bitwise the same sums as pc_conv3 HP per output (same K order: chunk, tap,
// k step, product order).
// ---------------------------------------------------------------------------------------------
#define PC3R_MAXPIX 384  // window pixels of a row-staged block (the head's shapes: 306-330)
template <int NT>
__global__ __launch_bounds__(512) void pc_conv3r_kernel(PcGeom g, Pc3 h, const __bf16* __restrict__ Xh,
                                                        const __bf16* __restrict__ Wk, int kpad,
                                                        const float* __restrict__ bias, float* __restrict__ Y, int ldy,
                                                        int accumulate, int zero_edge, PcScale sc, long long xpst,
                                                        long long wpst, unsigned* __restrict__ amax) {
  constexpr int BM = 256;
  constexpr int BR = 32 * NT;                                  // output channels per block
  constexpr int AI = (PC3R_MAXPIX * 4 + 511) / 512;            // window items (8 channels) per thread
  constexpr int BI = (3 * BR * 4 + 511) / 512;                 // 16-B weight items of one kernel row (kw <= 3)
  extern __shared__ __attribute__((aligned(16))) __bf16 pc3s[];
  __bf16* As = pc3s;                          // [plane][npix][PC2_P]
  __bf16* Bs = pc3s + 2 * h.npix * PC2_P;     // [plane][kw][BR][PC2_P]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, hh = lane >> 5;
  const int per_img = g.ho * g.wo;
  const long long m0 = (long long)blockIdx.x * BM;
  const int n0 = blockIdx.y * BR;
  const int img0 = (int)(m0 / per_img);
  const int oy0 = (int)(m0 - (long long)img0 * per_img) / g.wo;
  const int iy0 = oy0 + h.oy_off, ix0 = h.ox_off;
  const int nbr = g.kw * BR;  // staged weight rows of one kernel row

  int aoff[AI];  // (element offsets: the head's activations hold < 2^31 elements, pc3r_ok)
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int it = tid + 512 * i;
    aoff[i] = -2;
    if (it < h.npix * 4) {
      const int pix = it >> 2, part = it & 3;
      const int il = pix / (h.PR * h.PC);
      const int r2 = pix - il * h.PR * h.PC;
      const int pr = r2 / h.PC, pc = r2 - pr * h.PC;
      const int iy = iy0 + pr, ix = ix0 + pc;
      aoff[i] = (iy >= 0 && iy < g.hi && ix >= 0 && ix < g.wi)
                    ? ((((img0 + il) * g.hi + iy) * g.wi + ix) * g.ldx + part * 8)
                    : -1;
    }
  }
  pc_bf16x8 rh[AI], rh1[AI], rb[BI], rb1[BI];
  auto load_window = [&](int c) {
    const int k0 = c * 32;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int ci = k0 + ((tid + 512 * i) & 3) * 8;
      const pc_bf16x8 z = {};
      const bool ok = aoff[i] >= 0 && ci < g.cin;
      rh[i] = ok ? *(const pc_bf16x8*)(Xh + aoff[i] + k0) : z;
      rh1[i] = ok ? *(const pc_bf16x8*)(Xh + xpst + aoff[i] + k0) : z;
    }
  };
  auto load_row = [&](int c, int ky) {  // kernel row ky's kw taps, chunk c
    const int k0 = c * 32;
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int it = tid + 512 * i, row = it >> 2, q = it & 3;
      const int kx = row / BR, n = row - kx * BR;
      const pc_bf16x8 z = {};
      const bool ok = row < nbr && n0 + n < g.cout;
      const long long wo = ((long long)(ky * g.kw + kx) * g.cout + n0 + n) * kpad + k0 + q * 8;
      rb[i] = ok ? *(const pc_bf16x8*)(Wk + wo) : z;
      rb1[i] = ok ? *(const pc_bf16x8*)(Wk + wpst + wo) : z;
    }
  };
  auto store_window = [&]() {
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      if (aoff[i] < -1) continue;
      const int it = tid + 512 * i;
      *(pc_bf16x8*)&As[(it >> 2) * PC2_P + (it & 3) * 8] = rh[i];
      *(pc_bf16x8*)&As[(h.npix + (it >> 2)) * PC2_P + (it & 3) * 8] = rh1[i];
    }
  };
  auto store_row = [&]() {
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int it = tid + 512 * i, row = it >> 2, q = it & 3;
      if (row < nbr) {
        *(pc_bf16x8*)&Bs[row * PC2_P + q * 8] = rb[i];
        *(pc_bf16x8*)&Bs[(nbr + row) * PC2_P + q * 8] = rb1[i];
      }
    }
  };

  int abase;
  {
    const int rows_img = h.R * g.wo;
    const int ml = wave * 32 + l32;
    const int il = ml / rows_img;
    const int rem = ml - il * rows_img;
    const int ry = rem / g.wo, rx = rem - ry * g.wo;
    abase = ((il * h.PR + ry) * h.PC + rx) * PC2_P + 8 * hh;
  }
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  const int nchunk = kpad / 32;
  load_window(0);
  load_row(0, 0);
  store_window();
  store_row();
  __syncthreads();
  for (int c = 0; c < nchunk; ++c) {
    for (int ky = 0; ky < g.kh; ++ky) {
      const bool last_row = ky + 1 == g.kh;
      const bool more = !last_row || c + 1 < nchunk;
      if (!last_row) {
        load_row(c, ky + 1);
      } else if (c + 1 < nchunk) {
        load_window(c + 1);
        load_row(c + 1, 0);
      }
      for (int kx = 0; kx < g.kw; ++kx) {
        const int toff = (g.mode == 0 ? ky * h.PC + kx : (g.kh - 1 - ky) * h.PC + (g.kw - 1 - kx)) * PC2_P;
        const __bf16* bt = Bs + (kx * BR + l32) * PC2_P + 8 * hh;
#pragma unroll
        for (int kq = 0; kq < 2; ++kq) {
          const pc_bf16x8 af = *(const pc_bf16x8*)&As[abase + toff + kq * 16];
          const pc_bf16x8 af1 = *(const pc_bf16x8*)&As[h.npix * PC2_P + abase + toff + kq * 16];
#pragma unroll
          for (int tn = 0; tn < NT; ++tn) {
            const pc_bf16x8 bf = *(const pc_bf16x8*)(bt + tn * 32 * PC2_P + kq * 16);
            const pc_bf16x8 bf1 = *(const pc_bf16x8*)(bt + (nbr + tn * 32) * PC2_P + kq * 16);
            acc[tn] = pc_mfma<true>(af, bf, acc[tn]);  // h0 h0' + h0 h1' + h1 h0' (pc_conv3 HP's order)
            acc[tn] = pc_mfma<true>(af, bf1, acc[tn]);
            acc[tn] = pc_mfma<true>(af1, bf, acc[tn]);
          }
        }
      }
      __syncthreads();  // every wave is done with this row's weights (and, after the last row, the window)
      if (more) {
        if (last_row) store_window();
        store_row();
        __syncthreads();
      }
    }
  }
  const float al = pc_alpha(sc);
  const long long mw = m0 + wave * 32;
  float am = 0.f;  // (amax: max |y| of the block's outputs, after the accumulate)
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const long long mm = mw + (r & 3) + 8 * (r >> 2) + 4 * hh;
    bool zero = false;
    if (zero_edge) {
      const int rr = (int)(mm % per_img);
      zero = zero_edge == 1 ? (rr / g.wo == 0) : (rr % g.wo == 0);
    }
#pragma unroll
    for (int tn = 0; tn < NT; ++tn) {
      const int n = n0 + tn * 32 + l32;
      if (n >= g.cout) continue;
      float val = zero ? 0.f : acc[tn][r] * al + (bias ? bias[n] : 0.f);
      float* p = Y + mm * ldy + n;
      if (accumulate) val += *p;
      *p = val;
      am = fmaxf(am, fabsf(val));
    }
  }
  if (amax) block_absmax_put(am, amax);
}

// LDS of a row-staged launch (the window's and one kernel row's weights, both planes)
size_t pc3r_lds(const PcGeom& g, const Pc3& h, int NT) {
  return (size_t)(h.npix + g.kw * 32 * NT) * PC2_P * 2 * 2;
}
bool pc3r_ok(const PcGeom& g, const Pc3& h, int NT) {
  return g.kw <= 3 && h.npix <= PC3R_MAXPIX && (long long)g.n * g.hi * g.wi * g.ldx < (1LL << 31) &&
         pc3r_lds(g, h, NT) <= 160 * 1024;
}

template <int NT>
void pc3r_launch(const PcGeom& g, const Pc3& h, const __bf16* x, const __bf16* w, int kpad, const float* bias, float* y,
                 int ldy, int accumulate, int zero_edge, const PcScale& sc, hipStream_t st, long long xpst,
                 long long wpst, unsigned* amax) {
  static bool attr = false;
  if (!attr) {
    const int mx = (PC3R_MAXPIX + 3 * 32 * NT) * PC2_P * 2 * 2;
    (void)hipFuncSetAttribute((const void*)pc_conv3r_kernel<NT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              mx < 160 * 1024 ? mx : 160 * 1024);
    attr = true;
  }
  const long long rows = (long long)g.n * g.ho * g.wo;
  const dim3 grid((unsigned)(rows / 256), (unsigned)((g.cout + 32 * NT - 1) / (32 * NT)));
  hipLaunchKernelGGL((pc_conv3r_kernel<NT>), grid, dim3(512), pc3r_lds(g, h, NT), st, g, h, x, w, kpad, bias, y, ldy,
                     accumulate, zero_edge, sc, xpst, wpst, amax);
}

// ---------------------------------------------------------------------------------------------
// Tap-row weight gradient (stride 1, both modes: the resnet convs and their input gradients' nin /
// dense layers viewed as 16-wide images): dW[tap][ci][co] = sum_p X[src(p, tap)][ci] . D[p][co].
// Block = 64 ci x 64 co x ONE kernel row ky (its kw taps), four waves of 32 x 32 x kw taps; K = a
// split of the output pixels in chunks of 128 (whole image rows).  Per chunk the block stages, pixel-
// major in bf16, the chunk's X row segment for kernel row ky (R rows x (wo + kw - 1) pixels: the kw
// taps of the row are pixel shifts of one window) and its D rows; per 16-pixel K step a wave reads
// one transposed D fragment (ds_read_b64_tr_b16) and, per tap, one transposed X fragment at the
// tap's shift.  Against pc_wgrad_kernel (one tap per block) X and D are read kh instead of kh x kw
// times and each barrier covers 8 x kw MFMAs instead of 4.  bsum: the bias gradient's per-split
// column sums (blocks of ky = 0 and the first ci tile, fp32 before the bf16 staging).
// ---------------------------------------------------------------------------------------------
typedef short pc_v4i16 __attribute__((ext_vector_type(4)));
typedef short pc_v8i16 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ pc_v4i16 pc_tr16(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) pc_v4i16*)(p));
}
__device__ __forceinline__ pc_bf16x8 pc_join(pc_v4i16 lo, pc_v4i16 hi) {
  pc_v8i16 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(pc_bf16x8, v);
}
struct Pw4 {
  int R, PC, npix;  // image rows per chunk, window pixels per row, window pixels
  int iy_off[2];    // per kernel row: window row 0's input row relative to the chunk's first output row
  int ix_off;       // window column 0's input column
  int nchunk, cps;  // chunks in all, chunks per split
};
#define PW4_CP 128     // output pixels per chunk
#define PW4_MAXPIX 144 // 8 rows x 18 (16-wide images, kw = 3)
#define PW4_P 72       // LDS pixel pitch (bf16): 64 channels + 8
// DB: D (the output gradient) stored bf16 -- its MFMA precision (the bias sum is then done upstream)
// HP (with H): both fp16 planes of x and dy staged (xpst / dpst apart), three products per fragment pair
template <bool XB, bool DB, bool H = false, bool HP = false>
__global__ __launch_bounds__(256) void pc_wgrad4_kernel(PcGeom g, Pw4 h, const void* __restrict__ Xv,
                                                        const void* __restrict__ Dv, int ldd, float* __restrict__ part,
                                                        float* __restrict__ bsum, long long xpst = 0,
                                                        long long dpst = 0) {
  static_assert(!HP || (XB && DB && H), "fused planes: 16-bit fp16 x and dy");
  const float* D = (const float*)Dv;
  constexpr int WI = (PW4_MAXPIX * 8 + 255) / 256;  // window items (8 channels) per thread
  constexpr int DI = (PW4_CP * 16 + 255) / 256;     // D items (4 columns) per thread
  __shared__ __attribute__((aligned(16))) __bf16 smem[(HP ? 2 : 1) * (PW4_MAXPIX + PW4_CP) * PW4_P];
  __bf16* Ws = smem;                    // [npix][PW4_P]
  __bf16* Dm = smem + h.npix * PW4_P;   // [128][PW4_P]
  __bf16* Ws1 = Dm + PW4_CP * PW4_P;    // HP: the second planes
  __bf16* Dm1 = Ws1 + h.npix * PW4_P;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = lane >> 4, i16 = lane & 15, q = i16 >> 2, p4 = i16 & 3, l32 = lane & 31, hh = lane >> 5;
  const int ci0 = blockIdx.x * 64, co0 = blockIdx.y * 64;
  const int ky = blockIdx.z % g.kh, split = blockIdx.z / g.kh;
  const int wm = wave & 1, wn = wave >> 1;
  const bool live = ci0 + wm * 32 < g.cin && co0 + wn * 32 < g.cout;
  const int per_img = g.ho * g.wo;
  const int c_beg = split * h.cps;
  const int c_end = c_beg + h.cps < h.nchunk ? c_beg + h.cps : h.nchunk;
  const bool bias_blk = bsum && ky == 0 && ci0 == 0;
  const int iy_off = ky == 0 ? h.iy_off[0] : h.iy_off[1];

  f32x16 acc[3];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  f32x4 bacc = {0.f, 0.f, 0.f, 0.f};  // bias column sums: this thread's column quad (tid & 15)

  f32x4 xa[XB ? 1 : WI][2];
  pc_bf16x8 xh[XB ? WI : 1], xh1[HP ? WI : 1];
  f32x4 dv[DI];
  pc_bf16x4 dr[HP ? DI : 1], dr1[HP ? DI : 1];  // HP: dy's raw 16-bit lanes
  auto load = [&](int c) {
    const long long p0 = (long long)c * PW4_CP;
    const int img = (int)(p0 / per_img);
    const int oy0 = (int)(p0 - (long long)img * per_img) / g.wo;
#pragma unroll
    for (int i = 0; i < WI; ++i) {
      const int it = tid + 256 * i;
      const int pix = it >> 3, c8 = (it & 7) * 8;
      long long off = -1;
      if (it < h.npix * 8 && ci0 + c8 < g.cin) {
        const int pr = pix / h.PC, pc = pix - pr * h.PC;
        const int iy = oy0 + iy_off + pr, ix = h.ix_off + pc;
        if (iy >= 0 && iy < g.hi && ix >= 0 && ix < g.wi)
          off = ((long long)(img * g.hi + iy) * g.wi + ix) * g.ldx + ci0 + c8;
      }
      if constexpr (XB) {
        pc_bf16x8 z = {};
        xh[i] = off >= 0 ? *(const pc_bf16x8*)((const __bf16*)Xv + off) : z;
        if constexpr (HP) xh1[i] = off >= 0 ? *(const pc_bf16x8*)((const __bf16*)Xv + xpst + off) : z;
      } else {
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        xa[i][0] = off >= 0 ? *(const f32x4*)((const float*)Xv + off) : z;
        xa[i][1] = off >= 0 ? *(const f32x4*)((const float*)Xv + off + 4) : z;
      }
    }
#pragma unroll
    for (int i = 0; i < DI; ++i) {
      const int it = tid + 256 * i;
      const int k = it >> 4, c4 = (it & 15) * 4;
      if constexpr (HP) {
        const pc_bf16x4 z4 = {};
        const __bf16* dp = (const __bf16*)Dv + (p0 + k) * ldd + co0 + c4;
        dr[i] = co0 + c4 < g.cout ? *(const pc_bf16x4*)dp : z4;
        dr1[i] = co0 + c4 < g.cout ? *(const pc_bf16x4*)(dp + dpst) : z4;
      } else if constexpr (DB)
        dv[i] = co0 + c4 < g.cout
                    ? __builtin_convertvector(*(const pc_bf16x4*)((const __bf16*)Dv + (p0 + k) * ldd + co0 + c4), f32x4)
                    : f32x4{0.f, 0.f, 0.f, 0.f};
      else
        dv[i] = co0 + c4 < g.cout ? *(const f32x4*)(D + (p0 + k) * ldd + co0 + c4) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < WI; ++i) {
      const int it = tid + 256 * i;
      if (it >= h.npix * 8) continue;
      __bf16* w = Ws + (it >> 3) * PW4_P + (it & 7) * 8;
      if constexpr (XB) {
        *(pc_bf16x8*)w = xh[i];
        if constexpr (HP) *(pc_bf16x8*)(Ws1 + (it >> 3) * PW4_P + (it & 7) * 8) = xh1[i];
      } else {
        const pc_f32x8 v8 = {xa[i][0][0], xa[i][0][1], xa[i][0][2], xa[i][0][3],
                             xa[i][1][0], xa[i][1][1], xa[i][1][2], xa[i][1][3]};
        *(pc_bf16x8*)w = __builtin_convertvector(v8, pc_bf16x8);
      }
    }
#pragma unroll
    for (int i = 0; i < DI; ++i) {
      const int it = tid + 256 * i;
      const int k = it >> 4, c4 = (it & 15) * 4;
      if constexpr (HP) {
        *(pc_bf16x4*)(Dm + k * PW4_P + c4) = dr[i];
        *(pc_bf16x4*)(Dm1 + k * PW4_P + c4) = dr1[i];
        continue;
      }
      if (bias_blk) bacc += dv[i];  // (the column quad it & 15 == tid & 15 for every i)
      *(pc_bf16x4*)(Dm + k * PW4_P + c4) = __builtin_convertvector(dv[i], pc_bf16x4);
    }
  };

  // lane roles of the transposed reads: pixel lk (+ 4) of a 16-pixel K step, channel / column quad
  const int lk = 8 * (grp >> 1) + q;
  const int cha = wm * 32 + 16 * (grp & 1) + 4 * p4;
  const int chb = wn * 32 + 16 * (grp & 1) + 4 * p4;
  if (c_beg < c_end) {
    load(c_beg);
    store();
  }
  __syncthreads();
  for (int c = c_beg; c < c_end; ++c) {
    if (c + 1 < c_end) load(c + 1);
    if (live) {
#pragma unroll 2
      for (int ks = 0; ks < PW4_CP / 16; ++ks) {
        const int k0 = ks * 16;
        const int wrow = k0 / g.wo, wcol = k0 - wrow * g.wo;  // the step's 16 pixels share one image row
        const int wp = wrow * h.PC + wcol + lk;
        const pc_bf16x8 bf =
            pc_join(pc_tr16(Dm + (k0 + lk) * PW4_P + chb), pc_tr16(Dm + (k0 + lk + 4) * PW4_P + chb));
        pc_bf16x8 bf1 = {};
        if constexpr (HP)
          bf1 = pc_join(pc_tr16(Dm1 + (k0 + lk) * PW4_P + chb), pc_tr16(Dm1 + (k0 + lk + 4) * PW4_P + chb));
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          if (kx < g.kw) {
            const int sh = g.mode == 0 ? kx : g.kw - 1 - kx;
            const __bf16* wa = Ws + (wp + sh) * PW4_P + cha;
            const pc_bf16x8 af = pc_join(pc_tr16(wa), pc_tr16(wa + 4 * PW4_P));
            acc[kx] = pc_mfma<H>(af, bf, acc[kx]);
            if constexpr (HP) {
              const __bf16* wa1 = Ws1 + (wp + sh) * PW4_P + cha;
              const pc_bf16x8 af1 = pc_join(pc_tr16(wa1), pc_tr16(wa1 + 4 * PW4_P));
              acc[kx] = pc_mfma<true>(af, bf1, acc[kx]);
              acc[kx] = pc_mfma<true>(af1, bf, acc[kx]);
            }
          }
        }
      }
    }
    __syncthreads();
    if (c + 1 < c_end) {
      store();
      __syncthreads();
    }
  }
  if (live) {
    float* out = part + (long long)split * g.kh * g.kw * g.cin * g.cout;
    const int n = co0 + wn * 32 + l32;
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {  // (unrolled: a runtime-indexed acc would live in scratch memory)
      if (kx >= g.kw) break;
      const int tap = ky * g.kw + kx;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = ci0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (m < g.cin && n < g.cout) out[((long long)tap * g.cin + m) * g.cout + n] = acc[kx][r];
      }
    }
  }
  if (bias_blk) {  // the 16 row lanes of each column quad combined in lane order through LDS
    float* red = (float*)smem;  // [16 row lanes][64]
    *(f32x4*)&red[(tid >> 4) * 64 + (tid & 15) * 4] = bacc;
    __syncthreads();
    if (tid < 64 && co0 + tid < g.cout) {
      float v = 0.f;
      for (int i = 0; i < 16; ++i) v += red[i * 64 + tid];
      bsum[(long long)split * g.cout + co0 + tid] = v;
    }
  }
}

// (measured on the B = 128 head shapes: the [2, 3] convs 1.2-1.45x faster than the one-tap kernel, the
// [2, 2] and 1x1 ones slower at two blocks per CU: kw = 3 only)
// any_kw: every kernel width (the fused-plane weight gradients, where a one-tap launch re-reads x and dy per tap)
bool pw4_plan(const PcGeom& g, long long rows, Pw4* out, bool any_kw = false) {
  if (g.s != 1 || g.kh > 2 || (any_kw ? g.kw > 3 : g.kw != 3) || g.wo % 16 || PW4_CP % g.wo || (g.ho * g.wo) % PW4_CP || rows % PW4_CP ||
      g.ldx % 8 || g.cin % 8)
    return false;
  Pw4 h;
  h.R = PW4_CP / g.wo;
  h.PC = g.wo + g.kw - 1;
  h.npix = h.R * h.PC;
  if (h.npix > PW4_MAXPIX) return false;
  for (int ky = 0; ky < 2; ++ky) h.iy_off[ky] = g.mode == 0 ? ky - g.pt : g.pt - ky;
  h.ix_off = g.mode == 0 ? -g.pl : g.pl - (g.kw - 1);
  h.nchunk = (int)(rows / PW4_CP);
  h.cps = 0;
  *out = h;
  return true;
}

// ---------------------------------------------------------------------------------------------
// weight gradient: block = one tap x 64 ci x 64 co (2 x 2 waves of 32 x 32), K = a split of the
// output rows in chunks of 32, staged through LDS transposed (row-contiguous per channel, so
// each MFMA fragment is one 16-B LDS read).  Partial slabs [split][tap][ci][co].
// ---------------------------------------------------------------------------------------------
#define PW_RP 72  // LDS row pitch (bf16): 64 rows + 8 pad
// bsum != NULL: the blocks of tap 0 and the first ci tile also sum their D rows per column (fp32,
// before the bf16 staging) into bsum[split][cout]: the conv's bias gradient without another pass over dy
// HP (with H): both fp16 planes of x (xpst apart) and of dy (dpst apart) staged, h0 d0 + h0 d1 + h1 d0 per fragment
// pair in ONE launch (svae_pcnn_conv_wgrad_planes); dy's 16-bit lanes are staged as raw bits
template <bool XB, bool DB, bool H = false, bool HP = false>
__global__ __launch_bounds__(256) void pc_wgrad_kernel(PcGeom g, const void* __restrict__ Xv,
                                                       const void* __restrict__ Dv, int ldd, long long rows,
                                                       long long rows_per_split, float* __restrict__ part,
                                                       float* __restrict__ bsum, long long xpst = 0,
                                                       long long dpst = 0) {
  static_assert(!HP || (XB && DB && H), "fused planes: 16-bit fp16 x and dy");
  constexpr int NPL = HP ? 2 : 1;
  __shared__ __attribute__((aligned(16))) __bf16 Xs[NPL][2][64 * PW_RP];
  __shared__ __attribute__((aligned(16))) __bf16 Ds[NPL][2][64 * PW_RP];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int nci = (g.cin + 63) / 64;
  const int ci0 = (blockIdx.x % nci) * 64, co0 = (blockIdx.x / nci) * 64;
  const int tap = blockIdx.y, split = blockIdx.z;
  const int ky = tap / g.kw, kx = tap - ky * g.kw;
  const int wm = wave & 1, wn = wave >> 1;
  const int per_img = g.ho * g.wo;
  const long long r0 = (long long)split * rows_per_split;
  long long r1 = r0 + rows_per_split;
  if (r1 > rows) r1 = rows;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  // staging role: rows lr and lr + 32 (lr = tid >> 3), channel quads q0 and q0 + 8; chunks of 64
  // rows, the next chunk loaded into registers while the current one's MFMAs run
  const int lr = tid >> 3, q0 = tid & 7;
  f32x4 xv[2][2], dv[2][2];
  pc_bf16x8 xb8[2], xb81[2];  // XB: channels 8 q0 .. 8 q0 + 7 of the row in one 16-B load
  pc_bf16x4 dh[HP ? 2 : 1][2][2];  // HP: dy's raw 16-bit lanes, both planes
  auto load = [&](long long rc) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const long long row = rc + lr + 32 * u;
      long long xo = -1;
      const float* dp = nullptr;
      const __bf16* dph = nullptr;
      if (row < r1) {
        const int img = (int)(row / per_img);
        const int rr = (int)(row - (long long)img * per_img);
        const int oy = rr / g.wo, ox = rr - (rr / g.wo) * g.wo;
        int iy, ix;
        if (pc_src(g, oy, ox, ky, kx, iy, ix)) xo = ((long long)(img * g.hi + iy) * g.wi + ix) * g.ldx;
        if constexpr (DB) dph = (const __bf16*)Dv + row * ldd;
        else dp = (const float*)Dv + row * ldd;
      }
      if constexpr (XB) {
        pc_bf16x8 z8 = {};
        const bool ok = xo >= 0 && ci0 + 8 * q0 < g.cin;
        xb8[u] = ok ? *(const pc_bf16x8*)((const __bf16*)Xv + xo + ci0 + 8 * q0) : z8;
        if constexpr (HP) xb81[u] = ok ? *(const pc_bf16x8*)((const __bf16*)Xv + xpst + xo + ci0 + 8 * q0) : z8;
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = (q0 + 8 * j) * 4;
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        if constexpr (!XB) xv[u][j] = (xo >= 0 && ci0 + c < g.cin) ? *(const f32x4*)((const float*)Xv + xo + ci0 + c) : z;
        if constexpr (HP) {
          const pc_bf16x4 z4 = {};
          const bool ok = dph && co0 + c < g.cout;
          dh[0][u][j] = ok ? *(const pc_bf16x4*)(dph + co0 + c) : z4;
          dh[1][u][j] = ok ? *(const pc_bf16x4*)(dph + dpst + co0 + c) : z4;
        } else if constexpr (DB)
          dv[u][j] = (dph && co0 + c < g.cout) ? __builtin_convertvector(*(const pc_bf16x4*)(dph + co0 + c), f32x4) : z;
        else
          dv[u][j] = (dp && co0 + c < g.cout) ? *(const f32x4*)(dp + co0 + c) : z;
      }
    }
  };
  const bool bias_blk = bsum && tap == 0 && ci0 == 0;
  f32x4 bacc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  auto store = [&](int buf) {
    if (bias_blk) {
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int j = 0; j < 2; ++j) bacc[j] += dv[u][j];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = (q0 + 8 * j) * 4;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if constexpr (XB) Xs[0][buf][(8 * q0 + 4 * j + e) * PW_RP + lr + 32 * u] = xb8[u][4 * j + e];
          else Xs[0][buf][(c + e) * PW_RP + lr + 32 * u] = (__bf16)xv[u][j][e];
          if constexpr (HP) {
            Xs[NPL - 1][buf][(8 * q0 + 4 * j + e) * PW_RP + lr + 32 * u] = xb81[u][4 * j + e];
            Ds[0][buf][(c + e) * PW_RP + lr + 32 * u] = dh[0][u][j][e];
            Ds[NPL - 1][buf][(c + e) * PW_RP + lr + 32 * u] = dh[HP ? 1 : 0][u][j][e];
          } else {
            Ds[0][buf][(c + e) * PW_RP + lr + 32 * u] = (__bf16)dv[u][j][e];
          }
        }
      }
  };
  if (r0 < r1) {
    load(r0);
    store(0);
  }
  __syncthreads();
  int buf = 0;
  for (long long rc = r0; rc < r1; rc += 64) {
    const bool more = rc + 64 < r1;
    if (more) load(rc + 64);
#pragma unroll
    for (int kq = 0; kq < 4; ++kq) {
      const pc_bf16x8 af = *(const pc_bf16x8*)&Xs[0][buf][(wm * 32 + l32) * PW_RP + kq * 16 + 8 * h];
      const pc_bf16x8 bf = *(const pc_bf16x8*)&Ds[0][buf][(wn * 32 + l32) * PW_RP + kq * 16 + 8 * h];
      acc = pc_mfma<H>(af, bf, acc);
      if constexpr (HP) {
        const pc_bf16x8 af1 = *(const pc_bf16x8*)&Xs[NPL - 1][buf][(wm * 32 + l32) * PW_RP + kq * 16 + 8 * h];
        const pc_bf16x8 bf1 = *(const pc_bf16x8*)&Ds[NPL - 1][buf][(wn * 32 + l32) * PW_RP + kq * 16 + 8 * h];
        acc = pc_mfma<true>(af, bf1, acc);
        acc = pc_mfma<true>(af1, bf, acc);
      }
    }
    if (more) store(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  float* out = part + ((long long)split * g.kh * g.kw + tap) * g.cin * g.cout;
  const int co = co0 + wn * 32 + l32;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int ci = ci0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (ci < g.cin && co < g.cout) out[(long long)ci * g.cout + co] = acc[r];
  }
  if (bias_blk) {  // column sums: the 32 row lanes combined in lane order through LDS (the loop's last barrier passed)
    float* red = (float*)&Xs[0][0][0];  // [32][64]
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[lr * 64 + (q0 + 8 * j) * 4 + e] = bacc[j][e];
    __syncthreads();
    if (tid < 64 && co0 + tid < g.cout) {
      float v = 0.f;
      for (int i = 0; i < 32; ++i) v += red[i * 64 + tid];
      bsum[(long long)split * g.cout + co0 + tid] = v;
    }
  }
}

// sc.a != NULL: the slabs are fp16-plane products, the sum is scaled by their inverse scales (exact)
__global__ void split_reduce_kernel(const float* __restrict__ part, int nsplit, long long n, float* __restrict__ out,
                                    PcScale sc = PcScale{nullptr, nullptr}) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const float al = pc_alpha(sc);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float s = 0.f;
    for (int k = 0; k < nsplit; ++k) s += part[(long long)k * n + i];
    out[i] = s * al;
  }
}

// (n % 4 == 0, 16-B part / out: four elements per thread, the same k order -- bitwise)
__global__ void split_reduce4_kernel(const float* __restrict__ part, int nsplit, long long n, float* __restrict__ out,
                                     PcScale sc) {
  const long long stride = (long long)gridDim.x * blockDim.x * 4;
  const float al = pc_alpha(sc);
  for (long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < nsplit; ++k) s += *(const f32x4*)&part[(long long)k * n + i];
    *(f32x4*)&out[i] = s * al;
  }
}
// the weight-gradient split-K partials into dW (scaled by the split mode's alpha)
static void split_reduce(const float* part, int nsplit, long long n, float* out, PcScale sc, hipStream_t st) {
  static const bool vec = svae_knob("SVAE_PC_SRED4", 1) != 0;
  if (vec && n % 4 == 0 && ((uintptr_t)part & 15) == 0 && ((uintptr_t)out & 15) == 0)
    hipLaunchKernelGGL(split_reduce4_kernel, dim3(blocks_for(n / 4)), dim3(256), 0, st, part, nsplit, n, out, sc);
  else
    hipLaunchKernelGGL(split_reduce_kernel, dim3(blocks_for(n)), dim3(256), 0, st, part, nsplit, n, out, sc);
}

// ---------------------------------------------------------------------------------------------
// column sums (bias gradients) and edge masks
// ---------------------------------------------------------------------------------------------
// stage 1: blockIdx.x = 64-column group, blockIdx.y = row split -> scratch[split][c]
__global__ __launch_bounds__(256) void colsum_part_kernel_pc(const float* __restrict__ x, long long rows, int c,
                                                             int ldx, int per_img, int wo, int mask_edge,
                                                             long long rows_per_split, float* __restrict__ part) {
  __shared__ float red[4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63), q = threadIdx.x >> 6;
  const long long r0 = (long long)blockIdx.y * rows_per_split;
  long long r1 = r0 + rows_per_split;
  if (r1 > rows) r1 = rows;
  float s = 0.f;
  if (col < c)
    for (long long r = r0 + q; r < r1; r += 4) {
      if (mask_edge) {
        const int rr = (int)(r % per_img);
        if (mask_edge == 1 ? (rr / wo == 0) : (rr % wo == 0)) continue;
      }
      s += x[r * ldx + col];
    }
  red[q][threadIdx.x & 63] = s;
  __syncthreads();
  if (q == 0 && col < c)
    part[(long long)blockIdx.y * c + col] =
        red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}
// stage 1, 4-column vector form (c, ldx % 4 == 0, 16-B x / part, rows < 2^31): 64 columns x 16 row lanes per
// block, one 16-byte load per row and lane, the lanes combined in a fixed order (the element form above runs at
// ~1 TB/s on its 4-byte loads and 64-bit row modulo)
__global__ __launch_bounds__(256) void colsum_part4_kernel_pc(const float* __restrict__ x, int rows, int c, int ldx,
                                                              int per_img, FastDiv dimg, int wo, FastDiv dwo,
                                                              int mask_edge, int rows_per_split,
                                                              float* __restrict__ part) {
  __shared__ f32x4 red[16][16];
  const int cq = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int col = blockIdx.x * 64 + cq * 4;
  const int r0 = blockIdx.y * rows_per_split;
  const int r1 = r0 + rows_per_split < rows ? r0 + rows_per_split : rows;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (col < c)
    for (int r = r0 + rl; r < r1; r += 16) {
      if (mask_edge) {
        const int rr = r - fdiv(r, dimg) * per_img;
        const int y = fdiv(rr, dwo);
        if (mask_edge == 1 ? (y == 0) : (rr - y * wo == 0)) continue;
      }
      s += *(const f32x4*)&x[(long long)r * ldx + col];
    }
  red[rl][cq] = s;
  __syncthreads();
  if (rl == 0 && col < c) {
    f32x4 t = red[0][cq];
#pragma unroll
    for (int j = 1; j < 16; ++j) t += red[j][cq];
    *(f32x4*)&part[(long long)blockIdx.y * c + col] = t;
  }
}
// stage 1 with max |x| (the split mode's gradient planes, svae_pcnn_colsum_absmax): the bias gradient's column
// partials and the fp16 planes' scale from ONE pass over dy (were colsum_part4 + absmax4: two reads of it)
__global__ __launch_bounds__(256) void colsum_amax4_kernel_pc(const float* __restrict__ x, int rows, int c, int ldx,
                                                              int rows_per_split, float* __restrict__ part,
                                                              unsigned* __restrict__ mx) {
  __shared__ f32x4 red[16][16];
  const int cq = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int col = blockIdx.x * 64 + cq * 4;
  const int r0 = blockIdx.y * rows_per_split;
  const int r1 = r0 + rows_per_split < rows ? r0 + rows_per_split : rows;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  float m = 0.f;
  if (col < c)
    for (int r = r0 + rl; r < r1; r += 16) {
      const f32x4 v = *(const f32x4*)&x[(long long)r * ldx + col];
      s += v;
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
    }
  red[rl][cq] = s;
  block_absmax_put(m, mx);  // (its barrier also orders red's stores before the reads below)
  __syncthreads();
  if (rl == 0 && col < c) {
    f32x4 t = red[0][cq];
#pragma unroll
    for (int j = 1; j < 16; ++j) t += red[j][cq];
    *(f32x4*)&part[(long long)blockIdx.y * c + col] = t;
  }
}
// stage 2, 4-column form (with the vector stage 1): 64 columns x 16 split lanes per block, one 16-byte load per
// split and lane (the element form's 4 lanes looped ns / 4 = 128-256 dependent loads: 39 us per call, r05_gpv)
__global__ __launch_bounds__(256) void colsum_fin4_kernel_pc(const float* __restrict__ part, int nsplit, int c,
                                                             float* __restrict__ out, int accumulate) {
  __shared__ f32x4 red[16][16];
  const int cq = threadIdx.x & 15, q = threadIdx.x >> 4;
  const int col = blockIdx.x * 64 + cq * 4;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (col < c)
    for (int k = q; k < nsplit; k += 16) s += *(const f32x4*)&part[(long long)k * c + col];
  red[q][cq] = s;
  __syncthreads();
  if (q == 0 && col < c) {
    f32x4 t = red[0][cq];
#pragma unroll
    for (int j = 1; j < 16; ++j) t += red[j][cq];
#pragma unroll
    for (int j = 0; j < 4; ++j) out[col + j] = accumulate ? out[col + j] + t[j] : t[j];
  }
}
// stage 2: 64 columns per block, 4 split-lanes, fixed-order combine
__global__ __launch_bounds__(256) void colsum_fin_kernel_pc(const float* __restrict__ part, int nsplit, int c,
                                                            float* __restrict__ out, int accumulate) {
  __shared__ float red[4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63), q = threadIdx.x >> 6;
  float s = 0.f;
  if (col < c)
    for (int k = q; k < nsplit; k += 4) s += part[(long long)k * c + col];
  red[q][threadIdx.x & 63] = s;
  __syncthreads();
  if (q == 0 && col < c) {
    const float v = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    out[col] = accumulate ? out[col] + v : v;
  }
}

__global__ void mask_edge_kernel(float* x, long long n_rows, int per_img, int wo, int c, int ldx, int mask_edge) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long total = n_rows * c;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const long long r = i / c;
    const int rr = (int)(r % per_img);
    if (mask_edge == 1 ? (rr / wo == 0) : (rr % wo == 0)) x[r * ldx + (int)(i % c)] = 0.f;
  }
}

// ---------------------------------------------------------------------------------------------
// elementwise ops
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float elu_f(float x) { return x > 0.f ? x : expm1f(x); }
__device__ __forceinline__ float delu_f(float x) { return x > 0.f ? 1.f : expf(x); }

// Vectorised forms (4 channels per thread, NL_RPB rows per block, 32-bit index math): the resnet
// nonlinearity with the training pass's dropout fused (y = f(x) * mask, nn.py:270-274), written fp32
// or bf16 -- bf16 when its only consumers are the bf16-MFMA convs, which round it the same way --
// and its backward dx (+)= f'(x) * (dy * mask).
#define NL_RPB 64
__device__ __forceinline__ void nl_fwd4(f32x4 v, int kind, f32x4& a, f32x4& b) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (kind == 0) {
      a[e] = fmaxf(v[e], 0.f);
    } else {
      a[e] = elu_f(v[e]);
      b[e] = elu_f(-v[e]);
    }
  }
}
// the training pass's dropout keep-mask drawn in the kernel (no mask tensor): element idx of the
// [rows][cy] mask keeps with probability keep (splitmix64 of seed + idx, 24-bit uniform) and
// scales by 1 / keep -- the same value in the forward, the backward and svae_pcnn_dropout_mask
__device__ __forceinline__ float drop_scale(unsigned long long seed, unsigned long long idx, float keep, float inv) {
  unsigned long long z = seed + idx * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.f / 16777216.f) < keep ? inv : 0.f;
}
__device__ __forceinline__ f32x4 drop_scale4(unsigned long long seed, unsigned long long idx, float keep, float inv) {
  return f32x4{drop_scale(seed, idx, keep, inv), drop_scale(seed, idx + 1, keep, inv),
               drop_scale(seed, idx + 2, keep, inv), drop_scale(seed, idx + 3, keep, inv)};
}
__global__ void dropout_mask_kernel(long long n, float keep, unsigned long long seed, float* __restrict__ out) {
  const float inv = 1.f / keep;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    out[i] = drop_scale(seed, (unsigned long long)i, keep, inv);
}

template <bool YB>
// amax != NULL: max |y| over the block into *amax (the split mode's absmax of this conv input, fused: bitwise the
// separate pass over y)
__global__ __launch_bounds__(256) void nonlin4_kernel(const float* __restrict__ x, long long rows, int c, int ldx,
                                                      int kind, const float* __restrict__ mask, float keep,
                                                      unsigned long long seed, void* __restrict__ y, int ldy,
                                                      unsigned* __restrict__ amax) {
  float am = 0.f;
  const bool hashed = !mask && keep < 1.f;
  const float inv = 1.f / keep;
  const int q = c >> 2, cy = kind == 2 ? 2 * c : c;
  const long long r0 = (long long)blockIdx.x * NL_RPB;
  const int nr = (int)(rows - r0 < NL_RPB ? rows - r0 : NL_RPB);
  for (int j = threadIdx.x; j < nr * q; j += 256) {
    const int rr = j / q;
    const int ch = (j - rr * q) * 4;
    const long long r = r0 + rr;
    f32x4 a, b = {0.f, 0.f, 0.f, 0.f};
    nl_fwd4(*(const f32x4*)(x + r * ldx + ch), kind, a, b);
    if (mask) {
      a *= *(const f32x4*)(mask + r * cy + ch);
      if (kind == 2) b *= *(const f32x4*)(mask + r * cy + c + ch);
    } else if (hashed) {
      a *= drop_scale4(seed, (unsigned long long)(r * cy + ch), keep, inv);
      if (kind == 2) b *= drop_scale4(seed, (unsigned long long)(r * cy + c + ch), keep, inv);
    }
    if constexpr (YB) {
      __bf16* yp = (__bf16*)y + r * ldy + ch;
      *(pc_bf16x4*)yp = __builtin_convertvector(a, pc_bf16x4);
      if (kind == 2) *(pc_bf16x4*)(yp + c) = __builtin_convertvector(b, pc_bf16x4);
    } else {
      float* yp = (float*)y + r * ldy + ch;
      *(f32x4*)yp = a;
      if (kind == 2) *(f32x4*)(yp + c) = b;
      if (amax)
#pragma unroll
        for (int j = 0; j < 4; ++j) am = fmaxf(am, fmaxf(fabsf(a[j]), fabsf(b[j])));  // (b = 0 unless kind 2)
    }
  }
  if (!YB && amax) block_absmax_put(am, amax);
}
__global__ __launch_bounds__(256) void nonlin4_bwd_kernel(const float* __restrict__ x, long long rows, int c, int ldx,
                                                          int kind, const float* __restrict__ mask, float keep,
                                                          unsigned long long seed, const float* __restrict__ dy,
                                                          int ldy, float* __restrict__ dx, int lddx, int accumulate) {
  const bool hashed = !mask && keep < 1.f;
  const float inv = 1.f / keep;
  const int q = c >> 2, cy = kind == 2 ? 2 * c : c;
  const long long r0 = (long long)blockIdx.x * NL_RPB;
  const int nr = (int)(rows - r0 < NL_RPB ? rows - r0 : NL_RPB);
  for (int j = threadIdx.x; j < nr * q; j += 256) {
    const int rr = j / q;
    const int ch = (j - rr * q) * 4;
    const long long r = r0 + rr;
    const f32x4 v = *(const f32x4*)(x + r * ldx + ch);
    f32x4 g = *(const f32x4*)(dy + r * ldy + ch), g2 = {0.f, 0.f, 0.f, 0.f};
    if (kind == 2) g2 = *(const f32x4*)(dy + r * ldy + c + ch);
    if (mask) {
      g *= *(const f32x4*)(mask + r * cy + ch);
      if (kind == 2) g2 *= *(const f32x4*)(mask + r * cy + c + ch);
    } else if (hashed) {
      g *= drop_scale4(seed, (unsigned long long)(r * cy + ch), keep, inv);
      if (kind == 2) g2 *= drop_scale4(seed, (unsigned long long)(r * cy + c + ch), keep, inv);
    }
    f32x4 d;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (kind == 0) d[e] = v[e] > 0.f ? g[e] : 0.f;  // tf.nn.relu: relu'(0) = 0
      else if (kind == 1) d[e] = g[e] * delu_f(v[e]);
      else d[e] = g[e] * delu_f(v[e]) - g2[e] * delu_f(-v[e]);
    }
    f32x4* p = (f32x4*)(dx + r * lddx + ch);
    *p = accumulate ? *p + d : d;
  }
}

// the same backward (kinds 0 / 1, written, not accumulated) with per-block column sums of the written
// gradient into part[block][c] (row lanes, then lanes in order: deterministic), dx fp32 or bf16
__global__ __launch_bounds__(256) void nonlin4_bwd_cs_kernel(const float* __restrict__ x, long long rows, int c,
                                                             int ldx, int kind, const float* __restrict__ mask,
                                                             float keep, unsigned long long seed,
                                                             const float* __restrict__ dy, int ldy, void* __restrict__ dxv,
                                                             int lddx, int out_bf16, float* __restrict__ part) {
  __shared__ f32x4 red[256];
  const int q = c >> 2;
  const int RL = 256 / q;
  const int tid = threadIdx.x, qi = tid % q, rl = tid / q;
  const long long r0 = (long long)blockIdx.x * NL_RPB;
  const int nr = (int)(rows - r0 < NL_RPB ? rows - r0 : NL_RPB);
  const bool hashed = !mask && keep < 1.f;
  const float inv = 1.f / keep;
  const int ch = qi * 4;
  f32x4 sum = {0.f, 0.f, 0.f, 0.f};
  if (rl < RL) {
    for (int rr = rl; rr < nr; rr += RL) {
      const long long r = r0 + rr;
      const f32x4 v = *(const f32x4*)(x + r * ldx + ch);
      f32x4 g = *(const f32x4*)(dy + r * ldy + ch);
      if (mask) g *= *(const f32x4*)(mask + r * c + ch);
      else if (hashed) g *= drop_scale4(seed, (unsigned long long)(r * c + ch), keep, inv);
      f32x4 d;
#pragma unroll
      for (int e = 0; e < 4; ++e) d[e] = kind == 0 ? (v[e] > 0.f ? g[e] : 0.f) : g[e] * delu_f(v[e]);
      if (out_bf16) *(pc_bf16x4*)((__bf16*)dxv + r * lddx + ch) = __builtin_convertvector(d, pc_bf16x4);
      else *(f32x4*)((float*)dxv + r * lddx + ch) = d;
      sum += d;
    }
  }
  red[tid] = sum;
  __syncthreads();
  if (tid < q) {
    f32x4 t = red[tid];
    for (int l = 1; l < RL; ++l) t += red[l * q + tid];
    *(f32x4*)(part + (long long)blockIdx.x * c + ch) = t;
  }
}

__global__ void nonlin_kernel(const float* __restrict__ x, long long rows, int c, int ldx, int kind,
                              float* __restrict__ y, int ldy) {
  const long long stride = (long long)gridDim.x * blockDim.x, total = rows * c;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const long long r = i / c;
    const int j = (int)(i - r * c);
    const float v = x[r * ldx + j];
    if (kind == 0) {
      y[r * ldy + j] = fmaxf(v, 0.f);
    } else if (kind == 1) {
      y[r * ldy + j] = elu_f(v);
    } else {
      y[r * ldy + j] = elu_f(v);
      y[r * ldy + c + j] = elu_f(-v);
    }
  }
}

__global__ void nonlin_bwd_kernel(const float* __restrict__ x, long long rows, int c, int ldx, int kind,
                                  const float* __restrict__ dy, int ldy, float* __restrict__ dx, int lddx,
                                  int accumulate) {
  const long long stride = (long long)gridDim.x * blockDim.x, total = rows * c;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const long long r = i / c;
    const int j = (int)(i - r * c);
    const float v = x[r * ldx + j];
    float d;
    if (kind == 0) d = v > 0.f ? dy[r * ldy + j] : 0.f;  // tf.nn.relu: relu'(0) = 0
    else if (kind == 1) d = dy[r * ldy + j] * delu_f(v);
    else d = dy[r * ldy + j] * delu_f(v) - dy[r * ldy + c + j] * delu_f(-v);
    float* p = dx + r * lddx + j;
    *p = accumulate ? *p + d : d;
  }
}

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

__global__ void gate_kernel(const float* __restrict__ x, int ldx, const float* __restrict__ c2,
                            const float* __restrict__ hp, long long rows, int per_img, int f, float* __restrict__ out,
                            int ldo) {
  const long long stride = (long long)gridDim.x * blockDim.x, total = rows * f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const long long r = i / f;
    const int j = (int)(i - r * f);
    const long long img = r / per_img;
    float a = c2[r * 2 * f + j], b = c2[r * 2 * f + f + j];
    if (hp) {
      a += hp[img * 2 * f + j];
      b += hp[img * 2 * f + f + j];
    }
    out[r * ldo + j] = x[r * ldx + j] + a * sigm(b);
  }
}

__global__ void gate_bwd_kernel(const float* __restrict__ c2, const float* __restrict__ hp,
                                const float* __restrict__ dout, int lddo, long long rows, int per_img, int f,
                                float* __restrict__ dc2) {
  const long long stride = (long long)gridDim.x * blockDim.x, total = rows * f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const long long r = i / f;
    const int j = (int)(i - r * f);
    const long long img = r / per_img;
    float a = c2[r * 2 * f + j], b = c2[r * 2 * f + f + j];
    if (hp) {
      a += hp[img * 2 * f + j];
      b += hp[img * 2 * f + f + j];
    }
    const float d = dout[r * lddo + j], sb = sigm(b);
    dc2[r * 2 * f + j] = d * sb;
    dc2[r * 2 * f + f + j] = d * a * sb * (1.f - sb);
  }
}

// Vectorised gated-resnet tail (4 channels per thread, GT_RPB rows of one image per block, 32-bit
// index math).  The backward also sums dc2 over the block's rows per column (fixed order: row lanes,
// then lanes in order) into part[block][2f]; gate_imgsum_kernel adds an image's blocks in order: the
// per-image d(h . hw) without re-reading dc2.
#define GT_RPB 64
__device__ __forceinline__ f32x4 sigm4(f32x4 v) {
  f32x4 r;
#pragma unroll
  for (int e = 0; e < 4; ++e) r[e] = 1.f / (1.f + expf(-v[e]));
  return r;
}
// amax != NULL: max |out| into *amax (the bound of the next split-mode nonlinearity's fp16 planes)
__global__ __launch_bounds__(256) void gate4_kernel(const float* __restrict__ x, int ldx, const float* __restrict__ c2,
                                                    const float* __restrict__ hp, long long rows, int per_img, int f,
                                                    float* __restrict__ out, int ldo, unsigned* __restrict__ amax) {
  float am = 0.f;
  const int q = f >> 2;
  const long long r0 = (long long)blockIdx.x * GT_RPB;
  const int nr = (int)(rows - r0 < GT_RPB ? rows - r0 : GT_RPB);
  const long long img = r0 / per_img;  // (per_img % GT_RPB == 0: one image per block)
  for (int j = threadIdx.x; j < nr * q; j += 256) {
    const int rr = j / q;
    const int ch = (j - rr * q) * 4;
    const long long r = r0 + rr;
    f32x4 a = *(const f32x4*)(c2 + r * 2 * f + ch), b = *(const f32x4*)(c2 + r * 2 * f + f + ch);
    if (hp) {
      a += *(const f32x4*)(hp + img * 2 * f + ch);
      b += *(const f32x4*)(hp + img * 2 * f + f + ch);
    }
    const f32x4 o = *(const f32x4*)(x + r * ldx + ch) + a * sigm4(b);
    *(f32x4*)(out + r * ldo + ch) = o;
    am = fmaxf(am, fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fmaxf(fabsf(o[2]), fabsf(o[3]))));
  }
  if (amax) block_absmax_put(am, amax);
}
__global__ __launch_bounds__(256) void gate4_bwd_kernel(const float* __restrict__ c2, const float* __restrict__ hp,
                                                        const float* __restrict__ dout, int lddo, long long rows,
                                                        int per_img, int f, void* __restrict__ dc2v, int out_bf16,
                                                        float* __restrict__ part) {
  __shared__ f32x4 red[256][2];
  const int q = f >> 2;
  const int RL = 256 / q;  // row lanes (q <= 256)
  const int tid = threadIdx.x, qi = tid % q, rl = tid / q;
  const long long r0 = (long long)blockIdx.x * GT_RPB;
  const int nr = (int)(rows - r0 < GT_RPB ? rows - r0 : GT_RPB);
  const long long img = r0 / per_img;
  const int ch = qi * 4;
  f32x4 sa = {0.f, 0.f, 0.f, 0.f}, sb = {0.f, 0.f, 0.f, 0.f};
  if (rl < RL) {
    f32x4 ha = {0.f, 0.f, 0.f, 0.f}, hb = {0.f, 0.f, 0.f, 0.f};
    if (hp) {
      ha = *(const f32x4*)(hp + img * 2 * f + ch);
      hb = *(const f32x4*)(hp + img * 2 * f + f + ch);
    }
    for (int rr = rl; rr < nr; rr += RL) {
      const long long r = r0 + rr;
      const f32x4 a = *(const f32x4*)(c2 + r * 2 * f + ch) + ha, b = *(const f32x4*)(c2 + r * 2 * f + f + ch) + hb;
      const f32x4 d = *(const f32x4*)(dout + r * lddo + ch), s = sigm4(b);
      const f32x4 da = d * s, db = d * a * s * (1.f - s);
      if (out_bf16) {  // read only as a bf16 MFMA operand (the conv's input gradient and weight gradient)
        __bf16* o = (__bf16*)dc2v + r * 2 * f + ch;
        *(pc_bf16x4*)o = __builtin_convertvector(da, pc_bf16x4);
        *(pc_bf16x4*)(o + f) = __builtin_convertvector(db, pc_bf16x4);
      } else {
        float* o = (float*)dc2v + r * 2 * f + ch;
        *(f32x4*)o = da;
        *(f32x4*)(o + f) = db;
      }
      sa += da;
      sb += db;
    }
  }
  if (!part) return;
  red[tid][0] = sa;
  red[tid][1] = sb;
  __syncthreads();
  if (tid < q) {
    f32x4 ta = red[tid][0], tb = red[tid][1];
    for (int l = 1; l < RL; ++l) {
      ta += red[l * q + tid][0];
      tb += red[l * q + tid][1];
    }
    *(f32x4*)(part + (long long)blockIdx.x * 2 * f + ch) = ta;
    *(f32x4*)(part + (long long)blockIdx.x * 2 * f + f + ch) = tb;
  }
}
// out[img][c] = sum of the image's bpi blocks' partials, in block order
__global__ void gate_imgsum_kernel(const float* __restrict__ part, int bpi, int nimg, int c, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nimg * c) return;
  const int img = i / c, col = i - img * c;
  float v = 0.f;
  for (int b = 0; b < bpi; ++b) v += part[((long long)img * bpi + b) * c + col];
  out[i] = v;
}
__global__ void copy4_kernel(const float* __restrict__ x, int ldx, long long rows, int c, float* __restrict__ y, int ldy,
                             int accumulate) {
  const int q = c >> 2;
  const long long r0 = (long long)blockIdx.x * GT_RPB;
  const int nr = (int)(rows - r0 < GT_RPB ? rows - r0 : GT_RPB);
  for (int j = threadIdx.x; j < nr * q; j += 256) {
    const int rr = j / q;
    const int ch = (j - rr * q) * 4;
    const long long r = r0 + rr;
    f32x4 v = *(const f32x4*)(x + r * ldx + ch);
    if (accumulate) v += *(const f32x4*)(y + r * ldy + ch);
    *(f32x4*)(y + r * ldy + ch) = v;
  }
}

// long-K form: one wave per output, lanes over K, a fixed butterfly sum (deterministic)
__global__ __launch_bounds__(256) void gemm_small_wave_kernel(const float* __restrict__ A, int lda, int ta,
                                                              const float* __restrict__ B, int ldb, int tb,
                                                              float* __restrict__ C, int ldc, int m, int n, int k,
                                                              float beta) {
  const int lane = threadIdx.x & 63;
  const long long o = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (o >= (long long)m * n) return;
  const int mi = (int)(o / n), ni = (int)(o - (long long)mi * n);
  float s = 0.f;
  for (int kk = lane; kk < k; kk += 64) {
    const float a = ta ? A[(long long)kk * lda + mi] : A[(long long)mi * lda + kk];
    const float b = tb ? B[(long long)ni * ldb + kk] : B[(long long)kk * ldb + ni];
    s = fmaf(a, b, s);
  }
  s = wave_sum(s);
  if (lane == 0) {
    float* p = C + (long long)mi * ldc + ni;
    *p = beta != 0.f ? beta * *p + s : s;
  }
}

__global__ void gemm_small_kernel(const float* __restrict__ A, int lda, int ta, const float* __restrict__ B, int ldb,
                                  int tb, float* __restrict__ C, int ldc, int m, int n, int k, float beta) {
  const long long stride = (long long)gridDim.x * blockDim.x, total = (long long)m * n;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int mi = (int)(i / n), ni = (int)(i - (long long)mi * n);
    float s = 0.f;
    for (int kk = 0; kk < k; ++kk) {
      const float a = ta ? A[(long long)kk * lda + mi] : A[(long long)mi * lda + kk];
      const float b = tb ? B[(long long)ni * ldb + kk] : B[(long long)kk * ldb + ni];
      s = fmaf(a, b, s);
    }
    float* p = C + (long long)mi * ldc + ni;
    *p = beta != 0.f ? beta * *p + s : s;
  }
}

// per-image channel sums: block (64-column group, image, pixel split) -> part[split][img][c],
// then a fixed-order sum over the splits
#define IMGSUM_PIX 256
__global__ __launch_bounds__(256) void imgsum_kernel(const float* __restrict__ x, int ldx, int per_img, int c,
                                                     float* __restrict__ part) {
  __shared__ float red[4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63), q = threadIdx.x >> 6, img = blockIdx.y;
  const int p0 = blockIdx.z * IMGSUM_PIX;
  const int p1 = p0 + IMGSUM_PIX < per_img ? p0 + IMGSUM_PIX : per_img;
  float s = 0.f;
  if (col < c)
    for (int p = p0 + q; p < p1; p += 4) s += x[((long long)img * per_img + p) * ldx + col];
  red[q][threadIdx.x & 63] = s;
  __syncthreads();
  if (q == 0 && col < c)
    part[((long long)blockIdx.z * gridDim.y + img) * c + col] =
        red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}

__global__ void copy_kernel(const float* __restrict__ x, int ldx, long long rows, int c, float* __restrict__ y,
                            int ldy, int accumulate) {
  const long long stride = (long long)gridDim.x * blockDim.x, total = rows * c;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const long long r = i / c;
    const int j = (int)(i - r * c);
    float v = x[r * ldx + j];
    if (accumulate) v += y[r * ldy + j];
    y[r * ldy + j] = v;
  }
}

__global__ void pad_ones_kernel(const float* __restrict__ x, long long rows, int c, float* __restrict__ y, int ldy) {
  const long long stride = (long long)gridDim.x * blockDim.x, total = rows * ldy;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const long long r = i / ldy;
    const int j = (int)(i - r * ldy);
    y[i] = j < c ? x[r * c + j] : (j == c ? 1.f : 0.f);
  }
}

// ---------------------------------------------------------------------------------------------
// discretized logistic mixture (nn.py:46-87): log p(x) per pixel and d(-log p)/dl in one pass
// ---------------------------------------------------------------------------------------------
#define PC_MAXMIX 16
__device__ __forceinline__ float softplus_f(float x) { return x > 0.f ? x + log1pf(expf(-x)) : log1pf(expf(x)); }

__global__ void mixlogistic_kernel(const float* __restrict__ x, const float* __restrict__ l, long long pixels, int M,
                                   float* __restrict__ logp, float* __restrict__ dl, float coef) {
  const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= pixels) return;
  const float* lp = l + p * 10 * M;
  const float x0 = x[p * 3], x1 = x[p * 3 + 1], x2 = x[p * 3 + 2];
  const float xs[3] = {x0, x1, x2};
  float lpj[PC_MAXMIX];
  // log_softmax of the logits
  float lmax = -INFINITY;
  for (int j = 0; j < M; ++j) lmax = fmaxf(lmax, lp[j]);
  float lsum = 0.f;
  for (int j = 0; j < M; ++j) lsum += expf(lp[j] - lmax);
  const float llse = lmax + logf(lsum);
  for (int j = 0; j < M; ++j) {
    float acc = lp[j] - llse;
    for (int c = 0; c < 3; ++c) {
      const float* pc = lp + M + c * 3 * M;
      float mean = pc[j];
      if (c == 1) mean += tanhf(lp[M + 0 * 3 * M + 2 * M + j]) * x0;
      if (c == 2) mean += tanhf(lp[M + 1 * 3 * M + 2 * M + j]) * x0 + tanhf(lp[M + 2 * 3 * M + 2 * M + j]) * x1;
      const float ls = fmaxf(pc[M + j], -7.f);
      const float cx = xs[c] - mean, inv = expf(-ls);
      const float plus_in = inv * (cx + 1.f / 255.f), min_in = inv * (cx - 1.f / 255.f);
      float v;
      if (xs[c] < -0.999f) {
        v = plus_in - softplus_f(plus_in);
      } else if (xs[c] > 0.999f) {
        v = -softplus_f(min_in);
      } else {
        const float cd = sigm(plus_in) - sigm(min_in);
        if (cd > 1e-5f) {
          v = logf(fmaxf(cd, 1e-12f));
        } else {
          const float mid = inv * cx;
          v = mid - ls - 2.f * softplus_f(mid) - logf(127.5f);
        }
      }
      acc += v;
    }
    lpj[j] = acc;
  }
  float mx = -INFINITY;
  for (int j = 0; j < M; ++j) mx = fmaxf(mx, lpj[j]);
  float se = 0.f;
  for (int j = 0; j < M; ++j) se += expf(lpj[j] - mx);
  const float out = mx + logf(se);
  logp[p] = out;
  if (!dl) return;
  // d(-out)/d lp_j = -w_j (w = softmax(lpj)); d/d logit_k = -(w_k - softmax(logit)_k)
  float* dp = dl + p * 10 * M;
  for (int j = 0; j < M; ++j) {
    const float w = expf(lpj[j] - out);
    dp[j] = -coef * (w - expf(lp[j] - llse));
    const float gw = -coef * w;  // d loss / d lp_cj for every c
    float dmean[3], dls[3];
    const float tc0 = tanhf(lp[M + 0 * 3 * M + 2 * M + j]), tc1 = tanhf(lp[M + 1 * 3 * M + 2 * M + j]),
                tc2 = tanhf(lp[M + 2 * 3 * M + 2 * M + j]);
    for (int c = 0; c < 3; ++c) {
      const float* pc = lp + M + c * 3 * M;
      float mean = pc[j];
      if (c == 1) mean += tc0 * x0;
      if (c == 2) mean += tc1 * x0 + tc2 * x1;
      const float lsr = pc[M + j];
      const float ls = fmaxf(lsr, -7.f);
      const float cx = xs[c] - mean, inv = expf(-ls);
      const float plus_in = inv * (cx + 1.f / 255.f), min_in = inv * (cx - 1.f / 255.f);
      float d_plus = 0.f, d_min = 0.f, d_mid = 0.f, d_ls_direct = 0.f;
      if (xs[c] < -0.999f) {
        d_plus = 1.f - sigm(plus_in);
      } else if (xs[c] > 0.999f) {
        d_min = -sigm(min_in);
      } else {
        const float sp = sigm(plus_in), sm = sigm(min_in), cd = sp - sm;
        if (cd > 1e-5f) {
          d_plus = sp * (1.f - sp) / cd;
          d_min = -sm * (1.f - sm) / cd;
        } else {
          d_mid = 1.f - 2.f * sigm(inv * cx);
          d_ls_direct = -1.f;
        }
      }
      // plus_in = inv (cx + 1/255): d/dcx = inv, d/dls = -plus_in (likewise min_in, mid)
      const float mid = inv * cx;
      const float dcx = (d_plus + d_min + d_mid) * inv;
      const float dlsv = -(d_plus * plus_in + d_min * min_in + d_mid * mid) + d_ls_direct;
      dmean[c] = -dcx * gw;
      dls[c] = (lsr >= -7.f) ? dlsv * gw : 0.f;  // tf.maximum routes the gradient to x when x >= y
    }
    for (int c = 0; c < 3; ++c) {
      dp[M + c * 3 * M + j] = dmean[c];
      dp[M + c * 3 * M + M + j] = dls[c];
    }
    // coeffs: m1 += tc0 x0, m2 += tc1 x0 + tc2 x1; d tanh = 1 - t^2
    dp[M + 0 * 3 * M + 2 * M + j] = dmean[1] * x0 * (1.f - tc0 * tc0);
    dp[M + 1 * 3 * M + 2 * M + j] = dmean[2] * x0 * (1.f - tc1 * tc1);
    dp[M + 2 * 3 * M + 2 * M + j] = dmean[2] * x1 * (1.f - tc2 * tc2);
  }
}

__global__ __launch_bounds__(256) void sum_kernel(const float* __restrict__ x, long long n, float* out, double* out64) {
  __shared__ double red[256];
  double s = 0.0;
  for (long long i = threadIdx.x; i < n; i += 256) s += x[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (out) out[0] = (float)red[0];
    if (out64) out64[0] = red[0];
  }
}

__global__ void sample_kernel(const float* __restrict__ l, const float* __restrict__ u_mix,
                              const float* __restrict__ u_log, int nimg, int per_img, int M, float* __restrict__ x,
                              int q0, int q1, int pix_stride) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const int nq = q1 - q0;
  if (i >= (long long)nimg * nq) return;
  const long long p = (i / nq) * per_img + q0 + (int)(i % nq);
  const float* lp = l + p * 10 * M;
  int sel = 0;
  float best = -INFINITY;
  for (int j = 0; j < M; ++j) {
    const float v = lp[j] - logf(-logf(u_mix[p * M + j]));
    if (v > best) {  // tf.argmax: first maximum
      best = v;
      sel = j;
    }
  }
  float xs[3], co[3];
  for (int c = 0; c < 3; ++c) {
    const float* pc = lp + M + c * 3 * M;
    const float u = u_log[p * 3 + c];
    xs[c] = pc[sel] + expf(fmaxf(pc[M + sel], -7.f)) * (logf(u) - logf(1.f - u));
    co[c] = tanhf(pc[2 * M + sel]);
  }
  const float x0 = fminf(fmaxf(xs[0], -1.f), 1.f);
  const float x1 = fminf(fmaxf(xs[1] + co[0] * x0, -1.f), 1.f);
  const float x2 = fminf(fmaxf(xs[2] + co[1] * x0 + co[2] * x1, -1.f), 1.f);
  float* o = x + p * pix_stride;
  o[0] = x0;
  o[1] = x1;
  o[2] = x2;
}

// d sample / d l (the reparameterised logistic draw of sample_kernel, nn.py:89-109): the selected
// component's mean, log-scale (unless clamped at -7: tf.maximum routes the gradient to the
// argument where it is >= -7) and tanh coefficients; the clip to [-1, 1] passes the gradient where
// its argument lies inside (tf.minimum / tf.maximum tie rules, both bounds inclusive).  The mixture
// indicator is piecewise constant: no gradient to the logits.  dl [pixels][10 M] is overwritten.
__global__ void sample_bwd_kernel(const float* __restrict__ l, const float* __restrict__ u_mix,
                                  const float* __restrict__ u_log, long long npix, int M,
                                  const float* __restrict__ dx, int dx_stride, float* __restrict__ dl) {
  const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npix) return;
  const float* lp = l + p * 10 * M;
  float* dp = dl + p * 10 * M;
  for (int j = 0; j < 10 * M; ++j) dp[j] = 0.f;
  int sel = 0;
  float best = -INFINITY;
  for (int j = 0; j < M; ++j) {
    const float v = lp[j] - logf(-logf(u_mix[p * M + j]));
    if (v > best) {
      best = v;
      sel = j;
    }
  }
  float xs[3], co[3], es[3], lg[3], lsr[3];
  for (int c = 0; c < 3; ++c) {
    const float* pc = lp + M + c * 3 * M;
    const float u = u_log[p * 3 + c];
    lsr[c] = pc[M + sel];
    es[c] = expf(fmaxf(lsr[c], -7.f));
    lg[c] = logf(u) - logf(1.f - u);
    xs[c] = pc[sel] + es[c] * lg[c];
    co[c] = tanhf(pc[2 * M + sel]);
  }
  const float v0 = xs[0];
  const float x0 = fminf(fmaxf(v0, -1.f), 1.f);
  const float v1 = xs[1] + co[0] * x0;
  const float x1 = fminf(fmaxf(v1, -1.f), 1.f);
  const float v2 = xs[2] + co[1] * x0 + co[2] * x1;
  const float* g = dx + p * dx_stride;
  auto in = [](float v) { return (v >= -1.f && v <= 1.f) ? 1.f : 0.f; };
  const float g2 = g[2] * in(v2);
  float gx1 = g[1] + g2 * co[2];
  const float g1 = gx1 * in(v1);
  float gx0 = g[0] + g2 * co[1] + g1 * co[0];
  const float g0 = gx0 * in(v0);
  const float gv[3] = {g0, g1, g2};
  const float dco[3] = {g1 * x0, g2 * x0, g2 * x1};
  for (int c = 0; c < 3; ++c) {
    float* dc = dp + M + c * 3 * M;
    dc[sel] = gv[c];                                                   // d mean
    dc[M + sel] = lsr[c] >= -7.f ? gv[c] * es[c] * lg[c] : 0.f;         // d log_scale
    dc[2 * M + sel] = dco[c] * (1.f - co[c] * co[c]);                   // d coeff (tanh')
  }
}

// highway backward (pixelvae.py:135-137): ds = r dout; dprev (+)= (1 - r) dout;
// dz[img] = sum_i dout (s - prev) * (hi - lo) sigmoid'(z + zb).  One block per image (fixed order).
__global__ __launch_bounds__(256) void highway_bwd_kernel(const float* __restrict__ s, const float* __restrict__ prev,
                                                          const float* __restrict__ z, const float* __restrict__ zb,
                                                          long long per_img, float lo, float hi,
                                                          const float* __restrict__ dout, float* __restrict__ ds,
                                                          float* __restrict__ dprev, int prev_acc,
                                                          float* __restrict__ dz) {
  __shared__ float red[256];
  const int b = blockIdx.x;
  const float zz = z[b] + (zb ? zb[0] : 0.f);
  const float sg = sigm(zz);
  const float r = lo + (hi - lo) * sg;
  const long long o = (long long)b * per_img;
  float acc = 0.f;
  for (long long i = threadIdx.x; i < per_img; i += 256) {
    const float d = dout[o + i];
    if (ds) ds[o + i] = r * d;
    if (dprev) dprev[o + i] = (prev_acc ? dprev[o + i] : 0.f) + (1.f - r) * d;
    acc += d * (s[o + i] - prev[o + i]);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) dz[b] = red[0] * (hi - lo) * sg * (1.f - sg);
}

// dropout with a given mask (nn.py:273-274, tf.nn.dropout): y = x * mask, mask = keep / keep_prob or 0;
// the backward is the same product on the gradient
__global__ void dropout_kernel(const float* __restrict__ x, long long rows, int c, int ldx, const float* __restrict__ mask,
                               float* __restrict__ y, int ldy) {
  const long long n = rows * c;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / c;
    const int k = (int)(i - r * c);
    y[r * ldy + k] = x[r * ldx + k] * mask[i];
  }
}

// per-image mean squared error and its gradient (the chain's reconstruction term on the head's
// output, compute_and_accumulate_loss :1146): rec[b] = mean_i (a - t)^2, da = coef * 2 (a - t) / per_img
__global__ __launch_bounds__(256) void sqerr_kernel(const float* __restrict__ a, const float* __restrict__ t,
                                                    long long per_img, float coef, float* __restrict__ rec,
                                                    float* __restrict__ da) {
  __shared__ float red[256];
  const long long o = (long long)blockIdx.x * per_img;
  float acc = 0.f;
  for (long long i = threadIdx.x; i < per_img; i += 256) {
    const float d = a[o + i] - t[o + i];
    acc += d * d;
    if (da) da[o + i] = coef * 2.f * d / (float)per_img;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0 && rec) rec[blockIdx.x] = red[0] / (float)per_img;
}

__global__ void highway_kernel(const float* __restrict__ s, const float* __restrict__ prev,
                               const float* __restrict__ z, const float* __restrict__ zb, long long per_img,
                               long long total, float lo, float hi, float* __restrict__ out) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const float b = zb ? zb[0] : 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const float r = lo + (hi - lo) * sigm(z[i / per_img] + b);
    out[i] = r * s[i] + (1.f - r) * prev[i];
  }
}
__global__ void ratio_kernel(const float* __restrict__ z, const float* __restrict__ zb, int nimg, float lo, float hi,
                             float* __restrict__ ratio) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nimg) ratio[i] = lo + (hi - lo) * sigm(z[i] + (zb ? zb[0] : 0.f));
}

// column moments in fp64, two passes (mean, then the centred second moment) over row blocks of
// rpb rows: block (column group of 64, row block) -> part[rb][c]; the second pass and the
// finaliser re-derive each column's mean from part in the same fixed order (deterministic)
#define WNI_MAXRB 512
__device__ __forceinline__ double wni_mean(const double* part, int nrb, int c, int col, long long rows) {
  double s = 0.0;
  for (int k = 0; k < nrb; ++k) s += part[(long long)k * c + col];
  return s / (double)rows;
}
__global__ __launch_bounds__(256) void wn_mom_kernel(const float* __restrict__ y, long long rows, int c, int ldy,
                                                     long long rpb, int nrb, int pass, double* part) {
  __shared__ double red[4][64];
  __shared__ double mean_s[64];
  const int t = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + t;
  const long long r0 = (long long)blockIdx.y * rpb;
  const long long r1 = r0 + rpb < rows ? r0 + rpb : rows;
  if (pass == 1 && q == 0) mean_s[t] = col < c ? wni_mean(part, nrb, c, col, rows) : 0.0;
  __syncthreads();
  const double mean = pass == 1 ? mean_s[t] : 0.0;
  double s = 0.0;
  if (col < c)
    for (long long r = r0 + q; r < r1; r += 4) {
      const double v = (double)y[r * ldy + col] - mean;
      s += pass == 1 ? v * v : v;
    }
  red[q][t] = s;
  __syncthreads();
  if (q == 0 && col < c)
    part[((long long)pass * nrb + blockIdx.y) * c + col] = red[0][t] + red[1][t] + red[2][t] + red[3][t];
}
__global__ void wn_init_fin_kernel(const double* part, int nrb, long long rows, int c, float init_scale, float* g,
                                   float* b) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= c) return;
  const double mean = wni_mean(part, nrb, c, col, rows);
  const double var = wni_mean(part + (long long)nrb * c, nrb, c, col, rows);
  const double si = init_scale / sqrt(var + 1e-10);
  g[col] = (float)(g[col] * si);
  b[col] = (float)(b[col] - mean * si);
}

__global__ void ema_kernel(float* avg, const float* p, long long n, float decay) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    avg[i] = decay * avg[i] + (1.f - decay) * p[i];  // tf.train.ExponentialMovingAverage
}

PcGeom make_geom(int n, int hi, int wi, int cin, int ldx, int ho, int wo, int cout, int kh, int kw, int s, int pt,
                 int pl, int mode) {
  PcGeom g;
  g.n = n; g.hi = hi; g.wi = wi; g.cin = cin; g.ldx = ldx;
  g.ho = ho; g.wo = wo; g.cout = cout;
  g.kh = kh; g.kw = kw; g.s = s; g.pt = pt; g.pl = pl; g.mode = mode;
  return g;
}
bool geom_ok(const PcGeom& g) {
  return g.n > 0 && g.hi > 0 && g.wi > 0 && g.cin > 0 && g.ho > 0 && g.wo > 0 && g.cout > 0 && g.kh > 0 &&
         g.kw > 0 && (g.s == 1 || g.s == 2) && (g.mode == 0 || g.mode == 1) && g.ldx >= g.cin && g.ldx % 4 == 0 &&
         g.cin % 4 == 0;
}

}  // namespace

// =============================================================================================
// C ABI
// =============================================================================================
extern "C" {

int svae_pcnn_wnorm(const float* V, const float* g, int taps, int cin, int cout, float* norm, void* wk_f, int kf,
                    void* wk_d, int kd, void* stream) {
  return svae_pcnn_wnorm_planes(V, g, taps, cin, cout, norm, wk_f, kf, wk_d, kd, 1, nullptr, stream);
}

int svae_pcnn_wnorm_planes(const float* V, const float* g, int taps, int cin, int cout, float* norm, void* wk_f,
                           int kf, void* wk_d, int kd, int planes, float* h16_scale, void* stream) {
  if (!V || !g || !norm || taps < 1 || cin < 1 || cout < 1 || planes < 1 || planes > PC_MAXPLANES ||
      (h16_scale && planes != 2))
    return bad("pcnn_wnorm: bad arguments");
  if ((wk_f && (kf < cin || kf % 16)) || (wk_d && (kd < cout || kd % 16))) return bad("pcnn_wnorm: bad padding");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(wn_norm_kernel, dim3(cout), dim3(256), 0, s, V, taps * cin, cout, norm);
  if (h16_scale) {  // max |W| for the fp16 planes' scale
    if (hipMemsetAsync(h16_scale + 1, 0, sizeof(float), s) != hipSuccess) return hipchk();
    hipLaunchKernelGGL(wn_absmax_kernel, dim3(cout), dim3(256), 0, s, V, g, norm, taps * cin, cout,
                       (unsigned*)(h16_scale + 1));
  }
  const long long n = (wk_f ? (long long)taps * cout * kf : 0) + (wk_d ? (long long)taps * cin * kd : 0);
  if (n) hipLaunchKernelGGL(wn_apply_kernel, dim3(blocks_for(n)), dim3(256), 0, s, V, g, norm, taps, cin, cout,
                            (__bf16*)wk_f, kf, (__bf16*)wk_d, kd, planes, h16_scale);
  return hipchk();
}

int svae_pcnn_wnorm_bwd(const float* V, const float* g, const float* norm, const float* dW, int taps, int cin,
                        int cout, float* dV, float* dg, void* stream) {
  if (!V || !g || !norm || !dW || !dV || !dg || taps < 1 || cin < 1 || cout < 1) return bad("pcnn_wnorm_bwd: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(wn_dg_kernel, dim3(cout), dim3(256), 0, s, V, dW, norm, taps * cin, cout, dg);
  const long long n = (long long)taps * cin * cout;
  hipLaunchKernelGGL(wn_dv_kernel, dim3(blocks_for(n)), dim3(256), 0, s, V, g, norm, dW, dg, n, cout, dV);
  return hipchk();
}

static int pcnn_conv_impl(const void* x, int n, int hi, int wi, int cin, int ldx, int x_bf16, const void* wk, int kpad,
                          const float* bias, float* y, int ho, int wo, int cout, int ldy, int kh, int kw, int s, int pt,
                          int pl, int mode, int accumulate, int zero_edge, const NlbArgs& nlb, void* stream,
                          const PcScale& sc = PcScale{nullptr, nullptr});

int svae_pcnn_conv(const void* x, int n, int hi, int wi, int cin, int ldx, int x_bf16, const void* wk, int kpad,
                   const float* bias, float* y, int ho, int wo, int cout, int ldy, int kh, int kw, int s, int pt,
                   int pl, int mode, int accumulate, int zero_edge, void* stream) {
  NlbArgs nlb{};
  return pcnn_conv_impl(x, n, hi, wi, cin, ldx, x_bf16, wk, kpad, bias, y, ho, wo, cout, ldy, kh, kw, s, pt, pl, mode,
                        accumulate, zero_edge, nlb, stream);
}

int svae_pcnn_conv_act_bwd(const float* dy, int n, int hi, int wi, int cin, int lddy, const void* wk, int kpad,
                           float* dsrc, int ho, int wo, int cout, int ldd, int kh, int kw, int s, int pt, int pl, int mode,
                           int accumulate, const float* src, int lds, int kind, const float* mask, float keep,
                           uint64_t seed, void* stream) {
  if (!src || lds < cout || kind < 0 || kind > 1 || (!mask && !(keep > 0.f))) return bad("pcnn_conv_act_bwd: bad arguments");
  NlbArgs nlb{src, lds, kind, mask, keep, (unsigned long long)seed, 1};
  return pcnn_conv_impl(dy, n, hi, wi, cin, lddy, 0, wk, kpad, nullptr, dsrc, ho, wo, cout, ldd, kh, kw, s, pt, pl, mode,
                        accumulate, 0, nlb, stream);
}

static int pcnn_conv_impl(const void* x, int n, int hi, int wi, int cin, int ldx, int x_bf16, const void* wk, int kpad,
                          const float* bias, float* y, int ho, int wo, int cout, int ldy, int kh, int kw, int s, int pt,
                          int pl, int mode, int accumulate, int zero_edge, const NlbArgs& nlb, void* stream,
                          const PcScale& sc) {
  const PcGeom g = make_geom(n, hi, wi, cin, ldx, ho, wo, cout, kh, kw, s, pt, pl, mode);
  const bool H = sc.a != nullptr;  // fp16 planes (the split mode): 16-bit storage only
  if (H && (!x_bf16 || !sc.b || nlb.on)) return bad("pcnn_conv: fp16 planes need 16-bit x and both scales");
  if (!x || !wk || !y || !geom_ok(g) || ldy < cout || kpad < cin || kpad % 16 || zero_edge < 0 || zero_edge > 2)
    return bad("pcnn_conv: bad arguments");
  if (x_bf16 && (cin % 8 || ldx % 8 || kpad % 32)) return bad("pcnn_conv: bf16 input needs cin, ldx % 8 == 0");
  const long long rows = (long long)n * ho * wo;
  hipStream_t st = (hipStream_t)stream;
  const __bf16* w = (const __bf16*)wk;
  const unsigned gx = (unsigned)((rows + 127) / 128);
  static const bool old = svae_knob("SVAE_PC_CONV1", 0) == 1;
  static const int pc3 = svae_knob("SVAE_PC3", 1);  // 0 = stride-1 convs on pc_conv2 too; 1 / 2 = halo kernel, TM
  if (kpad % 32 == 0 && !old) {  // LDS-staged kernels, up to 160 output channels per block
    const int n32 = (cout + 31) / 32;
    int tiles = (n32 + 4) / 5;
    int NT = (n32 + tiles - 1) / tiles;
    Pc3 h;
    size_t lds = 0;
    if (pc3 >= 1 && pc3 <= 2 && pc3_plan(g, kpad, pc3, &h, &lds)) {  // stride 1: one halo window per chunk
      // widest column tile (32 x NT): 64 columns for the forward convs (bf16 input, mode 0), 160 for the
      // input gradients (tools/bench_pcconv.py, B = 128: mode 0 0-30 % faster at NT = 2 against NT = 5,
      // mode 1 up to 55 % slower; NT = 3 slower for both); SVAE_PC3_NT overrides
      static const int nt_env = svae_knob("SVAE_PC3_NT", 0);
      const int nt_max = nt_env > 0 ? nt_env : (x_bf16 && mode == 0 ? 2 : 5);
      if (nt_max < NT) {
        tiles = (n32 + nt_max - 1) / nt_max;
        NT = (n32 + tiles - 1) / tiles;
      }
#define PC3_NT(TMV, XBV, HV)                                                                                \
  switch (NT) {                                                                                             \
    case 1: pc3_launch<1, TMV, XBV, HV>(g, h, x, w, kpad, bias, y, ldy, accumulate, zero_edge, nlb, sc, st); break; \
    case 2: pc3_launch<2, TMV, XBV, HV>(g, h, x, w, kpad, bias, y, ldy, accumulate, zero_edge, nlb, sc, st); break; \
    case 3: pc3_launch<3, TMV, XBV, HV>(g, h, x, w, kpad, bias, y, ldy, accumulate, zero_edge, nlb, sc, st); break; \
    case 4: pc3_launch<4, TMV, XBV, HV>(g, h, x, w, kpad, bias, y, ldy, accumulate, zero_edge, nlb, sc, st); break; \
    default: pc3_launch<5, TMV, XBV, HV>(g, h, x, w, kpad, bias, y, ldy, accumulate, zero_edge, nlb, sc, st); break; \
  }
      if (H) { PC3_NT(1, true, true) }
      else if (x_bf16) { PC3_NT(1, true, false) }
      else if (pc3 == 2) { PC3_NT(2, false, false) }
      else { PC3_NT(1, false, false) }
#undef PC3_NT
      return hipchk();
    }
    const dim3 grid(gx, tiles);
#define PC2_NT(XBV, HV)                                                                                               \
  switch (NT) {                                                                                                      \
    case 1: hipLaunchKernelGGL((pc_conv2_kernel<1, XBV, HV>), grid, dim3(256), 0, st, g, x, w, kpad, bias, y, ldy, accumulate, zero_edge, nlb, sc); break; \
    case 2: hipLaunchKernelGGL((pc_conv2_kernel<2, XBV, HV>), grid, dim3(256), 0, st, g, x, w, kpad, bias, y, ldy, accumulate, zero_edge, nlb, sc); break; \
    case 3: hipLaunchKernelGGL((pc_conv2_kernel<3, XBV, HV>), grid, dim3(256), 0, st, g, x, w, kpad, bias, y, ldy, accumulate, zero_edge, nlb, sc); break; \
    case 4: hipLaunchKernelGGL((pc_conv2_kernel<4, XBV, HV>), grid, dim3(256), 0, st, g, x, w, kpad, bias, y, ldy, accumulate, zero_edge, nlb, sc); break; \
    default: hipLaunchKernelGGL((pc_conv2_kernel<5, XBV, HV>), grid, dim3(256), 0, st, g, x, w, kpad, bias, y, ldy, accumulate, zero_edge, nlb, sc); break; \
  }
    if (H) { PC2_NT(true, true) } else if (x_bf16) { PC2_NT(true, false) } else { PC2_NT(false, false) }
#undef PC2_NT
    return hipchk();
  }
  if (x_bf16 || nlb.on || H) return bad("pcnn_conv: bf16 input / activation epilogue on the register-direct kernel (SVAE_PC_CONV1)");
  // register-direct kernel: two 32-column subtiles per wave (wider tiles measured slower here)
  const float* xf = (const float*)x;
  if (cout > 32)
    hipLaunchKernelGGL(pc_conv_kernel<2>, dim3(gx, (cout + 63) / 64), dim3(256), 0, st, g, xf, w, kpad, bias, y, ldy,
                       accumulate, zero_edge);
  else
    hipLaunchKernelGGL(pc_conv_kernel<1>, dim3(gx, 1), dim3(256), 0, st, g, xf, w, kpad, bias, y, ldy, accumulate,
                       zero_edge);
  return hipchk();
}

// The weight gradient as a sum of nprod operand products sum_p gather(xs[p])^T ds[p] (one product: the
// plain bf16 gradient; the split mode's plane products, svae_pcnn_conv_wgrad_planes): every product's
// launch writes its own ns partial slabs and ONE fixed-order reduce adds all nprod * ns of them.
static int pcnn_wgrad_impl(const void* const* xs, const void* const* ds, int nprod, int n, int hi, int wi, int cin,
                           int ldx, int x_bf16, int ldd, int dy_bf16, int ho, int wo, int cout, int kh, int kw, int s,
                           int pt, int pl, int mode, float* dW, float* dbias, float* scratch, int64_t scratch_elems,
                           void* stream, const PcScale& sc = PcScale{nullptr, nullptr}, long long xpst = -1,
                           long long dpst = -1) {
  const bool H = sc.a != nullptr;  // fp16 planes: both operands 16-bit, the reduce applies the scales
  const bool HP = H && xpst >= 0;  // ... both planes of each in one launch (the three products fused)
  if (H && (!x_bf16 || !dy_bf16 || !sc.b || dbias)) return bad("pcnn_wgrad: fp16 planes need 16-bit x and dy");
  const PcGeom g = make_geom(n, hi, wi, cin, ldx, ho, wo, cout, kh, kw, s, pt, pl, mode);
  bool ok = nprod >= 1 && nprod <= PC_MAXPLANES * (PC_MAXPLANES + 1) / 2;
  for (int p = 0; ok && p < nprod; ++p) ok = xs[p] && ds[p];
  if (!ok || !dW || !scratch || !geom_ok(g) || ldd < cout || ldd % 4 || cout % 4)
    return bad("pcnn_wgrad: bad arguments");
  if (dy_bf16 && dbias) return bad("pcnn_wgrad: the bias gradient needs the fp32 dy (sum it upstream)");
  if (dbias && nprod > 1) return bad("pcnn_wgrad: the bias gradient of a plane product (sum it upstream)");
  const long long rows = (long long)n * ho * wo;
  const int taps = kh * kw;
  const long long wsz = (long long)taps * cin * cout;
  hipStream_t st = (hipStream_t)stream;
  static const int pw4 = svae_knob("SVAE_PW4", 1);  // 0: every weight gradient on the one-tap kernel
  {
    PcGeom g4 = g;
    if (kh == 1 && kw == 1 && pt == 0 && pl == 0 && s == 1 && rows % 256 == 0) {  // 1x1: 16-wide images
      g4.n = (int)(rows / 256);
      g4.hi = g4.wi = g4.ho = g4.wo = 16;
    }
    Pw4 h;
    static const bool allkw = svae_knob("SVAE_PW4_ALLKW", 1) != 0;  // fused planes: [2, 2] / 1x1 on the tap-row kernel too (387 -> 440 img/s)
    if (pw4 && pw4_plan(g4, rows, &h, HP && allkw)) {
      const long long tiles4 = (long long)((cin + 63) / 64) * ((cout + 63) / 64) * kh;
      static const int tgt4 = svae_knob("SVAE_PW4_TARGET", 1024);  // blocks of the tap-row kernel
      long long ns = (tgt4 + tiles4 - 1) / tiles4;
      if (ns > h.nchunk) ns = h.nchunk;
      if (ns > scratch_elems / (nprod * wsz + cout)) ns = scratch_elems / (nprod * wsz + cout);
      if (ns < 1) return bad("pcnn_wgrad: scratch too small");
      h.cps = (int)((h.nchunk + ns - 1) / ns);
      ns = (h.nchunk + h.cps - 1) / h.cps;
      float* bpart = dbias ? scratch + nprod * ns * wsz : nullptr;
      const dim3 grid((unsigned)((cin + 63) / 64), (unsigned)((cout + 63) / 64), (unsigned)(kh * ns));
      for (int p = 0; p < nprod; ++p) {
        const void* x = xs[p];
        const void* dy = ds[p];
        float* slab = scratch + p * ns * wsz;
#define PW4_L(XBV, DBV) hipLaunchKernelGGL((pc_wgrad4_kernel<XBV, DBV>), grid, dim3(256), 0, st, g4, h, x, dy, ldd, slab, bpart, 0LL, 0LL)
        if (HP) hipLaunchKernelGGL((pc_wgrad4_kernel<true, true, true, true>), grid, dim3(256), 0, st, g4, h, x, dy, ldd,
                                   slab, bpart, xpst, dpst);
        else if (H) hipLaunchKernelGGL((pc_wgrad4_kernel<true, true, true>), grid, dim3(256), 0, st, g4, h, x, dy, ldd,
                                       slab, bpart, 0LL, 0LL);
        else if (x_bf16) { if (dy_bf16) PW4_L(true, true); else PW4_L(true, false); }
        else { if (dy_bf16) PW4_L(false, true); else PW4_L(false, false); }
#undef PW4_L
      }
      split_reduce(scratch, (int)(nprod * ns), wsz, dW, sc, st);
      if (dbias)
        hipLaunchKernelGGL(split_reduce_kernel, dim3(blocks_for(cout)), dim3(256), 0, st, bpart, (int)ns,
                           (long long)cout, dbias, PcScale{nullptr, nullptr});
      return hipchk();
    }
  }
  const int tiles = ((cin + 63) / 64) * ((cout + 63) / 64);
  // splits: ~2048 blocks, >= 256 rows (8 chunks) per split, bounded by the scratch slabs
  static const int tgt1 = svae_knob("SVAE_PW_TARGET", 2048);  // blocks of the one-tap kernel
  long long ns = (tgt1 + (long long)tiles * taps - 1) / ((long long)tiles * taps);
  const long long max_rows = (rows + 255) / 256;
  if (ns > max_rows) ns = max_rows;
  if (ns > scratch_elems / (nprod * wsz + cout)) ns = scratch_elems / (nprod * wsz + cout);  // slabs + bias partials
  if (ns < 1) return bad("pcnn_wgrad: scratch too small");
  long long rps = (rows + ns - 1) / ns;
  rps = (rps + 63) / 64 * 64;
  ns = (rows + rps - 1) / rps;
  float* bpart = dbias ? scratch + nprod * ns * wsz : nullptr;
  for (int p = 0; p < nprod; ++p) {
    const void* x = xs[p];
    const void* dy = ds[p];
    float* slab = scratch + p * ns * wsz;
#define PW1_L(XBV, DBV) hipLaunchKernelGGL((pc_wgrad_kernel<XBV, DBV>), dim3(tiles, taps, (unsigned)ns), dim3(256), 0, st, g, x, dy, \
                                           ldd, rows, rps, slab, bpart, 0LL, 0LL)
    if (HP) hipLaunchKernelGGL((pc_wgrad_kernel<true, true, true, true>), dim3(tiles, taps, (unsigned)ns), dim3(256), 0, st,
                               g, x, dy, ldd, rows, rps, slab, bpart, xpst, dpst);
    else if (H) hipLaunchKernelGGL((pc_wgrad_kernel<true, true, true>), dim3(tiles, taps, (unsigned)ns), dim3(256), 0, st,
                                   g, x, dy, ldd, rows, rps, slab, bpart, 0LL, 0LL);
    else if (x_bf16) { if (dy_bf16) PW1_L(true, true); else PW1_L(true, false); }
    else { if (dy_bf16) PW1_L(false, true); else PW1_L(false, false); }
#undef PW1_L
  }
  split_reduce(scratch, (int)(nprod * ns), wsz, dW, sc, st);
  if (dbias)
    hipLaunchKernelGGL(split_reduce_kernel, dim3(blocks_for(cout)), dim3(256), 0, st, bpart, (int)ns, (long long)cout,
                       dbias, PcScale{nullptr, nullptr});
  return hipchk();
}

int svae_pcnn_conv_wgrad(const void* x, int n, int hi, int wi, int cin, int ldx, int x_bf16, const void* dy, int ldd,
                         int dy_bf16, int ho, int wo, int cout, int kh, int kw, int s, int pt, int pl, int mode, float* dW,
                         float* dbias, float* scratch, int64_t scratch_elems, void* stream) {
  return pcnn_wgrad_impl(&x, &dy, 1, n, hi, wi, cin, ldx, x_bf16, ldd, dy_bf16, ho, wo, cout, kh, kw, s, pt, pl, mode,
                         dW, dbias, scratch, scratch_elems, stream);
}

// the split mode's products (i, j), i + j < planes, largest first: (0,0) (0,1) (1,0) (0,2) (1,1) (2,0)
static int pc_products(int planes, int* pi, int* pj) {
  int k = 0;
  for (int d = 0; d < planes; ++d)
    for (int i = 0; i <= d; ++i) {
      pi[k] = i;
      pj[k] = d - i;
      ++k;
    }
  return k;
}

int svae_pcnn_conv_wgrad_planes(const void* x, int n, int hi, int wi, int cin, int ldx, int x_bf16, int64_t x_pstride,
                                const void* dy, int ldd, int dy_bf16, int64_t dy_pstride, int planes,
                                const float* x_scale, const float* dy_scale, int ho, int wo, int cout, int kh, int kw,
                                int s, int pt, int pl, int mode, float* dW, float* scratch, int64_t scratch_elems,
                                void* stream) {
  if (!x || !dy || planes < 1 || planes > PC_MAXPLANES || x_pstride < 0 || dy_pstride < 0 ||
      (!x_scale != !dy_scale) || (x_scale && planes != 2))
    return bad("pcnn_wgrad_planes: bad arguments");
  if (x_scale && x_bf16 && dy_bf16 && svae_knob("SVAE_PC_HP", 1) != 0)  // the fp16 planes: one launch per slab set
    return pcnn_wgrad_impl(&x, &dy, 1, n, hi, wi, cin, ldx, x_bf16, ldd, dy_bf16, ho, wo, cout, kh, kw, s, pt, pl, mode,
                           dW, nullptr, scratch, scratch_elems, stream, PcScale{x_scale, dy_scale}, x_pstride, dy_pstride);
  int pi[PC_MAXPLANES * PC_MAXPLANES], pj[PC_MAXPLANES * PC_MAXPLANES];
  const int np = pc_products(planes, pi, pj);
  const void* xs[PC_MAXPLANES * PC_MAXPLANES];
  const void* ds[PC_MAXPLANES * PC_MAXPLANES];
  for (int p = 0; p < np; ++p) {  // (the X plane against the D plane: products (i, j) pair x_i with dy_j)
    xs[p] = (const char*)x + (x_bf16 ? 2 : 4) * x_pstride * pi[p];
    ds[p] = (const char*)dy + (dy_bf16 ? 2 : 4) * dy_pstride * pj[p];
  }
  return pcnn_wgrad_impl(xs, ds, np, n, hi, wi, cin, ldx, x_bf16, ldd, dy_bf16, ho, wo, cout, kh, kw, s, pt, pl, mode,
                         dW, nullptr, scratch, scratch_elems, stream, PcScale{x_scale, dy_scale});
}

// The fp16-plane conv in ONE launch of the halo kernel with both planes staged (pc_conv3 HP): 1 if the launch is
// not eligible (stride 2, a window or stage beyond the LDS budget) -- the caller then runs the three products
// amax != NULL: max |y| into *amax where the row-staged kernel runs (*done set); the caller takes a pass otherwise
static int pcnn_conv_hp(const void* x, int n, int hi, int wi, int cin, int ldx, long long xpst, const void* wk, int kpad,
                        long long wpst, const PcScale& sc, const float* bias, float* y, int ho, int wo, int cout, int ldy,
                        int kh, int kw, int s, int pt, int pl, int mode, int accumulate, int zero_edge, void* stream,
                        unsigned* amax = nullptr, bool* done = nullptr) {
  const PcGeom g = make_geom(n, hi, wi, cin, ldx, ho, wo, cout, kh, kw, s, pt, pl, mode);
  if (!geom_ok(g) || cin % 8 || ldx % 8 || kpad % 32 || ldy < cout) return 1;
  if (svae_knob("SVAE_PC_HP", 1) == 0) return 1;
  Pc3 h;
  size_t lds0 = 0;
  if (!pc3_plan(g, kpad, 1, &h, &lds0)) return 1;
  const int n32 = (cout + 31) / 32;
  const __bf16* w = (const __bf16*)wk;
  hipStream_t st = (hipStream_t)stream;
  if (svae_knob("SVAE_PC_RS", 1) != 0) {  // row-staged: up to 160 columns per block, one window per chunk
    const int rtiles = (n32 + 4) / 5;
    const int RNT = (n32 + rtiles - 1) / rtiles;
    // (a grid under one block per CU keeps the 64-column tiles: 16 x 16 x 160 at B = 128 has 128 row blocks,
    //  60 us on pc_conv3 HP's 384 blocks against 65 us on 128; tools/bench_pcconv_hp.py)
    const long long rblocks = (long long)g.n * g.ho * g.wo / 256 * rtiles;
    if (rblocks >= 256 && pc3r_ok(g, h, RNT)) {
      const __bf16* xh = (const __bf16*)x;
      switch (RNT) {
        case 1: pc3r_launch<1>(g, h, xh, w, kpad, bias, y, ldy, accumulate, zero_edge, sc, st, xpst, wpst, amax); break;
        case 2: pc3r_launch<2>(g, h, xh, w, kpad, bias, y, ldy, accumulate, zero_edge, sc, st, xpst, wpst, amax); break;
        case 3: pc3r_launch<3>(g, h, xh, w, kpad, bias, y, ldy, accumulate, zero_edge, sc, st, xpst, wpst, amax); break;
        case 4: pc3r_launch<4>(g, h, xh, w, kpad, bias, y, ldy, accumulate, zero_edge, sc, st, xpst, wpst, amax); break;
        default: pc3r_launch<5>(g, h, xh, w, kpad, bias, y, ldy, accumulate, zero_edge, sc, st, xpst, wpst, amax); break;
      }
      if (done) *done = true;
      return hipchk();
    }
  }
  int tiles = (n32 + 1) / 2;  // at most 64 columns per block: two planes of window and weights in LDS
  const int NT = (n32 + tiles - 1) / tiles;
  const size_t lds = (size_t)(h.npix + kh * kw * 32 * NT) * PC2_P * 2 * 2;
  if (lds > 160 * 1024) return 1;
  NlbArgs nlb{};
  if (NT == 1) pc3_launch<1, 1, true, true, true>(g, h, x, w, kpad, bias, y, ldy, accumulate, zero_edge, nlb, sc, st, xpst, wpst);
  else pc3_launch<2, 1, true, true, true>(g, h, x, w, kpad, bias, y, ldy, accumulate, zero_edge, nlb, sc, st, xpst, wpst);
  return hipchk();
}

int svae_pcnn_conv_planes(const void* x, int n, int hi, int wi, int cin, int ldx, int x_bf16, int64_t x_pstride,
                          const void* wk, int kpad, int planes, const float* x_scale, const float* w_scale,
                          const float* bias, float* y, int ho, int wo, int cout, int ldy, int kh, int kw, int s, int pt,
                          int pl, int mode, int accumulate, int zero_edge, void* stream) {
  if (!x || !wk || planes < 1 || planes > PC_MAXPLANES || x_pstride < 0 || (!x_scale != !w_scale) ||
      (x_scale && planes != 2))
    return bad("pcnn_conv_planes: bad arguments");
  const PcScale sc{x_scale, w_scale};
  if (x_scale && x_bf16) {  // the fp16 planes: all three products in one launch where the halo kernel takes it
    const int rc = pcnn_conv_hp(x, n, hi, wi, cin, ldx, x_pstride, wk, kpad, (long long)kh * kw * cout * kpad, sc, bias,
                                y, ho, wo, cout, ldy, kh, kw, s, pt, pl, mode, accumulate, zero_edge, stream);
    if (rc <= 0) return rc;
  }
  int pi[PC_MAXPLANES * PC_MAXPLANES], pj[PC_MAXPLANES * PC_MAXPLANES];
  const int np = pc_products(planes, pi, pj);
  const long long wst = (long long)kh * kw * cout * kpad;  // one weight plane (wk [tap][cout][kpad])
  NlbArgs nlb{};
  for (int p = 0; p < np; ++p) {  // the first product writes (or accumulates) with the bias, the rest add
    const void* xp = (const char*)x + (x_bf16 ? 2 : 4) * x_pstride * pi[p];
    const __bf16* wp = (const __bf16*)wk + wst * pj[p];
    const int rc = pcnn_conv_impl(xp, n, hi, wi, cin, ldx, x_bf16, wp, kpad, p ? nullptr : bias, y, ho, wo, cout, ldy,
                                  kh, kw, s, pt, pl, mode, p ? 1 : accumulate, zero_edge, nlb, stream, sc);
    if (rc) return rc;
  }
  return 0;
}

// x [rows][ldx] fp32 -> `planes` planes [rows][ldo] (plane p at p * rows * ldo, fp32 or bf16): plane p = bf16
// of what planes 0..p-1 left of x; stored fp32, the last plane keeps the exact remainder (a kernel that
// reads it as an MFMA operand rounds it to bf16 itself)
__global__ void split_planes_kernel(const float* __restrict__ x, long long rows, int c, int ldx, int planes,
                                    void* __restrict__ out, int ldo, int out_bf16) {
  const long long n = rows * c, pst = rows * ldo;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const long long r = i / c;
    const int ch = (int)(i - r * c);
    float v = x[r * ldx + ch];
    const long long o = r * ldo + ch;
    for (int p = 0; p < planes; ++p) {
      const __bf16 b = (__bf16)v;
      if (out_bf16) ((__bf16*)out)[o + p * pst] = b;
      else ((float*)out)[o + p * pst] = p == planes - 1 ? v : (float)b;
      v -= (float)b;
    }
  }
}

__global__ __launch_bounds__(256) void absmax_kernel(const float* __restrict__ x, long long rows, int c, int ldx,
                                                     unsigned* __restrict__ mx) {
  const long long n = rows * c;
  const long long stride = (long long)gridDim.x * blockDim.x;
  float m = 0.f;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const long long r = i / c;
    m = fmaxf(m, fabsf(x[r * ldx + (i - r * c)]));
  }
  block_absmax_put(m, mx);
}

// the two scaled fp16 planes of x (h16[1]: the bits of max|x|; h16[0] <- the inverse scale)
__global__ void split_h16_kernel(const float* __restrict__ x, long long rows, int c, int ldx, __bf16* __restrict__ out,
                                 int ldo, float* h16) {
  const long long n = rows * c, pst = rows * ldo;
  const int sh = h16_shift(__float_as_uint(h16[1]));
  if (blockIdx.x == 0 && threadIdx.x == 0) h16[0] = ldexpf(1.f, -sh);
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const long long r = i / c;
    const int ch = (int)(i - r * c);
    h16_put(out, r * ldo + ch, pst, x[r * ldx + ch], sh);
  }
}

// 4-channel vector forms (c, ldx, ldo % 4 == 0, 16-B x, 8-B out; rows * c / 4 < 2^31): one 16-byte load and one
// 8-byte store per plane for four elements, the row by a multiply-shift -- the same per-element arithmetic as
// absmax_kernel / split_h16_kernel above (bitwise), which ran at 1.5-2.5 TB/s on their 64-bit divisions and
// 2-byte stores (the c_pixelvae split head calls them once per conv input: 11 % of its step, r05_gpv)
__global__ __launch_bounds__(256) void absmax4_kernel(const float* __restrict__ x, int n4, int c4, FastDiv dc4, int ldx,
                                                      unsigned* __restrict__ mx) {
  float m = 0.f;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    const int r = fdiv(i, dc4);
    const f32x4 v = *(const f32x4*)&x[(long long)r * ldx + 4 * (i - r * c4)];
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
  }
  block_absmax_put(m, mx);
}
__global__ __launch_bounds__(256) void split_h16x4_kernel(const float* __restrict__ x, int n4, int c4, FastDiv dc4,
                                                          int ldx, __bf16* __restrict__ out, int ldo, long long pst,
                                                          float* h16) {
  const int sh = h16_shift(__float_as_uint(h16[1]));
  if (blockIdx.x == 0 && threadIdx.x == 0) h16[0] = ldexpf(1.f, -sh);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    const int r = fdiv(i, dc4), q = i - r * c4;
    const f32x4 v = *(const f32x4*)&x[(long long)r * ldx + 4 * q];
    unsigned short h0[4], h1[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float t = ldexpf(v[j], sh);
      const _Float16 a = (_Float16)t;
      const _Float16 b = (_Float16)(t - (float)a);
      h0[j] = __builtin_bit_cast(unsigned short, a);
      h1[j] = __builtin_bit_cast(unsigned short, b);
    }
    const long long o = (long long)r * ldo + 4 * q;
    *(u64*)(out + o) = (u64)h0[0] | ((u64)h0[1] << 16) | ((u64)h0[2] << 32) | ((u64)h0[3] << 48);
    *(u64*)(out + o + pst) = (u64)h1[0] | ((u64)h1[1] << 16) | ((u64)h1[2] << 32) | ((u64)h1[3] << 48);
  }
}

// svae_pcnn_conv_planes leaving max |y| in y_scale[1] (the consumer nonlinearity's fp16-plane bound): fused into
// the row-staged kernel's epilogue, else a pass over y after the conv
int svae_pcnn_conv_planes_amax(const void* x, int n, int hi, int wi, int cin, int ldx, int x_bf16, int64_t x_pstride,
                               const void* wk, int kpad, int planes, const float* x_scale, const float* w_scale,
                               const float* bias, float* y, int ho, int wo, int cout, int ldy, int kh, int kw, int s,
                               int pt, int pl, int mode, int accumulate, int zero_edge, float* y_scale, void* stream) {
  if (!y_scale || !y) return bad("pcnn_conv_planes_amax: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(y_scale + 1, 0, sizeof(float), st) != hipSuccess) return hipchk();
  bool done = false;
  if (x && wk && x_scale && w_scale && x_bf16 && planes == 2 && x_pstride >= 0) {
    const PcScale sc{x_scale, w_scale};
    const int rc = pcnn_conv_hp(x, n, hi, wi, cin, ldx, x_pstride, wk, kpad, (long long)kh * kw * cout * kpad, sc, bias,
                                y, ho, wo, cout, ldy, kh, kw, s, pt, pl, mode, accumulate, zero_edge, stream,
                                (unsigned*)(y_scale + 1), &done);
    if (rc < 0) return rc;
    if (rc == 0 && done) return 0;
    if (rc == 0) {  // (ran on pc_conv3 HP: the pass below)
      hipLaunchKernelGGL(absmax_kernel, dim3(blocks_for((long long)n * ho * wo * cout, 256, 2048)), dim3(256), 0, st, y,
                         (long long)n * ho * wo, cout, ldy, (unsigned*)(y_scale + 1));
      return hipchk();
    }
  }
  const int rc = svae_pcnn_conv_planes(x, n, hi, wi, cin, ldx, x_bf16, x_pstride, wk, kpad, planes, x_scale, w_scale,
                                       bias, y, ho, wo, cout, ldy, kh, kw, s, pt, pl, mode, accumulate, zero_edge, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(absmax_kernel, dim3(blocks_for((long long)n * ho * wo * cout, 256, 2048)), dim3(256), 0, st, y,
                     (long long)n * ho * wo, cout, ldy, (unsigned*)(y_scale + 1));
  return hipchk();
}

static int pcnn_split(const float* x, int64_t rows, int c, int ldx, int planes, void* out, int ldo, int out_bf16,
                      float* h16_scale, bool premax, void* stream) {
  if (!x || !out || rows < 1 || c < 1 || ldx < c || ldo < c || planes < 1 || planes > PC_MAXPLANES ||
      (h16_scale && (planes != 2 || !out_bf16)))
    return bad("pcnn_split_planes: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  if (h16_scale) {
    if (!premax && hipMemsetAsync(h16_scale + 1, 0, sizeof(float), st) != hipSuccess) return hipchk();
    static const bool vec = svae_knob("SVAE_PC_SPLIT4", 1) != 0;
    if (vec && c % 4 == 0 && ldx % 4 == 0 && ldo % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)out & 7) == 0 &&
        rows * (long long)c / 4 < (1LL << 31)) {
      const int c4 = c / 4, n4 = (int)(rows * c4);
      const FastDiv dc4 = make_fastdiv(c4);
      if (!premax)
        hipLaunchKernelGGL(absmax4_kernel, dim3(blocks_for(n4, 256, 1024)), dim3(256), 0, st, x, n4, c4, dc4, ldx,
                           (unsigned*)(h16_scale + 1));
      hipLaunchKernelGGL(split_h16x4_kernel, dim3(blocks_for(n4)), dim3(256), 0, st, x, n4, c4, dc4, ldx,
                         (__bf16*)out, ldo, (long long)rows * ldo, h16_scale);
      return hipchk();
    }
    if (!premax)
      hipLaunchKernelGGL(absmax_kernel, dim3(blocks_for(rows * c, 256, 2048)), dim3(256), 0, st, x, (long long)rows, c,
                         ldx, (unsigned*)(h16_scale + 1));
    hipLaunchKernelGGL(split_h16_kernel, dim3(blocks_for(rows * c)), dim3(256), 0, st, x, (long long)rows, c, ldx,
                       (__bf16*)out, ldo, h16_scale);
    return hipchk();
  }
  hipLaunchKernelGGL(split_planes_kernel, dim3(blocks_for(rows * c)), dim3(256), 0, st, x, (long long)rows, c, ldx,
                     planes, out, ldo, out_bf16);
  return hipchk();
}
int svae_pcnn_split_planes(const float* x, int64_t rows, int c, int ldx, int planes, void* out, int ldo, int out_bf16,
                           float* h16_scale, void* stream) {
  return pcnn_split(x, rows, c, ldx, planes, out, ldo, out_bf16, h16_scale, false, stream);
}
int svae_pcnn_split_h16_premax(const float* x, int64_t rows, int c, int ldx, void* out, int ldo, float* h16_scale,
                               void* stream) {
  if (!h16_scale) return bad("pcnn_split_h16_premax: bad arguments");
  return pcnn_split(x, rows, c, ldx, 2, out, ldo, 1, h16_scale, true, stream);
}

int svae_pcnn_colsum(const float* x, int64_t rows, int c, int ldx, int ho, int wo, int mask_edge, float* out,
                     int accumulate, float* scratch, void* stream) {
  if (!x || !out || !scratch || rows < 1 || c < 1 || ldx < c || (mask_edge && (ho < 1 || wo < 1)))
    return bad("pcnn_colsum: bad arguments");
  long long ns = (rows + 255) / 256;  // ~256 rows per block (1024-row blocks measured slower)
  if (ns > 1024) ns = 1024;
  if (ns * c > (1LL << 24)) ns = ((1LL << 24) / c > 0) ? (1LL << 24) / c : 1;
  const long long rps = (rows + ns - 1) / ns;
  hipStream_t st = (hipStream_t)stream;
  static const bool vec = svae_knob("SVAE_PC_COLSUM4", 1) != 0;
  if (vec && c % 4 == 0 && ldx % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)scratch & 15) == 0 &&
      rows < (1LL << 31) - rps) {
    hipLaunchKernelGGL(colsum_part4_kernel_pc, dim3((c + 63) / 64, (unsigned)ns), dim3(256), 0, st, x, (int)rows, c,
                       ldx, ho * wo, make_fastdiv(ho * wo), wo, make_fastdiv(wo), mask_edge, (int)rps, scratch);
    hipLaunchKernelGGL(colsum_fin4_kernel_pc, dim3((c + 63) / 64), dim3(256), 0, st, scratch, (int)ns, c, out,
                       accumulate);
    return hipchk();
  }
  hipLaunchKernelGGL(colsum_part_kernel_pc, dim3((c + 63) / 64, (unsigned)ns), dim3(256), 0, st, x, (long long)rows, c,
                     ldx, ho * wo, wo, mask_edge, rps, scratch);
  hipLaunchKernelGGL(colsum_fin_kernel_pc, dim3((c + 63) / 64), dim3(256), 0, st, scratch, (int)ns, c, out,
                     accumulate);
  return hipchk();
}

// im2col of a small-channel stride-1 mode-0 conv's input as the two scaled fp16 planes of a [rows][kc] operand:
// column k = (ky * kw + kx) * cin + ci holds x[img][oy - pt + ky][ox - pl + kx][ci] (0 outside the image and for
// k >= kh * kw * cin), so the conv runs as a 1x1 conv with K = kc (the head's 4-channel input convs: K = 8-24 in
// one 32-wide chunk instead of 32 per tap, and 2 planes / 3 products instead of 3 bf16 planes / 6 launches)
__global__ __launch_bounds__(256) void im2col_h16_kernel(const float* __restrict__ x, int hi, int wi, int cin, int ldx,
                                                         int ho, int wo, int kw, int pt, int pl, int kreal, long long rows,
                                                         int kc, __bf16* __restrict__ out, float* h16) {
  const int sh = h16_shift(__float_as_uint(h16[1]));
  if (blockIdx.x == 0 && threadIdx.x == 0) h16[0] = ldexpf(1.f, -sh);
  const long long n = rows * kc, pst = rows * kc;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / kc;
    const int k = (int)(i - r * kc);
    float v = 0.f;
    if (k < kreal) {
      const int tap = k / cin, ci = k - tap * cin;
      const int ky = tap / kw, kx = tap - ky * kw;
      const int img = (int)(r / ((long long)ho * wo));
      const int rr = (int)(r - (long long)img * ho * wo);
      const int oy = rr / wo, ox = rr - oy * wo;
      const int iy = oy - pt + ky, ix = ox - pl + kx;
      if (iy >= 0 && iy < hi && ix >= 0 && ix < wi) v = x[((long long)(img * hi + iy) * wi + ix) * ldx + ci];
    }
    h16_put(out, i, pst, v, sh);
  }
}

int svae_pcnn_im2col_h16(const float* x, int n, int hi, int wi, int cin, int ldx, int ho, int wo, int kh, int kw, int pt,
                         int pl, void* out, int kc, float* h16_scale, void* stream) {
  if (!x || !out || !h16_scale || n < 1 || hi < 1 || wi < 1 || cin < 1 || ldx < cin || ho < 1 || wo < 1 || kh < 1 ||
      kw < 1 || kc < kh * kw * cin || kc % 32)
    return bad("pcnn_im2col_h16: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  const long long rows = (long long)n * ho * wo;
  if (hipMemsetAsync(h16_scale + 1, 0, sizeof(float), st) != hipSuccess) return hipchk();
  // the planes' scale from max|x| (>= max over the gathered columns: every value fits)
  hipLaunchKernelGGL(absmax_kernel, dim3(blocks_for((long long)n * hi * wi * cin, 256, 2048)), dim3(256), 0, st, x,
                     (long long)n * hi * wi, cin, ldx, (unsigned*)(h16_scale + 1));
  hipLaunchKernelGGL(im2col_h16_kernel, dim3(blocks_for(rows * kc)), dim3(256), 0, st, x, hi, wi, cin, ldx, ho, wo, kw,
                     pt, pl, kh * kw * cin, rows, kc, (__bf16*)out, h16_scale);
  return hipchk();
}

int svae_pcnn_colsum_absmax(const float* x, int64_t rows, int c, int ldx, float* out, int accumulate, float* scratch,
                            float* h16_scale, void* stream) {
  if (!x || !out || !scratch || !h16_scale || rows < 1 || c < 1 || ldx < c) return bad("pcnn_colsum_absmax: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(h16_scale + 1, 0, sizeof(float), st) != hipSuccess) return hipchk();
  long long ns = (rows + 255) / 256;  // (svae_pcnn_colsum's split: the same column partials, bitwise)
  if (ns > 1024) ns = 1024;
  if (ns * c > (1LL << 24)) ns = ((1LL << 24) / c > 0) ? (1LL << 24) / c : 1;
  const long long rps = (rows + ns - 1) / ns;
  static const bool vec = svae_knob("SVAE_PC_COLSUM4", 1) != 0 && svae_knob("SVAE_PC_CSAMAX", 1) != 0;
  if (vec && c % 4 == 0 && ldx % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)scratch & 15) == 0 &&
      rows < (1LL << 31) - rps) {
    hipLaunchKernelGGL(colsum_amax4_kernel_pc, dim3((c + 63) / 64, (unsigned)ns), dim3(256), 0, st, x, (int)rows, c,
                       ldx, (int)rps, scratch, (unsigned*)(h16_scale + 1));
    hipLaunchKernelGGL(colsum_fin4_kernel_pc, dim3((c + 63) / 64), dim3(256), 0, st, scratch, (int)ns, c, out,
                       accumulate);
    return hipchk();
  }
  const int rc = svae_pcnn_colsum(x, rows, c, ldx, 1, 1, 0, out, accumulate, scratch, stream);
  if (rc) return rc;
  hipLaunchKernelGGL(absmax_kernel, dim3(blocks_for(rows * c, 256, 2048)), dim3(256), 0, st, x, (long long)rows, c, ldx,
                     (unsigned*)(h16_scale + 1));
  return hipchk();
}

int svae_pcnn_mask_edge(float* x, int n, int ho, int wo, int c, int ldx, int mask_edge, void* stream) {
  if (!x || n < 1 || ho < 1 || wo < 1 || c < 1 || ldx < c || mask_edge < 1 || mask_edge > 2)
    return bad("pcnn_mask_edge: bad arguments");
  const long long rows = (long long)n * ho * wo;
  hipLaunchKernelGGL(mask_edge_kernel, dim3(blocks_for(rows * c)), dim3(256), 0, (hipStream_t)stream, x, rows, ho * wo,
                     wo, c, ldx, mask_edge);
  return hipchk();
}

static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

static int pcnn_nonlin(const float* x, int64_t rows, int c, int ldx, int kind, const float* mask, float keep,
                       uint64_t seed, void* y, int ldy, int y_bf16, float* h16_scale, void* stream) {
  if (!x || !y || rows < 1 || c < 1 || kind < 0 || kind > 2 || ldx < c || ldy < (kind == 2 ? 2 * c : c))
    return bad("pcnn_nonlin: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  unsigned* amax = h16_scale ? (unsigned*)(h16_scale + 1) : nullptr;
  if (amax && hipMemsetAsync(amax, 0, sizeof(float), st) != hipSuccess) return hipchk();
  const bool vec = c % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && al16(x) && (!mask || al16(mask)) &&
                   (y_bf16 ? ((uintptr_t)y & 7) == 0 : al16(y));
  if (vec) {
    const dim3 grid((unsigned)((rows + NL_RPB - 1) / NL_RPB));
    if (y_bf16)
      hipLaunchKernelGGL(nonlin4_kernel<true>, grid, dim3(256), 0, st, x, (long long)rows, c, ldx, kind, mask, keep,
                         (unsigned long long)seed, y, ldy, nullptr);
    else
      hipLaunchKernelGGL(nonlin4_kernel<false>, grid, dim3(256), 0, st, x, (long long)rows, c, ldx, kind, mask, keep,
                         (unsigned long long)seed, y, ldy, amax);
    return hipchk();
  }
  if (mask || keep < 1.f || y_bf16) return bad("pcnn_nonlin: dropout or a bf16 output needs 4-channel aligned rows");
  if (amax) return bad("pcnn_nonlin_absmax: needs 4-channel aligned fp32 rows");
  hipLaunchKernelGGL(nonlin_kernel, dim3(blocks_for(rows * c)), dim3(256), 0, st, x, (long long)rows, c, ldx, kind,
                     (float*)y, ldy);
  return hipchk();
}
int svae_pcnn_nonlin(const float* x, int64_t rows, int c, int ldx, int kind, const float* mask, float keep,
                     uint64_t seed, void* y, int ldy, int y_bf16, void* stream) {
  return pcnn_nonlin(x, rows, c, ldx, kind, mask, keep, seed, y, ldy, y_bf16, nullptr, stream);
}
int svae_pcnn_nonlin_absmax(const float* x, int64_t rows, int c, int ldx, int kind, const float* mask, float keep,
                            uint64_t seed, float* y, int ldy, float* h16_scale, void* stream) {
  if (!h16_scale) return bad("pcnn_nonlin_absmax: bad arguments");
  return pcnn_nonlin(x, rows, c, ldx, kind, mask, keep, seed, y, ldy, 0, h16_scale, stream);
}

// the nonlinearity (with the seeded dropout) writing its output straight as the two scaled fp16 planes of the
// consuming conv's operand: the planes' exponent from a bound on max |y| known before the pass -- max |x| (left
// by x's producer, x_scale[1]), 1 for elu / concat_elu, over keep -- instead of the fp32 output, its absmax and a
// split pass.  h16_scale <- [2^-s, the bound]
__global__ __launch_bounds__(256) void nonlin4_h16_kernel(const float* __restrict__ x, long long rows, int c, int ldx,
                                                          int kind, const float* __restrict__ mask, float keep,
                                                          unsigned long long seed, float mask_max,
                                                          const float* __restrict__ x_scale, __bf16* __restrict__ out,
                                                          int ldo, float* h16) {
  const bool hashed = !mask && keep < 1.f;
  const float inv = 1.f / keep;
  float bound = x_scale[1];
  if (kind != 0) bound = fmaxf(bound, 1.f);
  bound = bound * mask_max * (1.f + 0x1p-20f);  // (rounded up: every |y| <= bound)
  const int sh = h16_shift(__float_as_uint(bound));
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    h16[0] = ldexpf(1.f, -sh);
    h16[1] = bound;
  }
  const int q = c >> 2, cy = kind == 2 ? 2 * c : c;
  const long long pst = rows * ldo;
  const long long r0 = (long long)blockIdx.x * NL_RPB;
  const int nr = (int)(rows - r0 < NL_RPB ? rows - r0 : NL_RPB);
  for (int j = threadIdx.x; j < nr * q; j += 256) {
    const int rr = j / q;
    const int ch = (j - rr * q) * 4;
    const long long r = r0 + rr;
    f32x4 a, b = {0.f, 0.f, 0.f, 0.f};
    nl_fwd4(*(const f32x4*)(x + r * ldx + ch), kind, a, b);
    if (mask) {
      a *= *(const f32x4*)(mask + r * cy + ch);
      if (kind == 2) b *= *(const f32x4*)(mask + r * cy + c + ch);
    } else if (hashed) {
      a *= drop_scale4(seed, (unsigned long long)(r * cy + ch), keep, inv);
      if (kind == 2) b *= drop_scale4(seed, (unsigned long long)(r * cy + c + ch), keep, inv);
    }
    for (int half = 0; half < (kind == 2 ? 2 : 1); ++half) {
      const f32x4 v = half ? b : a;
      unsigned short h0[4], h1[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float t = ldexpf(v[e], sh);
        const _Float16 u = (_Float16)t;
        const _Float16 l = (_Float16)(t - (float)u);
        h0[e] = __builtin_bit_cast(unsigned short, u);
        h1[e] = __builtin_bit_cast(unsigned short, l);
      }
      const long long o = r * ldo + ch + half * c;
      *(u64*)(out + o) = (u64)h0[0] | ((u64)h0[1] << 16) | ((u64)h0[2] << 32) | ((u64)h0[3] << 48);
      *(u64*)(out + o + pst) = (u64)h1[0] | ((u64)h1[1] << 16) | ((u64)h1[2] << 32) | ((u64)h1[3] << 48);
    }
  }
}

int svae_pcnn_nonlin_h16(const float* x, int64_t rows, int c, int ldx, int kind, const float* mask, float mask_max,
                         float keep, uint64_t seed, const float* x_scale, void* out, int ldo, float* h16_scale,
                         void* stream) {
  const int cy = kind == 2 ? 2 * c : c;
  if (!x || !x_scale || !out || !h16_scale || rows < 1 || c < 1 || kind < 0 || kind > 2 || ldx < c || ldo < cy ||
      !(keep > 0.f) || keep > 1.f || c % 4 || ldx % 4 || ldo % 4 || !al16(x) || ((uintptr_t)out & 7) ||
      (mask && (!al16(mask) || !(mask_max >= 0.f))))
    return bad("pcnn_nonlin_h16: bad arguments");
  // the largest factor the dropout applies: the mask tensor's maximum, or 1 / keep for the in-kernel mask
  const float mmax = mask ? (mask_max > 0.f ? mask_max : 1.f) : 1.f / keep;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(nonlin4_h16_kernel, dim3((unsigned)((rows + NL_RPB - 1) / NL_RPB)), dim3(256), 0, st, x,
                     (long long)rows, c, ldx, kind, mask, keep, (unsigned long long)seed, mmax, x_scale, (__bf16*)out,
                     ldo, h16_scale);
  return hipchk();
}

int svae_pcnn_nonlin_bwd(const float* x, int64_t rows, int c, int ldx, int kind, const float* mask, float keep,
                         uint64_t seed, const float* dy, int ldy, void* dx, int lddx, int dx_bf16, int accumulate,
                         float* dsum, float* scratch, void* stream) {
  if (!x || !dy || !dx || rows < 1 || c < 1 || kind < 0 || kind > 2) return bad("pcnn_nonlin_bwd: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  const bool vec = c % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && lddx % 4 == 0 && al16(x) && al16(dy) &&
                   (dx_bf16 ? ((uintptr_t)dx & 7) == 0 : al16(dx)) && (!mask || al16(mask));
  if (dx_bf16 || dsum) {  // written gradient (bf16 and / or with its column sums): relu / elu only
    if (!vec || kind == 2 || accumulate || c > 1024 || (dsum && !scratch))
      return bad("pcnn_nonlin_bwd: bf16 output / column sums need kind 0/1, a written aligned gradient");
    const long long nb = (rows + NL_RPB - 1) / NL_RPB;
    float* part = dsum ? scratch : nullptr;
    if (!part) return bad("pcnn_nonlin_bwd: bf16 output without column sums is not built");
    hipLaunchKernelGGL(nonlin4_bwd_cs_kernel, dim3((unsigned)nb), dim3(256), 0, st, x, (long long)rows, c, ldx, kind,
                       mask, keep, (unsigned long long)seed, dy, ldy, dx, lddx, dx_bf16, part);
    // the column sums of the per-block partials: the two-stage fixed-order column sum (not one thread per column)
    return svae_pcnn_colsum(part, nb, c, c, 1, 1, 0, dsum, 0, part + nb * c, stream);
  }
  if (vec) {
    hipLaunchKernelGGL(nonlin4_bwd_kernel, dim3((unsigned)((rows + NL_RPB - 1) / NL_RPB)), dim3(256), 0, st, x,
                       (long long)rows, c, ldx, kind, mask, keep, (unsigned long long)seed, dy, ldy, (float*)dx, lddx,
                       accumulate);
    return hipchk();
  }
  if (mask || keep < 1.f) return bad("pcnn_nonlin_bwd: dropout needs 4-channel aligned rows");
  hipLaunchKernelGGL(nonlin_bwd_kernel, dim3(blocks_for(rows * c)), dim3(256), 0, st, x, (long long)rows, c, ldx, kind,
                     dy, ldy, (float*)dx, lddx, accumulate);
  return hipchk();
}

static int pcnn_gate(const float* x, int ldx, const float* c2, const float* hp, int64_t rows, int pix_per_img, int f,
                     float* out, int ldo, float* out_scale, void* stream) {
  if (!x || !c2 || !out || rows < 1 || f < 1 || pix_per_img < 1 || rows % pix_per_img) return bad("pcnn_gate: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  unsigned* amax = out_scale ? (unsigned*)(out_scale + 1) : nullptr;
  if (amax && hipMemsetAsync(amax, 0, sizeof(float), st) != hipSuccess) return hipchk();
  if (f % 4 == 0 && ldx % 4 == 0 && ldo % 4 == 0 && pix_per_img % GT_RPB == 0 && al16(x) && al16(c2) && al16(out) &&
      (!hp || al16(hp))) {
    hipLaunchKernelGGL(gate4_kernel, dim3((unsigned)(rows / GT_RPB)), dim3(256), 0, st, x, ldx, c2, hp, (long long)rows,
                       pix_per_img, f, out, ldo, amax);
    return hipchk();
  }
  hipLaunchKernelGGL(gate_kernel, dim3(blocks_for(rows * f)), dim3(256), 0, st, x, ldx, c2, hp, (long long)rows,
                     pix_per_img, f, out, ldo);
  if (amax)
    hipLaunchKernelGGL(absmax_kernel, dim3(blocks_for(rows * f, 256, 2048)), dim3(256), 0, st, out, (long long)rows, f,
                       ldo, amax);
  return hipchk();
}
int svae_pcnn_gate(const float* x, int ldx, const float* c2, const float* hp, int64_t rows, int pix_per_img, int f,
                   float* out, int ldo, void* stream) {
  return pcnn_gate(x, ldx, c2, hp, rows, pix_per_img, f, out, ldo, nullptr, stream);
}
int svae_pcnn_gate_amax(const float* x, int ldx, const float* c2, const float* hp, int64_t rows, int pix_per_img, int f,
                        float* out, int ldo, float* out_scale, void* stream) {
  if (!out_scale) return bad("pcnn_gate_amax: bad arguments");
  return pcnn_gate(x, ldx, c2, hp, rows, pix_per_img, f, out, ldo, out_scale, stream);
}

int svae_pcnn_gate_bwd(const float* c2, const float* hp, const float* dout, int lddo, int64_t rows, int pix_per_img,
                       int f, void* dc2, int dc2_bf16, float* dhp, float* dsum, float* scratch, void* stream) {
  if (!c2 || !dout || !dc2 || rows < 1 || f < 1 || pix_per_img < 1 || rows % pix_per_img || ((dhp || dsum) && !scratch))
    return bad("pcnn_gate_bwd: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  const int nimg = (int)(rows / pix_per_img);
  if (f % 4 == 0 && f <= 1024 && lddo % 4 == 0 && pix_per_img % GT_RPB == 0 && al16(c2) && al16(dout) &&
      (dc2_bf16 ? ((uintptr_t)dc2 & 7) == 0 : al16(dc2)) && (!hp || al16(hp))) {
    const long long nb = rows / GT_RPB;
    const bool sums = dhp || dsum;
    hipLaunchKernelGGL(gate4_bwd_kernel, dim3((unsigned)nb), dim3(256), 0, st, c2, hp, dout, lddo, (long long)rows,
                       pix_per_img, f, dc2, dc2_bf16, sums ? scratch : nullptr);
    if (dhp)
      hipLaunchKernelGGL(gate_imgsum_kernel, dim3((nimg * 2 * f + 255) / 256), dim3(256), 0, st, scratch,
                         pix_per_img / GT_RPB, nimg, 2 * f, dhp);
    if (dsum)  // the sums over all rows: the two-stage fixed-order column sum of the block partials
      return svae_pcnn_colsum(scratch, nb, 2 * f, 2 * f, 1, 1, 0, dsum, 0, scratch + nb * 2 * f, stream);
    return hipchk();
  }
  if (dc2_bf16 || dsum) return bad("pcnn_gate_bwd: bf16 dc2 / column sums need the vectorised path");
  hipLaunchKernelGGL(gate_bwd_kernel, dim3(blocks_for(rows * f)), dim3(256), 0, st, c2, hp, dout, lddo, (long long)rows,
                     pix_per_img, f, (float*)dc2);
  if (dhp) return svae_pcnn_imgsum((const float*)dc2, 2 * f, nimg, pix_per_img, 2 * f, dhp, scratch, stream);
  return hipchk();
}

int svae_pcnn_gemm_small(const float* A, int lda, int ta, const float* B, int ldb, int tb, float* C, int ldc, int m,
                         int n, int k, float beta, void* stream) {
  if (!A || !B || !C || m < 1 || n < 1 || k < 1) return bad("pcnn_gemm_small: bad arguments");
  if (k >= 128) {  // a wave per output: the K loop of one thread would be latency-bound
    hipLaunchKernelGGL(gemm_small_wave_kernel, dim3((unsigned)(((long long)m * n + 3) / 4)), dim3(256), 0,
                       (hipStream_t)stream, A, lda, ta, B, ldb, tb, C, ldc, m, n, k, beta);
    return hipchk();
  }
  hipLaunchKernelGGL(gemm_small_kernel, dim3(blocks_for((long long)m * n)), dim3(256), 0, (hipStream_t)stream, A, lda,
                     ta, B, ldb, tb, C, ldc, m, n, k, beta);
  return hipchk();
}

int svae_pcnn_imgsum(const float* x, int ldx, int nimg, int pix_per_img, int c, float* out, float* scratch,
                     void* stream) {
  if (!x || !out || !scratch || nimg < 1 || pix_per_img < 1 || c < 1 || ldx < c) return bad("pcnn_imgsum: bad arguments");
  const int ps = (pix_per_img + IMGSUM_PIX - 1) / IMGSUM_PIX;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(imgsum_kernel, dim3((c + 63) / 64, nimg, ps), dim3(256), 0, st, x, ldx, pix_per_img, c, scratch);
  const long long n = (long long)nimg * c;
  hipLaunchKernelGGL(split_reduce_kernel, dim3(blocks_for(n)), dim3(256), 0, st, scratch, ps, n, out,
                     PcScale{nullptr, nullptr});
  return hipchk();
}

int svae_pcnn_copy(const float* x, int ldx, int64_t rows, int c, float* y, int ldy, int accumulate, void* stream) {
  if (!x || !y || rows < 1 || c < 1 || ldx < c || ldy < c) return bad("pcnn_copy: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  if (c % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && al16(x) && al16(y)) {
    hipLaunchKernelGGL(copy4_kernel, dim3((unsigned)((rows + GT_RPB - 1) / GT_RPB)), dim3(256), 0, st, x, ldx,
                       (long long)rows, c, y, ldy, accumulate);
    return hipchk();
  }
  hipLaunchKernelGGL(copy_kernel, dim3(blocks_for(rows * c)), dim3(256), 0, st, x, ldx, (long long)rows, c, y, ldy,
                     accumulate);
  return hipchk();
}

int svae_pcnn_pad_ones(const float* x, int64_t rows, int c, float* y, int ldy, void* stream) {
  if (!x || !y || rows < 1 || c < 1 || ldy < c + 1) return bad("pcnn_pad_ones: bad arguments");
  hipLaunchKernelGGL(pad_ones_kernel, dim3(blocks_for(rows * ldy)), dim3(256), 0, (hipStream_t)stream, x,
                     (long long)rows, c, y, ldy);
  return hipchk();
}

int svae_pcnn_mixlogistic(const float* x, const float* l, int64_t pixels, int m, float* logp, float* dl, float coef,
                          void* stream) {
  if (!x || !l || !logp || pixels < 1 || m < 1 || m > PC_MAXMIX) return bad("pcnn_mixlogistic: bad arguments");
  hipLaunchKernelGGL(mixlogistic_kernel, dim3((unsigned)((pixels + 127) / 128)), dim3(128), 0, (hipStream_t)stream, x,
                     l, (long long)pixels, m, logp, dl, coef);
  return hipchk();
}

int svae_pcnn_sum(const float* x, int64_t n, float* out, double* out64, void* stream) {
  if (!x || n < 1 || (!out && !out64)) return bad("pcnn_sum: bad arguments");
  hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, x, (long long)n, out, out64);
  return hipchk();
}

int svae_pcnn_sample(const float* l, const float* u_mix, const float* u_log, int nimg, int per_img, int m, float* x,
                     int q0, int q1, int pix_stride, void* stream) {
  if (!l || !u_mix || !u_log || !x || nimg < 1 || per_img < 1 || m < 1 || m > PC_MAXMIX || q0 < 0 || q1 <= q0 ||
      q1 > per_img || pix_stride < 3)
    return bad("pcnn_sample: bad arguments");
  const long long n = (long long)nimg * (q1 - q0);
  hipLaunchKernelGGL(sample_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, l, u_mix,
                     u_log, nimg, per_img, m, x, q0, q1, pix_stride);
  return hipchk();
}

int svae_pcnn_sample_bwd(const float* l, const float* u_mix, const float* u_log, int nimg, int per_img, int m,
                         const float* dx, int dx_stride, float* dl, void* stream) {
  if (!l || !u_mix || !u_log || !dx || !dl || nimg < 1 || per_img < 1 || m < 1 || m > PC_MAXMIX || dx_stride < 3)
    return bad("pcnn_sample_bwd: bad arguments");
  const long long n = (long long)nimg * per_img;
  hipLaunchKernelGGL(sample_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, l, u_mix,
                     u_log, n, m, dx, dx_stride, dl);
  return hipchk();
}

int svae_pcnn_highway_bwd(const float* s, const float* prev, const float* z, const float* zb, int nimg, int64_t per_img,
                          float lo, float hi, const float* dout, float* ds, float* dprev, int prev_acc, float* dz,
                          void* stream) {
  if (!s || !prev || !z || !dout || !dz || nimg < 1 || per_img < 1) return bad("pcnn_highway_bwd: bad arguments");
  hipLaunchKernelGGL(highway_bwd_kernel, dim3(nimg), dim3(256), 0, (hipStream_t)stream, s, prev, z, zb,
                     (long long)per_img, lo, hi, dout, ds, dprev, prev_acc, dz);
  return hipchk();
}

int svae_pcnn_sqerr(const float* a, const float* t, int nimg, int64_t per_img, float coef, float* rec, float* da,
                    void* stream) {
  if (!a || !t || nimg < 1 || per_img < 1 || (!rec && !da)) return bad("pcnn_sqerr: bad arguments");
  hipLaunchKernelGGL(sqerr_kernel, dim3(nimg), dim3(256), 0, (hipStream_t)stream, a, t, (long long)per_img, coef, rec, da);
  return hipchk();
}

int svae_pcnn_dropout_mask(int64_t n, float keep, uint64_t seed, float* out, void* stream) {
  if (!out || n < 1 || !(keep > 0.f) || keep > 1.f) return bad("pcnn_dropout_mask: bad arguments");
  hipLaunchKernelGGL(dropout_mask_kernel, dim3(blocks_for(n)), dim3(256), 0, (hipStream_t)stream, (long long)n, keep,
                     (unsigned long long)seed, out);
  return hipchk();
}

int svae_pcnn_dropout(const float* x, int64_t rows, int c, int ldx, const float* mask, float* y, int ldy, void* stream) {
  if (!x || !mask || !y || rows < 1 || c < 1 || ldx < c || ldy < c) return bad("pcnn_dropout: bad arguments");
  hipLaunchKernelGGL(dropout_kernel, dim3(blocks_for((long long)rows * c)), dim3(256), 0, (hipStream_t)stream, x,
                     (long long)rows, c, ldx, mask, y, ldy);
  return hipchk();
}

int svae_pcnn_highway(const float* s, const float* prev, const float* z, const float* zb, int nimg, int64_t per_img,
                      float lo, float hi, float* out, float* ratio, void* stream) {
  if (!s || !prev || !z || !out || nimg < 1 || per_img < 1) return bad("pcnn_highway: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  const long long total = (long long)nimg * per_img;
  hipLaunchKernelGGL(highway_kernel, dim3(blocks_for(total)), dim3(256), 0, st, s, prev, z, zb, (long long)per_img,
                     total, lo, hi, out);
  if (ratio) hipLaunchKernelGGL(ratio_kernel, dim3((nimg + 255) / 256), dim3(256), 0, st, z, zb, nimg, lo, hi, ratio);
  return hipchk();
}

int svae_pcnn_wn_init(const float* y, int64_t rows, int c, int ldy, float init_scale, float* g, float* b,
                      double* scratch, void* stream) {
  if (!y || !g || !b || !scratch || rows < 1 || c < 1 || ldy < c) return bad("pcnn_wn_init: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  long long nrb = (rows + 1023) / 1024;  // >= 1024 rows per block, at most WNI_MAXRB blocks per column group
  if (nrb > WNI_MAXRB) nrb = WNI_MAXRB;
  const long long rpb = (rows + nrb - 1) / nrb;
  nrb = (rows + rpb - 1) / rpb;
  const dim3 grid((c + 63) / 64, (unsigned)nrb);
  for (int pass = 0; pass < 2; ++pass)
    hipLaunchKernelGGL(wn_mom_kernel, grid, dim3(256), 0, st, y, (long long)rows, c, ldy, rpb, (int)nrb, pass, scratch);
  hipLaunchKernelGGL(wn_init_fin_kernel, dim3((c + 255) / 256), dim3(256), 0, st, scratch, (int)nrb, (long long)rows, c,
                     init_scale, g, b);
  return hipchk();
}

int svae_pcnn_adam(float* p, const float* g, float* m, float* v, int64_t n, float lr, int64_t step, float clip,
                   void* stream) {
  if (!p || !g || !m || !v || n < 1 || step < 1) return bad("pcnn_adam: bad arguments");
  const double b1 = 0.9, b2 = 0.999;
  const double lr_t = lr * sqrt(1.0 - pow(b2, (double)step)) / (1.0 - pow(b1, (double)step));
  adam_step(p, g, m, v, nullptr, n, (float)lr_t, (float)b1, (float)b2, 1e-8f, clip, 1, 0, (hipStream_t)stream);
  return hipchk();
}

int svae_pcnn_ema(float* avg, const float* p, int64_t n, float decay, void* stream) {
  if (!avg || !p || n < 1) return bad("pcnn_ema: bad arguments");
  hipLaunchKernelGGL(ema_kernel, dim3(blocks_for(n)), dim3(256), 0, (hipStream_t)stream, avg, p, (long long)n, decay);
  return hipchk();
}

}  // extern "C"
