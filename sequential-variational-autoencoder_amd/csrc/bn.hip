// Training-mode BatchNorm (center=True, scale=False, eps=1e-3; abstract_network.py:22) + activation.
//
// Forward statistics come from the producing GEMM's epilogue, added into fixed-point
// per-column accumulators (common.h stat_put); the apply pass finalises them in fp64.  The normalise +
// beta + shortcut + activation pass writes straight into the consumer's view
// (e.g. the channel half of a concat buffer, combine_noise sequential_vae.py:1833).
// Backward: dz = dy*act'(y) (act' from the stored output, TF tie rules),
// dpre = invstd*(dz - mean(dz) - xhat*mean(dz*xhat)), dbeta = sum(dz).
#include <cstdlib>

#include "common.h"
#include "knobs.h"
#include "kernels.h"

typedef __bf16 bf16x4_bn __attribute__((ext_vector_type(4)));

// BN output before the activation, per element through common.h bn_y1 (one expression shared
// by every kernel that needs it, so the backward's act' sign is bitwise the forward's)
__device__ __forceinline__ f32x4 bn_y(f32x4 x, f32x4 m, f32x4 is, f32x4 b) {
  f32x4 r;
#pragma unroll
  for (int e = 0; e < 4; ++e) r[e] = bn_y1(x[e], m[e], is[e], b[e]);
  return r;
}

// Elementwise BN passes: a block owns up to AP_QB channel quads (contiguous 16-B column
// segments of a row) and a range of rows.  It first finalises its channels' statistics from
// the fixed-point accumulators (fp64, the same expression for every block, so all blocks agree
// bitwise) into LDS; the blocks of row range 0 also store them for the backward.  This replaces
// a separate finalize launch per BN layer.
#define AP_QB 64

// SVAE_BN_W8=1: bf16-output BN passes with 8 channels per thread (one 16-byte store)
static bool bn_w8() {
  static const bool v = svae_knob("SVAE_BN_W8", 0) == 1;
  return v;
}

// shards so that at most ~16 row-blocks add into one accumulator line
// cap: 16 (bf16 mode) or 32 (split mode: +0.8 % there, -1 % in bf16; profiles/r04_shards_ab.txt); the
// apply blocks each gather nsh x 4 words per channel, the producers' atomics contend with fewer (SVAE_BN_SHMAX
// overrides: 8 -3 %, 4 -13 %)
int bn_acc_shards(long long rowblocks, int cap) {
  static const int over = svae_knob("SVAE_BN_SHMAX", 0);
  if (over > 0) cap = over;
  int n = 1;
  while (n < cap && (long long)n * 16 < rowblocks) n *= 2;
  return n;
}

// integer sum over the nsh shards of the accumulators of channels [c0, c0 + nch) into LDS
// tot[4 * nch] (exact and order-free), block-cooperative; ends with a barrier.  Each thread sums
// its word over a stride of shards in registers (independent loads, one L2 round trip), then
// the k threads that share a word combine by LDS integer atomics.
__device__ __forceinline__ void acc_gather(const u64* acc, long long sh, int nsh, int c0, int nch, u64* tot) {
  const int nw = 4 * nch;
  const int tid = threadIdx.x;
  const u64* base = acc + 4LL * c0;
  if (nw >= 256) {
    for (int w = tid; w < nw; w += 256) {
      u64 v = 0;
#pragma unroll 8
      for (int k = 0; k < nsh; ++k) v += base[k * sh + w];
      tot[w] = v;
    }
    __syncthreads();
    return;
  }
  int k = 256 / nw;  // threads per word
  if (k > nsh) k = nsh;
  for (int i = tid; i < nw; i += 256) tot[i] = 0;
  __syncthreads();
  if (tid < k * nw) {
    const int w = tid % nw, part = tid / nw;
    u64 v = 0;
#pragma unroll 4
    for (int j = part; j < nsh; j += k) v += base[j * sh + w];
    if (k == 1) tot[w] = v;
    else atomicAdd(&tot[w], v);
  }
  __syncthreads();
}

struct ApGrid {
  dim3 grid;
  int rpb;
};
// W = channels per thread: 4 (one 16-byte fp32 quad), or 8 for bf16 outputs (one 16-byte bf16 store)
static ApGrid ap_grid(long long rows, int C, int groups, int W = 4) {
  const int Q = C / W;
  const int QB = Q < AP_QB * 4 / W ? Q : AP_QB * 4 / W;
  const int RL = 256 / QB;
  const int gx = (Q + QB - 1) / QB;
  // >= rpt rows per thread (SVAE_AP_RPT, default 2) within a budget of SVAE_AP_CAP blocks (default
  // 4096): these latency-bound passes want blocks even though every block re-finalises its channels'
  // statistics (tools/gpu/r02_rpt.sh: 2 / 4096 is 1 % faster per step than round 1's 4 / 2048; 8, 16,
  // 32 rows per thread 3, 10, 25 % slower)
  static const int rpt = svae_knob("SVAE_AP_RPT", 2);
  long long want = (rows + (long long)rpt * RL - 1) / ((long long)rpt * RL);
  static const int capb = svae_knob("SVAE_AP_CAP", 4096);  // block budget of one pass
  long long cap = capb / ((long long)gx * groups);
  if (cap < 1) cap = 1;
  long long ry = want < cap ? want : cap;
  if (ry < 1) ry = 1;
  ApGrid g;
  g.rpb = (int)((rows + ry - 1) / ry);
  g.grid = dim3(gx, (unsigned)((rows + g.rpb - 1) / g.rpb), groups);
  return g;
}

// W = 8 (bf16 output, C % 8 == 0): each thread normalises 8 consecutive channels of a row and
// writes them as one 16-byte bf16 vector (write-through-friendly; W = 4 writes 8 bytes)
// PB: pre is stored as bf16 (common.h pf_ld4)
template <int W, bool PB>
__global__ __launch_bounds__(256) void bn_apply_kernel(const float* pre, int ldp, long long pre_gs, long long rows,
                                                       int C, const u64* acc, long long acc_gs, long long sh,
                                                       int nsh, float eps,
                                                       float* mean, float* invstd, long long ms_gs, const float* beta,
                                                       long long beta_gs, const float* res, int ldr, long long res_gs,
                                                       int act, float* out, int ldo, long long out_gs, int rpb,
                                                       int out_bf16) {
  __shared__ __attribute__((aligned(16))) float sm[2][AP_QB * 4];
  __shared__ u64 tot[4 * AP_QB * 4];
  const int group = blockIdx.z;
  const int Q = C / W;
  const int QB = Q < AP_QB * 4 / W ? Q : AP_QB * 4 / W;
  const int RL = 256 / QB;
  const int tid = threadIdx.x, qi = tid % QB, rl = tid / QB;
  const int q0 = blockIdx.x * QB;
  const int nch = min(QB * W, C - q0 * W);
  mean += group * ms_gs;
  invstd += group * ms_gs;
  if (acc) acc_gather(acc + group * acc_gs, sh, nsh, q0 * W, nch, tot);
  if (tid < nch) {
    const int c = q0 * W + tid;
    {
      float m, is;
      if (acc) {
        const double cnt = (double)rows;
        const double md = fx_get(tot + 4 * tid) / cnt;
        double var = fx_get(tot + 4 * tid + 2) / cnt - md * md;
        if (var < 0.0) var = 0.0;
        m = (float)md;
        is = (float)(1.0 / sqrt(var + (double)eps));
        if (blockIdx.y == 0) {
          mean[c] = m;
          invstd[c] = is;
        }
      } else {
        m = mean[c];
        is = invstd[c];
      }
      sm[0][tid] = m;
      sm[1][tid] = is;
    }
  }
  __syncthreads();
  const int q = q0 + qi;
  if (rl >= RL || q >= Q) return;
  const int c = q * W;
  pre = pf_at(pre, group * pre_gs, PB);
  if (res) res += group * res_gs;
  const long long r0 = (long long)blockIdx.y * rpb;
  const long long r1 = r0 + rpb < rows ? r0 + rpb : rows;
  if constexpr (W == 8) {  // (out_bf16)
    const f32x4 m0 = *(const f32x4*)&sm[0][qi * 8], is0 = *(const f32x4*)&sm[1][qi * 8];
    const f32x4 m1 = *(const f32x4*)&sm[0][qi * 8 + 4], is1 = *(const f32x4*)&sm[1][qi * 8 + 4];
    const f32x4 b0 = *(const f32x4*)(beta + group * beta_gs + c), b1 = *(const f32x4*)(beta + group * beta_gs + c + 4);
#pragma unroll 4
    for (long long r = r0 + rl; r < r1; r += RL) {
      f32x4 y0 = bn_y(pf_ld4(pre, r * ldp + c, PB), m0, is0, b0);
      f32x4 y1 = bn_y(pf_ld4(pre, r * ldp + c + 4, PB), m1, is1, b1);
      if (res) {
        y0 += *(const f32x4*)(res + r * ldr + c);
        y1 += *(const f32x4*)(res + r * ldr + c + 4);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        y0[e] = act_f(y0[e], act);
        y1[e] = act_f(y1[e], act);
      }
      const long long o = group * out_gs + r * ldo + c;  // bf16 elements (a multiple of 8)
      const bf16x4_bn h0 = __builtin_convertvector(y0, bf16x4_bn), h1 = __builtin_convertvector(y1, bf16x4_bn);
      const u64 u0 = __builtin_bit_cast(u64, h0), u1 = __builtin_bit_cast(u64, h1);
      const f32x4 bits = {__uint_as_float((unsigned)u0), __uint_as_float((unsigned)(u0 >> 32)),
                          __uint_as_float((unsigned)u1), __uint_as_float((unsigned)(u1 >> 32))};
      st_out16(out, o / 2, bits);
    }
    return;
  }
  const f32x4 m = *(const f32x4*)&sm[0][qi * 4], is = *(const f32x4*)&sm[1][qi * 4];
  const f32x4 b = *(const f32x4*)(beta + group * beta_gs + c);
#pragma unroll 4
  for (long long r = r0 + rl; r < r1; r += RL) {
    f32x4 y = bn_y(pf_ld4(pre, r * ldp + c, PB), m, is, b);
    if (res) y += *(const f32x4*)(res + r * ldr + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) y[e] = act_f(y[e], act);
    const long long o = group * out_gs + r * ldo + c;
    if (out_bf16)  // read only by bf16 GEMMs, which round it the same way while staging
      st_out8((__bf16*)out + o, __builtin_bit_cast(u64, __builtin_convertvector(y, bf16x4_bn)));
    else
      st_out16(out, o, y);
  }
}

void bn_apply(const float* pre, int ldp, long long pre_gs, long long rows, int C, const u64* acc, long long acc_gs,
              long long sh, int nsh, float eps, float* mean, float* invstd, long long ms_gs, const float* beta, long long beta_gs,
              const float* res, int ldr, long long res_gs, int act, float* out, int ldo, long long out_gs, int groups,
              hipStream_t s, int out_bf16, int pre_bf16) {
  if (out_bf16 && bn_w8() && C % 8 == 0 && ldo % 8 == 0 && out_gs % 8 == 0 && ((uintptr_t)out & 15) == 0) {
    const ApGrid g = ap_grid(rows, C, groups, 8);
    if (pre_bf16)
      hipLaunchKernelGGL((bn_apply_kernel<8, true>), g.grid, dim3(256), 0, s, pre, ldp, pre_gs, rows, C, acc, acc_gs, sh, nsh,
                         eps, mean, invstd, ms_gs, beta, beta_gs, res, ldr, res_gs, act, out, ldo, out_gs, g.rpb, out_bf16);
    else
      hipLaunchKernelGGL((bn_apply_kernel<8, false>), g.grid, dim3(256), 0, s, pre, ldp, pre_gs, rows, C, acc, acc_gs, sh, nsh,
                         eps, mean, invstd, ms_gs, beta, beta_gs, res, ldr, res_gs, act, out, ldo, out_gs, g.rpb, out_bf16);
    return;
  }
  const ApGrid g = ap_grid(rows, C, groups);
  if (pre_bf16)
    hipLaunchKernelGGL((bn_apply_kernel<4, true>), g.grid, dim3(256), 0, s, pre, ldp, pre_gs, rows, C, acc, acc_gs, sh, nsh,
                       eps, mean, invstd, ms_gs, beta, beta_gs, res, ldr, res_gs, act, out, ldo, out_gs, g.rpb, out_bf16);
  else
    hipLaunchKernelGGL((bn_apply_kernel<4, false>), g.grid, dim3(256), 0, s, pre, ldp, pre_gs, rows, C, acc, acc_gs, sh, nsh,
                       eps, mean, invstd, ms_gs, beta, beta_gs, res, ldr, res_gs, act, out, ldo, out_gs, g.rpb, out_bf16);
}

// Statistics finalised ONCE per BN layer (svae_ctx::bnfin): one thread per channel sums the accumulator
// shards and writes what every apply block would otherwise compute from its own gather (the same fp64
// expressions: bitwise the per-block path).  The apply passes then read two floats per channel.
// Forward: mean, invstd.  Backward: ab = [a = mean(dz) | b = mean(dz xhat)] per group, and dbeta.
__global__ __launch_bounds__(256) void bn_fin_kernel(const u64* acc, long long acc_gs, long long sh, int nsh,
                                                     long long rows, int C, float eps, float* mean, float* invstd,
                                                     long long ms_gs, float* ab, float* dbeta, long long dbeta_gs) {
  const int c = blockIdx.x * 256 + threadIdx.x, group = blockIdx.y;
  if (c >= C) return;
  const u64* base = acc + group * acc_gs + 4LL * c;
  u64 t[4] = {0, 0, 0, 0};
  for (int k = 0; k < nsh; ++k)
#pragma unroll
    for (int w = 0; w < 4; ++w) t[w] += base[k * sh + w];
  const double cnt = (double)rows;
  if (ab) {  // backward (bn_bwd_apply_kernel's expressions)
    const double sd = fx_get(t), sx = fx_get(t + 2);
    ab[group * 2LL * C + c] = (float)(sd / cnt);
    ab[group * 2LL * C + C + c] = (float)(sx / cnt);
    if (dbeta) dbeta[group * dbeta_gs + c] = (float)sd;
    return;
  }
  const double md = fx_get(t) / cnt;  // (bn_apply_kernel's expressions)
  double var = fx_get(t + 2) / cnt - md * md;
  if (var < 0.0) var = 0.0;
  mean[group * ms_gs + c] = (float)md;
  invstd[group * ms_gs + c] = (float)(1.0 / sqrt(var + (double)eps));
}

void bn_finalize(const u64* acc, long long acc_gs, long long sh, int nsh, long long rows, int C, float eps, float* mean,
                 float* invstd, long long ms_gs, float* ab, float* dbeta, long long dbeta_gs, int groups, hipStream_t s) {
  hipLaunchKernelGGL(bn_fin_kernel, dim3((C + 255) / 256, groups), dim3(256), 0, s, acc, acc_gs, sh, nsh, rows, C, eps,
                     mean, invstd, ms_gs, ab, dbeta, dbeta_gs);
}

#define BWD_RPB 256  // rows per row-block of the backward reduction
int bn_bwd_rowblocks(long long rows) { return (int)((rows + BWD_RPB - 1) / BWD_RPB); }

// y == nullptr: act' from the recomputed pre-activation bn_y(pre) (layers without a shortcut add)
template <bool PB, bool YB>
__global__ void bn_bwd_reduce_kernel(const float* dy, int lddy, long long dy_gs, const float* y, int ldy,
                                     long long y_gs, const float* pre, int ldp, long long pre_gs, long long rows,
                                     int C, const float* mean, const float* invstd, long long ms_gs, const float* beta,
                                     long long beta_gs, int act, u64* acc, long long acc_gs, long long sh,
                                     int nsh) {
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
  if (y) y = pf_at(y, group * y_gs, YB);
  pre = pf_at(pre, group * pre_gs, PB);
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
      const f32x4 xp = pf_ld4(pre, r * ldp + c, PB);
      f32x4 yy = y ? pf_ld4(y, r * ldy + c, YB) : bn_y(xp, m, is, bb);
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
  // one (channel, sum|sum*xhat) per thread, row lanes combined in a fixed order
  if (tid < 8 * QB) {
    const int cc = tid % (4 * QB), kind = tid / (4 * QB), qq = cc >> 2, e = cc & 3;
    const int q2 = blockIdx.x * QB + qq;
    if (q2 < Q) {
      float v = 0.f;
      for (int j = 0; j < RL; ++j) v += red[kind][j * QB + qq][e];
      fx_add(acc + (blockIdx.y & (nsh - 1)) * sh + group * acc_gs + 4LL * (q2 * 4 + e) + 2 * kind, v);
    }
  }
}

void bn_bwd_reduce(const float* dy, int lddy, long long dy_gs, const float* y, int ldy, long long y_gs,
                   const float* pre, int ldp, long long pre_gs, long long rows, int C, const float* mean,
                   const float* invstd, long long ms_gs, const float* beta, long long beta_gs, int act, u64* acc,
                   long long acc_gs, long long sh, int nsh, int groups, hipStream_t s, int pre_bf16, int y_bf16) {
  const int Q = C / 4;
  const int QB = Q < 16 ? Q : 16;
  dim3 grid((Q + QB - 1) / QB, (unsigned)bn_bwd_rowblocks(rows), groups);
#define BWR_LAUNCH(PB_, YB_)                                                                                 \
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<PB_, YB_>), grid, dim3(256), 0, s, dy, lddy, dy_gs, y, ldy, y_gs, pre, ldp, \
                     pre_gs, rows, C, mean, invstd, ms_gs, beta, beta_gs, act, acc, acc_gs, sh, nsh)
  const bool yb = y && y_bf16;
  if (pre_bf16) {
    if (yb) BWR_LAUNCH(true, true);
    else BWR_LAUNCH(true, false);
  } else {
    if (yb) BWR_LAUNCH(false, true);
    else BWR_LAUNCH(false, false);
  }
#undef BWR_LAUNCH
}

// W = 8 (bf16 dpre, C % 8 == 0): 8 channels per thread, one 16-byte bf16 store per row
template <int W, bool PB, bool YB>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const float* dy, int lddy, long long dy_gs, const float* y, int ldy, long long y_gs, const float* pre, int ldp,
    long long pre_gs, long long rows, int C, const float* mean, const float* invstd, long long ms_gs,
    const float* beta, long long beta_gs, const u64* acc, long long acc_gs, long long sh, int nsh, float* dbeta,
    long long dbeta_gs, int act,
    float* dpre, int lddp, long long dpre_gs, float* dres, int ldres, long long dres_gs, int res_acc, int rpb,
    int dpre_bf16, const float* ab) {
  __shared__ __attribute__((aligned(16))) float sm[2][AP_QB * 4];
  __shared__ u64 tot[4 * AP_QB * 4];
  const int group = blockIdx.z;
  const int Q = C / W;
  const int QB = Q < AP_QB * 4 / W ? Q : AP_QB * 4 / W;
  const int RL = 256 / QB;
  const int tid = threadIdx.x, qi = tid % QB, rl = tid / QB;
  const int q0 = blockIdx.x * QB;
  const int nch = min(QB * W, C - q0 * W);
  if (ab) {  // finalised by the producer's last block (BnFin mode 1; dbeta written there)
    if (tid < nch) {
      const int c = q0 * W + tid;
      sm[0][tid] = ab[group * 2LL * C + c];
      sm[1][tid] = ab[group * 2LL * C + C + c];
    }
  } else {
    acc_gather(acc + group * acc_gs, sh, nsh, q0 * W, nch, tot);
  }
  if (tid < nch && !ab) {
    const int c = q0 * W + tid;
    {
      const double sd = fx_get(tot + 4 * tid), sx = fx_get(tot + 4 * tid + 2);
      sm[0][tid] = (float)(sd / (double)rows);  // a = mean(dz)
      sm[1][tid] = (float)(sx / (double)rows);  // b = mean(dz*xhat)
      if (blockIdx.y == 0 && dbeta) dbeta[group * dbeta_gs + c] = (float)sd;
    }
  }
  __syncthreads();
  const int q = q0 + qi;
  if (rl >= RL || q >= Q) return;
  const int c = q * W;
  dy += group * dy_gs;
  if (y) y = pf_at(y, group * y_gs, YB);
  pre = pf_at(pre, group * pre_gs, PB);
  if (dres) dres += group * dres_gs;
  if constexpr (W == 8) {  // (dpre_bf16)
    const long long r0 = (long long)blockIdx.y * rpb;
    const long long r1 = r0 + rpb < rows ? r0 + rpb : rows;
    f32x4 mm[2], iss[2], bbb[2], aa[2], bq[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      mm[h] = *(const f32x4*)(mean + group * ms_gs + c + 4 * h);
      iss[h] = *(const f32x4*)(invstd + group * ms_gs + c + 4 * h);
      bbb[h] = y ? f32x4{0.f, 0.f, 0.f, 0.f} : *(const f32x4*)(beta + group * beta_gs + c + 4 * h);
      aa[h] = *(const f32x4*)&sm[0][qi * 8 + 4 * h];
      bq[h] = *(const f32x4*)&sm[1][qi * 8 + 4 * h];
    }
#pragma unroll 2
    for (long long r = r0 + rl; r < r1; r += RL) {
      u64 u[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 g = *(const f32x4*)(dy + r * lddy + c + 4 * h);
        const f32x4 xp = pf_ld4(pre, r * ldp + c + 4 * h, PB);
        const f32x4 yy = y ? pf_ld4(y, r * ldy + c + 4 * h, YB) : bn_y(xp, mm[h], iss[h], bbb[h]);
        const f32x4 xh = (xp - mm[h]) * iss[h];
        f32x4 dz;
#pragma unroll
        for (int e = 0; e < 4; ++e) dz[e] = g[e] * dact_from_y(yy[e], act);
        const f32x4 dp = iss[h] * (dz - aa[h] - xh * bq[h]);
        u[h] = __builtin_bit_cast(u64, __builtin_convertvector(dp, bf16x4_bn));
        if (dres) {
          f32x4* d = (f32x4*)(dres + r * ldres + c + 4 * h);
          *d = res_acc ? *d + dz : dz;
        }
      }
      const f32x4 bits = {__uint_as_float((unsigned)u[0]), __uint_as_float((unsigned)(u[0] >> 32)),
                          __uint_as_float((unsigned)u[1]), __uint_as_float((unsigned)(u[1] >> 32))};
      st_out16(dpre, (group * dpre_gs + r * lddp + c) / 2, bits);
    }
    return;
  }
  const f32x4 m = *(const f32x4*)(mean + group * ms_gs + c), is = *(const f32x4*)(invstd + group * ms_gs + c);
  const f32x4 bb = y ? f32x4{0.f, 0.f, 0.f, 0.f} : *(const f32x4*)(beta + group * beta_gs + c);
  const f32x4 a = *(const f32x4*)&sm[0][qi * 4], b = *(const f32x4*)&sm[1][qi * 4];
  const long long r0 = (long long)blockIdx.y * rpb;
  const long long r1 = r0 + rpb < rows ? r0 + rpb : rows;
#pragma unroll 2
  for (long long r = r0 + rl; r < r1; r += RL) {
    const f32x4 g = *(const f32x4*)(dy + r * lddy + c);
    const f32x4 xp = pf_ld4(pre, r * ldp + c, PB);
    const f32x4 yy = y ? pf_ld4(y, r * ldy + c, YB) : bn_y(xp, m, is, bb);
    const f32x4 xh = (xp - m) * is;
    f32x4 dz;
#pragma unroll
    for (int e = 0; e < 4; ++e) dz[e] = g[e] * dact_from_y(yy[e], act);
    const f32x4 dp = is * (dz - a - xh * b);
    const long long o = group * dpre_gs + r * lddp + c;
    if (dpre_bf16)  // consumed only by bf16 GEMMs, which round it the same way while staging
      st_out8((__bf16*)dpre + o, __builtin_bit_cast(u64, __builtin_convertvector(dp, bf16x4_bn)));
    else
      st_out16(dpre, o, dp);
    if (dres) {
      f32x4* d = (f32x4*)(dres + r * ldres + c);
      *d = res_acc ? *d + dz : dz;
    }
  }
}

void bn_bwd_apply(const float* dy, int lddy, long long dy_gs, const float* y, int ldy, long long y_gs,
                  const float* pre, int ldp, long long pre_gs, long long rows, int C, const float* mean,
                  const float* invstd, long long ms_gs, const float* beta, long long beta_gs, const u64* acc,
                  long long acc_gs, long long sh, int nsh, float* dbeta, long long dbeta_gs, int act, float* dpre, int lddp,
                  long long dpre_gs, float* dres, int ldres, long long dres_gs, int res_acc, int groups,
                  hipStream_t s, int dpre_bf16, int pre_bf16, const float* ab, int y_bf16) {
  const bool yb = y && y_bf16;
#define BWA_ONE(W_, PB_, YB_, G_)                                                                                  \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<W_, PB_, YB_>), G_.grid, dim3(256), 0, s, dy, lddy, dy_gs, y, ldy, y_gs, pre, \
                     ldp, pre_gs, rows, C, mean, invstd, ms_gs, beta, beta_gs, acc, acc_gs, sh, nsh, dbeta, dbeta_gs, act, \
                     dpre, lddp, dpre_gs, dres, ldres, dres_gs, res_acc, G_.rpb, dpre_bf16, ab)
#define BWA_LAUNCH(W_, G_)                                                                                          \
  if (pre_bf16) {                                                                                                  \
    if (yb) BWA_ONE(W_, true, true, G_);                                                                           \
    else BWA_ONE(W_, true, false, G_);                                                                             \
  } else {                                                                                                         \
    if (yb) BWA_ONE(W_, false, true, G_);                                                                          \
    else BWA_ONE(W_, false, false, G_);                                                                            \
  }
  if (dpre_bf16 && bn_w8() && C % 8 == 0 && lddp % 8 == 0 && dpre_gs % 8 == 0 && ((uintptr_t)dpre & 15) == 0) {
    const ApGrid g = ap_grid(rows, C, groups, 8);
    BWA_LAUNCH(8, g)
    return;
  }
  const ApGrid g = ap_grid(rows, C, groups);
  BWA_LAUNCH(4, g)
#undef BWA_LAUNCH
#undef BWA_ONE
}
