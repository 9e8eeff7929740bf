#include <cstdlib>
// Implicit-GEMM convolution / FC kernels on CDNA4 MFMA (fp32 parity path).
//
// Every conv-like op of the hot path is one of two GEMM shapes:
//
//  gather-GEMM   C[p][n] = sum_{tap,k} A[src(p,tap)][k] * B[tap][k][n]
//     conv2d fwd (CONV, B=[kh,kw,Cin,Cout] = KN)       abstract_network.py:18
//     conv2d_transpose fwd (CONVT, B=[kh,kw,Cout,Cin] = NK)  abstract_network.py:37,56
//     conv dgrad = CONVT with the conv weights read NK; conv-T dgrad = CONV with KN
//     fully_connected fwd/dgrad (DENSE)                 abstract_network.py:65
//  weight-GEMM   dW[tap][m][n] = sum_p G[src(p,tap)][m] * D[p][n]   (split over p)
//
// Tiles: 256 threads = 4 waves, each wave a (TM*32)x(TN*32) block of
// v_mfma_f32_32x32x2_f32 accumulators (exact fp32 fma chains).  A/B tiles are
// gathered global->registers->LDS (double buffered, one barrier per K step).
// The epilogue optionally emits per-column partial (sum, sum^2) for the
// following training-mode BatchNorm, so BN statistics cost no extra HBM pass.
#include "common.h"
#include "knobs.h"
#include "kernels.h"

#define BK 32
#define LDS_PAD 4

namespace {

struct RowCoord {
  int img;   // n * Hi * Wi (pixel base of the image in the gathered operand)
  int y, x;  // output coordinate (class-adjusted for CONVT)
  int valid;
};

__device__ __forceinline__ void tap_of(const ConvGeom& g, int cls, int t, int& ky, int& kx) {
  if (g.mode == GM_CONVT && g.stride == 2) {
    int half = g.ksz >> 1;
    int py = cls >> 1, px = cls & 1;
    ky = ((py + g.pad) & 1) + 2 * (t / half);
    kx = ((px + g.pad) & 1) + 2 * (t % half);
  } else {
    ky = t / g.ksz;
    kx = t % g.ksz;
  }
}

__device__ __forceinline__ int ntaps_of(const ConvGeom& g) {
  if (g.mode == GM_DENSE) return 1;
  if (g.mode == GM_CONVT && g.stride == 2) return (g.ksz >> 1) * (g.ksz >> 1);
  return g.ksz * g.ksz;
}

// pixel index (within the gathered operand) for row coordinate + tap, or -1
__device__ __forceinline__ long long src_pixel(const ConvGeom& g, const RowCoord& rc, int ky, int kx) {
  if (!rc.valid) return -1;
  if (g.mode == GM_DENSE) return rc.img;
  int iy, ix;
  if (g.mode == GM_CONV) {
    iy = rc.y * g.stride - g.pad + ky;
    ix = rc.x * g.stride - g.pad + kx;
  } else {
    iy = rc.y + g.pad - ky;
    ix = rc.x + g.pad - kx;
    if (g.stride == 2) { iy >>= 1; ix >>= 1; }  // exact: parity class guarantees even
  }
  if (iy < 0 || iy >= g.Hi || ix < 0 || ix >= g.Wi) return -1;
  return (long long)rc.img + (long long)iy * g.Wi + ix;
}

__device__ __forceinline__ RowCoord row_coord(const ConvGeom& g, int cls, int m, int rows) {
  RowCoord rc;
  rc.valid = m < rows;
  if (!rc.valid) { rc.img = rc.y = rc.x = 0; return rc; }
  if (g.mode == GM_DENSE) { rc.img = m; rc.y = rc.x = 0; return rc; }
  int Ho = g.Ho, Wo = g.Wo;
  if (g.mode == GM_CONVT && g.stride == 2) {
    int qh = Ho >> 1, qw = Wo >> 1;
    int n = m / (qh * qw);
    int r = m - n * qh * qw;
    int qy = r / qw, qx = r - (r / qw) * qw;
    rc.y = 2 * qy + (cls >> 1);
    rc.x = 2 * qx + (cls & 1);
    rc.img = n * g.Hi * g.Wi;
  } else {
    int n = m / (Ho * Wo);
    int r = m - n * Ho * Wo;
    rc.y = r / Wo;
    rc.x = r - rc.y * Wo;
    rc.img = n * g.Hi * g.Wi;
  }
  return rc;
}

__device__ __forceinline__ long long out_row(const ConvGeom& g, int cls, int m) {
  if (g.mode == GM_CONVT && g.stride == 2) {
    int qh = g.Ho >> 1, qw = g.Wo >> 1;
    int n = m / (qh * qw);
    int r = m - n * qh * qw;
    int qy = r / qw, qx = r - (r / qw) * qw;
    return ((long long)n * g.Ho + 2 * qy + (cls >> 1)) * g.Wo + 2 * qx + (cls & 1);
  }
  return m;
}

}  // namespace

// ---------------------------------------------------------------------------
// gather-GEMM forward
// ---------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN, bool B_NK, bool SMALLC>
__global__ __launch_bounds__(256) void igemm_fwd_kernel(FwdArgs a) {
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  constexpr int RA = BM / 32;                 // float4 A loads per thread
  constexpr int RB = BN / 32;                 // float4 B loads per thread
  constexpr int AS = BK + LDS_PAD;            // A row stride (floats)
  constexpr int BS_NK = BK + LDS_PAD;
  constexpr int BS_KN = BN + LDS_PAD;
  constexpr int BSZ = B_NK ? BN * BS_NK : BK * BS_KN;
  __shared__ __attribute__((aligned(16))) float As[2][BM * AS];
  __shared__ __attribute__((aligned(16))) float Bs[2][BSZ];

  const ConvGeom& g = a.g;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int wm0 = (wave / WN) * (TM * 32), wn0 = (wave % WN) * (TN * 32);
  const int group = blockIdx.z / a.nclass, cls = blockIdx.z - group * a.nclass;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;

  const float* A = a.A + group * a.a_gs;
  const float* Bw = a.B + group * a.b_gs;

  const int ntap = ntaps_of(g);
  const int Ktot = ntap * a.Cin;
  const int nk = SMALLC ? (Ktot + BK - 1) / BK : ntap * (a.Cin / BK);
  const int kq = (tid & 7) * 4;

  RowCoord rc[RA];
#pragma unroll
  for (int i = 0; i < RA; ++i) rc[i] = row_coord(g, cls, m0 + (tid >> 3) + 32 * i, a.rows);

  f32x4 ra[RA], rb[RB];

  auto load_tile = [&](int kc) {
    if (!SMALLC) {
      const int cpt = a.Cin / BK;
      const int t = kc / cpt;
      const int ci0 = (kc - t * cpt) * BK;
      int ky, kx;
      tap_of(g, cls, t, ky, kx);
#pragma unroll
      for (int i = 0; i < RA; ++i) {
        long long sp = src_pixel(g, rc[i], ky, kx);
        if (sp >= 0) ra[i] = *(const f32x4*)(A + sp * a.lda + ci0 + kq);
        else ra[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      const float* Bt = Bw + (long long)(ky * g.ksz + kx) * a.b_tap;
      if (g.mode == GM_DENSE) Bt = Bw;
      if (B_NK) {
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          int n = n0 + (tid >> 3) + 32 * i;
          rb[i] = n < a.N ? *(const f32x4*)(Bt + (long long)n * a.ldb + ci0 + kq) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      } else {
        constexpr int QN = BN / 4;
        constexpr int KSTEP = 256 / QN;
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          int kk = tid / QN + KSTEP * i;
          int n = n0 + (tid % QN) * 4;
          rb[i] = n < a.N ? *(const f32x4*)(Bt + (long long)(ci0 + kk) * a.ldb + n) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    } else {
      // generic element-wise gather (Cin not a multiple of BK: first layers, tiny test nets)
#pragma unroll
      for (int i = 0; i < RA; ++i) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          int k = kc * BK + kq + e;
          float v = 0.f;
          if (k < Ktot) {
            int t = k / a.Cin, ci = k - t * a.Cin;
            int ky, kx;
            tap_of(g, cls, t, ky, kx);
            long long sp = src_pixel(g, rc[i], ky, kx);
            if (sp >= 0) v = A[sp * a.lda + ci];
          }
          ra[i][e] = v;
        }
      }
      if (B_NK) {
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          int n = n0 + (tid >> 3) + 32 * i;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            int k = kc * BK + kq + e;
            float v = 0.f;
            if (k < Ktot && n < a.N) {
              int t = k / a.Cin, ci = k - t * a.Cin;
              int ky, kx;
              tap_of(g, cls, t, ky, kx);
              long long tg = g.mode == GM_DENSE ? 0 : (ky * g.ksz + kx);
              v = Bw[tg * a.b_tap + (long long)n * a.ldb + ci];
            }
            rb[i][e] = v;
          }
        }
      } else {
        constexpr int QN = BN / 4;
        constexpr int KSTEP = 256 / QN;
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          int kk = tid / QN + KSTEP * i;
          int n = n0 + (tid % QN) * 4;
          int k = kc * BK + kk;
          f32x4 v = {0.f, 0.f, 0.f, 0.f};
          if (k < Ktot && n < a.N) {
            int t = k / a.Cin, ci = k - t * a.Cin;
            int ky, kx;
            tap_of(g, cls, t, ky, kx);
            long long tg = g.mode == GM_DENSE ? 0 : (ky * g.ksz + kx);
            v = *(const f32x4*)(Bw + tg * a.b_tap + (long long)ci * a.ldb + n);
          }
          rb[i] = v;
        }
      }
    }
  };

  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < RA; ++i) *(f32x4*)&As[buf][((tid >> 3) + 32 * i) * AS + kq] = ra[i];
    if (B_NK) {
#pragma unroll
      for (int i = 0; i < RB; ++i) *(f32x4*)&Bs[buf][((tid >> 3) + 32 * i) * BS_NK + kq] = rb[i];
    } else {
      constexpr int QN = BN / 4;
      constexpr int KSTEP = 256 / QN;
#pragma unroll
      for (int i = 0; i < RB; ++i) *(f32x4*)&Bs[buf][(tid / QN + KSTEP * i) * BS_KN + (tid % QN) * 4] = rb[i];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  load_tile(0);
  store_tile(0);
  __syncthreads();

  for (int kc = 0; kc < nk; ++kc) {
    const int cur = kc & 1;
    if (kc + 1 < nk) load_tile(kc + 1);
#pragma unroll
    for (int ks = 0; ks < BK / 8; ++ks) {
      f32x4 af[TM], bf[TN];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) af[tm] = *(const f32x4*)&As[cur][(wm0 + tm * 32 + l32) * AS + ks * 8 + 4 * h];
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        if (B_NK) {
          bf[tn] = *(const f32x4*)&Bs[cur][(wn0 + tn * 32 + l32) * BS_NK + ks * 8 + 4 * h];
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) bf[tn][j] = Bs[cur][(ks * 8 + 4 * h + j) * BS_KN + wn0 + tn * 32 + l32];
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn)
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[tm][j], bf[tn][j], acc[tm][tn], 0, 0, 0);
    }
    if (kc + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
  }

  // ------------------------------------------------------------------ epilogue
  float* Cp = a.C + group * a.c_gs;
  const float* bias = a.bias ? a.bias + group * a.bias_gs : nullptr;
  float csum[TN], csq[TN];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) { csum[tn] = 0.f; csq[tn] = 0.f; }
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + wm0 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (m >= a.rows) continue;
      const long long orow = out_row(g, cls, m);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int n = n0 + wn0 + tn * 32 + l32;
        if (n >= a.N) continue;
        float v = acc[tm][tn][r];
        csum[tn] += v;
        csq[tn] += v * v;
        if (bias) v += bias[n];
        v = act_f(v, a.act);
        float* dst = Cp + orow * a.ldc + n;
        if (a.accumulate) v += *dst;
        *dst = v;
      }
    }
  }
  if (a.stats) {
    // per-column partial (sum, sum^2) of this block's valid rows -> fixed-point accumulators
    float* red = &As[0][0];  // reuse: [WM][BN] sums then [WM][BN] squares
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      csum[tn] += __shfl_xor(csum[tn], 32, 64);
      csq[tn] += __shfl_xor(csq[tn], 32, 64);
    }
    __syncthreads();
    if (h == 0) {
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        red[(wave / WN) * BN + wn0 + tn * 32 + l32] = csum[tn];
        red[WM * BN + (wave / WN) * BN + wn0 + tn * 32 + l32] = csq[tn];
      }
    }
    __syncthreads();
    if (tid < BN) {
      const int n = n0 + tid;
      if (n < a.N) {
        float s = 0.f, q = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) { s += red[w * BN + tid]; q += red[WM * BN + w * BN + tid]; }
        const int rb = cls * gridDim.x + blockIdx.x;
        stat_put(a.stats + (rb & (a.s_nsh - 1)) * a.s_sh + group * a.s_gs, n, s, q);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// weight-gradient GEMM: part[split][tap][m][n] = sum_{p in split} G[src(p,tap)][m] * D[p][n]
// ---------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN, bool VECG>
__global__ __launch_bounds__(256) void wgrad_kernel(WgArgs a) {
  static_assert(WM * WN == 4, "4 waves");
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  static_assert(TM >= 1 && TN >= 1, "tile");
  constexpr int ASx = BM + LDS_PAD, BSx = BN + LDS_PAD;
  constexpr int QM = BM / 4, QN = BN / 4;
  constexpr int KSA = 256 / QM, KSB = 256 / QN;
  constexpr int RA = BK / KSA, RB = BK / KSB;
  __shared__ __attribute__((aligned(16))) float As[2][BK * ASx];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK * BSx];

  const ConvGeom& g = a.g;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int wm0 = (wave / WN) * (TM * 32), wn0 = (wave % WN) * (TN * 32);
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  int z = blockIdx.z;
  const int split = z % a.nsplit; z /= a.nsplit;
  const int tap = z % a.ntap;
  const int group = z / a.ntap;
  const int ky = tap / g.ksz, kx = tap - (tap / g.ksz) * g.ksz;

  const float* G = a.G + group * a.g_gs;
  const float* D = a.D + group * a.d_gs;
  const int p_begin = split * a.chunk;
  const int p_end = min(a.rows, p_begin + a.chunk);
  const int nk = (p_end - p_begin + BK - 1) / BK;

  f32x4 ra[RA], rb[RB];
  auto load_tile = [&](int kc) {
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      const int kk = tid / QM + KSA * i;
      const int mq = m0 + (tid % QM) * 4;
      const int p = p_begin + kc * BK + kk;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (p < p_end) {
        RowCoord rc = row_coord(g, 0, p, a.rows);
        long long sp = src_pixel(g, rc, ky, kx);
        if (sp >= 0) {
          const float* src = G + sp * a.ldg + mq;
          if (VECG) {
            if (mq < a.M) v = *(const f32x4*)src;
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = (mq + e < a.M) ? src[e] : 0.f;
          }
        }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int kk = tid / QN + KSB * i;
      const int nq = n0 + (tid % QN) * 4;
      const int p = p_begin + kc * BK + kk;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (p < p_end && nq < a.N) v = *(const f32x4*)(D + (long long)p * a.ldd + nq);
      rb[i] = v;
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < RA; ++i) *(f32x4*)&As[buf][(tid / QM + KSA * i) * ASx + (tid % QM) * 4] = ra[i];
#pragma unroll
    for (int i = 0; i < RB; ++i) *(f32x4*)&Bs[buf][(tid / QN + KSB * i) * BSx + (tid % QN) * 4] = rb[i];
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (nk > 0) {
    load_tile(0);
    store_tile(0);
  }
  __syncthreads();
  for (int kc = 0; kc < nk; ++kc) {
    const int cur = kc & 1;
    if (kc + 1 < nk) load_tile(kc + 1);
#pragma unroll
    for (int ks = 0; ks < BK / 8; ++ks) {
      float af[TM][4], bf[TN][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) af[tm][j] = As[cur][(ks * 8 + 4 * h + j) * ASx + wm0 + tm * 32 + l32];
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) bf[tn][j] = Bs[cur][(ks * 8 + 4 * h + j) * BSx + wn0 + tn * 32 + l32];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn)
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[tm][j], bf[tn][j], acc[tm][tn], 0, 0, 0);
    }
    if (kc + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
  }

  // partial slab: part[group][split][tap][m][n]
  float* P = a.part + group * a.p_gs + ((long long)split * a.ntap + tap) * (long long)a.M * a.N;
#pragma unroll
  for (int tm = 0; tm < TM; ++tm)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + wm0 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (m >= a.M) continue;
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int n = n0 + wn0 + tn * 32 + l32;
        if (n < a.N) P[(long long)m * a.N + n] = acc[tm][tn][r];
      }
    }
}

// sum the split slabs: out[tap][m][n] (rows m < msplit -> out0, else out1)
__device__ __forceinline__ float* wred_dst(float* out0, long long o0_gs, int msplit, float* out1, long long o1_gs,
                                           int group, int tap, int M, int m, int N, int n) {
  if (m < msplit) return out0 + group * o0_gs + ((long long)tap * msplit + m) * N + n;
  if (!out1) return nullptr;  // rows routed to an absent second output are dropped
  return out1 + group * o1_gs + ((long long)tap * (M - msplit) + (m - msplit)) * N + n;
}

// out[tap][m][n] (= or +=) sum_sp part[group][sp][tap][m][n], summed in split order (deterministic).
// VEC: 4 consecutive n per thread (N % 4 == 0), four independent partial sums over the splits.
// out[tap][m][n] (= or +=) sum_sp part[group][sp][tap][m][n].  A block is QB float4 columns x
// SL split lanes (QB*SL = 256): split lane l sums splits l, l+SL, ... with two partial sums,
// then the SL partials are combined in LDS in lane order -- a fixed order, so deterministic.
template <int SL>
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* part, long long p_gs, int nsplit, int ntap,
                                                           int M, int N, float* out0, long long o0_gs, int msplit,
                                                           float* out1, long long o1_gs, int accumulate) {
  constexpr int QB = 256 / SL;
  __shared__ f32x4 red[SL][QB];
  const int group = blockIdx.y;
  const long long per = (long long)ntap * M * N;
  const int ql = threadIdx.x % QB, sl = threadIdx.x / QB;
  const long long q = (long long)blockIdx.x * QB + ql;
  const bool ok = q * 4 < per;
  const float* p = part + group * p_gs + (ok ? q * 4 : 0);
  f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0;
  int sp = sl;
  for (; sp + SL < nsplit; sp += 2 * SL) {
    s0 += *(const f32x4*)(p + sp * per);
    s1 += *(const f32x4*)(p + (sp + SL) * per);
  }
  if (sp < nsplit) s0 += *(const f32x4*)(p + sp * per);
  red[sl][ql] = s0 + s1;
  __syncthreads();
  if (sl != 0 || !ok) return;
  f32x4 s = red[0][ql];
#pragma unroll
  for (int l = 1; l < SL; ++l) s += red[l][ql];
  const long long i = q * 4;
  const int tap = (int)(i / ((long long)M * N));
  const int rem = (int)(i - (long long)tap * M * N);
  const int m = rem / N, n = rem - m * N;
  float* dst = wred_dst(out0, o0_gs, msplit, out1, o1_gs, group, tap, M, m, N, n);
  if (!dst) return;
  if (accumulate) s += *(const f32x4*)dst;
  *(f32x4*)dst = s;
}

__global__ void wgrad_reduce_scalar_kernel(const float* part, long long p_gs, int nsplit, int ntap, int M, int N,
                                           float* out0, long long o0_gs, int msplit, float* out1, long long o1_gs,
                                           int accumulate) {
  const int group = blockIdx.y;
  const long long per = (long long)ntap * M * N;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < per; i += (long long)gridDim.x * blockDim.x) {
    const float* p = part + group * p_gs + i;
    float s = 0.f;
    for (int sp = 0; sp < nsplit; ++sp) s += p[sp * per];
    const int tap = (int)(i / ((long long)M * N));
    const int rem = (int)(i - (long long)tap * M * N);
    const int m = rem / N, n = rem - m * N;
    float* dst = wred_dst(out0, o0_gs, msplit, out1, o1_gs, group, tap, M, m, N, n);
    if (!dst) continue;
    *dst = accumulate ? *dst + s : s;
  }
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN, bool NK, bool SC>
static void launch_fwd(const FwdArgs& a, int groups, hipStream_t s) {
  FwdArgs b = a;
  b.mtiles = (a.rows + BM - 1) / BM;
  dim3 grid(b.mtiles, (a.N + BN - 1) / BN, groups * a.nclass);
  hipLaunchKernelGGL((igemm_fwd_kernel<BM, BN, WM, WN, NK, SC>), grid, dim3(256), 0, s, b);
}

template <int BM, int BN, int WM, int WN>
static void dispatch_fwd_nk(const FwdArgs& a, int groups, bool nk, bool sc, hipStream_t s) {
  if (nk) {
    if (sc) launch_fwd<BM, BN, WM, WN, true, true>(a, groups, s);
    else launch_fwd<BM, BN, WM, WN, true, false>(a, groups, s);
  } else {
    if (sc) launch_fwd<BM, BN, WM, WN, false, true>(a, groups, s);
    else launch_fwd<BM, BN, WM, WN, false, false>(a, groups, s);
  }
}

int igemm_fwd_bm(const FwdArgs& a) {
  // must mirror the tile choice in igemm_fwd (stats partial row-block count)
  if (smallc_ok(a, false)) return smallc_bm();  // smallc.hip pixel blocks
  int N = a.N;
  long long rows = (long long)a.rows * a.nclass;
  if (N <= 32) return 256;
  if (N <= 64) return 128;
  if (rows >= 16384) return 128;
  return 64;
}

void igemm_fwd(FwdArgs a, int groups, hipStream_t s) {
  if (smallc_ok(a, false)) {
    conv_smallc(a, groups, false, s);
    return;
  }
  const bool nk = a.b_nk != 0;
  const bool sc = (a.Cin % BK) != 0;
  const int bm = igemm_fwd_bm(a);
  if (a.N <= 32) dispatch_fwd_nk<256, 32, 4, 1>(a, groups, nk, sc, s);
  else if (a.N <= 64) dispatch_fwd_nk<128, 64, 2, 2>(a, groups, nk, sc, s);
  else if (bm == 128) dispatch_fwd_nk<128, 128, 2, 2>(a, groups, nk, sc, s);
  else dispatch_fwd_nk<64, 128, 1, 4>(a, groups, nk, sc, s);
}

template <int BM, int BN, int WM, int WN>
static void launch_wg(const WgArgs& a, int groups, bool vec, hipStream_t s) {
  dim3 grid((a.M + BM - 1) / BM, (a.N + BN - 1) / BN, groups * a.ntap * a.nsplit);
  if (vec) hipLaunchKernelGGL((wgrad_kernel<BM, BN, WM, WN, true>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((wgrad_kernel<BM, BN, WM, WN, false>), grid, dim3(256), 0, s, a);
}

void wgrad(WgArgs a, int groups, hipStream_t s) {
  const bool vec = (a.M % 4 == 0) && (a.ldg % 4 == 0);
  if (a.M <= 32) launch_wg<32, 128, 1, 4>(a, groups, vec, s);
  else if (a.N <= 32) launch_wg<128, 32, 4, 1>(a, groups, vec, s);
  else if (a.M >= 128 && a.N >= 128) launch_wg<128, 128, 2, 2>(a, groups, vec, s);
  else launch_wg<64, 64, 2, 2>(a, groups, vec, s);
}

void wgrad_reduce(const float* part, long long p_gs, int nsplit, int ntap, int M, int N, float* out0, long long o0_gs,
                  int msplit, float* out1, long long o1_gs, int accumulate, int groups, hipStream_t s) {
  long long per = (long long)ntap * M * N;
  const bool vec = (N % 4 == 0) && (p_gs % 4 == 0) && (o0_gs % 4 == 0) && (o1_gs % 4 == 0);
  if (!vec) {
    int blocks = (int)std::min<long long>((per + 255) / 256, 8192);
    hipLaunchKernelGGL(wgrad_reduce_scalar_kernel, dim3(blocks, groups), dim3(256), 0, s, part, p_gs, nsplit, ntap, M,
                       N, out0, o0_gs, msplit, out1, o1_gs, accumulate);
    return;
  }
  const long long nq = per / 4;
  // split lanes: enough blocks to stream the slab at full bandwidth even for small outputs
  // SVAE_WRED_SLMAX / SVAE_WRED_BLOCKS: split-lane cap and block target (A/B knobs)
  static const int sl_max = svae_knob("SVAE_WRED_SLMAX", 16);
  static const int blk_target = svae_knob("SVAE_WRED_BLOCKS", 1024);
  int sl = 1;
  while (sl < sl_max && sl < nsplit && (nq * sl) / 256 * groups < blk_target) sl *= 4;
  const int qb = 256 / sl;
  dim3 grid((unsigned)((nq + qb - 1) / qb), groups);
#define WRED(SLV)                                                                                                    \
  hipLaunchKernelGGL(wgrad_reduce_kernel<SLV>, grid, dim3(256), 0, s, part, p_gs, nsplit, ntap, M, N, out0, o0_gs, \
                     msplit, out1, o1_gs, accumulate)
  if (sl == 1) WRED(1);
  else if (sl == 4) WRED(4);
  else if (sl == 16) WRED(16);
  else WRED(64);
#undef WRED
}
