// bf16-MFMA implicit-GEMM kernels (throughput mode, dtype=1).
//
// Same two GEMM shapes as gemm.hip (gather-GEMM for conv / conv-T / FC forward and
// input-gradient; weight-GEMM for weight gradients) on v_mfma_f32_32x32x16_bf16 with fp32
// accumulation.  Activations stay fp32 in HBM and are rounded to bf16 while they are
// staged into LDS; weights come from bf16 "shadow" copies (both N and T layouts,
// refreshed from the fp32 master once per step) so every B tile is a 16-byte row load.
// LDS tiles are [row][k] bf16 with an 80-byte row pitch (conflict-free ds_read_b128 of
// the 8-element k fragments).  Weight-GEMM operands are pixel-major in HBM and are
// transposed in registers (4 pixels x 4 channels -> 4 x ds_write_b64).
#include "common.h"
#include "kernels.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));

#define BKB 32     // k per LDS stage (2 MFMA k-steps of 16)
#define ROWP 40    // LDS row pitch in bf16 (80 B)

namespace {

struct RowCoordB {
  int img, y, x, valid;
};

__device__ __forceinline__ void tap_of_b(const ConvGeom& g, int cls, int t, int& ky, int& kx) {
  if (g.mode == GM_CONVT && g.stride == 2) {
    int half = g.ksz >> 1;
    ky = (((cls >> 1) + g.pad) & 1) + 2 * (t / half);
    kx = (((cls & 1) + g.pad) & 1) + 2 * (t % half);
  } else {
    ky = t / g.ksz;
    kx = t % g.ksz;
  }
}
__device__ __forceinline__ int ntaps_of_b(const ConvGeom& g) {
  if (g.mode == GM_DENSE) return 1;
  if (g.mode == GM_CONVT && g.stride == 2) return (g.ksz >> 1) * (g.ksz >> 1);
  return g.ksz * g.ksz;
}
__device__ __forceinline__ long long src_pixel_b(const ConvGeom& g, const RowCoordB& rc, int ky, int kx) {
  if (!rc.valid) return -1;
  if (g.mode == GM_DENSE) return rc.img;
  int iy, ix;
  if (g.mode == GM_CONV) {
    iy = rc.y * g.stride - g.pad + ky;
    ix = rc.x * g.stride - g.pad + kx;
  } else {
    iy = rc.y + g.pad - ky;
    ix = rc.x + g.pad - kx;
    if (g.stride == 2) { iy >>= 1; ix >>= 1; }
  }
  if (iy < 0 || iy >= g.Hi || ix < 0 || ix >= g.Wi) return -1;
  return (long long)rc.img + (long long)iy * g.Wi + ix;
}
__device__ __forceinline__ RowCoordB row_coord_b(const ConvGeom& g, int cls, int m, int rows) {
  RowCoordB rc;
  rc.valid = m < rows;
  if (!rc.valid) { rc.img = rc.y = rc.x = 0; return rc; }
  if (g.mode == GM_DENSE) { rc.img = m; rc.y = rc.x = 0; return rc; }
  if (g.mode == GM_CONVT && g.stride == 2) {
    int qh = g.Ho >> 1, qw = g.Wo >> 1;
    int n = m / (qh * qw);
    int r = m - n * qh * qw;
    int qy = r / qw;
    rc.y = 2 * qy + (cls >> 1);
    rc.x = 2 * (r - qy * qw) + (cls & 1);
    rc.img = n * g.Hi * g.Wi;
  } else {
    int n = m / (g.Ho * g.Wo);
    int r = m - n * g.Ho * g.Wo;
    rc.y = r / g.Wo;
    rc.x = r - rc.y * g.Wo;
    rc.img = n * g.Hi * g.Wi;
  }
  return rc;
}
__device__ __forceinline__ long long out_row_b(const ConvGeom& g, int cls, int m) {
  if (g.mode == GM_CONVT && g.stride == 2) {
    int qh = g.Ho >> 1, qw = g.Wo >> 1;
    int n = m / (qh * qw);
    int r = m - n * qh * qw;
    int qy = r / qw, qx = r - (r / qw) * qw;
    return ((long long)n * g.Ho + 2 * qy + (cls >> 1)) * g.Wo + 2 * qx + (cls & 1);
  }
  return m;
}
__device__ __forceinline__ bf16x8 cvt8(f32x4 a, f32x4 b) {
  f32x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_convertvector(v, bf16x8);
}

}  // namespace

// ---------------------------------------------------------------------------
// gather-GEMM forward, bf16 MFMA.  A fp32 (gathered, converted), B bf16 NK [tap][n][k].
// ---------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN, bool SMALLC>
__global__ __launch_bounds__(256) void igemm_bf16_kernel(FwdArgs a) {
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  constexpr int CA = BM * 4;               // 8-k chunks per A tile
  constexpr int CB = BN * 4;
  constexpr int RA = (CA + 255) / 256;
  constexpr int RB = (CB + 255) / 256;
  __shared__ __attribute__((aligned(16))) __bf16 As[2][BM * ROWP];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[2][BN * ROWP];

  const ConvGeom& g = a.g;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int wm0 = (wave / WN) * (TM * 32), wn0 = (wave % WN) * (TN * 32);
  const int ks = a.ksplit;
  const BlockXYZ blk = xcd_block();
  const int split = blk.z % ks;
  const int zc = blk.z / ks;
  const int group = zc / a.nclass, cls = zc - group * a.nclass;
  const int m0 = blk.x * BM, n0 = blk.y * BN;
  const float* A = a.A + group * a.a_gs;
  const __bf16* Bw = (const __bf16*)a.Bh + group * a.b_gs;
  const int ntap = ntaps_of_b(g);
  const int Ktot = ntap * a.Cin;
  const int nk_all = SMALLC ? (Ktot + BKB - 1) / BKB : ntap * (a.Cin / BKB);
  const int kbeg = (int)((long long)nk_all * split / ks), kend = (int)((long long)nk_all * (split + 1) / ks);
  const int nk = kend - kbeg;
  const int k8 = (tid & 3) * 8;

  RowCoordB rc[RA];
#pragma unroll
  for (int i = 0; i < RA; ++i) rc[i] = row_coord_b(g, cls, m0 + (tid >> 2) + 64 * i, a.rows);

  bf16x8 ra[RA], rb[RB];
  const bf16x8 zero8 = {};

  auto load_tile = [&](int kc) {
    if (!SMALLC) {
      const int cpt = a.Cin / BKB;
      const int t = kc / cpt;
      const int ci0 = (kc - t * cpt) * BKB;
      int ky, kx;
      tap_of_b(g, cls, t, ky, kx);
#pragma unroll
      for (int i = 0; i < RA; ++i) {
        ra[i] = zero8;
        if (tid + 256 * i < CA) {
          long long sp = src_pixel_b(g, rc[i], ky, kx);
          if (sp >= 0) {
            const float* p = A + sp * a.lda + ci0 + k8;
            ra[i] = cvt8(*(const f32x4*)p, *(const f32x4*)(p + 4));
          }
        }
      }
      const __bf16* Bt = Bw + (g.mode == GM_DENSE ? 0LL : (long long)(ky * g.ksz + kx) * a.b_tap);
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        rb[i] = zero8;
        const int q = tid + 256 * i;
        const int n = n0 + (q >> 2);
        if (q < CB && n < a.N) rb[i] = *(const bf16x8*)(Bt + (long long)n * a.ldb + ci0 + k8);
      }
    } else {
#pragma unroll
      for (int i = 0; i < RA; ++i) {
        f32x8 v = {};
        if (tid + 256 * i < CA) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            int k = kc * BKB + k8 + e;
            if (k < Ktot) {
              int t = k / a.Cin, ci = k - t * a.Cin;
              int ky, kx;
              tap_of_b(g, cls, t, ky, kx);
              long long sp = src_pixel_b(g, rc[i], ky, kx);
              if (sp >= 0) v[e] = A[sp * a.lda + ci];
            }
          }
        }
        ra[i] = __builtin_convertvector(v, bf16x8);
      }
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        rb[i] = zero8;
        const int q = tid + 256 * i;
        const int n = n0 + (q >> 2);
        if (q < CB && n < a.N) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            int k = kc * BKB + k8 + e;
            if (k < Ktot) {
              int t = k / a.Cin, ci = k - t * a.Cin;
              int ky, kx;
              tap_of_b(g, cls, t, ky, kx);
              long long tg = g.mode == GM_DENSE ? 0 : (ky * g.ksz + kx);
              rb[i][e] = Bw[tg * a.b_tap + (long long)n * a.ldb + ci];
            }
          }
        }
      }
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < RA; ++i)
      if (tid + 256 * i < CA) *(bf16x8*)&As[buf][((tid >> 2) + 64 * i) * ROWP + k8] = ra[i];
#pragma unroll
    for (int i = 0; i < RB; ++i)
      if (tid + 256 * i < CB) *(bf16x8*)&Bs[buf][((tid + 256 * i) >> 2) * ROWP + k8] = rb[i];
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (nk > 0) {
    load_tile(kbeg);
    store_tile(0);
  }
  __syncthreads();
  for (int kc = 0; kc < nk; ++kc) {
    const int cur = kc & 1;
    if (kc + 1 < nk) load_tile(kbeg + kc + 1);
#pragma unroll
    for (int kq = 0; kq < BKB / 16; ++kq) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) af[tm] = *(const bf16x8*)&As[cur][(wm0 + tm * 32 + l32) * ROWP + kq * 16 + 8 * h];
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) bfr[tn] = *(const bf16x8*)&Bs[cur][(wn0 + tn * 32 + l32) * ROWP + kq * 16 + 8 * h];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[tm], bfr[tn], acc[tm][tn], 0, 0, 0);
    }
    if (kc + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
  }

  if (ks > 1) {  // raw partial tile -> slab[split][out_row][n]; bias/act/stats in splitk_reduce
    float* P = a.part + (long long)group * ks * a.rows_total * a.N + (long long)split * a.rows_total * a.N;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm0 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m >= a.rows) continue;
        const long long orow = out_row_b(g, cls, m);
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          const int n = n0 + wn0 + tn * 32 + l32;
          if (n < a.N) P[orow * a.N + n] = acc[tm][tn][r];
        }
      }
    return;
  }

  // epilogue (identical contract to the fp32 kernel)
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
      const long long orow = out_row_b(g, cls, m);
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
    float* red = (float*)&As[0][0];
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
        const long long rb_idx = (long long)cls * gridDim.x + blk.x;  // ks == 1 here
        float* st = a.stats + group * a.s_gs + rb_idx * 2 * a.N;
        st[n] = s;
        st[a.N + n] = q;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// weight-GEMM, bf16 MFMA, taps merged into M:  rows r = tap*M + m of
//   part[split][r][n] = sum_{p in split} G[src(p, tap)][m] * D[p][n]
// (small-channel layers fill all waves; one dY tile feeds every tap of the row tile)
// ---------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN, bool VECG>
__global__ __launch_bounds__(256) void wgrad_bf16_kernel(WgArgs a) {
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  constexpr int QMc = BM / 4, QNc = BN / 4;                  // channel quads
  constexpr int UA = QMc * (BKB / 4), UB = QNc * (BKB / 4);  // 4x4 units per tile
  constexpr int RA = (UA + 255) / 256, RB = (UB + 255) / 256;
  __shared__ __attribute__((aligned(16))) __bf16 As[2][BM * ROWP];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[2][BN * ROWP];

  const ConvGeom& g = a.g;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int wm0 = (wave / WN) * (TM * 32), wn0 = (wave % WN) * (TN * 32);
  const BlockXYZ blk = xcd_block();
  const int r0 = blk.x * BM, n0 = blk.y * BN;
  const int split = blk.z % a.nsplit;
  const int group = blk.z / a.nsplit;
  const int Mtot = a.ntap * a.M;
  const float* G = a.G + group * a.g_gs;
  const float* D = a.D + group * a.d_gs;
  const int p_begin = split * a.chunk;
  const int p_end = min(a.rows, p_begin + a.chunk);
  const int nk = (p_end - p_begin + BKB - 1) / BKB;

  auto pix = [&](int p) {  // row-space pixel -> coordinates, division-free
    RowCoordB rc;
    rc.valid = p < a.rows;
    if (g.mode == GM_DENSE) { rc.img = p; rc.y = rc.x = 0; return rc; }
    const int n = fdiv(p, g.dHW);
    const int r = p - n * g.dHW.d;
    rc.y = fdiv(r, g.dW);
    rc.x = r - rc.y * g.Wo;
    rc.img = n * g.Hi * g.Wi;
    return rc;
  };
  // per-unit (tap, channel) of the A rows this thread stages (fixed over the K loop)
  int utap[RA], um[RA];
#pragma unroll
  for (int i = 0; i < RA; ++i) {
    const int r = r0 + ((tid + 256 * i) % QMc) * 4;
    utap[i] = r / a.M;
    um[i] = r - utap[i] * a.M;
  }

  f32x4 va[RA][4], vb[RB][4];
  auto load_tile = [&](int kc) {
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      const int u = tid + 256 * i;
      const int pq = u / QMc;
      const int r = r0 + (u % QMc) * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        const int p = p_begin + kc * BKB + pq * 4 + j;
        if (u < UA && p < p_end && r < Mtot) {
          RowCoordB rc = pix(p);
          if (VECG) {
            const int tap = utap[i];
            long long sp = src_pixel_b(g, rc, tap / g.ksz, tap % g.ksz);
            if (sp >= 0) v = *(const f32x4*)(G + sp * a.ldg + um[i]);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int re = r + e;
              if (re < Mtot) {
                const int tap = re / a.M, m = re - (re / a.M) * a.M;
                long long sp = src_pixel_b(g, rc, tap / g.ksz, tap % g.ksz);
                if (sp >= 0) v[e] = G[sp * a.ldg + m];
              }
            }
          }
        }
        va[i][j] = v;
      }
    }
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int u = tid + 256 * i;
      const int nq = u % QNc, pq = u / QNc;
      const int nc = n0 + nq * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        const int p = p_begin + kc * BKB + pq * 4 + j;
        if (u < UB && p < p_end && nc < a.N) v = *(const f32x4*)(D + (long long)p * a.ldd + nc);
        vb[i][j] = v;
      }
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      const int u = tid + 256 * i;
      if (u >= UA) continue;
      const int mq = u % QMc, pq = u / QMc;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        f32x4 col = {va[i][0][c], va[i][1][c], va[i][2][c], va[i][3][c]};
        *(bf16x4*)&As[buf][(mq * 4 + c) * ROWP + pq * 4] = __builtin_convertvector(col, bf16x4);
      }
    }
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int u = tid + 256 * i;
      if (u >= UB) continue;
      const int nq = u % QNc, pq = u / QNc;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        f32x4 col = {vb[i][0][c], vb[i][1][c], vb[i][2][c], vb[i][3][c]};
        *(bf16x4*)&Bs[buf][(nq * 4 + c) * ROWP + pq * 4] = __builtin_convertvector(col, bf16x4);
      }
    }
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
    for (int ks = 0; ks < BKB / 16; ++ks) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) af[tm] = *(const bf16x8*)&As[cur][(wm0 + tm * 32 + l32) * ROWP + ks * 16 + 8 * h];
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) bfr[tn] = *(const bf16x8*)&Bs[cur][(wn0 + tn * 32 + l32) * ROWP + ks * 16 + 8 * h];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[tm], bfr[tn], acc[tm][tn], 0, 0, 0);
    }
    if (kc + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
  }
  float* P = a.part + group * a.p_gs + (long long)split * Mtot * a.N;
#pragma unroll
  for (int tm = 0; tm < TM; ++tm)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = r0 + wm0 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (m >= Mtot) continue;
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int n = n0 + wn0 + tn * 32 + l32;
        if (n < a.N) P[(long long)m * a.N + n] = acc[tm][tn][r];
      }
    }
}

// ---------------------------------------------------------------------------
// bf16 weight shadows: N = plain conversion; T = per-tap transpose of [rows][cols]
// ---------------------------------------------------------------------------
__global__ void shadow_n_kernel(const float* w, __bf16* out, long long n) {
  for (long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n;
       i += (long long)gridDim.x * blockDim.x * 4) {
    if (i + 3 < n) {
      f32x4 v = *(const f32x4*)(w + i);
      *(bf16x4*)(out + i) = __builtin_convertvector(v, bf16x4);
    } else {
      for (long long j = i; j < n; ++j) out[j] = (__bf16)w[j];
    }
  }
}

// one 32x32 tile per block; tiles enumerated by the host table (tensor, tap, r0, c0)
__global__ __launch_bounds__(256) void shadow_t_kernel(const float* w, __bf16* out, const int4* tiles,
                                                       const long long* offs) {
  __shared__ float t[32][33];
  const int4 d = tiles[blockIdx.x];  // x: tensor index, y: tap, z: r0, w: c0
  const long long off = offs[3 * d.x];
  const int R = (int)offs[3 * d.x + 1], Cc = (int)offs[3 * d.x + 2];
  const float* src = w + off + (long long)d.y * R * Cc;
  __bf16* dst = out + off + (long long)d.y * R * Cc;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int i = ty; i < 32; i += 8) {
    int r = d.z + i, c = d.w + tx;
    t[i][tx] = (r < R && c < Cc) ? src[(long long)r * Cc + c] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    int c = d.w + i, r = d.z + tx;
    if (r < R && c < Cc) dst[(long long)c * R + r] = (__bf16)t[tx][i];
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
// sum the K-split slabs; bias / act / accumulate into C; per-column (sum, sum^2) of the
// raw sums per 256-row block -> stats[rb][2][N]  (same contract as the GEMM epilogue)
#define SKR_ROWS 64
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* part, int ks, int rows_total, int N,
                                                            float* C, long long c_gs, int ldc, const float* bias,
                                                            long long bias_gs, int act, int accumulate, float* stats,
                                                            long long s_gs) {
  __shared__ f32x4 red[2][256];
  const int group = blockIdx.z;
  const int qi = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int n = (blockIdx.x * 16 + qi) * 4;
  const long long slab = (long long)rows_total * N;
  const float* P = part + (long long)group * ks * slab;
  float* Cg = C + group * c_gs;
  const float* bs = bias ? bias + group * bias_gs : nullptr;
  f32x4 s1 = {0.f, 0.f, 0.f, 0.f}, s2 = {0.f, 0.f, 0.f, 0.f};
  if (n < N) {
    const int r0 = blockIdx.y * SKR_ROWS;
    const int r1 = min(rows_total, r0 + SKR_ROWS);
    for (int r = r0 + rl; r < r1; r += 16) {
      f32x4 v = *(const f32x4*)(P + (long long)r * N + n);
#pragma unroll 4
      for (int k = 1; k < ks; ++k) v += *(const f32x4*)(P + k * slab + (long long)r * N + n);
      s1 += v;
      s2 += v * v;
      if (bs) v += *(const f32x4*)(bs + n);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = act_f(v[e], act);
      f32x4* d = (f32x4*)(Cg + (long long)r * ldc + n);
      *d = accumulate ? *d + v : v;
    }
  }
  if (!stats) return;
  red[0][threadIdx.x] = s1;
  red[1][threadIdx.x] = s2;
  __syncthreads();
  if (rl == 0 && n < N) {
    for (int j = 1; j < 16; ++j) {
      s1 += red[0][j * 16 + qi];
      s2 += red[1][j * 16 + qi];
    }
    float* st = stats + group * s_gs + (long long)blockIdx.y * 2 * N;
    *(f32x4*)(st + n) = s1;
    *(f32x4*)(st + N + n) = s2;
  }
}

template <int BM, int BN, int WM, int WN>
static void launch_bf16(const FwdArgs& a, int groups, bool sc, hipStream_t s) {
  dim3 grid((a.rows + BM - 1) / BM, (a.N + BN - 1) / BN, groups * a.nclass * a.ksplit);
  if (sc) hipLaunchKernelGGL((igemm_bf16_kernel<BM, BN, WM, WN, true>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((igemm_bf16_kernel<BM, BN, WM, WN, false>), grid, dim3(256), 0, s, a);
}

static int bf16_bm(const FwdArgs& a) {
  if (a.N <= 32) return 256;
  if (a.N <= 64) return 128;
  return igemm_fwd_bm(a) == 128 ? 128 : 64;
}
static int bf16_bn(const FwdArgs& a) { return a.N <= 32 ? 32 : (a.N <= 64 ? 64 : 128); }

int igemm_bf16_plan(const FwdArgs& a, int groups, int* ksplit) {
  const int bm = bf16_bm(a), bn = bf16_bn(a);
  const long long blocks = (long long)((a.rows + bm - 1) / bm) * ((a.N + bn - 1) / bn) * a.nclass * groups;
  const int ntap = a.g.mode == GM_DENSE ? 1 : (a.g.mode == GM_CONVT && a.g.stride == 2 ? 4 : 16);
  const int Ktot = ntap * a.Cin;
  const int nk = (a.Cin % BKB) ? (Ktot + BKB - 1) / BKB : ntap * (a.Cin / BKB);
  int ks = 1;
  if (blocks < 512 && a.part) {
    ks = (int)std::min<long long>((768 + blocks - 1) / blocks, 8);
    ks = std::min(ks, nk / 4);  // keep >= 4 K steps per split
    const long long rows_total = (long long)a.rows * a.nclass;
    while (ks > 1 && (long long)ks * rows_total * a.N * groups > a.part_cap) --ks;
    if (ks < 2) ks = 1;
  }
  if (ksplit) *ksplit = ks;
  if (ks == 1) return a.nclass * ((a.rows + bm - 1) / bm);
  return (int)(((long long)a.rows * a.nclass + SKR_ROWS - 1) / SKR_ROWS);
}

const char* kernel_name(int kid) {
  static const char* names[KID_COUNT] = {
      "none", "none",
      "igemm_bf16_kernel<256, 32, 4, 1, false>", "igemm_bf16_kernel<256, 32, 4, 1, true>",
      "igemm_bf16_kernel<128, 64, 2, 2, false>", "igemm_bf16_kernel<128, 64, 2, 2, true>",
      "igemm_bf16_kernel<128, 128, 2, 2, false>", "igemm_bf16_kernel<128, 128, 2, 2, true>",
      "igemm_bf16_kernel<64, 128, 1, 4, false>", "igemm_bf16_kernel<64, 128, 1, 4, true>",
      "wgrad_bf16_kernel<128, 32, 4, 1, true>", "wgrad_bf16_kernel<128, 32, 4, 1, false>",
      "wgrad_bf16_kernel<128, 64, 2, 2, true>", "wgrad_bf16_kernel<128, 64, 2, 2, false>",
      "wgrad_bf16_kernel<128, 128, 2, 2, true>", "wgrad_bf16_kernel<128, 128, 2, 2, false>"};
  return (kid >= 0 && kid < KID_COUNT) ? names[kid] : "none";
}

int igemm_bf16_kid(const FwdArgs& a) {
  const int sc = (a.Cin % BKB) != 0;
  if (a.N <= 32) return KID_IGEMM_BF16_256x32 + sc;
  if (a.N <= 64) return KID_IGEMM_BF16_128x64 + sc;
  if (bf16_bm(a) == 128) return KID_IGEMM_BF16_128x128 + sc;
  return KID_IGEMM_BF16_64x128 + sc;
}

int wgrad_bf16_kid(const WgArgs& a) {
  const int scalar = !((a.M % 4 == 0) && (a.ldg % 4 == 0));
  if (a.N <= 32) return KID_WGRAD_BF16_128x32 + scalar;
  if (a.N <= 64) return KID_WGRAD_BF16_128x64 + scalar;
  return KID_WGRAD_BF16_128x128 + scalar;
}

int igemm_bf16(FwdArgs a, int groups, hipStream_t s, hipEvent_t after) {
  const bool sc = (a.Cin % BKB) != 0;
  int ks = 1;
  const int nrb = igemm_bf16_plan(a, groups, &ks);
  a.ksplit = ks;
  a.rows_total = a.rows * a.nclass;
  switch (igemm_bf16_kid(a) & ~1) {
    case KID_IGEMM_BF16_256x32: launch_bf16<256, 32, 4, 1>(a, groups, sc, s); break;
    case KID_IGEMM_BF16_128x64: launch_bf16<128, 64, 2, 2>(a, groups, sc, s); break;
    case KID_IGEMM_BF16_128x128: launch_bf16<128, 128, 2, 2>(a, groups, sc, s); break;
    default: launch_bf16<64, 128, 1, 4>(a, groups, sc, s); break;
  }
  if (after) hipEventRecord(after, s);
  if (ks > 1) {
    dim3 grid((a.N + 63) / 64, nrb, groups);
    hipLaunchKernelGGL(splitk_reduce_kernel, grid, dim3(256), 0, s, a.part, ks, a.rows_total, a.N, a.C, a.c_gs, a.ldc,
                       a.bias, a.bias_gs, a.act, a.accumulate, a.stats, a.s_gs);
  }
  return nrb;
}

template <int BM, int BN, int WM, int WN>
static void launch_wg_bf16(const WgArgs& a, int groups, bool vec, hipStream_t s) {
  dim3 grid((a.ntap * a.M + BM - 1) / BM, (a.N + BN - 1) / BN, groups * a.nsplit);
  if (vec) hipLaunchKernelGGL((wgrad_bf16_kernel<BM, BN, WM, WN, true>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((wgrad_bf16_kernel<BM, BN, WM, WN, false>), grid, dim3(256), 0, s, a);
}

// tiles of the tap-merged weight-GEMM (for the split heuristic)
int wgrad_bf16_tiles(const WgArgs& a) {
  const int bn = a.N <= 32 ? 32 : (a.N <= 64 ? 64 : 128);
  return ((a.ntap * a.M + 127) / 128) * ((a.N + bn - 1) / bn);
}

void wgrad_bf16(WgArgs a, int groups, hipStream_t s, hipEvent_t after) {
  const int kid = wgrad_bf16_kid(a);
  const bool vec = !(kid & 1);
  a.g.dHW = make_fastdiv(a.g.Ho * a.g.Wo);
  a.g.dW = make_fastdiv(a.g.Wo);
  switch (kid & ~1) {
    case KID_WGRAD_BF16_128x32: launch_wg_bf16<128, 32, 4, 1>(a, groups, vec, s); break;
    case KID_WGRAD_BF16_128x64: launch_wg_bf16<128, 64, 2, 2>(a, groups, vec, s); break;
    default: launch_wg_bf16<128, 128, 2, 2>(a, groups, vec, s); break;
  }
  if (after) hipEventRecord(after, s);
}

void shadow_weights(const float* w, void* wn, void* wt, long long n, const void* tiles, int ntiles, const void* offs,
                    hipStream_t s) {
  long long q = (n + 3) / 4;
  int blocks = (int)std::min<long long>((q + 255) / 256, 8192);
  hipLaunchKernelGGL(shadow_n_kernel, dim3(blocks), dim3(256), 0, s, w, (__bf16*)wn, n);
  if (ntiles > 0)
    hipLaunchKernelGGL(shadow_t_kernel, dim3(ntiles), dim3(256), 0, s, w, (__bf16*)wt, (const int4*)tiles,
                       (const long long*)offs);
}
