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
#include <cstdlib>

#include "common.h"
#include "knobs.h"
#include "kernels.h"
#include "opload.h"

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
template <int BM, int BN, int WM, int WN, bool SMALLC, bool ABF>
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
  const long long a0 = group * a.a_gs;  // element offset of this group's A (fp32 or bf16)
  constexpr bool abf = ABF;
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
            const long long off = a0 + sp * a.lda + ci0 + k8;
            ra[i] = abf ? *(const bf16x8*)((const __bf16*)a.A + off)
                        : cvt8(*(const f32x4*)(a.A + off), *(const f32x4*)(a.A + off + 4));
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
              if (sp >= 0) v[e] = ld1(a.A, a0 + sp * a.lda + ci, abf);
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
  // fused backward-BN reductions (BwStat): per-column mean / invstd / beta of dy's BN layer
  const bool bwm = a.bw.pre != nullptr;
  float bwmean[TN], bwis[TN], bwb[TN];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    const int n = n0 + wn0 + tn * 32 + l32;
    bwmean[tn] = bwis[tn] = bwb[tn] = 0.f;
    if (bwm && n < a.bw.C) {
      bwmean[tn] = a.bw.mean[group * a.bw.ms_gs + n];
      bwis[tn] = a.bw.invstd[group * a.bw.ms_gs + n];
      bwb[tn] = a.bw.y ? 0.f : a.bw.beta[group * a.bw.beta_gs + n];
    }
  }
  // batches of 8 rows, all loads of a batch before its stores (see igemm_halo_kernel)
  float biasv[TN];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    const int n = n0 + wn0 + tn * 32 + l32;
    biasv[tn] = (bias && n < a.N) ? bias[n] : 0.f;
  }
  const bool pbf = a.bw.pre_bf16 != 0;
  const float* bwpre = bwm ? pf_at(a.bw.pre, group * a.bw.pre_gs, pbf) : nullptr;
  const bool ybf = a.bw.y_bf16 != 0;
  const float* bwy = (bwm && a.bw.y) ? pf_at(a.bw.y, group * a.bw.y_gs, ybf) : nullptr;
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
    for (int rb = 0; rb < 16; rb += 8) {
      long long orow[8];
      bool mok[8];
      float cv[8][TN], pv[8][TN], yv[8][TN];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = rb + i;
        const int m = m0 + wm0 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        mok[i] = m < a.rows;
        orow[i] = mok[i] ? out_row_b(g, cls, m) : 0;
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          const int n = n0 + wn0 + tn * 32 + l32;
          const bool ok = mok[i] && n < a.N;
          const bool bwc = ok && bwm && n < a.bw.C;
          cv[i][tn] = (ok && a.accumulate) ? Cp[orow[i] * a.ldc + n] : 0.f;
          pv[i][tn] = bwc ? pf_ld(bwpre, orow[i] * a.bw.ldp + n, pbf) : 0.f;
          yv[i][tn] = (bwc && bwy) ? pf_ld(bwy, orow[i] * a.bw.ldy + n, ybf) : 0.f;
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if (!mok[i]) continue;
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          const int n = n0 + wn0 + tn * 32 + l32;
          if (n >= a.N) continue;
          float v = acc[tm][tn][rb + i];
          if (a.c_bf16) v = bf_rnd(v);  // bf16-stored pre-BN output: the statistics of the stored values
          if (!bwm) {
            csum[tn] += v;
            csq[tn] += v * v;
          }
          if (bias) v += biasv[tn];
          v = act_f(v, a.act);
          if (a.accumulate) v += cv[i][tn];
          if (a.c_bf16) ((__bf16*)a.C)[group * a.c_gs + orow[i] * a.ldc + n] = (__bf16)v;
          else Cp[orow[i] * a.ldc + n] = v;
          if (bwm && n < a.bw.C)
            bw_term_v(v, pv[i][tn], bwmean[tn], bwis[tn], bwb[tn], bwy != nullptr, yv[i][tn], a.bw.act, csum[tn],
                      csq[tn]);
        }
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
      const int SC = bwm ? a.bw.C : a.N;  // stats columns (row-block stride 2*SC)
      if (n < SC) {
        float s = 0.f, q = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) { s += red[w * BN + tid]; q += red[WM * BN + w * BN + tid]; }
        const int rb = cls * gridDim.x + blk.x;
        stat_put(a.stats + (rb & (a.s_nsh - 1)) * a.s_sh + group * a.s_gs, n, s, q);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Halo-tile gather-GEMM (conv / conv-T forward and input gradient, bf16 MFMA).
// A block owns BM row-space pixels that form whole image rows (or whole images).  For each
// 32-channel chunk of the gathered operand the block stages the input window those pixels
// touch -- PR x PC pixels per image, zero-padded at the borders -- in LDS once, as bf16 with an
// 80-byte pixel pitch, and every tap of the chunk reads its A fragments from that window at a
// fixed (dy, dx) shift.  The per-tap gather of the plain kernel re-reads every input element
// through L2 once per tap (16x); here each element is read once per block (plus the halo).
// Weights keep the per-(chunk, tap) double-buffered B tiles of the plain kernel.
//   CONV          iy = ry*s - pad + ky         window rows (R-1)*s + 4, dy = ky
//   CONVT s=1     iy = ry + pad - ky           window rows R + 3,       dy = 3 - ky
//   CONVT s=2     class (cy,cx), ky = k0+2*ty  window rows R + 1,       dy = 1 - ty
// ---------------------------------------------------------------------------
#define HALO_CK 32   // channels per window stage
#define HALO_PI 8    // window items (8 channels each) per thread and stage: npix*4 <= 256*HALO_PI

struct HaloArgs {
  FwdArgs f;
  int Hr, Wr;        // row-space image dims (per parity class for CONVT s2)
  int R, nimg;       // image rows per block (per image) and images per block
  int PR, PC;        // window dims per image
  int sy;            // row-space -> input stride (CONV stride, else 1)
  int npix;          // nimg * PR * PC
  // launch-constant divisors (multiply-shift): no integer divisions in the index decode
  FastDiv d_win, d_pc, d_img, d_wr, d_rimg, d_q, d_qw;  // PR*PC, PC, Hr*Wr, Wr, R*Wr, (Ho/2)*(Wo/2), Wo/2
};
__device__ __forceinline__ long long out_row_h(const HaloArgs& h, const ConvGeom& g, int cls, int m) {
  if (g.mode == GM_CONVT && g.stride == 2) {
    const int n = fdiv(m, h.d_q);
    const int r = m - n * h.d_q.d;
    const int qy = fdiv(r, h.d_qw), qx = r - qy * h.d_qw.d;
    return ((long long)n * g.Ho + 2 * qy + (cls >> 1)) * g.Wo + 2 * qx + (cls & 1);
  }
  return m;
}
static void halo_divisors(HaloArgs& h, const ConvGeom& g) {
  h.d_win = make_fastdiv(h.PR * h.PC);
  h.d_pc = make_fastdiv(h.PC);
  h.d_img = make_fastdiv(h.Hr * h.Wr);
  h.d_wr = make_fastdiv(h.Wr);
  h.d_rimg = make_fastdiv(h.R * h.Wr);
  h.d_q = make_fastdiv((g.Ho >> 1) * (g.Wo >> 1));
  h.d_qw = make_fastdiv(g.Wo >> 1);
}

// bf16-A instances up to 128x64 at 4 waves per SIMD (128 VGPRs, 8-32 bytes of spill): +0.8 % of the step
// in a same-box A/B; the fp32-A instances spill 70-90 bytes there and were 1 % slower
template <int BM, int BN, int WM, int WN, bool S2T, bool ABF>
__global__ __launch_bounds__(256, (ABF && BN * BM <= 8192) ? 4 : 2) void igemm_halo_kernel(HaloArgs h) {
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  constexpr int NTAP = S2T ? 4 : 16;
  constexpr int P = 4;  // B-fragment prefetch distance in taps (NTAP % P == 0)
  extern __shared__ __attribute__((aligned(16))) __bf16 hsm[];
  const FwdArgs& a = h.f;
  const ConvGeom& g = a.g;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int wm0 = (wave / WN) * (TM * 32), wn0 = (wave % WN) * (TN * 32);
  const int ks = a.ksplit;
  const BlockXYZ blk = xcd_block();
  const int split = blk.z % ks;
  const int zc = blk.z / ks;
  const int group = zc / a.nclass, cls = zc - group * a.nclass;
  const int m0 = blk.x * BM, n0 = blk.y * BN;
  const long long a0 = group * a.a_gs;  // element offset of this group's A (fp32 or bf16)
  constexpr bool abf = ABF;
  const __bf16* Bw = (const __bf16*)a.Bh + group * a.b_gs;
  const int nchunk = a.Cin / HALO_CK;
  const int cbeg = (int)((long long)nchunk * split / ks), cend = (int)((long long)nchunk * (split + 1) / ks);

  // ---- block window origin and per-tap geometry (uniform) ----
  const int per_img = h.Hr * h.Wr;
  const int img0 = fdiv(m0, h.d_img);
  const int ry0 = fdiv(m0 - img0 * per_img, h.d_wr);
  int oy_min, ox_min, tap0, toff0, tsgn;
  if (S2T) {
    const int cy = cls >> 1, cx = cls & 1;
    const int ky0 = (cy + g.pad) & 1, kx0 = (cx + g.pad) & 1;
    oy_min = (cy + g.pad - ky0) / 2 - 1;
    ox_min = (cx + g.pad - kx0) / 2 - 1;
    tap0 = ky0 * 4 + kx0;  // B tap of t: tap0 + 8*(t>>1) + 2*(t&1)
    toff0 = h.PC + 1;      // window shift of t: (1-(t>>1))*PC + (1-(t&1))
    tsgn = -1;
  } else if (g.mode == GM_CONV) {
    oy_min = ox_min = -g.pad;
    tap0 = 0;
    toff0 = 0;  // shift of tap t: (t>>2)*PC + (t&3)
    tsgn = 1;
  } else {
    oy_min = ox_min = g.pad - 3;
    tap0 = 0;
    toff0 = 3 * h.PC + 3;  // shift: (3-(t>>2))*PC + (3-(t&3))
    tsgn = -1;
  }
  const int iy_base = ry0 * h.sy + oy_min;

  // ---- window staging: per-thread item offsets, identical for every chunk ----
  int woff[HALO_PI];
#pragma unroll
  for (int i = 0; i < HALO_PI; ++i) {
    const int it = tid + 256 * i;
    woff[i] = -2;  // -2: no item, -1: zero (outside the image)
    if (it < h.npix * 4) {
      const int pix = it >> 2, part = it & 3;
      const int il = fdiv(pix, h.d_win);
      const int r2 = pix - il * h.PR * h.PC;
      const int pr = fdiv(r2, h.d_pc), pc = r2 - pr * h.PC;
      const int iy = iy_base + pr, ix = ox_min + pc;
      woff[i] = (iy >= 0 && iy < g.Hi && ix >= 0 && ix < g.Wi)
                    ? (((img0 + il) * g.Hi + iy) * g.Wi + ix) * a.lda + part * 8
                    : -1;
    }
  }
  // staged in two halves (items [0, PI/2) and [PI/2, PI)) to halve the registers in flight
  constexpr int HP = HALO_PI / 2;
  f32x4 wv[HP][2];
  auto load_window = [&](int chunk, int half) {
    const long long ac = a0 + chunk * HALO_CK;
#pragma unroll
    for (int j = 0; j < HP; ++j) {
      const int i = half * HP + j;
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      wv[j][0] = z;
      wv[j][1] = z;
      if (woff[i] >= 0) ld8_raw(a.A, ac + woff[i], abf, wv[j][0], wv[j][1]);
    }
  };
  auto store_window = [&](int buf, int half) {
    __bf16* W = hsm + buf * h.npix * ROWP;
#pragma unroll
    for (int j = 0; j < HP; ++j) {
      const int i = half * HP + j;
      const int it = tid + 256 * i;
      if (woff[i] >= -1) *(bf16x8*)&W[(it >> 2) * ROWP + (it & 3) * 8] = raw8_bf(wv[j][0], wv[j][1], abf);
    }
  };

  // ---- A fragment bases (window pixel of tap shift 0) ----
  int abase[TM];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int ml = wm0 + tm * 32 + l32;
    const int rows_img = h.R * h.Wr;
    const int il = fdiv(ml, h.d_rimg);
    const int rem = ml - il * rows_img;
    const int ryl = fdiv(rem, h.d_wr), rx = rem - ryl * h.Wr;
    abase[tm] = ((il * h.PR + ryl * h.sy) * h.PC + rx * h.sy) * ROWP + 8 * hh;
  }

  // ---- B fragments straight from the bf16 shadow (L2-resident), P taps ahead ----
  bool nok[TN];
  const __bf16* bptr[TN];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    const int n = n0 + wn0 + tn * 32 + l32;
    nok[tn] = (n0 + wn0 + tn * 32) < a.N;  // uniform per 32-column group
    bptr[tn] = Bw + (long long)((nok[tn] && n < a.N) ? n : 0) * a.ldb + 8 * hh;  // N < 32: clamp, discard
  }
  bf16x8 bq[P][TN][2];
  auto load_b = [&](int slot, int chunk, int t) {
    const int tap = S2T ? tap0 + 8 * (t >> 1) + 2 * (t & 1) : t;
    const long long off = (long long)tap * a.b_tap + chunk * HALO_CK;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
      for (int kq = 0; kq < 2; ++kq) bq[slot][tn][kq] = *(const bf16x8*)(bptr[tn] + off + kq * 16);
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (cbeg < cend) {
    load_window(cbeg, 0);
    store_window(0, 0);
    load_window(cbeg, 1);
#pragma unroll
    for (int t = 0; t < P; ++t) load_b(t, cbeg, t);
    store_window(0, 1);
  }
  __syncthreads();
  for (int c = cbeg; c < cend; ++c) {
    const int buf = (c - cbeg) & 1;
    const bool has_next = c + 1 < cend;
    const __bf16* W = hsm + buf * h.npix * ROWP;
#pragma unroll
    for (int t = 0; t < NTAP; ++t) {
      // next chunk's window: half 0 issued at tap 0 and stored at NTAP/2-1, half 1 at NTAP/2 .. NTAP-1
      if (has_next && (t == 0 || t == NTAP / 2)) load_window(c + 1, t == 0 ? 0 : 1);
      const int shift = S2T ? toff0 + tsgn * ((t >> 1) * h.PC + (t & 1)) : toff0 + tsgn * ((t >> 2) * h.PC + (t & 3));
      const int sh = shift * ROWP;
#pragma unroll
      for (int kq = 0; kq < 2; ++kq) {
        bf16x8 af[TM];
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) af[tm] = *(const bf16x8*)&W[abase[tm] + sh + kq * 16];
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn)
            if (nok[tn])
              acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[tm], bq[t % P][tn][kq], acc[tm][tn], 0, 0, 0);
      }
      // refill this slot with the fragments P taps ahead
      if (t + P < NTAP) load_b(t % P, c, t + P);
      else if (has_next) load_b(t % P, c + 1, t + P - NTAP);
      if (has_next && (t == NTAP / 2 - 1 || t == NTAP - 1)) store_window(buf ^ 1, t == NTAP - 1 ? 1 : 0);
    }
    __syncthreads();
  }

  if (ks > 1) {  // raw partial tile -> slab[split][out_row][n]; bias/act/stats in splitk_reduce
    float* Pp = a.part + (long long)group * ks * a.rows_total * a.N + (long long)split * a.rows_total * a.N;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm0 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        const long long orow = out_row_h(h, g, cls, m);
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          const int n = n0 + wn0 + tn * 32 + l32;
          if (nok[tn] && n < a.N) Pp[orow * a.N + n] = acc[tm][tn][r];
        }
      }
    return;
  }

  float* Cp = a.C + group * a.c_gs;
  const float* bias = a.bias ? a.bias + group * a.bias_gs : nullptr;
  float csum[TN], csq[TN];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) { csum[tn] = 0.f; csq[tn] = 0.f; }
  // fused backward-BN reductions (BwStat): per-column mean / invstd / beta of dy's BN layer
  const bool bwm = a.bw.pre != nullptr;
  float bwmean[TN], bwis[TN], bwb[TN];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    const int n = n0 + wn0 + tn * 32 + l32;
    bwmean[tn] = bwis[tn] = bwb[tn] = 0.f;
    if (bwm && n < a.bw.C) {
      bwmean[tn] = a.bw.mean[group * a.bw.ms_gs + n];
      bwis[tn] = a.bw.invstd[group * a.bw.ms_gs + n];
      bwb[tn] = a.bw.y ? 0.f : a.bw.beta[group * a.bw.beta_gs + n];
    }
  }
  // batches of 8 rows: every global load of a batch (accumulate target, BN-backward pre / y) is
  // issued before the first store, so the batch pays one memory round trip, not one per element
  // (C may alias nothing it reads here, but the compiler cannot know that across the stores)
  float biasv[TN];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    const int n = n0 + wn0 + tn * 32 + l32;
    biasv[tn] = (bias && nok[tn] && n < a.N) ? bias[n] : 0.f;
  }
  const bool pbf = a.bw.pre_bf16 != 0;
  const float* bwpre = bwm ? pf_at(a.bw.pre, group * a.bw.pre_gs, pbf) : nullptr;
  const bool ybf = a.bw.y_bf16 != 0;
  const float* bwy = (bwm && a.bw.y) ? pf_at(a.bw.y, group * a.bw.y_gs, ybf) : nullptr;
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
    for (int rb = 0; rb < 16; rb += 8) {
      long long orow[8];
      float cv[8][TN], pv[8][TN], yv[8][TN];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = rb + i;
        const int m = m0 + wm0 + tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        orow[i] = out_row_h(h, g, cls, m);
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          const int n = n0 + wn0 + tn * 32 + l32;
          const bool ok = nok[tn] && n < a.N;
          const bool bwc = ok && bwm && n < a.bw.C;
          cv[i][tn] = (ok && a.accumulate) ? Cp[orow[i] * a.ldc + n] : 0.f;
          pv[i][tn] = bwc ? pf_ld(bwpre, orow[i] * a.bw.ldp + n, pbf) : 0.f;
          yv[i][tn] = (bwc && bwy) ? pf_ld(bwy, orow[i] * a.bw.ldy + n, ybf) : 0.f;
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          const int n = n0 + wn0 + tn * 32 + l32;
          if (!nok[tn] || n >= a.N) continue;
          float v = acc[tm][tn][rb + i];
          if (a.c_bf16) v = bf_rnd(v);  // bf16-stored pre-BN output: the statistics of the stored values
          if (!bwm) {
            csum[tn] += v;
            csq[tn] += v * v;
          }
          if (bias) v += biasv[tn];
          v = act_f(v, a.act);
          if (a.accumulate) v += cv[i][tn];
          if (a.c_bf16) ((__bf16*)a.C)[group * a.c_gs + orow[i] * a.ldc + n] = (__bf16)v;
          else Cp[orow[i] * a.ldc + n] = v;
          if (bwm && n < a.bw.C)
            bw_term_v(v, pv[i][tn], bwmean[tn], bwis[tn], bwb[tn], bwy != nullptr, yv[i][tn], a.bw.act, csum[tn],
                      csq[tn]);
        }
      }
    }
  }
  if (a.stats) {
    float* red = (float*)hsm;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      csum[tn] += __shfl_xor(csum[tn], 32, 64);
      csq[tn] += __shfl_xor(csq[tn], 32, 64);
    }
    __syncthreads();
    if (hh == 0) {
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        red[(wave / WN) * BN + wn0 + tn * 32 + l32] = csum[tn];
        red[WM * BN + (wave / WN) * BN + wn0 + tn * 32 + l32] = csq[tn];
      }
    }
    __syncthreads();
    if (tid < BN) {
      const int n = n0 + tid;
      const int SC = bwm ? a.bw.C : a.N;  // stats columns (row-block stride 2*SC)
      if (n < SC) {
        float s = 0.f, q = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) { s += red[w * BN + tid]; q += red[WM * BN + w * BN + tid]; }
        const int rb = cls * gridDim.x + blk.x;
        stat_put(a.stats + (rb & (a.s_nsh - 1)) * a.s_sh + group * a.s_gs, n, s, q);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Halo weight-GEMM (conv / conv-T weight gradient, bf16 MFMA, gfx950 transposed LDS reads).
//   dW[tap][m][n] = sum_p G[src(p, tap)][m] * D[p][n],  src = (y*s - pad + ky, x*s - pad + kx)
// A block owns 32 G-channels x BN D-channels and all 16 taps (wave w: kernel row ky = w, kx 0..3)
// and walks chunks of CP row-space pixels (whole image rows, or whole images).  Per chunk it
// stages, once, the G input window those pixels touch (halo included) and the D rows, both
// pixel-major bf16 exactly as they lie in HBM (no register transpose).  MFMA fragments need
// K = pixels contiguous per channel: ds_read_b64_tr_b16 delivers 4 consecutive pixels of one
// channel per lane, so every tap's A fragment is the window read at a pixel shift.
//   G window pitch: 64 B (s = 1) / 96 B (s = 2) -> conflict-free transposed reads;
//   D rows (BN = 64): 8-byte slot XOR 8 on pixel bit 1 -> conflict-free.
// ---------------------------------------------------------------------------
#define WH_WPI 12  // window items (4 channels each, 8 per pixel) per thread: npix*8 <= 256*WH_WPI
#define WH_DPI 8   // D items per thread: CP*BN/4 <= 256*WH_DPI


typedef short v4i16 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4i16 lds_tr16(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(p));
}
__device__ __forceinline__ bf16x8 join_tr(v4i16 lo, v4i16 hi) {
  typedef short v8i16 __attribute__((ext_vector_type(8)));
  v8i16 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

template <int BN, int S, int OPB>
__global__ __launch_bounds__(256, (BN == 32 && S == 1) ? 2 : 1) void wgrad_halo_kernel(WHaloArgs h) {
  constexpr int NS = BN / 32;              // 32-column MFMA subtiles
  constexpr int GP = S == 1 ? 32 : 48;     // window pixel pitch (bf16)
  extern __shared__ __attribute__((aligned(16))) __bf16 wsm[];
  const WgArgs& a = h.w;
  const ConvGeom& g = a.g;
  __bf16* Gw = wsm;
  __bf16* Dt = wsm + h.npix * GP;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int grp = lane >> 4, i16 = lane & 15, q = i16 >> 2, p4 = i16 & 3;
  const BlockXYZ blk = xcd_block();
  const int m0 = blk.x * 32, n0 = blk.y * BN;
  const int split = blk.z % a.nsplit, group = blk.z / a.nsplit;
  const long long gg0 = group * a.g_gs, dd0 = group * a.d_gs;  // element offsets (fp32 or bf16)
  constexpr bool gbf = (OPB & 1) != 0, dbf = (OPB & 2) != 0;  // G / D stored as bf16
  const int cbeg = (int)((long long)h.nchunk * split / a.nsplit);
  const int cend = (int)((long long)h.nchunk * (split + 1) / a.nsplit);
  const int per_img = g.Ho * g.Wo;

  // window items: chunk-invariant relative offset (from the chunk's window origin) + row index
  int wrel[WH_WPI], wpr[WH_WPI];
#pragma unroll
  for (int i = 0; i < WH_WPI; ++i) {
    const int it = tid + 256 * i;
    wrel[i] = 0;
    wpr[i] = -1;  // -1: no item
    if (it < h.npix * 8) {
      const int pix = it >> 3, part = it & 7;
      const int il = pix / (h.PR * h.PC);
      const int r2 = pix - il * h.PR * h.PC;
      const int pr = r2 / h.PC, pc = r2 - pr * h.PC;
      const int ix = pc - g.pad;
      wrel[i] = ((il * g.Hi + pr) * g.Wi + ix) * a.ldg + m0 + part * 4;
      wpr[i] = (ix >= 0 && ix < g.Wi) ? pr : -2;  // -2: column outside the image (zero)
    }
  }

  // per-lane fragment geometry: the 4 pixels of this lane's transposed read, per K step
  f32x16 acc[4][NS];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NS; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int lgR = h.lgImgPix - h.lgWo;
  // Chunk c+1's G window and D rows are loaded into registers while chunk c computes (one
  // chunk of MFMA work hides the HBM latency); they are converted and stored to LDS after the
  // chunk's closing barrier.
  f32x4 gv[WH_WPI], dv[WH_DPI];
  auto load_chunk = [&](int c) {
    const int row0 = c * h.CP;
    const int img0 = row0 / per_img;
    const int ry0 = (row0 - img0 * per_img) >> h.lgWo;
    const int iy0 = ry0 * S - g.pad;  // input row of window row 0
    const long long gc = gg0 + ((long long)img0 * g.Hi + iy0) * g.Wi * a.ldg;
#pragma unroll
    for (int i = 0; i < WH_WPI; ++i) {
      gv[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int iy = iy0 + wpr[i];
      if (wpr[i] >= 0 && iy >= 0 && iy < g.Hi) gv[i] = ld4_raw(a.G, gc + wrel[i], gbf);
    }
    const long long dc = dd0 + (long long)row0 * a.ldd + n0;
#pragma unroll
    for (int i = 0; i < WH_DPI; ++i) {
      const int it = tid + 256 * i;
      if (it < h.CP * (BN / 4)) {
        const int k = it / (BN / 4), slot = it - k * (BN / 4);
        dv[i] = ld4_raw(a.D, dc + (long long)k * a.ldd + slot * 4, dbf);
      }
    }
  };
  auto store_chunk = [&]() {
#pragma unroll
    for (int i = 0; i < WH_WPI; ++i) {
      if (wpr[i] == -1) continue;
      const int it = tid + 256 * i;
      *(bf16x4*)&Gw[(it >> 3) * GP + (it & 7) * 4] = raw4_bf(gv[i], gbf);
    }
#pragma unroll
    for (int i = 0; i < WH_DPI; ++i) {
      const int it = tid + 256 * i;
      if (it < h.CP * (BN / 4)) {
        const int k = it / (BN / 4), slot = it - k * (BN / 4);
        const int sw = BN == 64 ? (slot ^ (((k >> 1) & 1) << 3)) : slot;
        *(bf16x4*)&Dt[k * BN + sw * 4] = raw4_bf(dv[i], dbf);
      }
    }
  };
  if (cbeg < cend) load_chunk(cbeg);
  for (int c = cbeg; c < cend; ++c) {
    store_chunk();
    __syncthreads();
    if (c + 1 < cend) load_chunk(c + 1);
    // ---- K steps of 16 pixels ----
    for (int kk = 0; kk < h.CP / 16; ++kk) {
      int wp[2], kr[2];
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int k = kk * 16 + 8 * (grp >> 1) + 4 * r + q;
        kr[r] = k;
        const int il = k >> h.lgImgPix;
        const int ry = (k >> h.lgWo) & ((1 << lgR) - 1);
        const int rx = k & ((1 << h.lgWo) - 1);
        wp[r] = (il * h.PR + ry * S) * h.PC + rx * S;
      }
      bf16x8 bfr[NS];
#pragma unroll
      for (int ns = 0; ns < NS; ++ns) {
        v4i16 t[2];
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          const int slot = ns * 8 + 4 * (grp & 1) + p4;
          const int sw = BN == 64 ? (slot ^ (((kr[r] >> 1) & 1) << 3)) : slot;
          t[r] = lds_tr16(&Dt[kr[r] * BN + sw * 4]);
        }
        bfr[ns] = join_tr(t[0], t[1]);
      }
      const int ch = 16 * (grp & 1) + 4 * p4;
#pragma unroll
      for (int kx = 0; kx < 4; ++kx) {
        const int shift = wave * h.PC + kx;  // tap (ky = wave, kx)
        const bf16x8 af = join_tr(lds_tr16(&Gw[(wp[0] + shift) * GP + ch]), lds_tr16(&Gw[(wp[1] + shift) * GP + ch]));
#pragma unroll
        for (int ns = 0; ns < NS; ++ns)
          acc[kx][ns] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr[ns], acc[kx][ns], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  // ---- partial dW[tap][m][n] of this split (or the gradient itself when nsplit == 1) ----
  float* out = a.part + group * a.p_gs + (long long)split * 16 * a.M * a.N;
#pragma unroll
  for (int kx = 0; kx < 4; ++kx) {
    const int tap = wave * 4 + kx;
#pragma unroll
    for (int ns = 0; ns < NS; ++ns) {
      const int n = n0 + ns * 32 + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        out[((long long)tap * a.M + m) * a.N + n] = acc[kx][ns][r];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// weight-GEMM, bf16 MFMA, taps merged into M:  rows r = tap*M + m of
//   part[split][r][n] = sum_{p in split} G[src(p, tap)][m] * D[p][n]
// (small-channel layers fill all waves; one dY tile feeds every tap of the row tile)
// ---------------------------------------------------------------------------
// NSP > 1 (split mode, dtype bf16x6): both operands staged as NSP bf16 planes (opload.h split4) in ONE
// LDS buffer (two barriers per K chunk instead of double buffering), mfma_split products: the FC
// weight gradients (K = the batch: NSP = 3, six products) and the tap-merged conv weight gradients
// without a halo kernel (NSP = 2, three products, as wgrad_halo2 / wgrad_smallc)
template <int BM, int BN, int WM, int WN, bool VECG, int NSP = 1>
__global__ __launch_bounds__(256) void wgrad_bf16_kernel(WgArgs a) {
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  constexpr int QMc = BM / 4, QNc = BN / 4;                  // channel quads
  constexpr int UA = QMc * (BKB / 4), UB = QNc * (BKB / 4);  // 4x4 units per tile
  constexpr int RA = (UA + 255) / 256, RB = (UB + 255) / 256;
  constexpr int NBUF = NSP == 1 ? 2 : 1;
  __shared__ __attribute__((aligned(16))) __bf16 As[NBUF][NSP][BM * ROWP];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[NBUF][NSP][BN * ROWP];

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
  const long long gg0 = group * a.g_gs, dd0 = group * a.d_gs;  // element offsets (fp32 or bf16)
  const bool gbf = a.g_bf16 != 0, dbf = a.d_bf16 != 0;
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
  // staging unit u -> (channel quad, pixel quad): eight consecutive lanes take the eight pixel quads of one
  // channel quad, so the transposed 8-byte LDS stores of 32 lanes (4 channel quads x 8 pixel quads, rows 4
  // apart at an 80-B pitch) hit 64 distinct banks (u % QMc put 32 channel quads of one pixel quad on 4 bank
  // offsets: 8-way conflicts); the global loads still use whole 128-B lines (8 channel quads x 8 pixels)
  constexpr int PQ = BKB / 4;  // pixel quads per K chunk
  // per-unit (tap, channel) of the A rows this thread stages (fixed over the K loop)
  int utap[RA], um[RA], uky[RA], ukx[RA];
#pragma unroll
  for (int i = 0; i < RA; ++i) {
    const int r = r0 + ((tid + 256 * i) / PQ) * 4;
    utap[i] = r / a.M;
    um[i] = r - utap[i] * a.M;
    uky[i] = utap[i] / g.ksz;
    ukx[i] = utap[i] - uky[i] * g.ksz;
  }

  f32x4 va[RA][4], vb[RB][4];
  auto load_tile = [&](int kc) {
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      const int u = tid + 256 * i;
      const int pq = u % PQ;
      const int r = r0 + (u / PQ) * 4;
      if (VECG) {
        // a quad of 4 row-space pixels never crosses an image row (chunks are 32-aligned and
        // every row-space width is a multiple of 4): decode it once, step x by the stride
        const int p0 = p_begin + kc * BKB + pq * 4;
        const bool uok = u < UA && r < Mtot && p0 < p_end;
        const RowCoordB rc = pix(uok ? p0 : 0);
        int iy = 0, ix0 = 0;
        if (g.mode == GM_DENSE) {
          iy = 0;
          ix0 = 0;
        } else {
          iy = rc.y * g.stride - g.pad + uky[i];
          ix0 = rc.x * g.stride - g.pad + ukx[i];
        }
        const bool rowok = uok && (g.mode == GM_DENSE || (iy >= 0 && iy < g.Hi));
        const long long gp = gg0 + (g.mode == GM_DENSE ? (long long)p0 * a.ldg
                                                       : ((long long)rc.img + (long long)iy * g.Wi + ix0) * a.ldg) +
                             um[i];
        const int step = g.mode == GM_DENSE ? a.ldg : g.stride * a.ldg;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f32x4 v = {0.f, 0.f, 0.f, 0.f};
          const int ix = ix0 + j * g.stride;
          const bool ok = rowok && (p0 + j < p_end) && (g.mode == GM_DENSE || (ix >= 0 && ix < g.Wi));
          if (ok) v = ld4_raw(a.G, gp + (long long)j * step, gbf);
          va[i][j] = v;
        }
        continue;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        const int p = p_begin + kc * BKB + pq * 4 + j;
        if (u < UA && p < p_end && r < Mtot) {
          RowCoordB rc = pix(p);
          if (VECG) {
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int re = r + e;
              if (re < Mtot) {
                const int tap = re / a.M, m = re - (re / a.M) * a.M;
                long long sp = src_pixel_b(g, rc, tap / g.ksz, tap % g.ksz);
                if (sp >= 0) v[e] = ld1(a.G, gg0 + sp * a.ldg + m, gbf);
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
      const int nq = u / PQ, pq = u % PQ;
      const int nc = n0 + nq * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        const int p = p_begin + kc * BKB + pq * 4 + j;
        if (u < UB && p < p_end && nc < a.N) v = ld4_raw(a.D, dd0 + (long long)p * a.ldd + nc, dbf);
        vb[i][j] = v;
      }
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      const int u = tid + 256 * i;
      if (u >= UA) continue;
      const int mq = u / PQ, pq = u % PQ;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const bool rg = VECG && gbf;  // raw bf16 bits (the scalar gather path holds fp32 values)
        f32x4 col = {raw4_elem(va[i][0], c, rg), raw4_elem(va[i][1], c, rg), raw4_elem(va[i][2], c, rg),
                     raw4_elem(va[i][3], c, rg)};
        if constexpr (NSP == 1) {
          *(bf16x4*)&As[buf][0][(mq * 4 + c) * ROWP + pq * 4] = __builtin_convertvector(col, bf16x4);
        } else {
          bf16x4 pl[NSP];
          split4<NSP>(col, pl);
#pragma unroll
          for (int q = 0; q < NSP; ++q) *(bf16x4*)&As[buf][q][(mq * 4 + c) * ROWP + pq * 4] = pl[q];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int u = tid + 256 * i;
      if (u >= UB) continue;
      const int nq = u / PQ, pq = u % PQ;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        f32x4 col = {raw4_elem(vb[i][0], c, dbf), raw4_elem(vb[i][1], c, dbf), raw4_elem(vb[i][2], c, dbf),
                     raw4_elem(vb[i][3], c, dbf)};
        if constexpr (NSP == 1) {
          *(bf16x4*)&Bs[buf][0][(nq * 4 + c) * ROWP + pq * 4] = __builtin_convertvector(col, bf16x4);
        } else {
          bf16x4 pl[NSP];
          split4<NSP>(col, pl);
#pragma unroll
          for (int q = 0; q < NSP; ++q) *(bf16x4*)&Bs[buf][q][(nq * 4 + c) * ROWP + pq * 4] = pl[q];
        }
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
    const int cur = NSP == 1 ? (kc & 1) : 0;
    if (kc + 1 < nk) load_tile(kc + 1);
#pragma unroll
    for (int ks = 0; ks < BKB / 16; ++ks) {
      bf16x8 af[TM][NSP], bfr[TN][NSP];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int q = 0; q < NSP; ++q)
          af[tm][q] = *(const bf16x8*)&As[cur][q][(wm0 + tm * 32 + l32) * ROWP + ks * 16 + 8 * h];
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int q = 0; q < NSP; ++q)
          bfr[tn][q] = *(const bf16x8*)&Bs[cur][q][(wn0 + tn * 32 + l32) * ROWP + ks * 16 + 8 * h];
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) acc[tm][tn] = mfma_split<NSP>(af[tm], bfr[tn], acc[tm][tn]);
    }
    if constexpr (NSP == 1) {
      if (kc + 1 < nk) store_tile(cur ^ 1);
      __syncthreads();
    } else {  // one buffer: every wave done reading it before the next chunk is stored
      __syncthreads();
      if (kc + 1 < nk) {
        store_tile(0);
        __syncthreads();
      }
    }
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
// split mode (nsp planes): plane p holds bf16(w - sum of the earlier planes) (opload.h split4)
__global__ void shadow_n_kernel(const float* w, __bf16* out, long long n, int nsp, long long plane, const int* wtab) {
  for (long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n;
       i += (long long)gridDim.x * blockDim.x * 4) {
    if (i + 3 < n) {
      f32x4 v = *(const f32x4*)(w + i);
      bool bfp = true;  // the bf16 planes (split mode: only the tensors flagged in the table)
      if (nsp == 3) {  // split mode: the fp16 planes too
        _Float16 h0[4], h1[4];
        const int tv = wtab ? wtab[i >> 6] : (H16_WS | WTAB_BF16);
        bfp = wtab_bf16(tv);
        for (int e = 0; e < 4; ++e) h16_pair(v[e], wtab_exp(tv), h0[e], h1[e]);
        for (int e = 0; e < 4; ++e) {
          ((_Float16*)out)[H16_PLANE * plane + i + e] = h0[e];
          ((_Float16*)out)[(H16_PLANE + 1) * plane + i + e] = h1[e];
        }
      }
      if (bfp)
      for (int p = 0; p < nsp; ++p) {
        const bf16x4 h = __builtin_convertvector(v, bf16x4);
        *(bf16x4*)(out + p * plane + i) = h;
        v = v - __builtin_convertvector(h, f32x4);
      }
    } else {
      for (long long j = i; j < n; ++j) {
        float v = w[j];
        const int tv = wtab ? wtab[j >> 6] : (H16_WS | WTAB_BF16);
        if (nsp == 3)
          h16_pair(v, wtab_exp(tv), ((_Float16*)out)[H16_PLANE * plane + j], ((_Float16*)out)[(H16_PLANE + 1) * plane + j]);
        if (nsp != 3 || wtab_bf16(tv))
        for (int p = 0; p < nsp; ++p) {
          const __bf16 h = (__bf16)v;
          out[p * plane + j] = h;
          v -= (float)h;
        }
      }
    }
  }
}

// one 32x32 tile per block; tiles enumerated by the host table (tensor, tap, r0, c0)
__global__ __launch_bounds__(256) void shadow_t_kernel(const float* w, __bf16* out, const int4* tiles,
                                                       const long long* offs, int nsp, long long plane, const int* wtab) {
  __shared__ float t[32][33];
  const int4 d = tiles[blockIdx.x];  // x: tensor index, y: tap, z: r0, w: c0
  const long long off = offs[3 * d.x];
  const int R = (int)offs[3 * d.x + 1], Cc = (int)offs[3 * d.x + 2];
  const float* src = w + off + (long long)d.y * R * Cc;
  __bf16* dst = out + off + (long long)d.y * R * Cc;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int tv = (nsp == 3 && wtab) ? wtab[off >> 6] : (H16_WS | WTAB_BF16);
  const int ex = wtab_exp(tv);
  const int np = (nsp != 3 || wtab_bf16(tv)) ? nsp : 0;  // bf16 planes written (split mode: flagged tensors)
  for (int i = ty; i < 32; i += 8) {
    int r = d.z + i, c = d.w + tx;
    t[i][tx] = (r < R && c < Cc) ? src[(long long)r * Cc + c] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    int c = d.w + i, r = d.z + tx;
    if (r < R && c < Cc) {
      float v = t[tx][i];
      if (nsp == 3)  // split mode: the fp16 planes too
        h16_pair(v, ex, ((_Float16*)dst)[H16_PLANE * plane + (long long)c * R + r],
                 ((_Float16*)dst)[(H16_PLANE + 1) * plane + (long long)c * R + r]);
      for (int p = 0; p < np; ++p) {
        const __bf16 h = (__bf16)v;
        dst[p * plane + (long long)c * R + r] = h;
        v -= (float)h;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
// sum the K-split slabs; bias / act / accumulate into C; per-column (sum, sum^2) of the
// raw sums per 64-row block -> fixed-point column accumulators (same contract as the GEMM epilogue)
#define SKR_ROWS 64
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* part, int ks, int rows_total, int N,
                                                            float* C, long long c_gs, int ldc, const float* bias,
                                                            long long bias_gs, int act, int accumulate, u64* stats,
                                                            long long s_gs, long long s_sh, int s_nsh, BwStat bw,
                                                            int rpb, int c_bf16) {
  __shared__ f32x4 red[2][256];
  const int group = blockIdx.z;
  const int qi = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int n = (blockIdx.x * 16 + qi) * 4;
  const long long slab = (long long)rows_total * N;
  const float* P = part + (long long)group * ks * slab;
  float* Cg = C + group * c_gs;
  const float* bs = bias ? bias + group * bias_gs : nullptr;
  f32x4 s1 = {0.f, 0.f, 0.f, 0.f}, s2 = {0.f, 0.f, 0.f, 0.f};
  const bool bwq = bw.pre && n < bw.C;  // fused backward-BN terms on this column quad
  f32x4 bm = {0.f, 0.f, 0.f, 0.f}, bi = bm, bb = bm;
  if (bwq) {
    bm = *(const f32x4*)(bw.mean + group * bw.ms_gs + n);
    bi = *(const f32x4*)(bw.invstd + group * bw.ms_gs + n);
    if (!bw.y) bb = *(const f32x4*)(bw.beta + group * bw.beta_gs + n);
  }
  if (n < N) {
    const int r0 = blockIdx.y * rpb;  // rows per block: SKR_ROWS, or 16 for the few-row FC layers
    const int r1 = min(rows_total, r0 + rpb);
    // up to SKR_ROWS / 16 rows per thread: every load of all of them (slabs, accumulate target,
    // BN-backward pre / y) before the first store
    constexpr int NRT = SKR_ROWS / 16;
    f32x4 v[NRT], pr[NRT], yr[NRT];
    const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
    const f32x4 bsv = bs ? *(const f32x4*)(bs + n) : z4;
#pragma unroll
    for (int i = 0; i < NRT; ++i) {
      const int r = r0 + rl + 16 * i;
      v[i] = pr[i] = yr[i] = z4;
      if (r >= r1) continue;
      v[i] = *(const f32x4*)(P + (long long)r * N + n);
#pragma unroll 8
      for (int k = 1; k < ks; ++k) v[i] += *(const f32x4*)(P + k * slab + (long long)r * N + n);
      if (bwq) {
        pr[i] = pf_ld4(bw.pre, group * bw.pre_gs + (long long)r * bw.ldp + n, bw.pre_bf16 != 0);
        if (bw.y) yr[i] = pf_ld4(bw.y, group * bw.y_gs + (long long)r * bw.ldy + n, bw.y_bf16 != 0);
      }
    }
    f32x4 cv[NRT];
#pragma unroll
    for (int i = 0; i < NRT; ++i) {
      const int r = r0 + rl + 16 * i;
      cv[i] = (accumulate && r < r1) ? *(const f32x4*)(Cg + (long long)r * ldc + n) : z4;
    }
#pragma unroll
    for (int i = 0; i < NRT; ++i) {
      const int r = r0 + rl + 16 * i;
      if (r >= r1) continue;
      f32x4 w = v[i];
      if (c_bf16) {  // bf16-stored pre-BN output: the statistics of the stored values
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = bf_rnd(w[e]);
      }
      if (!bw.pre) {
        s1 += w;
        s2 += w * w;
      }
      if (bs) w += bsv;
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] = act_f(w[e], act);
      if (accumulate) w += cv[i];
      if (c_bf16)
        *(pf_bf16x4*)((__bf16*)C + group * c_gs + (long long)r * ldc + n) = __builtin_convertvector(w, pf_bf16x4);
      else
        *(f32x4*)(Cg + (long long)r * ldc + n) = w;
      if (bwq) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float sd = s1[e], sx = s2[e];
          bw_term_v(w[e], pr[i][e], bm[e], bi[e], bb[e], bw.y != nullptr, yr[i][e], bw.act, sd, sx);
          s1[e] = sd;
          s2[e] = sx;
        }
      }
    }
  }
  if (!stats) return;
  red[0][threadIdx.x] = s1;
  red[1][threadIdx.x] = s2;
  __syncthreads();
  const int SC = bw.pre ? bw.C : N;  // stats columns (row-block stride 2*SC)
  // one (column, sum|sum^2) per thread: the row lanes are combined in a fixed order and the
  // atomics issue in parallel
  if (threadIdx.x < 128) {
    const int cc = threadIdx.x & 63, kind = threadIdx.x >> 6, qq = cc >> 2, e = cc & 3;
    const int n2 = blockIdx.x * 64 + cc;
    if (n2 < SC) {
      float v = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) v += red[kind][j * 16 + qq][e];
      fx_add(stats + (blockIdx.y & (s_nsh - 1)) * s_sh + group * s_gs + 4LL * n2 + 2 * kind, v);
    }
  }
}

template <int BM, int BN, int WM, int WN>
static void launch_bf16(const FwdArgs& a, int groups, bool sc, hipStream_t s) {
  dim3 grid((a.rows + BM - 1) / BM, (a.N + BN - 1) / BN, groups * a.nclass * a.ksplit);
  if (a.a_bf16) {
    if (sc) hipLaunchKernelGGL((igemm_bf16_kernel<BM, BN, WM, WN, true, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((igemm_bf16_kernel<BM, BN, WM, WN, false, true>), grid, dim3(256), 0, s, a);
  } else {
    if (sc) hipLaunchKernelGGL((igemm_bf16_kernel<BM, BN, WM, WN, true, false>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((igemm_bf16_kernel<BM, BN, WM, WN, false, false>), grid, dim3(256), 0, s, a);
  }
}

static int bf16_bm(const FwdArgs& a) {
  if (a.N <= 32) return 256;
  if (a.N <= 64) return 128;
  return igemm_fwd_bm(a) == 128 ? 128 : 64;
}
static int bf16_bn(const FwdArgs& a) { return a.N <= 32 ? 32 : (a.N <= 64 ? 64 : 128); }

// ---- halo-tile planner: which (BM, BN) instance, window geometry, split-K ----
struct HaloPlan {
  bool ok = false;
  int bm = 0, bn = 0, kid = KID_NONE, ks = 1, nrb = 0;
  HaloArgs h;
  size_t lds = 0;
};
#define HALO_LDS_MAX (80 * 1024)  // two blocks per CU

// the large tile is kept only when it fills this many blocks; below it the smaller tile (no or
// less split-K) wins (tools/bench_gather.py: 16x16 / 8x8 conv-T layers).  SVAE_HALO_FILL overrides.
static int halo_fill() {
  static const int v = svae_knob("SVAE_HALO_FILL", 512);
  return v;
}

static HaloPlan halo_plan(const FwdArgs& a, int groups) {
  HaloPlan p;
  const ConvGeom& g = a.g;
  // N: multiples of 32, or a single partial 32-column tile (the 3/4-channel image-space layers)
  if (g.mode == GM_DENSE || g.ksz != 4 || a.Cin % HALO_CK != 0 || !a.Bh || (a.N % 32 != 0 && a.N > 32)) return p;
  const bool s2t = g.mode == GM_CONVT && g.stride == 2;
  const int Hr = s2t ? g.Ho / 2 : g.Ho, Wr = s2t ? g.Wo / 2 : g.Wo;
  const int sy = g.mode == GM_CONV ? g.stride : 1;
  const int span = s2t ? 2 : 4;
  if (g.mode == GM_CONVT && g.stride > 2) return p;
  // measured (tools/bench_gather.py, profiles/r01_v10_gather_microbench.txt): the v2 kernel is
  // faster than the per-tap kernel on every CelebA layer shape, 4x4 .. 32x32; only the LDS
  // window capacity below excludes shapes
  const int bn = a.N <= 32 ? 32 : (a.N <= 64 ? 64 : 128);
  const int cands[2] = {bn == 32 ? 256 : 128, bn == 32 ? 128 : 64};
  const int per_img = Hr * Wr;
  // the smaller tile of the two (128x32 / 64x64 / 64x128) by default since the gather-GEMMs run at
  // 4 waves per SIMD (v42: +0.8 % of the step over 4 same-box rounds); SVAE_HALO_SMALL=0 restores the
  // larger tile where it fills halo_fill() blocks
  static const bool small_only = svae_knob("SVAE_HALO_SMALL", 1) != 0;
  for (int ci = small_only ? 1 : 0; ci < 2; ++ci) {
    const int bm = cands[ci];
    if (bm % Wr != 0 || a.rows % bm != 0) continue;
    if (!(per_img % bm == 0 || bm % per_img == 0)) continue;
    HaloArgs h;
    h.Hr = Hr;
    h.Wr = Wr;
    h.R = bm >= per_img ? Hr : bm / Wr;
    h.nimg = bm >= per_img ? bm / per_img : 1;
    h.sy = sy;
    h.PR = (h.R - 1) * sy + span;
    h.PC = (Wr - 1) * sy + span;
    h.npix = h.nimg * h.PR * h.PC;
    if (h.npix * 4 > 256 * HALO_PI) continue;
    const size_t lds = (size_t)(2 * h.npix) * ROWP * sizeof(__bf16);
    if (lds > HALO_LDS_MAX) continue;
    const long long blocks = (long long)(a.rows / bm) * ((a.N + bn - 1) / bn) * a.nclass * groups;
    if (ci == 0 && blocks < halo_fill()) {  // prefer the smaller tile when the large one underfills
      const int bm2 = cands[1];
      if (bm2 % Wr == 0 && a.rows % bm2 == 0 && (per_img % bm2 == 0 || bm2 % per_img == 0)) {
        const int R2 = bm2 >= per_img ? Hr : bm2 / Wr, n2 = bm2 >= per_img ? bm2 / per_img : 1;
        const int np2 = n2 * ((R2 - 1) * sy + span) * ((Wr - 1) * sy + span);
        if (np2 * 4 <= 256 * HALO_PI && (size_t)(2 * np2) * ROWP * sizeof(__bf16) <= HALO_LDS_MAX) continue;
      }
    }
    p.ok = true;
    p.bm = bm;
    p.bn = bn;
    halo_divisors(h, g);
    p.h = h;
    p.lds = lds;
    const int nchunk = a.Cin / HALO_CK;
    int ks = 1;
    if (blocks < 512 && a.part && a.N % 4 == 0) {  // the split-K reduce works on column quads
      ks = (int)std::min<long long>((768 + blocks - 1) / blocks, 8);
      ks = std::min(ks, nchunk);
      const long long rows_total = (long long)a.rows * a.nclass;
      while (ks > 1 && (long long)ks * rows_total * a.N * groups > a.part_cap) --ks;
      if (ks < 2) ks = 1;
    }
    p.ks = ks;
    // a split of one chunk never prefetches a second window: one LDS buffer, so that three blocks
    // (the register limit) instead of two fit a CU and hide each other's window-load latency
    static const bool two_buf = svae_knob("SVAE_HALO_1BUF", 1) == 0;
    if (!two_buf && (nchunk + ks - 1) / ks <= 1) p.lds = (size_t)h.npix * ROWP * sizeof(__bf16);
    p.nrb = ks == 1 ? a.nclass * (a.rows / bm) : (int)(((long long)a.rows * a.nclass + SKR_ROWS - 1) / SKR_ROWS);
    if (bn == 32) p.kid = bm == 256 ? KID_HALO_256x32 : KID_HALO_128x32;
    else if (bn == 64) p.kid = bm == 128 ? KID_HALO_128x64 : KID_HALO_64x64;
    else p.kid = bm == 128 ? KID_HALO_128x128 : KID_HALO_64x128;
    return p;
  }
  return p;
}

template <int BM, int BN, int WM, int WN>
static void launch_halo(const HaloArgs& h, int groups, size_t lds, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)igemm_halo_kernel<BM, BN, WM, WN, false, false>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, HALO_LDS_MAX);
    hipFuncSetAttribute((const void*)igemm_halo_kernel<BM, BN, WM, WN, true, false>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, HALO_LDS_MAX);
    hipFuncSetAttribute((const void*)igemm_halo_kernel<BM, BN, WM, WN, false, true>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, HALO_LDS_MAX);
    hipFuncSetAttribute((const void*)igemm_halo_kernel<BM, BN, WM, WN, true, true>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, HALO_LDS_MAX);
    attr = true;
  }
  const FwdArgs& a = h.f;
  dim3 grid(a.rows / BM, (a.N + BN - 1) / BN, groups * a.nclass * a.ksplit);
  const bool s2t = a.g.mode == GM_CONVT && a.g.stride == 2;
  if (a.a_bf16) {
    if (s2t) hipLaunchKernelGGL((igemm_halo_kernel<BM, BN, WM, WN, true, true>), grid, dim3(256), lds, s, h);
    else hipLaunchKernelGGL((igemm_halo_kernel<BM, BN, WM, WN, false, true>), grid, dim3(256), lds, s, h);
  } else {
    if (s2t) hipLaunchKernelGGL((igemm_halo_kernel<BM, BN, WM, WN, true, false>), grid, dim3(256), lds, s, h);
    else hipLaunchKernelGGL((igemm_halo_kernel<BM, BN, WM, WN, false, false>), grid, dim3(256), lds, s, h);
  }
}

// the wave-split kernel (halo_kw.hip) is tried first wherever it fits: 32-column tiles, four waves
// over the taps (tools/bench_gather.py: 16x16 layers 39->27 / 24->18 us, 8x8 s2 conv-T 20->15).
// Until v42 the one-chunk 32x32 layers stayed on the tiled kernel (the wave split was 3-7 % slower
// per launch there); at 4 waves per SIMD (v41) the wave split on every layer is 2.3 % faster per
// step (v43, same-box A/B).  SVAE_KW: 0 = only instead of split-K, 1 = layers with >= 2 chunks
static bool kw_first(const FwdArgs& a, const HaloPlan& hp) {
  static const int mode = svae_knob("SVAE_KW", 2);  // 0 = only instead of split-K, 2 = wherever it fits
  if (hp.ks > 1) return true;
  if (mode == 2) return true;
  return mode == 1 && a.Cin >= 2 * HALO_CK;
}

static int halo_disabled() {
  static const int v = svae_knob("SVAE_NO_HALO", 0) == 1;
  return v;
}

// per-tap kernel (igemm_bf16_kernel) split-K and stats row-blocks
static int pertap_plan(const FwdArgs& a, int groups, int* ksplit) {
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

bool igemm_split_ok(const FwdArgs& a, int groups) {
  return a.Bh && !a.a_bf16 &&
         (dense_kw_ok(a, groups) || halo_x3_plan(a, groups) > 0 || halo_kw_plan(a, groups) > 0 || smalln_ok(a));
}

// bf16-stored pre-BN outputs (FwdArgs::c_bf16): every bf16 launch path of a BN-statistics GEMM implements
// them (wave-split / tiled halo, per-tap, their split-K reduce, the small-channel conv) except dense_kw
// (FC layers keep fp32 pre); the consumer-side BN launches run on halo_kw, which implements them too
bool igemm_c_bf16_ok(const FwdArgs& a, int groups) {
  if (a.nsp > 1 || !a.stats || a.bias || a.act != ACT_NONE || a.accumulate || a.bw.pre) return false;
  if (a.ldc % 4 || a.c_gs % 4 || ((uintptr_t)a.C & 7)) return false;
  if (a.ain.acc) return halo_kw_plan(a, groups) > 0;  // (the consumer-side BN launch: halo_kw only)
  return !dense_kw_ok(a, groups);
}

// the launch runs on halo_kw (igemm_bf16_path's choice), whose epilogue implements FwdArgs::fin
bool igemm_fin_ok(const FwdArgs& a, int groups) {
  if (!a.stats) return false;
  if (a.ain.acc) return halo_kw_plan(a, groups) > 0;
  if (a.nsp > 1) return !dense_kw_ok(a, groups) && halo_kw_plan(a, groups) > 0;
  if (smallc_ok(a, true) || dense_kw_ok(a, groups) || halo_disabled()) return false;
  const HaloPlan hp = halo_plan(a, groups);
  return hp.ok && kw_first(a, hp) && halo_kw_plan(a, groups) > 0;
}

int igemm_bf16_plan(const FwdArgs& a, int groups, int* ksplit) {
  if (a.ain.acc) {  // consumer-side BN of A: the wave-split halo gather only
    if (ksplit) *ksplit = 1;
    return halo_kw_plan(a, groups);
  }
  if (a.nsp > 1) {  // split-bf16 planes: dense_kw, halo_kw or the small-N conv-T (igemm_split_ok)
    if (ksplit) *ksplit = 1;
    if (dense_kw_ok(a, groups)) return dense_kw_nrb(a);
    const int nx3 = halo_x3_plan(a, groups);  // the fp16-plane gather (halo_x3.hip) first
    if (nx3 > 0) return nx3;
    const int nrb = halo_kw_plan(a, groups);
    return nrb > 0 ? nrb : 0;  // (convt_smalln: no statistics)
  }
  if (smallc_ok(a, true)) {
    if (ksplit) *ksplit = 1;
    return smallc_nrb(a);
  }
  if (dense_kw_ok(a, groups)) {  // FC layers: K over the waves of a block (dense_kw.hip)
    if (ksplit) *ksplit = 1;
    return dense_kw_nrb(a);
  }
  // (no shortcut for convt_smalln: it only takes launches without stats, and the plan is asked
  //  before a.stats is set -- a BN layer must plan as the kernel that will carry its stats)
  {
    const int nx3 = halo_x3_plan(a, groups);  // the lean wave-split gather (halo_x3.hip) first
    if (nx3 > 0) {
      if (ksplit) *ksplit = 1;
      return nx3;
    }
  }
  if (!halo_disabled()) {
    const HaloPlan hp = halo_plan(a, groups);
    if (hp.ok) {
      if (kw_first(a, hp)) {  // K split over the waves of one block where it fits
        const int nrb = halo_kw_plan(a, groups);
        if (nrb) {
          if (ksplit) *ksplit = 1;
          return nrb;
        }
      }
      if (ksplit) *ksplit = hp.ks;
      return hp.nrb;
    }
  }
  return pertap_plan(a, groups, ksplit);
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
      "wgrad_bf16_kernel<128, 128, 2, 2, true>", "wgrad_bf16_kernel<128, 128, 2, 2, false>",
      "igemm_halo_kernel<256, 32, 4, 1>", "igemm_halo_kernel<128, 32, 4, 1>",
      "igemm_halo_kernel<128, 64, 2, 2>", "igemm_halo_kernel<64, 64, 2, 2>",
      "igemm_halo_kernel<128, 128, 2, 2>", "igemm_halo_kernel<64, 128, 1, 4>",
      "wgrad_halo_kernel<32, 1>", "wgrad_halo_kernel<32, 2>", "wgrad_halo_kernel<64, 1>", "wgrad_halo_kernel<64, 2>",
      "wgrad_halo2_kernel (stride-1 halo weight-GEMM, all S = 1 instances)",
      "igemm_halo_kw_kernel (small-image gather-GEMM, K split over waves, all instances)",
      "wgrad_halo2_kernel (stride-2 halo weight-GEMM, all instances)",
      "gather_x3_kernel (wave-split halo gather: fp16 hi/lo planes in split mode, bf16 in bf16 mode; all instances)"};
  return (kid >= 0 && kid < KID_COUNT) ? names[kid] : "none";
}

int igemm_bf16_kid(const FwdArgs& a) {
  if (a.ain.acc) return halo_kw_plan(a, 1) > 0 ? KID_HALO_KW : KID_NONE;
  if (a.nsp > 1) {
    if (dense_kw_ok(a, 1)) return KID_NONE;
    if (halo_x3_plan(a, 1) > 0) return KID_HALO_X3;
    return halo_kw_plan(a, 1) > 0 ? KID_HALO_KW : KID_NONE;
  }
  if (halo_x3_plan(a, 1) > 0) return KID_HALO_X3;
  if (!halo_disabled()) {
    const HaloPlan hp = halo_plan(a, 1);
    if (hp.ok) return (kw_first(a, hp) && halo_kw_plan(a, 1)) ? KID_HALO_KW : hp.kid;
  }
  const int sc = (a.Cin % BKB) != 0;
  if (a.N <= 32) return KID_IGEMM_BF16_256x32 + sc;
  if (a.N <= 64) return KID_IGEMM_BF16_128x64 + sc;
  if (bf16_bm(a) == 128) return KID_IGEMM_BF16_128x128 + sc;
  return KID_IGEMM_BF16_64x128 + sc;
}

int wgrad_bf16_kid(const WgArgs& a) {
  // the vector gather decodes a quad of 4 row-space pixels once: they must lie on one image row
  // (row-space width a multiple of 4; a 2-wide layer took pixels of the next row at the wrong place)
  const int scalar = !((a.M % 4 == 0) && (a.ldg % 4 == 0) && (a.g.mode == GM_DENSE || a.g.Wo % 4 == 0));
  if (a.N <= 32) return KID_WGRAD_BF16_128x32 + scalar;
  if (a.N <= 64) return KID_WGRAD_BF16_128x64 + scalar;
  return KID_WGRAD_BF16_128x128 + scalar;
}

int igemm_bf16(FwdArgs a, int groups, hipStream_t s, hipEvent_t after) {
  return igemm_bf16_path(a, groups, 2, s, after);
}

int igemm_bf16_path(FwdArgs a, int groups, int path, hipStream_t s, hipEvent_t after) {
  if (a.ain.acc) {  // consumer-side BN of A (the caller checked halo_kw_plan)
    const int nrb = halo_kw(a, groups, s);
    if (after) hipEventRecord(after, s);
    return nrb;
  }
  if (a.nsp > 1 && !igemm_split_ok(a, groups)) return -2;  // no split kernel for this shape
  if (path == 2 && a.nsp <= 1 && smallc_ok(a, true)) {
    conv_smallc(a, groups, true, s);
    if (after) hipEventRecord(after, s);
    return smallc_nrb(a);
  }
  if (path == 2 && a.nsp <= 1 && smalln_ok(a)) {
    convt_smalln(a, groups, s);
    if (after) hipEventRecord(after, s);
    return 0;  // no stats (smalln_ok requires none)
  }
  if (path == 2 && dense_kw_ok(a, groups)) {
    const int ks = dense_kw(a, dense_kw_ks(a), s);
    if (after) hipEventRecord(after, s);
    if (ks > 1) {
      const int rpb = dense_kw_rpb(a);
      dim3 grid((a.N + 63) / 64, (a.rows + rpb - 1) / rpb, 1);
      hipLaunchKernelGGL(splitk_reduce_kernel, grid, dim3(256), 0, s, a.part, ks, a.rows, a.N, a.C, a.c_gs, a.ldc,
                         a.bias, a.bias_gs, a.act, a.accumulate, a.stats, a.s_gs, a.s_sh, a.s_nsh, a.bw, rpb, a.c_bf16);
    }
    return dense_kw_nrb(a);
  }
  if (a.nsp > 1) {  // igemm_split_ok: the wave-split halo gather takes every other split shape
    if (halo_x3_plan(a, groups) <= 0 && halo_kw_plan(a, groups) <= 0 && smalln_ok(a)) {  // the N <= 16 stride-2 conv-T (output layer, layer-0 dgrad)
      convt_smalln(a, groups, s);
      if (after) hipEventRecord(after, s);
      return 0;
    }
    int nrb = halo_x3(a, groups, s);  // the fp16-plane gather (halo_x3.hip) where it fits
    if (nrb < 0) nrb = halo_kw(a, groups, s);
    if (after) hipEventRecord(after, s);
    return nrb;
  }
  if (path == 2) {  // the lean wave-split gather (halo_x3.hip) where it fits
    const int nrb = halo_x3(a, groups, s);
    if (nrb >= 0) {
      if (after) hipEventRecord(after, s);
      return nrb;
    }
  }
  if (path == 1 || (path == 2 && !halo_disabled())) {
    HaloPlan hp = halo_plan(a, groups);
    if (!hp.ok && path == 1) return -1;
    if (hp.ok && path == 2 && kw_first(a, hp)) {  // K over the block's waves
      const int nrb = halo_kw(a, groups, s);
      if (nrb > 0) {
        if (after) hipEventRecord(after, s);
        return nrb;
      }
    }
    if (hp.ok) {
      a.ksplit = hp.ks;
      a.rows_total = a.rows * a.nclass;
      hp.h.f = a;
      switch (hp.kid) {
        case KID_HALO_256x32: launch_halo<256, 32, 4, 1>(hp.h, groups, hp.lds, s); break;
        case KID_HALO_128x32: launch_halo<128, 32, 4, 1>(hp.h, groups, hp.lds, s); break;
        case KID_HALO_128x64: launch_halo<128, 64, 2, 2>(hp.h, groups, hp.lds, s); break;
        case KID_HALO_64x64: launch_halo<64, 64, 2, 2>(hp.h, groups, hp.lds, s); break;
        case KID_HALO_128x128: launch_halo<128, 128, 2, 2>(hp.h, groups, hp.lds, s); break;
        default: launch_halo<64, 128, 1, 4>(hp.h, groups, hp.lds, s); break;
      }
      if (after) hipEventRecord(after, s);
      if (hp.ks > 1) {
        dim3 grid((a.N + 63) / 64, hp.nrb, groups);
        hipLaunchKernelGGL(splitk_reduce_kernel, grid, dim3(256), 0, s, a.part, hp.ks, a.rows_total, a.N, a.C, a.c_gs,
                           a.ldc, a.bias, a.bias_gs, a.act, a.accumulate, a.stats, a.s_gs, a.s_sh, a.s_nsh, a.bw, SKR_ROWS, a.c_bf16);
      }
      return hp.nrb;
    }
  }
  const bool sc = (a.Cin % BKB) != 0;
  int ks = 1;
  const int nrb = pertap_plan(a, groups, &ks);
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
                       a.bias, a.bias_gs, a.act, a.accumulate, a.stats, a.s_gs, a.s_sh, a.s_nsh, a.bw, SKR_ROWS, a.c_bf16);
  }
  return nrb;
}

template <int BM, int BN, int WM, int WN>
static void launch_wg_bf16(const WgArgs& a, int groups, bool vec, hipStream_t s) {
  dim3 grid((a.ntap * a.M + BM - 1) / BM, (a.N + BN - 1) / BN, groups * a.nsplit);
  if (a.nsp == 3) {
    if (vec) hipLaunchKernelGGL((wgrad_bf16_kernel<BM, BN, WM, WN, true, 3>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((wgrad_bf16_kernel<BM, BN, WM, WN, false, 3>), grid, dim3(256), 0, s, a);
  } else if (a.nsp == 2) {
    if (vec) hipLaunchKernelGGL((wgrad_bf16_kernel<BM, BN, WM, WN, true, 2>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((wgrad_bf16_kernel<BM, BN, WM, WN, false, 2>), grid, dim3(256), 0, s, a);
  } else {
    if (vec) hipLaunchKernelGGL((wgrad_bf16_kernel<BM, BN, WM, WN, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((wgrad_bf16_kernel<BM, BN, WM, WN, false>), grid, dim3(256), 0, s, a);
  }
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

// ---- halo weight-GEMM planner ----
static int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return (1 << l) == v ? l : -1;
}

int wgrad_halo_plan(const WgArgs& a, int groups, WHaloPlanOut* out) {
  const ConvGeom& g = a.g;
  if (g.mode != GM_CONV || g.ksz != 4 || a.ntap != 16 || (g.stride != 1 && g.stride != 2)) return 0;
  if (a.M % 32 != 0 || a.N % 32 != 0 || a.ldg % 4 != 0 || a.ldd % 4 != 0) return 0;
  const int lgWo = ilog2(g.Wo), per_img = g.Ho * g.Wo;
  if (lgWo < 2 || ilog2(per_img) < 0 || g.Ho != g.Wo) return 0;
  const int bn = 32;  // BN = 64 needs 128 accumulators per lane (1 wave/SIMD): not used
  const int S = g.stride;
  const int GP = S == 1 ? 32 : 48;
  for (int CP = 128; CP >= 32; CP >>= 1) {
    if (a.rows % CP != 0 || CP < g.Wo) continue;
    WHaloArgs h;
    h.CP = CP;
    h.lgWo = lgWo;
    if (CP <= per_img) {
      h.R = CP / g.Wo;
      h.img_per_ch = 1;
      h.ch_per_img = per_img / CP;
      h.lgImgPix = ilog2(CP);  // a chunk never spans images: image index term stays 0
    } else {
      h.R = g.Ho;
      h.img_per_ch = CP / per_img;
      h.ch_per_img = 0;
      h.lgImgPix = ilog2(per_img);
    }
    h.PR = (h.R - 1) * S + 4;
    h.PC = (g.Wo - 1) * S + 4;
    h.npix = h.img_per_ch * h.PR * h.PC;
    if (h.npix * 8 > 256 * WH_WPI || CP * bn / 4 > 256 * WH_DPI) continue;
    const size_t lds = ((size_t)h.npix * GP + (size_t)CP * bn) * sizeof(__bf16);
    if (lds > 64 * 1024) continue;
    h.nchunk = a.rows / CP;
    out->h = h;
    out->bn = bn;
    out->lds = lds;
    out->tiles = (a.M / 32) * (a.N / bn);
    return 1;
  }
  return 0;
}

static int wgrad_halo_disabled() {
  static const int v = svae_knob("SVAE_NO_HALO", 0) == 1;
  return v;
}
int wgrad_halo_enabled() { return !wgrad_halo_disabled(); }

void wgrad_halo(const WHaloPlanOut& pl, const WgArgs& a, int groups, hipStream_t s, hipEvent_t after) {
  WHaloArgs h = pl.h;
  h.w = a;
  dim3 grid(a.M / 32, a.N / pl.bn, groups * a.nsplit);
  const int op = (a.g_bf16 ? 1 : 0) | (a.d_bf16 ? 2 : 0);  // operand storage: compile-time in the kernel
#define WHL(BN_, S_)                                                                                   \
  switch (op) {                                                                                        \
    case 0: hipLaunchKernelGGL((wgrad_halo_kernel<BN_, S_, 0>), grid, dim3(256), pl.lds, s, h); break; \
    case 1: hipLaunchKernelGGL((wgrad_halo_kernel<BN_, S_, 1>), grid, dim3(256), pl.lds, s, h); break; \
    case 2: hipLaunchKernelGGL((wgrad_halo_kernel<BN_, S_, 2>), grid, dim3(256), pl.lds, s, h); break; \
    default: hipLaunchKernelGGL((wgrad_halo_kernel<BN_, S_, 3>), grid, dim3(256), pl.lds, s, h); break; \
  }
  if (pl.bn == 32) {
    if (a.g.stride == 1) { WHL(32, 1) } else { WHL(32, 2) }
  } else {
    if (a.g.stride == 1) { WHL(64, 1) } else { WHL(64, 2) }
  }
#undef WHL
  if (after) hipEventRecord(after, s);
}

void shadow_weights(const float* w, void* wn, void* wt, long long n, const void* tiles, int ntiles, const void* offs,
                    int nsp, long long plane, hipStream_t s, const int* wtab) {
  long long q = (n + 3) / 4;
  int blocks = (int)std::min<long long>((q + 255) / 256, 8192);
  hipLaunchKernelGGL(shadow_n_kernel, dim3(blocks), dim3(256), 0, s, w, (__bf16*)wn, n, nsp, plane, wtab);
  if (ntiles > 0)
    hipLaunchKernelGGL(shadow_t_kernel, dim3(ntiles), dim3(256), 0, s, w, (__bf16*)wt, (const int4*)tiles,
                       (const long long*)offs, nsp, plane, wtab);
}

void shadow_t_tiles(const float* w, void* wt, const void* tiles, int ntiles, const void* offs, int nsp, long long plane,
                    hipStream_t s, const int* wtab) {
  if (ntiles > 0)
    hipLaunchKernelGGL(shadow_t_kernel, dim3(ntiles), dim3(256), 0, s, w, (__bf16*)wt, (const int4*)tiles,
                       (const long long*)offs, nsp, plane, wtab);
}

// ---------------------------------------------------------------------------
// the fp16 weight planes' per-tensor exponents (common.h h16_wexp): max |w| per tensor -> exponent table
// ---------------------------------------------------------------------------
__device__ float wexp_block_max(const float* w, long long n) {  // max |w[0..n)| over the block (256 threads)
  __shared__ float wm[4];
  float m = 0.f;
  for (long long i = threadIdx.x; i < n; i += blockDim.x) m = fmaxf(m, fabsf(w[i]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  return fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
}

// one block per tensor: its exponent into every 64-float block entry the tensor covers
__device__ int wexp_set(const float* w, const long long* info, int t, int* wtab) {
  const long long off = info[4 * t], n = info[4 * t + 1];
  const int e = h16_wexp(wexp_block_max(w + off, n));
  for (long long b = (off >> 6) + threadIdx.x; b < ((off + n + 63) >> 6); b += blockDim.x)
    wtab[b] = (wtab[b] & ~0xffff) | (e & 0xffff);  // (the bf16-planes flag stays)
  return e;
}

__global__ __launch_bounds__(256) void wexp_refresh_kernel(const float* w, const long long* info, int* wtab, int* ovf) {
  wexp_set(w, info, blockIdx.x, wtab);
  if (blockIdx.x == 0 && threadIdx.x == 0) *ovf = 0;  // the shadow pass that follows rewrites every plane
}

// one block (runs in every split-mode forward; returns at once unless an Adam update raised the flag)
__global__ __launch_bounds__(256) void wexp_fixup_kernel(const float* w, const long long* info, int ntensor, int* wtab,
                                                         int* ovf, _Float16* wn, _Float16* wt, long long plane) {
  if (*ovf == 0) return;
  for (int t = 0; t < ntensor; ++t) {
    const int e = wexp_set(w, info, t, wtab);
    const long long off = info[4 * t], n = info[4 * t + 1];
    const int R = (int)info[4 * t + 2], Cc = (int)info[4 * t + 3];
    const long long per = (long long)R * Cc;
    for (long long i = threadIdx.x; i < n; i += blockDim.x) {
      _Float16 h0, h1;
      h16_pair(w[off + i], e, h0, h1);
      wn[H16_PLANE * plane + off + i] = h0;  // N layout
      wn[(H16_PLANE + 1) * plane + off + i] = h1;
      const long long tap = i / per, rc = i - tap * per;  // per-tap transpose: [tap][r][c] -> [tap][c][r]
      const int r = (int)(rc / Cc), c = (int)(rc - (long long)r * Cc);
      const long long j = off + tap * per + (long long)c * R + r;
      wt[H16_PLANE * plane + j] = h0;
      wt[(H16_PLANE + 1) * plane + j] = h1;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *ovf = 0;
}

void wexp_refresh(const float* w, const long long* info, int ntensor, int* wtab, int* ovf, hipStream_t s) {
  if (ntensor > 0) hipLaunchKernelGGL(wexp_refresh_kernel, dim3(ntensor), dim3(256), 0, s, w, info, wtab, ovf);
}

void wexp_fixup(const float* w, const long long* info, int ntensor, int* wtab, int* ovf, void* wn, void* wt,
                long long plane, hipStream_t s) {
  if (ntensor > 0)
    hipLaunchKernelGGL(wexp_fixup_kernel, dim3(1), dim3(256), 0, s, w, info, ntensor, wtab, ovf, (_Float16*)wn,
                       (_Float16*)wt, plane);
}
