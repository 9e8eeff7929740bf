// Small-image halo gather-GEMM with the K dimension split over the block's waves (bf16 MFMA).
//
// The 8x8 and 4x4 layers of the ladders (CelebA: every level-2 conv / conv-T, the encoder's last
// conv, and their input gradients) have only 8K or 2K output pixels per chain step.  Tiled like
// the larger layers they give 128-256 blocks, so igemm_halo_kernel splits K over the grid and a
// separate splitk_reduce pass sums fp32 partial slabs (up to 6 x 4 MB written, read back, one more
// launch).  Here a block owns BM x 32 outputs and all of K: each of its four waves runs a quarter
// of the taps of every 32-channel chunk (kernel row ky = wave; for stride-2 conv-T classes one tap
// each) over the SAME staged input window, and the four partial tiles are summed in LDS in a fixed
// wave order before one epilogue (bias / act / accumulate, forward BN statistics or the fused
// backward-BN partials, exactly the splitk_reduce contract).  32-column tiles give >= 512 blocks.
//
// Window geometry, staging and A-fragment addressing follow igemm_halo_kernel (gemm_bf16.hip):
//   CONV          iy = ry*s - pad + ky         window rows (R-1)*s + 4, dy = ky
//   CONVT s=1     iy = ry + pad - ky           window rows R + 3,       dy = 3 - ky
//   CONVT s=2     class (cy,cx), ky = k0+2*ty  window rows R + 1,       dy = 1 - ty
#include <cstdlib>

#include "common.h"
#include "kernels.h"
#include "knobs.h"
#include "opload.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x8 __attribute__((ext_vector_type(8)));

#define KW_CK 32   // channels per window stage
#define KW_ROWP 40 // LDS pixel pitch in bf16 (80 B: conflict-free 16-B fragment reads)
#define KW_PI 4    // window items (8 channels) per thread: npix * 4 <= 256 * KW_PI
#ifndef KW_OCC
#define KW_OCC 4   // waves per SIMD of the bf16-A 32-column instances (5 spills 38 VGPRs)
#endif
#ifndef KW_OCC_BR
#define KW_OCC_BR 5  // the same with the two-tap B ring
#endif
#ifndef KW_OCC_H16
#define KW_OCC_H16 4  // the split mode's fp16-plane instances (two planes: ~24 VGPRs fewer than three)
#endif
#ifndef KW_OCC_H16_64
#define KW_OCC_H16_64 3  // (4 spills 8-26 VGPRs)
#endif
#ifndef KW_OCC_H16_128
#define KW_OCC_H16_128 2
#endif
#ifndef KW_OCC_S32
#define KW_OCC_S32 3  // split-mode 32-row instances with the B ring (4 spills 17-18 VGPRs)
#endif

struct KwArgs {
  FwdArgs f;
  int Hr, Wr;   // row-space image dims (per parity class for conv-T stride 2)
  int R, nimg;  // image rows per block (per image), images per block
  int PR, PC;   // window dims per image
  int sy;       // row-space -> input stride (conv stride, else 1)
  int npix;     // nimg * PR * PC
  // launch-constant divisors (multiply-shift): the kernel's index decode has no integer divisions
  FastDiv d_win, d_pc, d_img, d_wr, d_rimg, d_q, d_qw;  // PR*PC, PC, Hr*Wr, Wr, R*Wr, (Ho/2)*(Wo/2), Wo/2
  int ntx, nty, ntz;  // tiles along rows / columns / (groups x classes)
  int tpb;            // tiles per block: 1 = one tile per block (3-D grid); > 1 = persistent (1-D grid)
  int vec;            // 16-byte epilogue (every epilogue operand row 16-byte aligned; SVAE_KW_VEC)
  int ain_off;        // byte offset of the consumer-side BN table [3][Cin] in dynamic LDS (f.ain.acc != nullptr)
  int slot_off;       // NS = 2: byte offset of the [2][4] wave maxima of |A| in dynamic LDS
};

namespace {

__device__ __forceinline__ long long kw_out_row(const KwArgs& h, const ConvGeom& g, int cls, int m) {
  if (g.mode == GM_CONVT && g.stride == 2) {
    const int n = fdiv(m, h.d_q);
    const int r = m - n * h.d_q.d;
    const int qy = fdiv(r, h.d_qw), qx = r - qy * h.d_qw.d;
    return ((long long)n * g.Ho + 2 * qy + (cls >> 1)) * g.Wo + 2 * qx + (cls & 1);
  }
  return m;
}

// The epilogue with 16-byte accesses (h.vec: every operand row 16-byte aligned): thread = 4
// consecutive columns of BM / (256 / (BN / 4)) rows.  The four waves' partial tiles (red, [4][BM][BN]
// fp32) are summed in wave order, then bias / act / accumulate, one 16-byte store per row, the
// forward BN statistics or the fused backward-BN partials per column (row groups summed in LDS in a
// fixed order: deterministic).  Stores go through st_out16 (write-through in SVAE_WT builds: a
// 16-byte sc1 store costs what a plain one does, a 4-byte one six times as much per byte).
template <int BM, int BN, bool PB, bool YB>
__device__ __forceinline__ void kw_epilogue_vec(const KwArgs& h, float* red, int tid, int m0, int n0, int group, int cls) {
  const FwdArgs& a = h.f;
  const ConvGeom& g = a.g;
  constexpr int TPR = BN / 4;       // threads per row
  constexpr int NRG = 256 / TPR;    // row groups
  constexpr int NR = BM / NRG > 0 ? BM / NRG : 1;
  const int c4 = (tid % TPR) * 4, rg = tid / TPR;
  const int n = n0 + c4;
  float* Cp = a.C + group * a.c_gs;
  const bool bwm = a.bw.pre != nullptr;
  const bool bwc = bwm && n < a.bw.C;  // (bw.C % 4 == 0: whole quads)
  f32x4 bm = {0.f, 0.f, 0.f, 0.f}, bi = bm, bb = bm, biasv = bm;
  if (bwc) {
    bm = *(const f32x4*)&a.bw.mean[group * a.bw.ms_gs + n];
    bi = *(const f32x4*)&a.bw.invstd[group * a.bw.ms_gs + n];
    if (!a.bw.y) bb = *(const f32x4*)&a.bw.beta[group * a.bw.beta_gs + n];
  }
  if (a.bias) biasv = *(const f32x4*)&a.bias[group * a.bias_gs + n];
  constexpr bool pbf = PB;  // (compile-time: a run-time choice per load serialises the batch's loads)
  const float* bwpre = bwc ? pf_at(a.bw.pre, group * a.bw.pre_gs, pbf) : nullptr;
  const float* bwy = (bwc && a.bw.y) ? pf_at(a.bw.y, group * a.bw.y_gs, YB) : nullptr;
  const bool rows_ok = rg < BM;  // (NRG > BM: the extra row groups idle)
  long long orow[NR];
  f32x4 cv[NR], pv[NR], yv[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) {  // every global load before the first store
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    cv[i] = pv[i] = yv[i] = z;
    orow[i] = 0;
    if (!rows_ok) continue;
    orow[i] = kw_out_row(h, g, cls, m0 + rg + i * NRG);
    if (a.accumulate) cv[i] = *(const f32x4*)&Cp[orow[i] * a.ldc + n];
    if (bwpre) pv[i] = pf_ld4(bwpre, orow[i] * a.bw.ldp + n, pbf);
    if (bwy) yv[i] = pf_ld4(bwy, orow[i] * a.bw.ldy + n, YB);
  }
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    if (!rows_ok) continue;
    const int m = rg + i * NRG;
    f32x4 v = *(const f32x4*)&red[(0 * BM + m) * BN + c4];
#pragma unroll
    for (int w = 1; w < 4; ++w) v += *(const f32x4*)&red[(w * BM + m) * BN + c4];
    if (a.c_bf16) {  // bf16-stored pre-BN output: the statistics of the stored values
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = bf_rnd(v[j]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float x = v[j];
      if (!bwm) {
        s1[j] += x;
        s2[j] += x * x;
      }
      if (a.bias) x += biasv[j];
      x = act_f(x, a.act);
      if (a.accumulate) x += cv[i][j];
      v[j] = x;
      if (bwc) bw_term_v(x, pv[i][j], bm[j], bi[j], bb[j], bwy != nullptr, yv[i][j], a.bw.act, s1[j], s2[j]);
    }
    if (a.c_bf16)
      st_out8((__bf16*)a.C + group * a.c_gs + orow[i] * a.ldc + n, __builtin_bit_cast(u64, __builtin_convertvector(v, pf_bf16x4)));
    else
      st_out16(Cp, orow[i] * a.ldc + n, v);
  }
  if (a.stats) {
    __syncthreads();  // every wave is done reading red
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      red[rg * BN + c4 + j] = s1[j];
      red[NRG * BN + rg * BN + c4 + j] = s2[j];
    }
    __syncthreads();
    if (tid < BN) {
      const int SC = bwm ? a.bw.C : a.N;  // stats columns (row-block stride 2*SC)
      if (n0 + tid < SC) {
        float sa = 0.f, qa = 0.f;
        for (int j = 0; j < NRG; ++j) {
          sa += red[j * BN + tid];
          qa += red[NRG * BN + j * BN + tid];
        }
        const int rb = cls * h.ntx + m0 / BM;
        stat_put(a.stats + (rb & (a.s_nsh - 1)) * a.s_sh + group * a.s_gs, n0 + tid, sa, qa);
      }
    }
    if (a.fin.cnt) bn_fin_arrive(a.fin, group, (int*)red);
  }
}

// bf16-A 32-column instances at 4 waves per SIMD (<= 128 VGPRs, no spills; was 132 -> 3 waves): +0.3 %
// of the step in a same-box A/B (tools/gpu/r02_libab.sh); the fp32-A ones would spill
// NS = 3: the split-bf16 mode (dtype bf16x6, opload.h split8 / mfma_split): the fp32 window is
// staged as three bf16 planes (one LDS buffer, restaged under a second barrier per chunk) and every
// A x B fragment pair runs the six plane products; B comes from the three shadow planes
// PST: the persistent form (h.tpb > 1 tiles per block, 1-D grid); without it the tile loop runs once
// BR: B fragments through a two-tap register ring (tap u + 1's loads issued under tap u's MFMAs; the
// next chunk's first tap under the last) instead of a whole chunk of taps one chunk ahead: 16-tap
// instances only; frees (NTW - 2) x TN x 2 x NS fragment registers (split mode: 48 VGPRs)
// PI: window items per thread (npix * 4 <= 256 * PI); 3 frees 8 (fp32) window registers
// AIN: the bf16-A instances that take the consumer-side BN (a bf16-stored pre-BN tensor); the fp32-A ones
// take it at run time (in the bf16-A ones it would cost the default instances 12-15 spilled VGPRs)
template <int BM, int BN, bool S2T, bool ABF, int NS = 1, bool PST = false, bool BR = false, int PI = KW_PI,
          bool AIN = false>
__global__ __launch_bounds__(256, AIN ? (S2T ? 4 : 3) : (ABF && BN == 32 && BM <= 64 && !PST) ? ((BR || S2T) ? KW_OCC_BR : KW_OCC)
                                                                         : NS == 2 ? (BM == 128 ? KW_OCC_H16_128 : BM == 64 ? KW_OCC_H16_64 : KW_OCC_H16)
                                                                         : ((NS == 3 && BR) ? (BM == 32 ? KW_OCC_S32 : (BM == 128 ? 2 : 3)) : 2))
void igemm_halo_kw_kernel(KwArgs h) {
  static_assert(NS == 1 || ((NS == 2 || NS == 3) && !ABF), "split planes from fp32 activations only");
  static_assert(!BR || !S2T, "the B ring: 16-tap instances");
  static_assert(!(PST && NS == 2), "the fp16 planes' running exponent is per tile");
  constexpr int TM = BM / 32;
  constexpr int TN = BN / 32;
  constexpr int NTAP = S2T ? 4 : 16;
  constexpr int NTW = NTAP / 4;  // taps per wave (and B prefetch distance: one chunk ahead)
  constexpr int NBQ = BR ? 2 : NTW;  // B fragment slots
  extern __shared__ __attribute__((aligned(16))) __bf16 ksm[];
  const FwdArgs& a = h.f;
  const ConvGeom& g = a.g;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  constexpr bool abf = ABF;
#ifdef SVAE_EXP_STAMPS  // timing experiment: per-wave phase stamps (s_memtime) into the split-K scratch
  unsigned long long* stamp_p = (unsigned long long*)a.part +
      ((long long)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) * 4 + wave) * 16;
#define KW_STAMP(i) do { if (lane == 0 && (i) < 16) stamp_p[(i)] = __builtin_readcyclecounter(); } while (0)
#else
#define KW_STAMP(i) do {} while (0)
#endif
  KW_STAMP(0);
  const int nchunk = a.Cin / KW_CK;
  const int per_img = h.Hr * h.Wr;

  // ---- tiles of this block: one (3-D XCD-ordered grid), or a contiguous run of tpb tiles of the
  // linear order (x fastest, then y, then z) in the persistent form (1-D grid): tile i + 1's
  // window and B fragments are loaded while tile i's last chunk computes and its epilogue runs ----
  long long t_cur, t_end;
  int bx, by, bz;
  if constexpr (!PST) {
    const BlockXYZ blk = xcd_block();
    bx = blk.x; by = blk.y; bz = blk.z;
    t_cur = 0; t_end = 1;
  } else {
    const long long ntiles = (long long)h.ntx * h.nty * h.ntz;
    t_cur = (long long)blockIdx.x * h.tpb;
    t_end = t_cur + h.tpb < ntiles ? t_cur + h.tpb : ntiles;
    bx = (int)(t_cur % h.ntx); by = (int)((t_cur / h.ntx) % h.nty); bz = (int)(t_cur / ((long long)h.ntx * h.nty));
  }

  // per-tile geometry (uniform): the current tile's, and the next one's while its loads are issued
  struct TileG {
    int m0, n0, group, cls, tap0;
  };
  auto tile_geo = [&](int x, int y, int z) {
    TileG q;
    q.group = z / a.nclass;
    q.cls = z - q.group * a.nclass;
    q.m0 = x * BM;
    q.n0 = y * BN;
    q.tap0 = 0;
    if (S2T) {
      const int cy = q.cls >> 1, cx = q.cls & 1;
      q.tap0 = ((cy + g.pad) & 1) * 4 + ((cx + g.pad) & 1);
    }
    return q;
  };
  // tap shift constants (the same for every tile of a launch)
  int toff0, tsgn;
  if (S2T) {
    toff0 = h.PC + 1;
    tsgn = -1;
  } else if (g.mode == GM_CONV) {
    toff0 = 0;
    tsgn = 1;
  } else {
    toff0 = 3 * h.PC + 3;
    tsgn = -1;
  }

  int woff[PI];
  auto set_window = [&](const TileG& q) {  // window item offsets of tile q (igemm_halo_kernel's origin)
    int oy_min, ox_min;
    if (S2T) {
      const int cy = q.cls >> 1, cx = q.cls & 1;
      const int ky0 = (cy + g.pad) & 1, kx0 = (cx + g.pad) & 1;
      oy_min = (cy + g.pad - ky0) / 2 - 1;
      ox_min = (cx + g.pad - kx0) / 2 - 1;
    } else if (g.mode == GM_CONV) {
      oy_min = ox_min = -g.pad;
    } else {
      oy_min = ox_min = g.pad - 3;
    }
    const int img0 = fdiv(q.m0, h.d_img);
    const int ry0 = fdiv(q.m0 - img0 * per_img, h.d_wr);
    const int iy_base = ry0 * h.sy + oy_min;
#pragma unroll
    for (int i = 0; i < PI; ++i) {
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
  };
  f32x4 wv[PI][2];
  auto load_window = [&](const TileG& q, int chunk) {
    const long long ac = q.group * a.a_gs + chunk * KW_CK;
#pragma unroll
    for (int i = 0; i < PI; ++i) {
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      wv[i][0] = z;
      wv[i][1] = z;
      if (woff[i] >= 0) ld8_raw(a.A, ac + woff[i], abf, wv[i][0], wv[i][1]);
    }
  };
  // consumer-side BN (a.ain): a = act(bn_y(pre)) of the chunk's 8 channels of this thread (every item of
  // a thread has the same channel part tid & 3), table [mean | invstd | beta][Cin] in LDS
  const bool ain = (!ABF || AIN) && a.ain.acc != nullptr;
  const float* ain_tbl = (const float*)((const char*)ksm + h.ain_off);
  auto ain_apply = [&](f32x4& lo, f32x4& hi, int chunk) {
    const int c0 = chunk * KW_CK + (tid & 3) * 8;
    const f32x4 m0 = *(const f32x4*)&ain_tbl[c0], m1 = *(const f32x4*)&ain_tbl[c0 + 4];
    const f32x4 s0 = *(const f32x4*)&ain_tbl[a.Cin + c0], s1 = *(const f32x4*)&ain_tbl[a.Cin + c0 + 4];
    const f32x4 b0 = *(const f32x4*)&ain_tbl[2 * a.Cin + c0], b1 = *(const f32x4*)&ain_tbl[2 * a.Cin + c0 + 4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      lo[j] = act_f(bn_y1(lo[j], m0[j], s0[j], b0[j]), a.ain.act);
      hi[j] = act_f(bn_y1(hi[j], m1[j], s1[j], b1[j]), a.ain.act);
    }
  };
  // NS == 2 (scaled fp16 planes): the block-wide running max of |A| over the chunks staged so far and
  // its exponent hs (A is staged as A * 2^hs; every wave's accumulator is kept in the current units and
  // shrunk by the exponent step when a chunk raises the max, exact powers of two)
  [[maybe_unused]] int hs = 0;
  [[maybe_unused]] float hmax = 0.f;
  [[maybe_unused]] float* hslot = (float*)((char*)ksm + h.slot_off);
  auto wave_max_put = [&](int parity) {  // this wave's max |A| of the registers holding the next chunk
    float m = 0.f;
#pragma unroll
    for (int i = 0; i < PI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) m = fmaxf(m, fmaxf(fabsf(wv[i][0][j]), fabsf(wv[i][1][j])));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if (lane == 0) hslot[parity * 4 + wave] = m;
  };
  auto take_scale = [&](int parity) {  // (after a barrier) the new exponent; returns the step (<= 0)
    const float m = fmaxf(fmaxf(hslot[parity * 4], hslot[parity * 4 + 1]), fmaxf(hslot[parity * 4 + 2], hslot[parity * 4 + 3]));
    hmax = fmaxf(hmax, m);
    const int ns = h16_exp(hmax);
    const int d = ns - hs;
    hs = ns;
    return d;
  };
  // NS == 1: buffer `buf` of two; NS == 3 / 2: plane p of the one buffer at p * npix * KW_ROWP
  auto store_window = [&](int buf, int chunk) {
    __bf16* W = ksm + buf * h.npix * KW_ROWP;
#pragma unroll
    for (int i = 0; i < PI; ++i) {
      const int it = tid + 256 * i;
      if (woff[i] < -1) continue;
      if (ain && woff[i] >= 0) {  // (padding stays 0)
        if constexpr (ABF) {  // bf16-stored pre: widen, apply, round back (bn_apply's bf16 output, bitwise)
          const ol_f32x8 w8 = __builtin_convertvector(__builtin_bit_cast(bf16x8, wv[i][0]), ol_f32x8);
          f32x4 lo = {w8[0], w8[1], w8[2], w8[3]}, hi = {w8[4], w8[5], w8[6], w8[7]};
          ain_apply(lo, hi, chunk);
          wv[i][0] = __builtin_bit_cast(f32x4, raw8_bf(lo, hi, false));
        } else {
          ain_apply(wv[i][0], wv[i][1], chunk);
        }
      }
      const int o = (it >> 2) * KW_ROWP + (it & 3) * 8;
      if constexpr (NS == 1) {
        *(bf16x8*)&W[o] = raw8_bf(wv[i][0], wv[i][1], abf);
      } else {
        bf16x8 pl[NS];
#ifdef SVAE_EXP_NOSPLIT  // timing experiment (wrong results): one conversion, copied to every plane
        pl[0] = raw8_bf(wv[i][0], wv[i][1], false);
        for (int p = 1; p < NS; ++p) pl[p] = pl[0];
#else
        if constexpr (NS == 2) split8_h16(wv[i][0], wv[i][1], hs, pl);
        else split8<NS>(wv[i][0], wv[i][1], pl);
#endif
#pragma unroll
        for (int p = 0; p < NS; ++p) *(bf16x8*)&ksm[p * h.npix * KW_ROWP + o] = pl[p];
      }
    }
  };

  // ---- A fragment bases: the whole BM-row tile, every wave (the same for every tile) ----
  int abase[TM];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int ml = tm * 32 + l32;
    const int rows_img = h.R * h.Wr;
    const int il = fdiv(ml, h.d_rimg);
    const int rem = ml - il * rows_img;
    const int ryl = fdiv(rem, h.d_wr), rx = rem - ryl * h.Wr;
    abase[tm] = ((il * h.PR + ryl * h.sy) * h.PC + rx * h.sy) * KW_ROWP + 8 * hh;
  }

  // ---- this wave's taps: t = wave * NTW + u; B fragments one chunk ahead ----
  bf16x8 bq[NBQ][TN][2][NS];
  auto load_b = [&](const TileG& q, int slot, int u, int chunk) {
    const __bf16* bptr = (const __bf16*)a.Bh + q.group * a.b_gs + (long long)(q.n0 + l32) * a.ldb + 8 * hh;
    const int t = wave * NTW + u;
    const int tap = S2T ? q.tap0 + 8 * (t >> 1) + 2 * (t & 1) : t;
#ifdef SVAE_EXP_BL1  // timing experiment (wrong results): every B fragment from one L1-resident tap / chunk
    const long long off = 0 * (tap + chunk);
#else
    const long long off = (long long)tap * a.b_tap + chunk * KW_CK;
#endif
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
      for (int kq = 0; kq < 2; ++kq)
#pragma unroll
        for (int p = 0; p < NS; ++p)
          bq[slot][tn][kq][p] = *(const bf16x8*)(bptr + p * a.b_plane + (long long)tn * 32 * a.ldb + off + kq * 16);
  };

  TileG cur = tile_geo(bx, by, bz);
  if (ain) {  // finalise the producer's statistics of every input channel (bn_apply's expression)
    float* tbl = (float*)((char*)ksm + h.ain_off);
    const int g = cur.group;
    for (int c = tid; c < a.Cin; c += 256) {
      if (a.ain.fin) {  // the producer's last block finalised them (BnFin)
        tbl[c] = a.ain.mean[g * a.ain.ms_gs + c];
        tbl[a.Cin + c] = a.ain.invstd[g * a.ain.ms_gs + c];
        tbl[2 * a.Cin + c] = a.ain.beta[g * a.ain.beta_gs + c];
        continue;
      }
      const u64* base = a.ain.acc + g * a.ain.acc_gs + 4LL * c;
      u64 t[4] = {0, 0, 0, 0};
      for (int k = 0; k < a.ain.nsh; ++k)
#pragma unroll
        for (int w = 0; w < 4; ++w) t[w] += base[k * a.ain.sh + w];
      const double cnt = (double)a.ain.rows;
      const double md = fx_get(t) / cnt;
      double var = fx_get(t + 2) / cnt - md * md;
      if (var < 0.0) var = 0.0;
      const float m = (float)md, is = (float)(1.0 / sqrt(var + (double)a.ain.eps));
      tbl[c] = m;
      tbl[a.Cin + c] = is;
      tbl[2 * a.Cin + c] = a.ain.beta[g * a.ain.beta_gs + c];
      if (bx == 0 && by == 0 && a.ain.mean) {
        a.ain.mean[g * a.ain.ms_gs + c] = m;
        a.ain.invstd[g * a.ain.ms_gs + c] = is;
      }
    }
    __syncthreads();
  }
  KW_STAMP(13);
  set_window(cur);
  load_window(cur, 0);
  if constexpr (BR) {
    load_b(cur, 0, 0, 0);
  } else {
#pragma unroll
    for (int u = 0; u < NTW; ++u) load_b(cur, u, u, 0);
  }
  if constexpr (NS == 1) {
    store_window(0, 0);
    __syncthreads();
  }
  KW_STAMP(14);
  if constexpr (NS == 2) {
    wave_max_put(0);
    __syncthreads();
  }
  KW_STAMP(1);
  for (;;) {
    // the next tile of this block (persistent form)
    const bool has_tile = PST && t_cur + 1 < t_end;
    TileG nxt = cur;
    if (has_tile) {
      const long long tn_ = t_cur + 1;
      nxt = tile_geo((int)(tn_ % h.ntx), (int)((tn_ / h.ntx) % h.nty), (int)(tn_ / ((long long)h.ntx * h.nty)));
    }
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    for (int c = 0; c < nchunk; ++c) {
      const int buf = NS == 1 ? (c & 1) : 0;
      const bool has_next = c + 1 < nchunk;
      if constexpr (NS > 1) {  // one buffer of NS planes: stage chunk c, then prefetch c + 1
        if constexpr (NS == 2) {
          const int d = take_scale(c & 1);
          if (d != 0) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
              for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = __builtin_ldexpf(acc[i][j][r], d);
          }
        }
        store_window(0, c);
        __syncthreads();
      }
      if (c < 4) KW_STAMP(2 + 2 * c);
      if constexpr (!BR) {
        if (has_next) {
          load_window(cur, c + 1);
        } else if (has_tile) {  // the next tile's first window, under this chunk's MFMAs and the epilogue
          set_window(nxt);
          load_window(nxt, 0);
        }
      }
      const __bf16* W = ksm + buf * h.npix * KW_ROWP;
#pragma unroll
      for (int u = 0; u < NTW; ++u) {
        if constexpr (BR) {  // the ring: the next tap's B (this chunk's, or the next chunk's first)
          if (u + 1 < NTW) load_b(cur, (u + 1) & 1, u + 1, c);
          else if (has_next) load_b(cur, (u + 1) & 1, 0, c + 1);
          else if (has_tile) load_b(nxt, (u + 1) & 1, 0, 0);  // persistent: the next tile's first tap
          // the next chunk's (or tile's) window after tap 1's B loads (in-order vmcnt: a later B wait
          // also waits for it)
          if (u == 0) {
            if (has_next) {
              load_window(cur, c + 1);
            } else if (has_tile) {
              set_window(nxt);
              load_window(nxt, 0);
            }
          }
        }
        const int t = wave * NTW + u;
        const int shift = S2T ? toff0 + tsgn * ((t >> 1) * h.PC + (t & 1)) : toff0 + tsgn * ((t >> 2) * h.PC + (t & 3));
        const int sh = shift * KW_ROWP;
#pragma unroll
        for (int kq = 0; kq < 2; ++kq) {
          bf16x8 af[TM][NS];
#pragma unroll
          for (int tm = 0; tm < TM; ++tm)
#pragma unroll
            for (int p = 0; p < NS; ++p) af[tm][p] = *(const bf16x8*)&W[p * h.npix * KW_ROWP + abase[tm] + sh + kq * 16];
#pragma unroll
          for (int tm = 0; tm < TM; ++tm)
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
              if constexpr (NS == 2) acc[tm][tn] = mfma_h16(af[tm], bq[BR ? (u & 1) : u][tn][kq], acc[tm][tn]);
              else acc[tm][tn] = mfma_split<NS>(af[tm], bq[BR ? (u & 1) : u][tn][kq], acc[tm][tn]);
            }
        }
        if constexpr (!BR) {
          if (has_next) load_b(cur, u, u, c + 1);
          else if (has_tile) load_b(nxt, u, u, 0);
        }
      }
      if (c < 4) KW_STAMP(3 + 2 * c);
      if constexpr (NS == 1) {
        if (has_next) store_window(buf ^ 1, c + 1);
      }
      if constexpr (NS == 2) {
        if (has_next) wave_max_put((c + 1) & 1);
      }
      __syncthreads();
    }
    KW_STAMP(10);

    // ---- sum the four waves' partial tiles in LDS (fixed order), then one epilogue ----
    const int m0 = cur.m0, n0 = cur.n0, group = cur.group, cls = cur.cls;
    float* red = (float*)ksm;  // [4][BM][BN]
    [[maybe_unused]] int wex = H16_WS;  // the weight planes' exponent (split mode)
    if constexpr (NS == 2) wex = a.wexp ? wtab_exp(a.wexp[group * a.wexp_gs]) : H16_WS;
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          red[(wave * BM + m) * BN + tn * 32 + l32] = NS == 2 ? __builtin_ldexpf(acc[tm][tn][r], -(hs + wex)) : acc[tm][tn][r];
        }
    __syncthreads();
    KW_STAMP(11);
    if (h.vec) {  // 16-byte epilogue: 4 consecutive columns per thread (write-through-friendly stores)
      if (a.bw.pre_bf16) {
        if (a.bw.y_bf16) kw_epilogue_vec<BM, BN, true, true>(h, red, tid, cur.m0, cur.n0, cur.group, cur.cls);
        else kw_epilogue_vec<BM, BN, true, false>(h, red, tid, cur.m0, cur.n0, cur.group, cur.cls);
      } else {
        if (a.bw.y_bf16) kw_epilogue_vec<BM, BN, false, true>(h, red, tid, cur.m0, cur.n0, cur.group, cur.cls);
        else kw_epilogue_vec<BM, BN, false, false>(h, red, tid, cur.m0, cur.n0, cur.group, cur.cls);
      }
      KW_STAMP(12);
      if (!has_tile) break;
      __syncthreads();
      cur = nxt;
      ++t_cur;
      if constexpr (NS == 1) {
        store_window(0, 0);
        __syncthreads();
      }
      continue;
    }
    constexpr int NRG = 256 / BN;  // row groups
    const int col = tid % BN, rg = tid / BN;
    const int n = n0 + col;
    float* Cp = a.C + group * a.c_gs;
    const float* bias = a.bias ? a.bias + group * a.bias_gs : nullptr;
    const bool bwm = a.bw.pre != nullptr;
    const bool bwc = bwm && n < a.bw.C;
    float bm = 0.f, bi = 0.f, bb = 0.f;
    if (bwc) {
      bm = a.bw.mean[group * a.bw.ms_gs + n];
      bi = a.bw.invstd[group * a.bw.ms_gs + n];
      bb = a.bw.y ? 0.f : a.bw.beta[group * a.bw.beta_gs + n];
    }
    float s1 = 0.f, s2 = 0.f;
    // every global load (accumulate target, BN-backward pre / y) before the first store: one
    // memory round trip for the thread's BM / NRG rows, not one per row
    constexpr int NR = BM / NRG;
    long long orow[NR];
    float cv[NR], pv[NR], yv[NR];
    const bool pbf = a.bw.pre_bf16 != 0;
    const float* bwpre = bwc ? pf_at(a.bw.pre, group * a.bw.pre_gs, pbf) : nullptr;
    const bool ybf = a.bw.y_bf16 != 0;
    const float* bwy = (bwc && a.bw.y) ? pf_at(a.bw.y, group * a.bw.y_gs, ybf) : nullptr;
    const float biasv = bias ? bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      orow[i] = kw_out_row(h, g, cls, m0 + rg + i * NRG);
      cv[i] = a.accumulate ? Cp[orow[i] * a.ldc + n] : 0.f;
      pv[i] = bwpre ? pf_ld(bwpre, orow[i] * a.bw.ldp + n, pbf) : 0.f;
      yv[i] = bwy ? pf_ld(bwy, orow[i] * a.bw.ldy + n, ybf) : 0.f;
    }
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int m = rg + i * NRG;
      float v = red[(0 * BM + m) * BN + col];
#pragma unroll
      for (int w = 1; w < 4; ++w) v += red[(w * BM + m) * BN + col];
      if (a.c_bf16) v = bf_rnd(v);  // bf16-stored pre-BN output: the statistics of the stored values
      if (!bwm) {
        s1 += v;
        s2 += v * v;
      }
      if (bias) v += biasv;
      v = act_f(v, a.act);
      if (a.accumulate) v += cv[i];
      if (a.c_bf16) ((__bf16*)a.C)[group * a.c_gs + orow[i] * a.ldc + n] = (__bf16)v;
#ifdef SVAE_EXP_NOSTORE  // timing experiment (wrong results): the epilogue without its stores
      else if (v != v) st_out(&Cp[orow[i] * a.ldc + n], v);
#else
      else st_out(&Cp[orow[i] * a.ldc + n], v);
#endif
      if (bwc) bw_term_v(v, pv[i], bm, bi, bb, bwy != nullptr, yv[i], a.bw.act, s1, s2);
    }
    KW_STAMP(15);
    if (a.stats) {
      __syncthreads();  // every wave is done reading red
      red[tid] = s1;
      red[256 + tid] = s2;
      __syncthreads();
      if (tid < BN) {
        const int SC = bwm ? a.bw.C : a.N;  // stats columns (row-block stride 2*SC)
        if (n0 + tid < SC) {
          float s = 0.f, q = 0.f;
#pragma unroll
          for (int j = 0; j < NRG; ++j) {
            s += red[j * BN + tid];
            q += red[256 + j * BN + tid];
          }
          const int rb = cls * h.ntx + m0 / BM;
          stat_put(a.stats + (rb & (a.s_nsh - 1)) * a.s_sh + group * a.s_gs, n0 + tid, s, q);
        }
      }
      if (a.fin.cnt) bn_fin_arrive(a.fin, group, (int*)red);
    }
    KW_STAMP(12);
    if (!has_tile) break;
    // ---- the next tile: its window (prefetched above) into LDS once every wave is done with red ----
    __syncthreads();
    cur = nxt;
    ++t_cur;
    if constexpr (NS == 1) {
      store_window(0, 0);
      __syncthreads();
    }
  }
}

}  // namespace

// ---- planner: eligible shapes, BM, window geometry, LDS, stats row-blocks ----
static int kw_bn_mode() {  // SVAE_KW_BN: 32 (default) or 64 column tiles
  static const int v = svae_knob("SVAE_KW_BN", 32);
  return v;
}

static bool split_pi3() {  // SVAE_KW_PI3=0: split instances keep 4 window items per thread
  static const bool v = svae_knob("SVAE_KW_PI3", 1) != 0;
  return v;
}

// split mode: SVAE_KW_SPLIT_BM=32 takes 32-row tiles (4 waves per SIMD) instead of 64 where both fit
static int split_bm_max() {
#ifndef KW_SPLIT_BM_DEFAULT
#define KW_SPLIT_BM_DEFAULT 64
#endif
  static const int v = svae_knob("SVAE_KW_SPLIT_BM", KW_SPLIT_BM_DEFAULT);
  return v;
}

static bool kw_plan(const FwdArgs& a, int groups, KwArgs* out, int* bm_out, int* bn_out, size_t* lds_out) {
  const ConvGeom& g = a.g;
  if (g.mode == GM_DENSE || g.ksz != 4 || g.pad != 1 || !a.Bh || a.Cin % KW_CK != 0 || a.N % 32 != 0) return false;
  const bool s2t = g.mode == GM_CONVT && g.stride == 2;
  if (g.mode == GM_CONVT && g.stride > 2) return false;
  const int Hr = s2t ? g.Ho / 2 : g.Ho, Wr = s2t ? g.Wo / 2 : g.Wo;
  const int sy = g.mode == GM_CONV ? g.stride : 1;
  const int span = s2t ? 2 : 4;
  const int per_img = Hr * Wr;
  static const int bm_max = svae_knob("SVAE_KW_BM", 64);  // (bf16 instances; the split ones: split_bm_max())
  for (int bm : {128, 64, 32}) {
    if (bm > (a.nsp > 1 ? split_bm_max() : bm_max)) continue;
    if (bm % Wr != 0 || a.rows % bm != 0) continue;
    if (!(per_img % bm == 0 || bm % per_img == 0)) continue;
    KwArgs h;
    h.Hr = Hr;
    h.Wr = Wr;
    h.R = bm >= per_img ? Hr : bm / Wr;
    h.nimg = bm >= per_img ? bm / per_img : 1;
    h.sy = sy;
    h.PR = (h.R - 1) * sy + span;
    h.PC = (Wr - 1) * sy + span;
    h.npix = h.nimg * h.PR * h.PC;
    if (h.npix * 4 > 256 * KW_PI) continue;
    h.d_win = make_fastdiv(h.PR * h.PC);
    h.d_pc = make_fastdiv(h.PC);
    h.d_img = make_fastdiv(Hr * Wr);
    h.d_wr = make_fastdiv(Wr);
    h.d_rimg = make_fastdiv(h.R * Wr);
    h.d_q = make_fastdiv((g.Ho >> 1) * (g.Wo >> 1));
    h.d_qw = make_fastdiv(g.Wo >> 1);
    int bn = 32;
    if (kw_bn_mode() == 64 && a.nsp <= 1 && a.N % 64 == 0 &&
        (long long)(a.rows / bm) * (a.N / 64) * a.nclass * groups >= 512)
      bn = 64;
    const long long blocks = (long long)(a.rows / bm) * (a.N / bn) * a.nclass * groups;
    if (blocks < 256 && bm > 32) continue;  // the smaller tile doubles the blocks
    *out = h;
    *bm_out = bm;
    *bn_out = bn;
    // NS = 1: two window buffers; NS = 3 (split planes): one buffer of three planes
    const int wbufs = a.nsp > 1 ? (a.h16 ? 2 : 3) : 2;  // (h16: one buffer of two fp16 planes)
    if (a.nsp > 1 && (a.a_bf16 || bm > split_bm_max())) continue;  // split instances: fp32 A
    *lds_out = std::max((size_t)(wbufs * h.npix) * KW_ROWP * sizeof(__bf16), (size_t)4 * bm * bn * sizeof(float));
    return true;
  }
  return false;
}

static bool kw_disabled() {
  static const bool v = svae_knob("SVAE_NO_KW", 0) == 1;
  return v;
}

int halo_kw_plan(const FwdArgs& a, int groups) {
  if (kw_disabled()) return 0;
  if (a.ain.acc && a.Cin % 8) return 0;  // consumer-side BN: A is the pre-BN tensor (fp32, or bf16-stored)
  KwArgs h;
  int bm, bn;
  size_t lds;
  if (!kw_plan(a, groups, &h, &bm, &bn, &lds)) return 0;
  if (a.ain.acc && a.a_bf16 && (bn != 32 || bm > 64)) return 0;  // the AIN instances
  return a.nclass * (a.rows / bm);
}

int halo_kw(const FwdArgs& a, int groups, hipStream_t s) {
  KwArgs h;
  int bm, bn;
  size_t lds;
  if (kw_disabled() || !kw_plan(a, groups, &h, &bm, &bn, &lds)) return -1;
  h.f = a;
  const bool s2t = a.g.mode == GM_CONVT && a.g.stride == 2;
  dim3 grid(a.rows / bm, a.N / bn, groups * a.nclass);
  h.f.fin.nblk = (a.rows / bm) * (a.N / bn) * a.nclass;  // tiles per group (last-arriver finalisation)
  h.ntx = (int)grid.x;
  h.nty = (int)grid.y;
  h.ntz = (int)grid.z;
  h.tpb = 1;
  h.ain_off = 0;
  h.slot_off = 0;
  if (a.ain.acc) {  // the consumer-side BN table [3][Cin] after the window / reduction region
    if (a.Cin % 8) return -1;
    h.ain_off = (int)((lds + 15) / 16 * 16);
    lds = (size_t)h.ain_off + 3 * (size_t)a.Cin * sizeof(float);
  }
  {  // SVAE_KW_VEC=1: the 16-byte epilogue where every row of C (and of the BN-backward operands) is aligned
    static const int vec_mode = svae_knob("SVAE_KW_VEC", 0);
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    // bf16-stored pre (written, or read by the fused backward-BN terms): always the 8-byte vector form
    const bool pbf = a.c_bf16 || (a.bw.pre && a.bw.pre_bf16);
    bool ok = (vec_mode != 0 || pbf) && a.ldc % 4 == 0 && a.c_gs % 4 == 0 && al16(a.C) && (!a.bias || (al16(a.bias) && a.bias_gs % 4 == 0));
    if (a.bw.pre)
      ok = ok && a.bw.C % 4 == 0 && a.bw.ldp % 4 == 0 && a.bw.pre_gs % 4 == 0 && al16(a.bw.pre) && al16(a.bw.mean) &&
           al16(a.bw.invstd) && a.bw.ms_gs % 4 == 0 &&
           (a.bw.y ? (a.bw.ldy % 4 == 0 && a.bw.y_gs % 4 == 0 && al16(a.bw.y)) : (al16(a.bw.beta) && a.bw.beta_gs % 4 == 0));
    h.vec = ok ? 1 : 0;
  }
  // persistent form (SVAE_KW_PERSIST=1): where the tiles exceed the resident blocks, each block runs
  // a contiguous run of tiles with the next tile's window / B loads under the current tile's last
  // chunk and epilogue
  static const int persist = svae_knob("SVAE_KW_PERSIST", 0);
  if (persist && a.nsp <= 1 && a.a_bf16 && bn == 32 && bm == 64 && !a.ain.acc) {  // the persistent instances
    const int occ_w = 2;
    const int occ_l = (int)std::max<size_t>(1, (size_t)163840 / std::max<size_t>(lds, 1));
    const long long slots = 256LL * std::min(occ_w, occ_l) * (persist > 1 ? persist : 1);
    const long long ntiles = (long long)h.ntx * h.nty * h.ntz;
    if (ntiles > slots) {
      h.tpb = (int)((ntiles + slots - 1) / slots);
      grid = dim3((unsigned)((ntiles + h.tpb - 1) / h.tpb), 1, 1);
    }
  }
  // SVAE_KW_BRING: the two-tap B register ring on the 16-tap instances (bit 0: split mode, bit 1: bf16).
  // Default 1: the split instances go from 2 to 3 waves per SIMD (bf16x6 step 18.74 -> 18.08 ms,
  // profiles/r04_ab1.txt); the bf16 ones would need a fifth wave and spill (8 % slower)
  static const int bring = svae_knob("SVAE_KW_BRING", 1);
  if (a.nsp > 1 && a.h16) {  // split mode, scaled fp16 planes (opload.h split8_h16 / mfma_h16): 3 MFMAs per pair
    static bool attr = false;
    if (!attr) {
      for (const void* f : {(const void*)igemm_halo_kw_kernel<64, 32, true, false, 2>,
                            (const void*)igemm_halo_kw_kernel<32, 32, true, false, 2>,
                            (const void*)igemm_halo_kw_kernel<128, 32, true, false, 2>,
                            (const void*)igemm_halo_kw_kernel<64, 32, false, false, 2, false, true, 3>,
                            (const void*)igemm_halo_kw_kernel<32, 32, false, false, 2, false, true, 3>,
                            (const void*)igemm_halo_kw_kernel<64, 32, false, false, 2, false, true>,
                            (const void*)igemm_halo_kw_kernel<32, 32, false, false, 2, false, true>,
                            (const void*)igemm_halo_kw_kernel<128, 32, false, false, 2, false, true>})
        hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 98304);
      attr = true;
    }
    h.f.Bh = (const __bf16*)a.Bh + 3 * a.b_plane;  // the fp16 planes
    h.slot_off = (int)((lds + 15) / 16 * 16);
    lds = (size_t)h.slot_off + 8 * sizeof(float);
    const bool pi3 = h.npix * 4 <= 256 * 3;
    if (bm == 128) {
      if (s2t) hipLaunchKernelGGL((igemm_halo_kw_kernel<128, 32, true, false, 2>), grid, dim3(256), lds, s, h);
      else hipLaunchKernelGGL((igemm_halo_kw_kernel<128, 32, false, false, 2, false, true>), grid, dim3(256), lds, s, h);
    } else if (bm == 64) {
      if (s2t) hipLaunchKernelGGL((igemm_halo_kw_kernel<64, 32, true, false, 2>), grid, dim3(256), lds, s, h);
      else if (pi3) hipLaunchKernelGGL((igemm_halo_kw_kernel<64, 32, false, false, 2, false, true, 3>), grid, dim3(256), lds, s, h);
      else hipLaunchKernelGGL((igemm_halo_kw_kernel<64, 32, false, false, 2, false, true>), grid, dim3(256), lds, s, h);
    } else {
      if (s2t) hipLaunchKernelGGL((igemm_halo_kw_kernel<32, 32, true, false, 2>), grid, dim3(256), lds, s, h);
      else if (pi3) hipLaunchKernelGGL((igemm_halo_kw_kernel<32, 32, false, false, 2, false, true, 3>), grid, dim3(256), lds, s, h);
      else hipLaunchKernelGGL((igemm_halo_kw_kernel<32, 32, false, false, 2, false, true>), grid, dim3(256), lds, s, h);
    }
    return a.nclass * (a.rows / bm);
  }
  if (a.nsp > 1) {  // split-bf16 planes (fp32 A): 64 / 32-row tiles, 32 columns
    static bool attr = false;
    if (!attr) {
      for (const void* f : {(const void*)igemm_halo_kw_kernel<64, 32, true, false, 3>,
                            (const void*)igemm_halo_kw_kernel<64, 32, false, false, 3>,
                            (const void*)igemm_halo_kw_kernel<32, 32, true, false, 3>,
                            (const void*)igemm_halo_kw_kernel<32, 32, false, false, 3>,
                            (const void*)igemm_halo_kw_kernel<64, 32, false, false, 3, false, true>,
                            (const void*)igemm_halo_kw_kernel<32, 32, false, false, 3, false, true>,
                            (const void*)igemm_halo_kw_kernel<64, 32, false, false, 3, false, true, 3>,
                            (const void*)igemm_halo_kw_kernel<32, 32, false, false, 3, false, true, 3>,
                            (const void*)igemm_halo_kw_kernel<128, 32, true, false, 3>,
                            (const void*)igemm_halo_kw_kernel<128, 32, false, false, 3, false, true>})
        hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 98304);
      attr = true;
    }
    const bool br = (bring & 1) != 0;
    const bool pi3 = h.npix * 4 <= 256 * 3 && split_pi3();
    // SVAE_KW_PERSIST_SPLIT=k: the 64-row split ring instances persistent over 256 x 3 x k blocks (the
    // next tile's window and first B fragments load under the current tile's last chunk)
    static const int persist_split = svae_knob("SVAE_KW_PERSIST_SPLIT", 0);
    if (persist_split && br && pi3 && bm == 64 && !s2t && !a.ain.acc) {
      const long long slots = 256LL * 3 * persist_split;
      const long long ntiles = (long long)h.ntx * h.nty * h.ntz;
      if (ntiles > slots) {
        h.tpb = (int)((ntiles + slots - 1) / slots);
        grid = dim3((unsigned)((ntiles + h.tpb - 1) / h.tpb), 1, 1);
        static bool attrp = false;
        if (!attrp) {
          hipFuncSetAttribute((const void*)igemm_halo_kw_kernel<64, 32, false, false, 3, true, true, 3>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 98304);
          attrp = true;
        }
        hipLaunchKernelGGL((igemm_halo_kw_kernel<64, 32, false, false, 3, true, true, 3>), grid, dim3(256), lds, s, h);
        return a.nclass * (a.rows / bm);
      }
    }
    if (bm == 128) {  // 128-row tiles: each B fragment serves four row fragments
      if (s2t) hipLaunchKernelGGL((igemm_halo_kw_kernel<128, 32, true, false, 3>), grid, dim3(256), lds, s, h);
      else hipLaunchKernelGGL((igemm_halo_kw_kernel<128, 32, false, false, 3, false, true>), grid, dim3(256), lds, s, h);
    } else if (bm == 64) {
      if (s2t) hipLaunchKernelGGL((igemm_halo_kw_kernel<64, 32, true, false, 3>), grid, dim3(256), lds, s, h);
      else if (br && pi3) hipLaunchKernelGGL((igemm_halo_kw_kernel<64, 32, false, false, 3, false, true, 3>), grid, dim3(256), lds, s, h);
      else if (br) hipLaunchKernelGGL((igemm_halo_kw_kernel<64, 32, false, false, 3, false, true>), grid, dim3(256), lds, s, h);
      else hipLaunchKernelGGL((igemm_halo_kw_kernel<64, 32, false, false, 3>), grid, dim3(256), lds, s, h);
    } else {
      if (s2t) hipLaunchKernelGGL((igemm_halo_kw_kernel<32, 32, true, false, 3>), grid, dim3(256), lds, s, h);
      else if (br && pi3) hipLaunchKernelGGL((igemm_halo_kw_kernel<32, 32, false, false, 3, false, true, 3>), grid, dim3(256), lds, s, h);
      else if (br) hipLaunchKernelGGL((igemm_halo_kw_kernel<32, 32, false, false, 3, false, true>), grid, dim3(256), lds, s, h);
      else hipLaunchKernelGGL((igemm_halo_kw_kernel<32, 32, false, false, 3>), grid, dim3(256), lds, s, h);
    }
    return a.nclass * (a.rows / bm);
  }
#define KW_LAUNCH(BM_, BN_)                                                                                  \
  if (h.tpb > 1 && a.a_bf16 && BN_ == 32 && BM_ == 64) {  /* persistent: the bf16-A 64x32 instances */     \
    if (s2t) hipLaunchKernelGGL((igemm_halo_kw_kernel<64, 32, true, true, 1, true>), grid, dim3(256), lds, s, h); \
    else hipLaunchKernelGGL((igemm_halo_kw_kernel<64, 32, false, true, 1, true>), grid, dim3(256), lds, s, h);    \
  } else if (a.a_bf16 && a.ain.acc) {  /* consumer-side BN of a bf16 pre-BN tensor (halo_kw_plan: BN 32, BM <= 64) */ \
    if (s2t) hipLaunchKernelGGL((igemm_halo_kw_kernel<BM_, BN_, true, true, 1, false, false, KW_PI, true>), grid, dim3(256), lds, s, h); \
    else hipLaunchKernelGGL((igemm_halo_kw_kernel<BM_, BN_, false, true, 1, false, false, KW_PI, true>), grid, dim3(256), lds, s, h); \
  } else if (a.a_bf16) {                                                                                     \
    if (s2t) hipLaunchKernelGGL((igemm_halo_kw_kernel<BM_, BN_, true, true>), grid, dim3(256), lds, s, h);    \
    else if ((bring & 2) && BN_ == 32 && BM_ <= 64)                                                          \
      hipLaunchKernelGGL((igemm_halo_kw_kernel<BM_, BN_, false, true, 1, false, true>), grid, dim3(256), lds, s, h); \
    else hipLaunchKernelGGL((igemm_halo_kw_kernel<BM_, BN_, false, true>), grid, dim3(256), lds, s, h);       \
  } else {                                                                                                   \
    if (s2t) hipLaunchKernelGGL((igemm_halo_kw_kernel<BM_, BN_, true, false>), grid, dim3(256), lds, s, h);   \
    else hipLaunchKernelGGL((igemm_halo_kw_kernel<BM_, BN_, false, false>), grid, dim3(256), lds, s, h);      \
  }
  if (bm == 128) {
    static bool attr = false;
    if (!attr) {  // 4 x 128 x 32 fp32 partial tiles: 64 KB
      for (const void* f : {(const void*)igemm_halo_kw_kernel<128, 32, true, false>,
                            (const void*)igemm_halo_kw_kernel<128, 32, false, false>,
                            (const void*)igemm_halo_kw_kernel<128, 32, true, true>,
                            (const void*)igemm_halo_kw_kernel<128, 32, false, true>})
        hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 98304);
      attr = true;
    }
    KW_LAUNCH(128, 32)
  } else if (bm == 64 && bn == 64) {
    static bool attr = false;
    if (!attr) {  // 4 x 64 x 64 fp32 partial tiles: 64 KB
      for (const void* f : {(const void*)igemm_halo_kw_kernel<64, 64, true, false>,
                            (const void*)igemm_halo_kw_kernel<64, 64, false, false>,
                            (const void*)igemm_halo_kw_kernel<64, 64, true, true>,
                            (const void*)igemm_halo_kw_kernel<64, 64, false, true>})
        hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 98304);
      attr = true;
    }
    KW_LAUNCH(64, 64)
  } else if (bm == 64) {
    KW_LAUNCH(64, 32)
  } else if (bn == 64) {
    KW_LAUNCH(32, 64)
  } else {
    KW_LAUNCH(32, 32)
  }
#undef KW_LAUNCH
  return a.nclass * (a.rows / bm);
}
