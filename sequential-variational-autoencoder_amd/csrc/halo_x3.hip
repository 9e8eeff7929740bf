// The split mode's wave-split halo gather on scaled fp16 hi/lo planes (dtype bf16x6; opload.h
// split8_h16 / mfma_h16): every conv / conv-T forward and input gradient with >= 1 channel chunk of 32
// and 32-column output tiles.
//
// A block owns BM output rows x 32 columns and all of K.  Per 32-channel chunk it stages the input
// window of its rows (plus the 4x4 halo) in LDS once, as the two fp16 planes of A * 2^hs (hs: the
// block's running exponent, below), and its four waves run the MFMAs against that window:
//   16-tap layers (conv s1 / s2, conv-T s1): wave w takes kernel row ky = w (four taps); the four
//       partial tiles are summed in LDS in wave order before one epilogue (deterministic).
//   stride-2 conv-T: the block covers all four output-parity classes of its rows, wave w the class
//       (cy, cx) = (w >> 1, w & 1) with that class's four taps over one union window; the waves' tiles
//       are disjoint, so there is no reduction (halo_kw.hip ran one class per block, one tap per wave).
// B (the weights) comes from the two scaled fp16 weight planes H16_PLANE.. of the engine's shadows,
// one tap of fragments ahead in registers.
//
// Scaling: fp16 has 11 significant bits and a narrow exponent range, so the block scales A by a power
// of two 2^hs with max|A| * 2^hs in [2^14, 2^15) over the chunks staged so far (the running maximum
// only grows, so hs only falls; the accumulators are rescaled by the same exact power of two when it
// does).  Weights carry their tensor's exponent 2^e (common.h h16_pair).  The epilogue multiplies by 2^-(hs + e).
#include "common.h"
#include "kernels.h"
#include "knobs.h"
#include "opload.h"

typedef __bf16 x3_16x8 __attribute__((ext_vector_type(8)));  // 8 raw 16-bit lanes (fp16 bits)

#define X3_CK 32    // channels per window stage
#define X3_ROWP 40  // LDS pixel pitch in 16-bit elements (80 B: conflict-free 16-B fragment reads)
#ifndef X3_OCC_S32
#define X3_OCC_S32 3  // 32-row split instances: 3 waves per SIMD (at 4 the PI = 4 instance spilt 20 VGPRs; 14.93 vs 15.04 ms, profiles/r05_x3_occ_ab.txt)
#endif
#define X3_OCC(BM, NP, PI) \
  ((PI) > 4 ? 2 : (NP) == 2 ? ((BM) == 128 ? 2 : (BM) == 64 ? 3 : X3_OCC_S32) : ((BM) == 128 ? 2 : 4))
#ifndef X3_PI8
#define X3_PI8 1  // 64-row tiles of the stride-2 convs with 8 window items per thread (their windows are 4x)
#endif
#ifndef X3_PERM
#define X3_PERM 1  // the conflict-free window image (x3_lane_pix); 0: round 5's pixel-order lanes, compact rows
#endif
#ifndef X3_BMMAX
#define X3_BMMAX 128  // largest row tile (16-tap layers; the stride-2 conv-T takes <= 64: four classes per block)
#endif

struct X3Args {
  const float* A; long long a_gs; int lda;
  const __bf16* Bh; long long b_gs; int ldb; long long b_tap, b_plane;  // fp16 plane h0 at Bh, h1 at Bh + b_plane
  float* C; long long c_gs; int ldc;
  u64* stats; long long s_gs, s_sh; int s_nsh;
  const float* bias; long long bias_gs;
  BwStat bw;
  int Cin, act, accumulate;
  int c_bf16;        // (bf16 mode) C is the bf16-stored pre-BN output
  int mode;          // GM_CONV / GM_CONVT
  int Hi, Wi, Ho, Wo;
  int Hr, Wr;        // row space per class
  int R, PR, PC, sy, npix;
  // LDS image of the window (conflict-free A-fragment reads, x3_lane_pix): row pitch PCP >= PC pixels, nlds
  // pixels in all; dint: the stride-2 convs' window columns de-interleaved (even columns, then from PCh the odd
  // ones); pm: the lane -> output pixel order of a 32-row tile (0 identity, 1 16-wide rows, 2 8-wide rows)
  int PCP, PCh, nlds, dint, pm;
  int oy0, ox0;      // window origin (conv-T stride 2: the union of the four classes' windows)
  int toff0, tsgn;   // tap shift: LDS pixel offset of tap t = toff0 + tsgn * (row(t) * PCP + col(t))
  FastDiv d_win, d_pc, d_img, d_wr, d_rimg;
  int slot_off;      // byte offset of the [2][4] wave maxima of |A| in dynamic LDS
  void* stamps;      // (SVAE_EXP_STAMPS builds: the phase stamps, in the split-K scratch)
  const int* wexp; long long wexp_gs;  // the weight planes' exponent of group g (nullptr: H16_WS)
};

namespace {

// Conflict-free A-fragment reads.  A ds_read_b128 serves its 64 lanes in four groups of 16 lanes, {0-3, 12-15,
// 20-27} and {4-11, 16-19, 28-31} of each half-wave; a group is conflict-free when its 16 pixels hit 16 distinct
// 16-byte bank slots, which at the 80-B pixel pitch (slot = 5 * pixel mod 16) means 16 distinct pixel positions
// mod 16.  A 32-row tile of a 32-wide row space is 32 consecutive pixels of one row: every group reads 16
// consecutive positions.  In 16- and 8-wide row spaces the tile's rows jump by the window pitch and groups
// collided (2-3 way; 5.9 conflict cycles per LDS instruction on the 8x8 layers, profiles/r06_p1_sq.txt).  So
// the lanes take the tile's pixels in a group-aware order: pm 1 (16-wide) gives each group one row of 16
// consecutive pixels; pm 2 (8-wide) gives each group 4 rows x 4 columns, with the LDS row pitch PCP = 12 (stride
// 1 / conv-T) or 18 (stride-2 conv, whose de-interleaved rows are 2 * 18 = 4 mod 16 apart), so its rows sit
// 0 / 4 / 8 / 12 slots apart.  The output pixel of accumulator row m is then x3_lane_pix(m); the epilogue reads
// the reduced tile through the inverse (x3_pix_lane).  Bitwise the same results (every output element sums the
// same products in the same order).
__device__ __forceinline__ int x3_rank_lane(int g, int k) {  // the lane of rank k (0..15) in group g
  return g == 0 ? (k < 4 ? k : (k < 8 ? k + 8 : k + 12)) : (k < 8 ? k + 4 : (k < 12 ? k + 8 : k + 16));
}
__device__ __forceinline__ int x3_lane_pix(int l, int pm) {  // tile-local output pixel of lane l (0..31)
  if (pm == 0) return l;
  const int g = (l < 4 || (l >= 12 && l < 16) || (l >= 20 && l < 28)) ? 0 : 1;
  const int k = g == 0 ? (l < 4 ? l : (l < 16 ? l - 8 : l - 12)) : (l < 12 ? l - 4 : (l < 20 ? l - 8 : l - 16));
  return pm == 1 ? g * 16 + k : (k >> 2) * 8 + g * 4 + (k & 3);
}
__device__ __forceinline__ int x3_pix_lane(int p, int pm) {  // inverse: the lane (accumulator row) of pixel p
  if (pm == 0) return p;
  const int g = pm == 1 ? (p >> 4) : ((p >> 2) & 1);
  const int k = pm == 1 ? (p & 15) : ((p >> 3) * 4 + (p & 3));
  return x3_rank_lane(g, k);
}

// NP = 2: the split mode (fp32 A, scaled fp16 hi/lo planes, three MFMAs per fragment pair).
// NP = 1: the bf16 mode (A fp32 or, ABF, stored bf16; one bf16 plane; bf16-stored pre-BN outputs c_bf16 and
//         the fused backward-BN terms on bf16-stored pre / y).
// RD: the B (weight) fragment ring.  2: two taps of fragments, the next tap's loaded while the current one's
// MFMAs run (the next chunk's window loaded after tap 1's).  4 (the split mode, one block per CU): a slot per
// tap of the wave's kernel row, refilled with the same tap of the NEXT chunk right after its MFMAs, and the
// next chunk's window loaded right after the barrier, before those refills -- every tap's fragments are then
// a whole chunk ahead, and (vmcnt counts in issue order) no tap's wait includes the window's loads.  32 more
// VGPRs: one wave per SIMD, for the launches whose grid is one block per CU anyway.
template <int BM, bool CPW, int PI, int NP = 2, bool ABF = false, int RD = 2>
__global__ __launch_bounds__(256, RD == 4 ? 1 : X3_OCC(BM, NP, PI)) void gather_x3_kernel(X3Args h) {
  static_assert(RD == 2 || (RD == 4 && NP == 2), "the full-chunk ring: split mode");
  static_assert(NP == 2 || NP == 1, "fp16 hi/lo planes or one bf16 plane");
  static_assert(NP == 1 || !ABF, "the split planes come from fp32 activations");
  constexpr int TM = BM / 32;
  extern __shared__ __attribute__((aligned(16))) __bf16 xsm[];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
#ifdef SVAE_EXP_STAMPS  // timing experiment: per-wave phase stamps (s_memtime) into the split-K scratch
  unsigned long long* stamp_p = (unsigned long long*)h.stamps +
      ((long long)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) * 4 + wave) * 16;
#define X3_STAMP(i) do { if (lane == 0 && (i) < 16) stamp_p[(i)] = __builtin_readcyclecounter(); } while (0)
#else
#define X3_STAMP(i) do {} while (0)
#endif
  X3_STAMP(0);
  const BlockXYZ blk = xcd_block();
  const int m0 = blk.x * BM, n0 = blk.y * 32, group = blk.z;
  const int nchunk = h.Cin / X3_CK;
  // the split mode's weight-plane exponent (the epilogue's unscale), read with a vector-memory load whose
  // value is first used in the epilogue: a scalar load would be waited for before the window's addresses are
  // even computed (lgkmcnt is not in order), this one completes under the window's own wait (num_records 0
  // without a table: the load returns 0, decoded as H16_WS below)
  [[maybe_unused]] int wraw = 0;
  if constexpr (NP == 2) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(h.wexp ? h.wexp + group * h.wexp_gs : nullptr), (short)0, h.wexp ? 4 : 0, 0x00020000);
    wraw = __builtin_amdgcn_raw_buffer_load_b32(r, 0, 0, 0);
  }
  const int per_img = h.Hr * h.Wr;

  // ---- window items: PI per thread, 8 channels each (item it = pixel it / 4, channel part it % 4) ----
  int woff[PI], wpos[PI];  // global element offset; LDS element offset (the pixel's slot in the window image)
  {
    const int img0 = fdiv(m0, h.d_img);
    const int ry0 = fdiv(m0 - img0 * per_img, h.d_wr);
    const int iy_base = ry0 * h.sy + h.oy0;
#pragma unroll
    for (int i = 0; i < PI; ++i) {
      const int it = tid + 256 * i;
      woff[i] = -2;  // -2: no item, -1: zero (outside the image)
      if (it < h.npix * 4) {
        const int pix = it >> 2, part = it & 3;
        const int il = fdiv(pix, h.d_win);
        const int r2 = pix - il * h.PR * h.PC;
        const int pr = fdiv(r2, h.d_pc), pc = r2 - pr * h.PC;
        const int iy = iy_base + pr, ix = h.ox0 + pc;
        woff[i] = (iy >= 0 && iy < h.Hi && ix >= 0 && ix < h.Wi) ? (((img0 + il) * h.Hi + iy) * h.Wi + ix) * h.lda + part * 8
                                                                 : -1;
        const int cs = h.dint ? ((pc & 1) ? h.PCh + (pc >> 1) : (pc >> 1)) : pc;
        wpos[i] = ((il * h.PR + pr) * h.PCP + cs) * X3_ROWP + part * 8;
      }
    }
  }
  f32x4 wv[PI][2];
  const float* Ag = ABF ? (const float*)((const __bf16*)h.A + group * h.a_gs) : h.A + group * h.a_gs;
  auto load_window = [&](int chunk) {
#pragma unroll
    for (int i = 0; i < PI; ++i) {
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      wv[i][0] = z;
      wv[i][1] = z;
      if (woff[i] >= 0) ld8_raw(Ag, woff[i] + chunk * X3_CK, ABF, wv[i][0], wv[i][1]);
    }
  };

  // ---- the block's running max |A| and exponent hs (A staged as A * 2^hs) ----
  int hs = 0;
  float hmax = 0.f;
  float* hslot = (float*)((char*)xsm + h.slot_off);
  auto wave_max_put = [&](int parity) {  // this wave's max |A| over the registers holding the next chunk
    float m = 0.f;
#pragma unroll
    for (int i = 0; i < PI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) m = fmaxf(m, fmaxf(fabsf(wv[i][0][j]), fabsf(wv[i][1][j])));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if (lane == 0) hslot[parity * 4 + wave] = m;
  };
  auto store_window = [&]() {
#pragma unroll
    for (int i = 0; i < PI; ++i) {
      if (woff[i] < -1) continue;
      const int o = wpos[i];
      if constexpr (NP == 2) {
        x3_16x8 pl[2];
        split8_h16(wv[i][0], wv[i][1], hs, pl);
        *(x3_16x8*)&xsm[o] = pl[0];
        *(x3_16x8*)&xsm[h.nlds * X3_ROWP + o] = pl[1];
      } else {
        *(x3_16x8*)&xsm[o] = raw8_bf(wv[i][0], wv[i][1], ABF);
      }
    }
  };

  // ---- A fragment bases (this wave's class offset for the stride-2 conv-T) ----
  const int cls = CPW ? wave : 0;
  const int cyo = CPW ? (wave >> 1) : 0, cxo = CPW ? (wave & 1) : 0;
  int abase[TM];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int ml = tm * 32 + x3_lane_pix(l32, h.pm);
    const int rows_img = h.R * h.Wr;
    const int il = fdiv(ml, h.d_rimg);
    const int rem = ml - il * rows_img;
    const int ryl = fdiv(rem, h.d_wr), rx = rem - ryl * h.Wr;
    // (de-interleaved stride-2 windows: output column rx reads slot rx + the tap's column slot)
    abase[tm] = ((il * h.PR + ryl * h.sy + cyo) * h.PCP + (h.dint ? rx : rx * h.sy + cxo)) * X3_ROWP + 8 * hh;
  }
  // this wave's taps u = 0..3: 16-tap layers kernel row ky = wave; conv-T stride 2 class `cls`'s 2 x 2
  auto tap_of = [&](int u) {
    if constexpr (CPW) {
      const int cy = cls >> 1, cx = cls & 1;
      return ((cy + 1) & 1) * 4 + ((cx + 1) & 1) + 8 * (u >> 1) + 2 * (u & 1);  // (pad 1)
    } else {
      return wave * 4 + u;
    }
  };
  auto shift_of = [&](int u) {
    if constexpr (CPW) return h.toff0 + h.tsgn * ((u >> 1) * h.PCP + (u & 1));
    else return h.dint ? wave * h.PCP + ((u & 1) ? h.PCh + (u >> 1) : (u >> 1)) : h.toff0 + h.tsgn * (wave * h.PCP + u);
  };
  x3_16x8 bq[RD][2][NP];  // [ring slot][kq][plane]
  const __bf16* bbase = h.Bh + group * h.b_gs + (long long)(n0 + l32) * h.ldb + 8 * hh;
  auto load_b = [&](int slot, int u, int chunk) {
    const __bf16* p = bbase + (long long)tap_of(u) * h.b_tap + chunk * X3_CK;
#pragma unroll
    for (int kq = 0; kq < 2; ++kq) {
      bq[slot][kq][0] = *(const x3_16x8*)(p + kq * 16);
      if constexpr (NP == 2) bq[slot][kq][1] = *(const x3_16x8*)(p + h.b_plane + kq * 16);
    }
  };

  X3_STAMP(13);
  load_window(0);
  if constexpr (RD == 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) load_b(u, u, 0);
  } else {
    load_b(0, 0, 0);
  }
  X3_STAMP(14);
  if constexpr (NP == 2) {
    wave_max_put(0);
    __syncthreads();
  }
  X3_STAMP(1);

  f32x16 acc[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;

  for (int c = 0; c < nchunk; ++c) {
    const bool has_next = c + 1 < nchunk;
    if constexpr (NP == 2) {  // the chunk's exponent (the running max only grows: a step d <= 0 shrinks the accumulators exactly)
      const float* sl = hslot + (c & 1) * 4;
      hmax = fmaxf(hmax, fmaxf(fmaxf(sl[0], sl[1]), fmaxf(sl[2], sl[3])));
      const int ns = h16_exp(hmax);
      const int d = ns - hs;
      hs = ns;
      if (d != 0 && c > 0) {  // (before the first chunk the accumulators are zero)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][r] = __builtin_ldexpf(acc[i][r], d);
      }
    }
    store_window();
    __syncthreads();
    if (c < 4) X3_STAMP(2 + 2 * c);
    if (RD == 4 && has_next) load_window(c + 1);  // (older than this chunk's B refills)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if constexpr (RD == 2) {
        // the ring: the next tap's B (this chunk's, or the next chunk's first)
        if (u + 1 < 4) load_b((u + 1) & 1, u + 1, c);
        else if (has_next) load_b(0, 0, c + 1);
        // the next chunk's window after tap 1's B loads (in-order vmcnt: a later B wait also waits for it)
        if (u == 0 && has_next) load_window(c + 1);
      }
      const int slot = RD == 4 ? u : (u & 1);
      const int sh = shift_of(u) * X3_ROWP;
#pragma unroll
      for (int kq = 0; kq < 2; ++kq) {
        x3_16x8 af[TM][NP];
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          af[tm][0] = *(const x3_16x8*)&xsm[abase[tm] + sh + kq * 16];
          if constexpr (NP == 2) af[tm][1] = *(const x3_16x8*)&xsm[h.nlds * X3_ROWP + abase[tm] + sh + kq * 16];
        }
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
          if constexpr (NP == 2) acc[tm] = mfma_h16(af[tm], bq[slot][kq], acc[tm]);
          else acc[tm] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[tm][0], bq[slot][kq][0], acc[tm], 0, 0, 0);
        }
      }
      if (RD == 4 && has_next) load_b(slot, u, c + 1);  // this tap of the next chunk, a whole chunk ahead
    }
    if (c < 4) X3_STAMP(3 + 2 * c);
    if constexpr (NP == 2) {
      if (has_next) wave_max_put((c + 1) & 1);
    }
    __syncthreads();
  }
  X3_STAMP(10);

  // ---- epilogue operands (independent of the accumulators): set up, and the first row batch's loads issued
  // before the tiles go through LDS, so their latency runs under the reduction ----
  // 16-byte epilogue: thread = 4 consecutive columns x rows rg, rg + 32, ... (8 threads per 128-B row)
  constexpr int ROWS = CPW ? 4 * BM : BM;  // output rows of the block (CPW: the four classes' tiles)
  constexpr int NR = ROWS / 32;
  const int c4 = (tid & 7) * 4, rg = tid >> 3;
  const int n = n0 + c4;
  float* Cp = h.C + group * h.c_gs;
  const bool bwm = h.bw.pre != nullptr;
  const bool bwc = bwm && n < h.bw.C;
  f32x4 bm = {0.f, 0.f, 0.f, 0.f}, bi = bm, bb = bm, biasv = bm;
  if (bwc) {
    bm = *(const f32x4*)&h.bw.mean[group * h.bw.ms_gs + n];
    bi = *(const f32x4*)&h.bw.invstd[group * h.bw.ms_gs + n];
    if (!h.bw.y) bb = *(const f32x4*)&h.bw.beta[group * h.bw.beta_gs + n];
  }
  if (h.bias) biasv = *(const f32x4*)&h.bias[group * h.bias_gs + n];
  // bf16-stored pre / y (bf16 mode): compile-time per instance only where NP == 1 (h.bw.*_bf16 checked by the plan)
  const bool pbf = NP == 1 && h.bw.pre_bf16, ybf = NP == 1 && h.bw.y_bf16;
  const float* bwpre = bwc ? pf_at(h.bw.pre, group * h.bw.pre_gs, pbf) : nullptr;
  const float* bwy = (bwc && h.bw.y) ? pf_at(h.bw.y, group * h.bw.y_gs, ybf) : nullptr;
  constexpr int NB = NR < 4 ? NR : 4;  // rows per batch: every global load of a batch before its first store
  static_assert(NR % NB == 0, "row batches");
  long long orow[NB];
  f32x4 cv[NB], pv[NB], yv[NB];
  auto fetch = [&](int i0) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int vr = rg + 32 * (i0 + b);
      if constexpr (CPW) {  // class k = (cy, cx), row m -> output pixel (2 qy + cy, 2 qx + cx)
        const int k = vr / BM;
        const int row = m0 + vr % BM;
        const int img = fdiv(row, h.d_img);
        const int r2 = row - img * per_img;
        const int qy = fdiv(r2, h.d_wr), qx = r2 - qy * h.Wr;
        orow[b] = ((long long)img * h.Ho + 2 * qy + (k >> 1)) * h.Wo + 2 * qx + (k & 1);
      } else {
        orow[b] = m0 + vr;
      }
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      cv[b] = pv[b] = yv[b] = z;
      if (h.accumulate) cv[b] = *(const f32x4*)&Cp[orow[b] * h.ldc + n];
      if (bwpre) pv[b] = pf_ld4(bwpre, orow[b] * h.bw.ldp + n, pbf);
      if (bwy) yv[b] = pf_ld4(bwy, orow[b] * h.bw.ldy + n, ybf);
    }
  };
  fetch(0);

  // ---- the waves' tiles into LDS (in the units of C), then one epilogue over the block ----
  float* red = (float*)xsm;  // [4][BM][32]
  // (the split mode's tiles in units of 2^(hs + H16_WS), shared by the block's waves: the reduced sums are
  // unscaled below -- exact, as every partial carries the same power of two)
  const int usc = NP == 2 ? -(hs + (h.wexp ? wtab_exp(wraw) : H16_WS)) : 0;
#pragma unroll
  for (int tm = 0; tm < TM; ++tm)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = tm * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
      red[(wave * BM + m) * 32 + l32] = acc[tm][r];
    }
  __syncthreads();
  X3_STAMP(11);

  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i0 = 0; i0 < NR; i0 += NB) {
    if (i0 > 0) fetch(i0);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int vr = rg + 32 * (i0 + b);
      const int vq = (vr & ~31) | x3_pix_lane(vr & 31, h.pm);  // the accumulator row of output row vr
      f32x4 v = *(const f32x4*)&red[vq * 32 + c4];
      if constexpr (!CPW) {
#pragma unroll
        for (int w = 1; w < 4; ++w) v += *(const f32x4*)&red[(w * BM + vq) * 32 + c4];
      }
      if constexpr (NP == 2) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = __builtin_ldexpf(v[j], usc);
      }
      if (NP == 1 && h.c_bf16) {  // bf16-stored pre-BN output: the statistics of the stored values
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
        if (h.bias) x += biasv[j];
        x = act_f(x, h.act);
        if (h.accumulate) x += cv[b][j];
        v[j] = x;
        if (bwc) bw_term_v(x, pv[b][j], bm[j], bi[j], bb[j], bwy != nullptr, yv[b][j], h.bw.act, s1[j], s2[j]);
      }
      if (NP == 1 && h.c_bf16)
        *(u64*)((__bf16*)h.C + group * h.c_gs + orow[b] * h.ldc + n) = __builtin_bit_cast(u64, __builtin_convertvector(v, pf_bf16x4));
      else
        *(f32x4*)&Cp[orow[b] * h.ldc + n] = v;
    }
  }
  X3_STAMP(15);
  if (h.stats) {
    __syncthreads();  // every wave is done reading red
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      red[rg * 32 + c4 + j] = s1[j];
      red[32 * 32 + rg * 32 + c4 + j] = s2[j];
    }
    __syncthreads();
    if (tid < 32) {
      const int SC = bwm ? h.bw.C : 0x7fffffff;  // stats columns
      if (n0 + tid < SC) {
        float sa = 0.f, qa = 0.f;
        for (int j = 0; j < 32; ++j) {  // fixed order: deterministic
          sa += red[j * 32 + tid];
          qa += red[32 * 32 + j * 32 + tid];
        }
        const int rb = blk.x;
        stat_put(h.stats + (rb & (h.s_nsh - 1)) * h.s_sh + group * h.s_gs, n0 + tid, sa, qa);
      }
    }
  }
  X3_STAMP(12);
}

}  // namespace

// ---- planner / launcher ----
// Eligible: 4x4 pad-1 conv (stride 1 / 2) and conv-T (stride 1 / 2) with Cin % 32 == 0, N % 32 == 0, fp32
// A and C, the fp16 weight planes (a.h16), 16-byte aligned epilogue operands, no consumer-side BN.
// the full-chunk B ring (RD = 4): 0 never, 1 where the grid is at most one block per CU (the occupancy the
// ring's registers cost is then not there to lose), 2 every split launch of 64 / 128 rows
#ifndef X3_RD_MODE
#define X3_RD_MODE 1
#endif
struct X3Plan {
  X3Args h;
  int bm, pi, rd;
  bool cpw;
  size_t lds;
  dim3 grid;
};

// (knob builds read these per call: the bitwise tests switch them between networks of one process)
static bool x3_bf16_on() { return svae_knob("SVAE_X3_BF16", 1) != 0; }  // 0: the bf16 mode's gathers on halo_kw
// SVAE_X3=0: every gather on halo_kw (the knob-only consumer-side BN / last-arriver paths' bitwise tests
// compare halo_kw with halo_kw)
static bool x3_on() { return svae_knob("SVAE_X3", 1) != 0; }

static bool x3_plan(const FwdArgs& a, int groups, X3Plan* out) {
  const ConvGeom& g = a.g;
  if (!x3_on() || !a.Bh || a.ain.acc || a.fin.cnt) return false;
  const bool split = a.nsp > 1;
  if (split ? (!a.h16 || a.a_bf16 || a.c_bf16) : !x3_bf16_on()) return false;
  if (a.c_bf16 && (a.accumulate || a.bias || a.act != ACT_NONE || ((uintptr_t)a.C & 7))) return false;
  if (g.mode == GM_DENSE || g.ksz != 4 || g.pad != 1 || a.Cin % X3_CK != 0 || a.N % 32 != 0) return false;
  if (g.mode == GM_CONVT && g.stride > 2) return false;
  if (split && a.bw.pre && (a.bw.pre_bf16 || a.bw.y_bf16)) return false;
  auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  auto al8 = [](const void* p) { return ((uintptr_t)p & 7) == 0; };
  if (a.ldc % 4 || a.c_gs % 4 || (!a.c_bf16 && !al16(a.C)) || (a.bias && (!al16(a.bias) || a.bias_gs % 4))) return false;
  if (a.bw.pre && (a.bw.C % 4 || a.bw.ldp % 4 || a.bw.pre_gs % 4 || !(a.bw.pre_bf16 ? al8(a.bw.pre) : al16(a.bw.pre)) ||
                   !al16(a.bw.mean) || !al16(a.bw.invstd) || a.bw.ms_gs % 4 ||
                   (a.bw.y ? (a.bw.ldy % 4 || a.bw.y_gs % 4 || !(a.bw.y_bf16 ? al8(a.bw.y) : al16(a.bw.y)))
                           : (!al16(a.bw.beta) || a.bw.beta_gs % 4))))
    return false;
  const bool s2t = g.mode == GM_CONVT && g.stride == 2;
  const int Hr = s2t ? g.Ho / 2 : g.Ho, Wr = s2t ? g.Wo / 2 : g.Wo;
  const int sy = g.mode == GM_CONV ? g.stride : 1;
  const int span = s2t ? 3 : 4;  // window rows beyond R - 1 (conv-T stride 2: the classes' union)
  const int per_img = Hr * Wr;
  // 128-row tiles on the 16-tap layers (the fixed per-block costs -- window prologue, epilogue -- over twice
  // the MFMA work: 0.74-0.97 of the 64-row time on those shapes, profiles/r05_m1_x3.txt); the stride-2
  // conv-T keeps <= 64 (its block already covers four classes: 128 rows left too few blocks, 1.6x)
  for (int bm : {128, 64, 32}) {
    if (bm > X3_BMMAX || (bm == 128 && s2t)) continue;
    if (bm % Wr != 0 || a.rows % bm != 0) continue;
    if (!(per_img % bm == 0 || bm % per_img == 0)) continue;
    X3Args& h = out->h;
    h.Hr = Hr;
    h.Wr = Wr;
    h.R = bm >= per_img ? Hr : bm / Wr;
    const int nimg = bm >= per_img ? bm / per_img : 1;
    h.sy = sy;
    h.PR = (h.R - 1) * sy + span;
    h.PC = (Wr - 1) * sy + span;
    h.npix = nimg * h.PR * h.PC;
    // the conflict-free window image (x3_lane_pix): lane order and row pitch by row-space width
    h.dint = (X3_PERM && sy == 2) ? 1 : 0;
    h.PCh = (h.PC + 1) / 2;
    h.pm = !X3_PERM ? 0 : Wr == 16 ? 1 : Wr == 8 ? 2 : 0;
    h.PCP = h.PC;
    if (h.pm == 2 && sy == 1) h.PCP = 12;                        // (PC = 11 / 10: rows 12 = -4 mod 16 slots apart)
    if (h.pm == 2 && sy == 2 && (2 * h.PC) % 16 != 4) h.pm = 0;  // (PC = 18: de-interleaved rows 36 = 4 mod 16 apart)
    h.nlds = nimg * h.PR * h.PCP;
    const int pi = (h.npix * 4 + 255) / 256;
    // the stride-2 convs' windows are four times a stride-1 one per output row: 64-row tiles take 8 items per
    // thread there (the 32-row tiles they fell back to ran 24 MFMAs per wave between two barriers)
    if (pi > ((X3_PI8 && bm == 64 && !s2t) ? 8 : 4)) continue;
    const long long blocks = (long long)(a.rows / bm) * (a.N / 32) * groups;
    if (blocks < 256 && bm > 32) continue;
    // stride-2 conv-T: one block per 4 classes' tiles; the 4x4-input levels give too few blocks
    // (halo_kw's one class per block, four times the blocks, is faster there: 29 vs 40 us, 14 vs 17 us)
    if (s2t && blocks < 512) return false;
    h.d_win = make_fastdiv(h.PR * h.PC);
    h.d_pc = make_fastdiv(h.PC);
    h.d_img = make_fastdiv(per_img);
    h.d_wr = make_fastdiv(Wr);
    h.d_rimg = make_fastdiv(h.R * Wr);
    if (s2t) {  // union origin of the four classes (pad 1: class 0 starts one row / column up)
      h.oy0 = h.ox0 = -1;
      h.toff0 = h.PCP + 1;
      h.tsgn = -1;
    } else if (g.mode == GM_CONV) {
      h.oy0 = h.ox0 = -g.pad;
      h.toff0 = 0;
      h.tsgn = 1;
    } else {
      h.oy0 = h.ox0 = g.pad - 3;
      h.toff0 = 3 * h.PCP + 3;
      h.tsgn = -1;
    }
    out->bm = bm;
    out->pi = pi <= 3 ? 3 : (pi <= 4 ? 4 : 8);
    out->cpw = s2t;
    out->rd = (split && bm >= 64 && (X3_RD_MODE == 2 || (X3_RD_MODE == 1 && blocks <= 256))) ? 4 : 2;
    const size_t win = (size_t)(split ? 2 : 1) * h.nlds * X3_ROWP * 2;  // NP planes
    const size_t red = (size_t)4 * bm * 32 * 4;
    h.slot_off = (int)((std::max(win, red) + 15) / 16 * 16);
    out->lds = (size_t)h.slot_off + 8 * sizeof(float);
    out->grid = dim3(a.rows / bm, a.N / 32, groups);
    return true;
  }
  return false;
}

int halo_x3_plan(const FwdArgs& a, int groups) {
  X3Plan p;
  if (!x3_plan(a, groups, &p)) return 0;
  return a.rows / p.bm;  // stats row-blocks (per group)
}

int halo_x3(const FwdArgs& a, int groups, hipStream_t s) {
  X3Plan p;
  if (!x3_plan(a, groups, &p)) return -1;
  X3Args& h = p.h;
  h.A = a.A; h.a_gs = a.a_gs; h.lda = a.lda;
  const bool split = a.nsp > 1;
  h.Bh = (const __bf16*)a.Bh + (split ? H16_PLANE * a.b_plane : 0);  // split: the fp16 planes of the shadow
  h.b_gs = a.b_gs; h.ldb = a.ldb; h.b_tap = a.b_tap; h.b_plane = a.b_plane;
  h.C = a.C; h.c_gs = a.c_gs; h.ldc = a.ldc;
  h.stats = a.stats; h.s_gs = a.s_gs; h.s_sh = a.s_sh; h.s_nsh = a.s_nsh;
  h.bias = a.bias; h.bias_gs = a.bias_gs;
  h.bw = a.bw;
  h.Cin = a.Cin; h.act = a.act; h.accumulate = a.accumulate;
  h.c_bf16 = a.c_bf16;
  h.mode = a.g.mode;
  h.Hi = a.g.Hi; h.Wi = a.g.Wi; h.Ho = a.g.Ho; h.Wo = a.g.Wo;
  h.stamps = a.part;
  h.wexp = a.wexp; h.wexp_gs = a.wexp_gs;
  static bool attr = false;
  if (!attr) {  // (LDS above the 64 KB default: the 128-row reduction tile)
#define X3_ATTR(BM_, CPW_, PI_, NP_, ABF_) \
    hipFuncSetAttribute((const void*)gather_x3_kernel<BM_, CPW_, PI_, NP_, ABF_>, hipFuncAttributeMaxDynamicSharedMemorySize, 98304); \
    if (NP_ == 2 && BM_ >= 64) hipFuncSetAttribute((const void*)gather_x3_kernel<BM_, CPW_, PI_, 2, false, (NP_ == 2 && BM_ >= 64) ? 4 : 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 98304);
    X3_ATTR(128, false, 3, 2, false) X3_ATTR(128, false, 4, 2, false) X3_ATTR(64, false, 3, 2, false)
    X3_ATTR(64, false, 4, 2, false) X3_ATTR(32, false, 3, 2, false) X3_ATTR(32, false, 4, 2, false)
    X3_ATTR(64, true, 3, 2, false) X3_ATTR(64, true, 4, 2, false) X3_ATTR(32, true, 3, 2, false)
    X3_ATTR(32, true, 4, 2, false)
    X3_ATTR(128, false, 4, 1, false) X3_ATTR(128, false, 4, 1, true) X3_ATTR(64, false, 4, 1, false)
    X3_ATTR(64, false, 4, 1, true) X3_ATTR(32, false, 4, 1, false) X3_ATTR(32, false, 4, 1, true)
    X3_ATTR(64, true, 4, 1, false) X3_ATTR(64, true, 4, 1, true) X3_ATTR(32, true, 4, 1, false)
    X3_ATTR(32, true, 4, 1, true)
    X3_ATTR(64, false, 8, 2, false) X3_ATTR(64, false, 8, 1, false) X3_ATTR(64, false, 8, 1, true)
#undef X3_ATTR
    attr = true;
  }
#define X3_LAUNCH(BM_, CPW_, PI_, NP_, ABF_) do { \
  if (NP_ == 2 && BM_ >= 64 && p.rd == 4) \
    hipLaunchKernelGGL((gather_x3_kernel<BM_, CPW_, PI_, 2, false, (NP_ == 2 && BM_ >= 64) ? 4 : 2>), p.grid, dim3(256), p.lds, s, h); \
  else \
    hipLaunchKernelGGL((gather_x3_kernel<BM_, CPW_, PI_, NP_, ABF_>), p.grid, dim3(256), p.lds, s, h); } while (0)
  // the bf16 mode (NP = 1): four window items per thread (registers to spare), A fp32 or bf16-stored
#define X3_BF(BM_, CPW_) \
  if (a.a_bf16) X3_LAUNCH(BM_, CPW_, 4, 1, true); else X3_LAUNCH(BM_, CPW_, 4, 1, false);
#define X3_SP(BM_, CPW_) \
  if (p.pi == 3) X3_LAUNCH(BM_, CPW_, 3, 2, false); else X3_LAUNCH(BM_, CPW_, 4, 2, false);
  if (p.pi == 8) {  // (64-row tiles of the stride-2 convs only)
    if (split) X3_LAUNCH(64, false, 8, 2, false);
    else if (a.a_bf16) X3_LAUNCH(64, false, 8, 1, true);
    else X3_LAUNCH(64, false, 8, 1, false);
    return a.rows / p.bm;
  }
  if (p.bm == 128) {
    if (split) { X3_SP(128, false) } else { X3_BF(128, false) }
  } else if (p.bm == 64) {
    if (p.cpw) { if (split) { X3_SP(64, true) } else { X3_BF(64, true) } }
    else { if (split) { X3_SP(64, false) } else { X3_BF(64, false) } }
  } else {
    if (p.cpw) { if (split) { X3_SP(32, true) } else { X3_BF(32, true) } }
    else { if (split) { X3_SP(32, false) } else { X3_BF(32, false) } }
  }
#undef X3_SP
#undef X3_BF
#undef X3_LAUNCH
  return a.rows / p.bm;
}
