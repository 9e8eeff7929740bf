// Dense (FC) GEMM with the K dimension split over the block's waves (bf16 MFMA, fp32 accumulate).
//
// The FC layers of the chain (the generator's top fc_bn_lrelu, abstract_network.py:64-71, and the
// encoder's last FC, and their input gradients) are [B=128 x K] . [K x N] with K = 384 .. 6144:
// one or two 128-row tiles, so the tiled kernel had to split K over the grid (up to 8 ways) and
// add a split-K reduce launch.  Here a block owns 32 rows x 32*TN columns and all of K; its four
// waves take interleaved 16-wide K steps (step j on wave j % 4), fragments straight from HBM/L2
// (each lane's A row is one batch row, 8 consecutive k; B from the [n][k] bf16 weight copy), and
// the four partial tiles are summed in LDS in a fixed wave order before one epilogue (bias, act,
// accumulate, forward BN column statistics -- the splitk_reduce contract).  Where that grid is
// short of 512 blocks (the encoder FC, N = 384, and the input gradients) K is also split over the
// grid (blockIdx.z), each split writing a raw fp32 slab that splitk_reduce sums in a fixed order.
#include <cstdlib>

#include "common.h"
#include "knobs.h"
#include "kernels.h"
#include "opload.h"

namespace {

typedef __bf16 dk_bf16x8 __attribute__((ext_vector_type(8)));

#ifndef DKW_U
#define DKW_U 4
#endif

// WK waves interleave the K steps of a 32-row tile; 4 / WK such tiles per block (BMR rows).
// WK = 4: 32-row blocks, K over the waves.  WK = 1: 128-row blocks (the whole batch), every wave
// its own 32 rows over the split's full K range, so each weight column is read by one block.
// NS = 3: split-bf16 planes (dtype bf16x6, opload.h): A split in registers, B from the three
// shadow planes, six MFMAs per fragment pair.  NS = 2: the split mode's scaled fp16 hi/lo planes
// (opload.h split8_h16 / mfma_h16, three MFMAs): A * 2^hs with a per-wave running exponent over the
// wave's K batches (the accumulators shrink by the exact power of two when it falls), B the shadow's
// fp16 planes (w * 2^e, e the tensor's exponent); each wave's partial tile is unscaled before the LDS sum
template <int TN, bool ABF, int WK, int NS = 1>
__global__ __launch_bounds__(256) void dense_kw_kernel(FwdArgs a) {
  constexpr int BN = 32 * TN, BMR = 32 * (4 / WK);
  __shared__ float red[WK][BMR][BN + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int wk = wave % WK, wr = wave / WK;
  // XCD-aware order: the row blocks of one column tile (which read the same weight columns) run
  // on one XCD and share its L2
  const BlockXYZ blk = xcd_block();
  const int m0 = blk.x * BMR, n0 = blk.y * BN;
  const int nks = a.Cin / 16, ks = gridDim.z, z = blk.z;
  const int j0 = (int)((long long)nks * z / ks), j1 = (int)((long long)nks * (z + 1) / ks);
  const int m = m0 + wr * 32 + l32;
  const bool mv = m < a.rows;
  const __bf16* Bw = (const __bf16*)a.Bh;  // (NS = 2: advanced to the fp16 planes below)
  [[maybe_unused]] const int wex = (NS == 2 && a.wexp) ? wtab_exp(a.wexp[0]) : H16_WS;
  f32x16 acc[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  const long long arow = (long long)m * a.lda;
  [[maybe_unused]] int hs = 0;
  [[maybe_unused]] float hmax = 0.f;
  if constexpr (NS == 2) Bw += H16_PLANE * a.b_plane;  // the fp16 planes of the shadow
  // DKW_U K steps per batch, all loads of a batch issued before its MFMAs (the per-wave chain is
  // latency-bound: a handful of K steps per wave, few waves per CU); steps past the split's end
  // load zero fragments
  for (int jb = j0 + wk; jb < j1; jb += WK * DKW_U) {
    dk_bf16x8 af[DKW_U][NS], bf[DKW_U][TN][NS];
    [[maybe_unused]] f32x4 alo[DKW_U], ahi[DKW_U];
#pragma unroll
    for (int u = 0; u < DKW_U; ++u) {
      const int j = jb + WK * u;
      const int k = 16 * j + 8 * h;
      f32x4 lo = {0.f, 0.f, 0.f, 0.f}, hi = lo;
      if (mv && j < j1) ld8_raw(a.A, arow + k, ABF, lo, hi);
      if constexpr (NS == 1) af[u][0] = raw8_bf(lo, hi, ABF);
      else if constexpr (NS == 2) {
        alo[u] = lo;
        ahi[u] = hi;
      } else split8<NS>(lo, hi, af[u]);
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        const int n = n0 + t * 32 + l32;
#pragma unroll
        for (int p = 0; p < NS; ++p) {
          bf[u][t][p] = dk_bf16x8{};
          if (n < a.N && j < j1) bf[u][t][p] = *(const dk_bf16x8*)(Bw + p * a.b_plane + (long long)n * a.ldb + k);
        }
      }
    }
    if constexpr (NS == 2) {  // the batch's max |A| over the wave, the running exponent, then the planes
      float mx = 0.f;
#pragma unroll
      for (int u = 0; u < DKW_U; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) mx = fmaxf(mx, fmaxf(fabsf(alo[u][e]), fabsf(ahi[u][e])));
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
      hmax = fmaxf(hmax, mx);
      const int ns = h16_exp(hmax);
      if (ns != hs) {
#pragma unroll
        for (int t = 0; t < TN; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[t][r] = __builtin_ldexpf(acc[t][r], ns - hs);
        hs = ns;
      }
#pragma unroll
      for (int u = 0; u < DKW_U; ++u) split8_h16(alo[u], ahi[u], hs, af[u]);
#pragma unroll
      for (int u = 0; u < DKW_U; ++u)
#pragma unroll
        for (int t = 0; t < TN; ++t) acc[t] = mfma_h16(af[u], bf[u][t], acc[t]);
    } else {
#pragma unroll
      for (int u = 0; u < DKW_U; ++u)
#pragma unroll
        for (int t = 0; t < TN; ++t) acc[t] = mfma_split<NS>(af[u], bf[u][t], acc[t]);
    }
  }
  if constexpr (NS == 2) {  // back to the units of C (the weight planes carry their tensor's exponent)
#pragma unroll
    for (int t = 0; t < TN; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = __builtin_ldexpf(acc[t][r], -(hs + wex));
  }
  // ---- the WK waves' partial tiles, summed in a fixed order ----
#pragma unroll
  for (int t = 0; t < TN; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wk][wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * h][t * 32 + l32] = acc[t][r];
  __syncthreads();
  constexpr int NRG = 256 / BN;  // row groups
  const int col = tid % BN, rg = tid / BN;
  const int n = n0 + col;
  if (ks > 1) {  // raw partial -> slab[split][row][n]; bias / act / stats in splitk_reduce
    if (n < a.N) {
      float* P = a.part + (long long)z * a.rows * a.N;
      for (int r = rg; r < BMR; r += NRG) {
        const int mm = m0 + r;
        if (mm >= a.rows) break;
        float v = red[0][r][col];
#pragma unroll
        for (int w = 1; w < WK; ++w) v += red[w][r][col];
        P[(long long)mm * a.N + n] = v;
      }
    }
    return;
  }
  float s1 = 0.f, s2 = 0.f;
  if (n < a.N) {
    const float bias = a.bias ? a.bias[n] : 0.f;
    for (int r = rg; r < BMR; r += NRG) {
      const int mm = m0 + r;
      if (mm >= a.rows) break;
      float v = red[0][r][col];
#pragma unroll
      for (int w = 1; w < WK; ++w) v += red[w][r][col];
      s1 += v;
      s2 += v * v;
      v = act_f(v + bias, a.act);
      float* dst = a.C + (long long)mm * a.ldc + n;
      if (a.accumulate) v += *dst;
      *dst = v;
    }
  }
  if (!a.stats) return;
  __syncthreads();  // every thread is done reading red
  float* sr = &red[0][0][0];
  sr[tid] = s1;
  sr[256 + tid] = s2;
  __syncthreads();
  if (tid < BN && n0 + tid < a.N) {
    float s = 0.f, q = 0.f;
#pragma unroll
    for (int g = 0; g < NRG; ++g) {
      s += sr[g * BN + tid];
      q += sr[256 + g * BN + tid];
    }
    stat_put(a.stats + (blk.x & (a.s_nsh - 1)) * a.s_sh, n0 + tid, s, q);
  }
}

bool dkw_disabled() {
  static const bool v = svae_knob("SVAE_NO_DKW", 0) == 1;
  return v;
}

}  // namespace

static int dkw_wk() {  // SVAE_DKW_WK: 4 (32-row blocks), 2 or 1 (128-row blocks)
  static const int v = [] {
    const int w = svae_knob("SVAE_DKW_WK", 4);
    return (w == 1 || w == 2) ? w : 4;
  }();
  return v;
}
static int dkw_bmr() { return 32 * (4 / dkw_wk()); }
static int dkw_bmr(const FwdArgs& a) { return a.nsp > 1 ? 32 : dkw_bmr(); }

static long long dkw_blocks(const FwdArgs& a) {
  return (long long)((a.rows + dkw_bmr(a) - 1) / dkw_bmr(a)) * (a.N / (a.N % 64 == 0 ? 64 : 32));
}

// K splits over the grid: double while the grid is short of the target, each split keeps >= mink
// K steps and the slabs fit the scratch
int dense_kw_ks(const FwdArgs& a) {
  const long long blocks = dkw_blocks(a);
  const int nks = a.Cin / 16;
  static const int tgt = svae_knob("SVAE_DKW_TGT", 512);
  static const int mink = svae_knob("SVAE_DKW_MINK", 8);
  int ks = 1;
  if (!a.part || a.ldc % 4) return 1;
  while (blocks * ks < tgt && nks / (2 * ks) >= mink && (long long)(2 * ks) * a.rows * a.N <= a.part_cap) ks *= 2;
  return ks;
}

bool dense_kw_ok(const FwdArgs& a, int groups) {
  if (dkw_disabled() || a.g.mode != GM_DENSE || groups != 1 || a.nclass != 1 || !a.Bh) return false;
  if (a.Cin % 16 || a.N % 32 || a.lda % 8 || a.ldb % 8 || a.rows < 1) return false;
  if (a.nsp > 1) return !a.a_bf16 && (dense_kw_ks(a) > 1 || !a.bw.pre);  // the split kernel: every FC shape
  if (dense_kw_ks(a) > 1) return true;
  // unsplit: only where the grid fills the chip and the per-wave K chain is short; the fused
  // backward-BN terms live in splitk_reduce only
  return !a.bw.pre && dkw_blocks(a) >= 256 && a.Cin <= 2048;
}

// rows per splitk_reduce block: 16-row groups where 64-row blocks would leave the reduce with
// fewer than 128 blocks (latency-bound), else 64 (fewer statistics atomics)
int dense_kw_rpb(const FwdArgs& a) { return (long long)((a.N + 63) / 64) * ((a.rows + 63) / 64) < 128 ? 16 : 64; }

int dense_kw_nrb(const FwdArgs& a) {
  if (dense_kw_ks(a) > 1) return (a.rows + dense_kw_rpb(a) - 1) / dense_kw_rpb(a);
  return (a.rows + dkw_bmr(a) - 1) / dkw_bmr(a);
}

int dense_kw(const FwdArgs& a, int ks, hipStream_t s) {
  const int tn = a.N % 64 == 0 ? 2 : 1, wk = dkw_wk();
  const dim3 grid((a.rows + dkw_bmr(a) - 1) / dkw_bmr(a), a.N / (32 * tn), ks);
#define DKW_L(TN_, WK_)                                                                         \
  if (a.a_bf16) hipLaunchKernelGGL((dense_kw_kernel<TN_, true, WK_>), grid, dim3(256), 0, s, a); \
  else hipLaunchKernelGGL((dense_kw_kernel<TN_, false, WK_>), grid, dim3(256), 0, s, a);
  if (a.nsp > 1 && a.h16) {  // split mode, scaled fp16 planes: fp32 A, 32-row blocks with K over the waves
    if (tn == 2) hipLaunchKernelGGL((dense_kw_kernel<2, false, 4, 2>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((dense_kw_kernel<1, false, 4, 2>), grid, dim3(256), 0, s, a);
  } else if (a.nsp > 1) {  // split-bf16 planes: fp32 A, 32-row blocks with K over the waves
    if (tn == 2) hipLaunchKernelGGL((dense_kw_kernel<2, false, 4, 3>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((dense_kw_kernel<1, false, 4, 3>), grid, dim3(256), 0, s, a);
  } else if (tn == 2) {
    if (wk == 4) { DKW_L(2, 4) } else if (wk == 2) { DKW_L(2, 2) } else { DKW_L(2, 1) }
  } else {
    if (wk == 4) { DKW_L(1, 4) } else if (wk == 2) { DKW_L(1, 2) } else { DKW_L(1, 1) }
  }
#undef DKW_L
  return ks;
}
