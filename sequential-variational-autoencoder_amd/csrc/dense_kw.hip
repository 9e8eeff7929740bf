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
#include "kernels.h"
#include "opload.h"

namespace {

typedef __bf16 dk_bf16x8 __attribute__((ext_vector_type(8)));

template <int TN, bool ABF>
__global__ __launch_bounds__(256) void dense_kw_kernel(FwdArgs a) {
  constexpr int BN = 32 * TN;
  __shared__ float red[4][32][BN + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l32 = lane & 31, h = lane >> 5;
  const int m0 = blockIdx.x * 32, n0 = blockIdx.y * BN;
  const int nks = a.Cin / 16, ks = gridDim.z, z = blockIdx.z;
  const int j0 = (int)((long long)nks * z / ks), j1 = (int)((long long)nks * (z + 1) / ks);
  const int m = m0 + l32;
  const bool mv = m < a.rows;
  const __bf16* Bw = (const __bf16*)a.Bh;
  f32x16 acc[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  const long long arow = (long long)m * a.lda;
#pragma unroll 2
  for (int j = j0 + wave; j < j1; j += 4) {
    const int k = 16 * j + 8 * h;
    f32x4 lo = {0.f, 0.f, 0.f, 0.f}, hi = lo;
    if (mv) ld8_raw(a.A, arow + k, ABF, lo, hi);
    const dk_bf16x8 af = raw8_bf(lo, hi, ABF);
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const int n = n0 + t * 32 + l32;
      dk_bf16x8 bf = {};
      if (n < a.N) bf = *(const dk_bf16x8*)(Bw + (long long)n * a.ldb + k);
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf, acc[t], 0, 0, 0);
    }
  }
  // ---- the four waves' partial tiles, summed in a fixed order ----
#pragma unroll
  for (int t = 0; t < TN; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wave][(r & 3) + 8 * (r >> 2) + 4 * h][t * 32 + l32] = acc[t][r];
  __syncthreads();
  constexpr int NRG = 256 / BN;  // row groups
  const int col = tid % BN, rg = tid / BN;
  const int n = n0 + col;
  if (ks > 1) {  // raw partial -> slab[split][row][n]; bias / act / stats in splitk_reduce
    if (n < a.N) {
      float* P = a.part + (long long)z * a.rows * a.N;
      for (int r = rg; r < 32; r += NRG) {
        const int mm = m0 + r;
        if (mm >= a.rows) break;
        float v = red[0][r][col];
#pragma unroll
        for (int w = 1; w < 4; ++w) v += red[w][r][col];
        P[(long long)mm * a.N + n] = v;
      }
    }
    return;
  }
  float s1 = 0.f, s2 = 0.f;
  if (n < a.N) {
    const float bias = a.bias ? a.bias[n] : 0.f;
    for (int r = rg; r < 32; r += NRG) {
      const int mm = m0 + r;
      if (mm >= a.rows) break;
      float v = red[0][r][col];
#pragma unroll
      for (int w = 1; w < 4; ++w) v += red[w][r][col];
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
    stat_put(a.stats + (blockIdx.x & (a.s_nsh - 1)) * a.s_sh, n0 + tid, s, q);
  }
}

bool dkw_disabled() {
  static const bool v = [] {
    const char* e = getenv("SVAE_NO_DKW");
    return e && e[0] == '1';
  }();
  return v;
}

}  // namespace

static long long dkw_blocks(const FwdArgs& a) {
  return (long long)((a.rows + 31) / 32) * (a.N / (a.N % 64 == 0 ? 64 : 32));
}

// K splits over the grid: double while the grid is short of 512 blocks, each split keeps >= 2
// K steps per wave and the slabs fit the scratch
int dense_kw_ks(const FwdArgs& a) {
  const long long blocks = dkw_blocks(a);
  const int nks = a.Cin / 16;
  int ks = 1;
  if (!a.part || a.ldc % 4) return 1;
  while (blocks * ks < 512 && nks / (2 * ks) >= 8 && (long long)(2 * ks) * a.rows * a.N <= a.part_cap) ks *= 2;
  return ks;
}

bool dense_kw_ok(const FwdArgs& a, int groups) {
  if (dkw_disabled() || a.g.mode != GM_DENSE || groups != 1 || a.nclass != 1 || !a.Bh) return false;
  if (a.Cin % 16 || a.N % 32 || a.lda % 8 || a.ldb % 8 || a.rows < 1) return false;
  if (dense_kw_ks(a) > 1) return true;
  // unsplit: only where the grid fills the chip and the per-wave K chain is short; the fused
  // backward-BN terms live in splitk_reduce only
  return !a.bw.pre && dkw_blocks(a) >= 256 && a.Cin <= 2048;
}

int dense_kw_nrb(const FwdArgs& a) { return dense_kw_ks(a) > 1 ? (a.rows + 63) / 64 : (a.rows + 31) / 32; }

int dense_kw(const FwdArgs& a, int ks, hipStream_t s) {
  const int tn = a.N % 64 == 0 ? 2 : 1;
  const dim3 grid((a.rows + 31) / 32, a.N / (32 * tn), ks);
  if (tn == 2) {
    if (a.a_bf16) hipLaunchKernelGGL((dense_kw_kernel<2, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((dense_kw_kernel<2, false>), grid, dim3(256), 0, s, a);
  } else {
    if (a.a_bf16) hipLaunchKernelGGL((dense_kw_kernel<1, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((dense_kw_kernel<1, false>), grid, dim3(256), 0, s, a);
  }
  return ks;
}
