// Image-space stride-2 4x4 convolutions with few input channels (Cin <= 4): one MFMA
// gather-GEMM per block over an LDS window of whole input rows.
//
//   * conv 0 of the recognition ladder and of every g_theta encoder step: conv2d of the image,
//     Cin = C = 3 (abstract_network.py:18 conv2d_bn_lrelu; sequential_vae.py:1738,1766);
//   * the output conv-T's input gradient: CONV gather over d[x_hat | ratio], Cin = C+1 = 4
//     (the adjoint of abstract_network.py:37 conv2d_t, sequential_vae.py:1723-1729).
//
// The generic gather-GEMMs reach Cin % 32 != 0 through an element-wise gather with a tap decode
// per element (igemm_fwd_kernel / igemm_bf16_kernel SMALLC): 60-80 us per launch for a 16.8 MB
// output.  Here a block owns 256 consecutive output pixels = R = 256/Wo whole output rows of one
// image, stages the (2R+2) x (Wi+2) input window once, channel-padded to 4 with zeros (TF SAME
// padding and the missing channel), and runs K = 16 taps x 4 channels from it:
//   BF   (bf16 model): 4 x v_mfma_f32_32x32x16_bf16 per 32x32 tile; lane h's 8 k values are
//        taps (ky, 2h) and (ky, 2h+1) x 4 channels = ONE 16-byte LDS read.  Operands are
//        RNE-rounded to bf16 exactly as the staging of the other bf16 gathers; B = the bf16
//        shadow weights a.Bh [tap][n][k];
//   fp32 (fp32 model, and the output conv-T input gradient in both): 32 x
//        v_mfma_f32_32x32x2_f32 per tile (exact fp32 fma chains); in step (tap, s) lane h holds
//        channel 2h+s, so one 8-byte LDS read feeds two MFMAs.
// The epilogue is the generic one: optional bias, activation, accumulate, and the per-column
// (sum, sum^2) BatchNorm partials of the block's 256 rows -> stats[rowblock = blockIdx.x].
// 128-pixel blocks (twice the blocks in flight) measured the same step time (19.12 vs 19.17 ms,
// 3 alternating bench pairs on one box), so the larger block with half the stats partials stays.
#include <type_traits>

#include "common.h"
#include "knobs.h"
#include "kernels.h"
#include "opload.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int SC_TM = 2;               // 32-pixel tiles per wave
constexpr int SC_BM = 4 * 32 * SC_TM;  // output pixels per block (4 waves)
constexpr int SC_SQ = 6;               // window items per thread (WR * WC <= 1536)

// PB: the fused backward-BN partials read a bf16-stored pre (a.bw.pre_bf16; compile-time: a run-time
// choice per load cost the output layer's input gradient 75 %)
template <int TN, int TM, bool BF, bool PB = false>
__global__ __launch_bounds__(256) void conv_smallc_kernel(FwdArgs a) {
  constexpr int BM = 128 * TM;
  // window: BF 8 B per pixel (4 x bf16), fp32 16 B per pixel; sized by the host (dynamic LDS)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ float red[2][4][TN * 32];

  const ConvGeom& g = a.g;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int group = blockIdx.z;
  const int HWo = g.Ho * g.Wo;
  const int p0 = blockIdx.x * BM;  // first output pixel (row space)
  const int img = p0 / HWo;
  const int oy0 = (p0 - img * HWo) / g.Wo;
  const int R = BM / g.Wo;
  const int WR = 2 * R + 2, WC = g.Wi + 2;
  const int iy0 = 2 * oy0 - g.pad;

  const float* A = a.A + group * a.a_gs + (long long)img * g.Hi * g.Wi * a.lda;

  // ---- stage the window (rows iy0 .. iy0+WR-1, cols -1 .. Wi), 4 channels, zeros outside: every
  //      item's loads issue before the first LDS store (one memory round trip per block, not one per
  //      256 items; WR * WC <= 256 * SC_SQ, host-checked)
  {
    f32x4 sv[SC_SQ];
#pragma unroll
    for (int i = 0; i < SC_SQ; ++i) {
      const int q = tid + 256 * i;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (q < WR * WC) {
        const int r = q / WC, col = q - r * WC;
        const int iy = iy0 + r, ix = col - 1;
        if (iy >= 0 && iy < g.Hi && ix >= 0 && ix < g.Wi) {
          const float* src = A + ((long long)iy * g.Wi + ix) * a.lda;
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (c < a.Cin) v[c] = src[c];
        }
      }
      sv[i] = v;
    }
#pragma unroll
    for (int i = 0; i < SC_SQ; ++i) {
      const int q = tid + 256 * i;
      if (q < WR * WC) {
        if (BF) ((bf16x4*)smem)[q] = __builtin_convertvector(sv[i], bf16x4);
        else ((f32x4*)smem)[q] = sv[i];
      }
    }
  }

  // ---- B fragments (registers, once per block)
  const int N = a.N;
  typedef typename std::conditional<BF, bf16x8, float>::type BFrag;
  constexpr int KSTEPS = BF ? 4 : 32;
  BFrag bfr[TN][KSTEPS];
  if constexpr (BF) {
    const __bf16* Bw = (const __bf16*)a.Bh + group * a.b_gs;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int n = tn * 32 + l32;
#pragma unroll
      for (int j = 0; j < KSTEPS; ++j) {
        bf16x8 w = {};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int tap = 4 * j + 2 * h + (e >> 2), c = e & 3;
          if (c < a.Cin) w[e] = Bw[tap * a.b_tap + (long long)n * a.ldb + c];
        }
        bfr[tn][j] = w;
      }
    }
  } else {
    const float* Bw = a.B + group * a.b_gs;
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int n = tn * 32 + l32;
#pragma unroll
      for (int j = 0; j < KSTEPS; ++j) {
        const int tap = j >> 1, c = 2 * h + (j & 1);
        float w = 0.f;
        if (c < a.Cin)
          w = a.b_nk ? Bw[tap * a.b_tap + (long long)n * a.ldb + c] : Bw[tap * a.b_tap + (long long)c * a.ldb + n];
        bfr[tn][j] = w;
      }
    }
  }
  __syncthreads();

  // ---- per-lane window base of its pixel in each tile: output (oy, ox) reads window row
  //      2(oy-oy0)+ky, col 2ox+kx
  int base[TM];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    const int pi = p0 - img * HWo + 32 * (wave * TM + tm) + l32;
    const int oy = pi / g.Wo, ox = pi - (pi / g.Wo) * g.Wo;
    base[tm] = 2 * (oy - oy0) * WC + 2 * ox;
  }

  f32x16 acc[TM][TN];
#pragma unroll
  for (int tm = 0; tm < TM; ++tm)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[tm][tn][r] = 0.f;

  if constexpr (BF) {
    const bf16x4* Wb = (const bf16x4*)smem;
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // ky = j; lane h: kx = 2h, 2h+1
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const bf16x8 av = *(const bf16x8*)&Wb[base[tm] + j * WC + 2 * h];
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bfr[tn][j], acc[tm][tn], 0, 0, 0);
      }
    }
  } else {
    const float* Wf = (const float*)smem;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int off = (t >> 2) * WC + (t & 3);
#pragma unroll
      for (int tm = 0; tm < TM; ++tm) {
        const f32x2 av = *(const f32x2*)&Wf[(base[tm] + off) * 4 + 2 * h];
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[0], bfr[tn][2 * t], acc[tm][tn], 0, 0, 0);
          acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[1], bfr[tn][2 * t + 1], acc[tm][tn], 0, 0, 0);
        }
      }
    }
  }

  // ---- epilogue (optionally with the fused backward-BN partials of the layer whose dy this is:
  //      BwStat, the halo_kw / igemm_halo contract; their pre / y rows load before any store)
  float* Cp = a.C + group * a.c_gs;
  const float* bias = a.bias ? a.bias + group * a.bias_gs : nullptr;
  float csum[TN], csq[TN];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) { csum[tn] = 0.f; csq[tn] = 0.f; }
  const bool bwm = a.bw.pre != nullptr;
  float bwmean[TN], bwis[TN], bwb[TN];
#pragma unroll
  for (int tn = 0; tn < TN; ++tn) {
    const int n = tn * 32 + l32;
    bwmean[tn] = bwis[tn] = bwb[tn] = 0.f;
    if (bwm && n < a.bw.C) {
      bwmean[tn] = a.bw.mean[group * a.bw.ms_gs + n];
      bwis[tn] = a.bw.invstd[group * a.bw.ms_gs + n];
      bwb[tn] = a.bw.y ? 0.f : a.bw.beta[group * a.bw.beta_gs + n];
    }
  }
  constexpr bool pbf = PB;
  const float* bwpre = bwm ? pf_at(a.bw.pre, group * a.bw.pre_gs, pbf) : nullptr;
  const bool ybf = a.bw.y_bf16 != 0;
  const float* bwy = (bwm && a.bw.y) ? pf_at(a.bw.y, group * a.bw.y_gs, ybf) : nullptr;
#pragma unroll
  for (int tm = 0; tm < TM; ++tm) {
    float pv[16][TN], yv[16][TN];
    if (bwm) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long long m = p0 + 32 * (wave * TM + tm) + (r & 3) + 8 * (r >> 2) + 4 * h;
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
          const int n = tn * 32 + l32;
          const bool bwc = n < a.bw.C;
          pv[r][tn] = bwc ? pf_ld(bwpre, m * a.bw.ldp + n, pbf) : 0.f;
          yv[r][tn] = (bwc && bwy) ? pf_ld(bwy, m * a.bw.ldy + n, ybf) : 0.f;
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const long long m = p0 + 32 * (wave * TM + tm) + (r & 3) + 8 * (r >> 2) + 4 * h;
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) {
        const int n = tn * 32 + l32;
        float v = acc[tm][tn][r];
        if (BF && a.c_bf16) v = bf_rnd(v);  // bf16-stored pre-BN output: the statistics of the stored values (bf16 model only)
        if (!bwm) {
          csum[tn] += v;
          csq[tn] += v * v;
        }
        if (bias) v += bias[n];
        v = act_f(v, a.act);
        if (BF && a.c_bf16) {
          ((__bf16*)a.C)[group * a.c_gs + m * a.ldc + n] = (__bf16)v;
          continue;
        }
        float* dst = Cp + m * a.ldc + n;
        if (a.accumulate) v += *dst;
        *dst = v;
        if (bwm && n < a.bw.C)
          bw_term_v(v, pv[r][tn], bwmean[tn], bwis[tn], bwb[tn], bwy != nullptr, yv[r][tn], a.bw.act, csum[tn], csq[tn]);
      }
    }
  }
  if (a.stats) {
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      csum[tn] += __shfl_xor(csum[tn], 32, 64);
      csq[tn] += __shfl_xor(csq[tn], 32, 64);
      if (h == 0) {
        red[0][wave][tn * 32 + l32] = csum[tn];
        red[1][wave][tn * 32 + l32] = csq[tn];
      }
    }
    __syncthreads();
    if (tid < (bwm ? a.bw.C : N)) {
      const float s = ((red[0][0][tid] + red[0][1][tid]) + red[0][2][tid]) + red[0][3][tid];
      const float q = ((red[1][0][tid] + red[1][1][tid]) + red[1][2][tid]) + red[1][3][tid];
      stat_put(a.stats + (blockIdx.x & (a.s_nsh - 1)) * a.s_sh + group * a.s_gs, tid, s, q);
    }
  }
}

int smallc_lds(const FwdArgs& a, bool bf) {
  const int R = SC_BM / a.g.Wo;
  return (2 * R + 2) * (a.g.Wi + 2) * (bf ? 8 : 16);
}

template <int TN, bool BF>
void launch_smallc(const FwdArgs& a, int groups, hipStream_t s) {
  dim3 grid(a.rows / SC_BM, 1, groups);
  if (a.bw.pre && a.bw.pre_bf16)
    hipLaunchKernelGGL((conv_smallc_kernel<TN, SC_TM, BF, true>), grid, dim3(256), smallc_lds(a, BF), s, a);
  else
    hipLaunchKernelGGL((conv_smallc_kernel<TN, SC_TM, BF>), grid, dim3(256), smallc_lds(a, BF), s, a);
}

// ---------------------------------------------------------------------------
// Stride-2 4x4 conv-T gathers with few output channels (N <= 16): the output conv-T of the
// decoder (F1 -> [x_hat | ratio], N = C+1 = 4; sequential_vae.py:1720,1727 via
// abstract_network.py:37) and the input gradient of layer-0 conv (CONVT gather over its dpre,
// N = C = 3).  On the 32-column tiles of the general gathers these cost what an N = 32 launch
// does (61 us at CelebA B=128) for a tenth of the output.
//
// A block owns R = 8 full-width output rows of one image; wave w owns output parity class
// (cy, cx) = (w >> 1, w & 1), whose pixels all use the same 4 taps (ky = ky0 + 2ty,
// kx = kx0 + 2tx) and read input pixel (qy + cy - ty, qx + cx - tx) for class pixel (qy, qx).
// The R/2 + 2 input rows (+1 column of zeros each side) of a 32-channel chunk are staged once
// as bf16 (80-byte pixel pitch), and every 16-pixel class-row segment is one
// v_mfma_f32_16x16x32_bf16 per tap: K = the chunk's 32 channels, N padded to 16.
// ---------------------------------------------------------------------------
constexpr int SN_R = 8;      // output rows per block
constexpr int SN_PITCH = 40; // LDS pixel pitch in bf16 (32 channels + 8 pad)
constexpr int SN_MAXT = 16;  // class-row tiles per wave: (R/2) x (Wi/16) <= 16  -> Wi <= 64
constexpr int SN_SQ = 2;     // window staging items per thread and batch (4 cost the kernel a wave per SIMD)

typedef float f32x8 __attribute__((ext_vector_type(8)));

// NS = 3 (split mode, dtype bf16x6): the fp32 window is staged as three bf16 planes (opload.h split8),
// B comes from the three weight planes (a.b_plane apart) and every fragment pair runs the six plane
// products (mfma_split16): an fp32-accurate conv-T on bf16 MFMA
template <int NS>
__device__ __forceinline__ f32x4 mfma_split16(const bf16x8 (&x)[NS], const bf16x8 (&y)[NS], f32x4 acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[0], y[0], acc, 0, 0, 0);
  if constexpr (NS >= 3) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[0], y[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[1], y[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[0], y[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[2], y[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x[1], y[1], acc, 0, 0, 0);
  }
  return acc;
}

// MT: class-row tiles per wave the kernel is compiled for (8: input rows up to 32 wide -- the 64x64 output
// layer; 16: up to 64).  The accumulators and the unrolled tile loop scale with it: at 16 the split
// instance needed 256 VGPRs + 91 AGPRs (one wave per SIMD)
template <int NS, int MT = SN_MAXT>
__global__ __launch_bounds__(256) void convt_smalln_kernel(FwdArgs a) {
  static_assert(NS == 1 || NS == 3, "one plane or the split mode's three");
  static_assert(MT <= SN_MAXT, "tiles per wave");
  extern __shared__ __attribute__((aligned(16))) __bf16 wsm[];
  const ConvGeom& g = a.g;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cy = wave >> 1, cx = wave & 1;
  const int r16 = lane & 15, kg = lane >> 4;
  const int bpi = g.Ho / SN_R;
  const int img = blockIdx.x / bpi;
  const int Y0 = (blockIdx.x - img * bpi) * SN_R;
  const int group = blockIdx.z;
  const int PR = SN_R / 2 + 2, PC = g.Wi + 2;
  const int iy0 = Y0 / 2 - 1;
  const int WT = g.Wi / 16;             // 16-pixel segments per class row
  const int ntile = (SN_R / 2) * WT;
  const long long a0 = group * a.a_gs + (long long)img * g.Hi * g.Wi * a.lda;  // element offset (fp32 or bf16 A)
  const bool abf = a.a_bf16 != 0;
  const __bf16* Bw = (const __bf16*)a.Bh + group * a.b_gs;
  const int ky0 = (cy + g.pad) & 1, kx0 = (cx + g.pad) & 1;
  const bool nvalid = r16 < a.N;
  const int wplane = PR * PC * SN_PITCH;  // LDS elements per window plane (NS = 3)

  f32x4 acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int ch = 0; ch < a.Cin; ch += 32) {
    if (ch) __syncthreads();  // previous chunk's window fully read
    // batches of SN_SQ items per thread: every load of a batch issues before its LDS stores (one
    // memory round trip per batch of 512 items)
    for (int b0 = 0; b0 < PR * PC * 4; b0 += 256 * SN_SQ) {
      f32x4 lo[SN_SQ], hi[SN_SQ];
#pragma unroll
      for (int i = 0; i < SN_SQ; ++i) {
        const int it = b0 + tid + 256 * i;
        lo[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        hi[i] = lo[i];
        if (it < PR * PC * 4) {
          const int pix = it >> 2, part = it & 3;
          const int pr = pix / PC, pc = pix - pr * PC;
          const int iy = iy0 + pr, ix = pc - 1;
          if (iy >= 0 && iy < g.Hi && ix >= 0 && ix < g.Wi)
            ld8_raw(a.A, a0 + ((long long)iy * g.Wi + ix) * a.lda + ch + part * 8, abf, lo[i], hi[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < SN_SQ; ++i) {
        const int it = b0 + tid + 256 * i;
        if (it < PR * PC * 4) {
          const int o = (it >> 2) * SN_PITCH + (it & 3) * 8;
          if constexpr (NS == 1) {
            *(bf16x8*)&wsm[o] = raw8_bf(lo[i], hi[i], abf);
          } else {
            bf16x8 pl[NS];
            split8<NS>(lo[i], hi[i], pl);
#pragma unroll
            for (int q = 0; q < NS; ++q) *(bf16x8*)&wsm[q * wplane + o] = pl[q];
          }
        }
      }
    }
    // this class's 4 tap fragments of the chunk (columns >= N are zero)
    bf16x8 bq[4][NS];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int tap = (ky0 + 2 * (t >> 1)) * 4 + kx0 + 2 * (t & 1);
#pragma unroll
      for (int q = 0; q < NS; ++q)
        bq[t][q] = nvalid ? *(const bf16x8*)(Bw + q * a.b_plane + tap * a.b_tap + (long long)r16 * a.ldb + ch + 8 * kg)
                          : bf16x8{};
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      if (i < ntile) {
        const int j = i / WT, hseg = i - j * WT;
        // class pixel (qy, qx) = (Y0/2 + j, 16*hseg + r16): window row qy + cy - ty - iy0
        const int wr = j + 1 + cy, wc = 16 * hseg + r16 + cx + 1;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int ty = t >> 1, tx = t & 1;
          bf16x8 af[NS];
#pragma unroll
          for (int q = 0; q < NS; ++q) af[q] = *(const bf16x8*)&wsm[q * wplane + ((wr - ty) * PC + wc - tx) * SN_PITCH + 8 * kg];
          acc[i] = mfma_split16<NS>(af, bq[t], acc[i]);
        }
      }
    }
  }

  float* Cp = a.C + group * a.c_gs;
  const float bv = nvalid && a.bias ? a.bias[group * a.bias_gs + r16] : 0.f;
  if (a.ldc == a.N) {
    // the block's SN_R output rows are one contiguous run of SN_R * Wo * N floats: assemble them in
    // LDS (the four classes interleave), then store the run with 16-byte vectors
    __syncthreads();  // every wave is done reading the window
    float* ot = (float*)wsm;  // [SN_R][Wo][N]
    if (nvalid) {
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        if (i < ntile) {
          const int j = i / WT, hseg = i - j * WT;
          const int y = 2 * j + cy;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int X = 2 * (16 * hseg + 4 * kg + e) + cx;
            ot[(y * g.Wo + X) * a.N + r16] = act_f(acc[i][e] + bv, a.act);
          }
        }
      }
    }
    __syncthreads();
    const int n = SN_R * g.Wo * a.N;
    float* dst = Cp + ((long long)img * g.Ho + Y0) * g.Wo * a.N;
    if ((n & 3) == 0 && (((long long)img * g.Ho + Y0) * g.Wo * a.N & 3) == 0) {
      for (int q = tid; q < n / 4; q += 256) {
        f32x4 v = *(const f32x4*)&ot[4 * q];
        if (a.accumulate) v += *(const f32x4*)(dst + 4 * q);
        *(f32x4*)(dst + 4 * q) = v;
      }
    } else {
      for (int q = tid; q < n; q += 256) dst[q] = a.accumulate ? dst[q] + ot[q] : ot[q];
    }
    return;
  }
  if (!nvalid) return;
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    if (i < ntile) {
      const int j = i / WT, hseg = i - j * WT;
      const int Y = Y0 + 2 * j + cy;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int X = 2 * (16 * hseg + 4 * kg + e) + cx;
        float v = acc[i][e] + bv;
        v = act_f(v, a.act);
        float* dst = Cp + (((long long)img * g.Ho + Y) * g.Wo + X) * a.ldc + r16;
        if (a.accumulate) v += *dst;
        *dst = v;
      }
    }
  }
}

}  // namespace

bool smallc_ok(const FwdArgs& a, bool bf) {
  const ConvGeom& g = a.g;
  if (smallc_disabled()) return false;
  if (g.mode != GM_CONV || g.ksz != 4 || g.stride != 2 || g.pad != 1 || a.nclass != 1) return false;
  if (a.Cin < 1 || a.Cin > 4) return false;
  if (a.bw.pre && (a.bw.C > a.N || !a.stats)) return false;  // fused BN-backward partials: N columns at most
  if (!(a.N == 32 || a.N == 64 || a.N == 128)) return false;
  if (g.Hi != 2 * g.Ho || g.Wi != 2 * g.Wo || g.Wo > SC_BM || SC_BM % g.Wo) return false;
  if ((g.Ho * g.Wo) % SC_BM || a.rows % SC_BM) return false;
  if (bf ? !a.Bh : !a.B) return false;
  if ((2 * (SC_BM / g.Wo) + 2) * (g.Wi + 2) > 256 * SC_SQ) return false;  // the staging's item budget
  return smallc_lds(a, bf) <= 64 * 1024;
}

int smallc_nrb(const FwdArgs& a) { return a.rows / SC_BM; }

bool smallc_disabled() {
  static const int off = svae_knob("SVAE_NO_SMALLC", 0) == 1;
  return off != 0;
}

void conv_smallc(const FwdArgs& a, int groups, bool bf, hipStream_t s) {
  if (bf) {
    if (a.N == 32) launch_smallc<1, true>(a, groups, s);
    else if (a.N == 64) launch_smallc<2, true>(a, groups, s);
    else launch_smallc<4, true>(a, groups, s);
  } else {
    if (a.N == 32) launch_smallc<1, false>(a, groups, s);
    else if (a.N == 64) launch_smallc<2, false>(a, groups, s);
    else launch_smallc<4, false>(a, groups, s);
  }
}

int smallc_bm() { return SC_BM; }

bool smalln_ok(const FwdArgs& a) {
  const ConvGeom& g = a.g;
  if (smallc_disabled()) return false;
  if (g.mode != GM_CONVT || g.ksz != 4 || g.stride != 2 || g.pad != 1 || a.nclass != 4) return false;
  if (a.N < 1 || a.N > 16 || a.Cin % 32 || !a.Bh || a.stats || a.bw.pre) return false;
  if (g.Ho != 2 * g.Hi || g.Wo != 2 * g.Wi || g.Ho % SN_R || g.Wi % 16) return false;
  if ((SN_R / 2) * (g.Wi / 16) > SN_MAXT) return false;
  if (a.ldb % 8 || a.b_tap % 8 || a.lda % 4) return false;  // 16-byte fragment / staging loads
  if (a.nsp > 1 && (a.nsp != 3 || a.a_bf16 || a.b_plane % 8)) return false;  // split: fp32 A, 3 planes
  const int planes = a.nsp > 1 ? 3 : 1;
  return (SN_R / 2 + 2) * (g.Wi + 2) * SN_PITCH * 2 * planes <= 64 * 1024 && SN_R * g.Wo * a.N * 4 <= 64 * 1024;
}

void convt_smalln(const FwdArgs& a, int groups, hipStream_t s) {
  const int planes = a.nsp > 1 ? 3 : 1;
  const int win = (SN_R / 2 + 2) * (a.g.Wi + 2) * SN_PITCH * 2 * planes;
  const int tile = a.ldc == a.N ? SN_R * a.g.Wo * a.N * 4 : 0;  // the assembled output rows
  const int lds = win > tile ? win : tile;
  dim3 grid(a.g.nimg * (a.g.Ho / SN_R), 1, groups);
  const bool small = (SN_R / 2) * (a.g.Wi / 16) <= 8;
  if (planes == 3) {
    if (small) hipLaunchKernelGGL((convt_smalln_kernel<3, 8>), grid, dim3(256), lds, s, a);
    else hipLaunchKernelGGL((convt_smalln_kernel<3>), grid, dim3(256), lds, s, a);
  } else {
    if (small) hipLaunchKernelGGL((convt_smalln_kernel<1, 8>), grid, dim3(256), lds, s, a);
    else hipLaunchKernelGGL((convt_smalln_kernel<1>), grid, dim3(256), lds, s, a);
  }
}
