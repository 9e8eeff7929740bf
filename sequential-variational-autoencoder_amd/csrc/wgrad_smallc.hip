// Weight gradient of the image-space stride-2 4x4 layers with <= 4 image channels (bf16 MFMA).
//
//   dW[tap][ci][co] = sum_p x[src(p, tap)][ci] * dpre[p][co],   src = (2*oy - 1 + ky, 2*ox - 1 + kx)
//
// the first conv of every recognition ladder (conv2d_bn_lrelu abstract_network.py:17-24 on the
// 64x64x3 image, sequential_vae.py:1553-1560) and of every generator encoder (:1764-1770).  The
// generic tap-merged weight-GEMM (gemm_bf16.hip wgrad_bf16_kernel) gave this shape a 128-row tile
// for M' = 16 taps * 3 channels = 48 and gathered every operand element from HBM per tap: 17 TF/s,
// ~190 us at the tail of the backward for the T-batched recognition layer.
//
// Here a block walks chunks of 256 output pixels (8 output rows of one image):
//   1. the 2R+2 input rows the chunk touches are copied into LDS as fp32 (contiguous rows,
//      16-byte loads; the zero columns / rows of the padding are LDS zeros),
//   2. each thread builds its pixel's im2col vector (16 taps x Cin, bf16) in LDS, as 32-column
//      planes [pixel][32] with a 64-byte pitch,
//   3. the dpre rows of the chunk (bf16, 64 bytes per pixel per 32-column tile) are staged next
//      to them, and the four waves run K steps of 16 pixels over the chunk with the gfx950
//      transposed LDS read (ds_read_b64_tr_b16) for both fragments -- the same fragment layout as
//      wgrad_halo2.hip -- one 32x32x16 MFMA per plane.
// The next chunk's input rows and dpre rows are loaded into registers while the current chunk
// computes.  The four waves' accumulators are summed in LDS in wave order, and the block writes
// its split's partial [16][Cin][N] (the TF layout itself when there is one split); wgrad_reduce
// sums the splits in split order.  Deterministic.
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "knobs.h"
#include "kernels.h"
#include "opload.h"

typedef __bf16 sc_bf16x8 __attribute__((ext_vector_type(8)));
typedef float sc_f32x8 __attribute__((ext_vector_type(8)));
typedef short sc_v4i16 __attribute__((ext_vector_type(4)));
typedef short sc_v8i16 __attribute__((ext_vector_type(8)));

namespace {

constexpr int SC_CP = 256;    // output pixels per chunk
constexpr int SC_WO = 32;     // output width (chunk = 8 whole output rows)
constexpr int SC_R = SC_CP / SC_WO;
constexpr int SC_WR = 2 * SC_R + 2;  // input rows per chunk
constexpr int SC_WI = 2 * SC_WO;     // input width
constexpr int SC_WC = SC_WI + 2;     // window columns (one zero column each side)

__device__ __forceinline__ sc_v4i16 sc_tr16(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) sc_v4i16*)(p));
}
__device__ __forceinline__ sc_bf16x8 sc_join(sc_v4i16 lo, sc_v4i16 hi) {
  sc_v8i16 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(sc_bf16x8, v);
}

struct SCArgs {
  const float* X; long long x_gs;        // input image, fp32 NHWC [B][64][64][CI] (row-contiguous)
  const void* D; long long d_gs; int ldd;  // dpre [B*32*32][ldd]: bf16 (NSP = 1) or fp32 (NSP = 2)
  float* part; long long p_gs;           // [split][16][CI][N] partials (or dW when nsplit == 1)
  int N, nsplit, nchunk, Hi;             // Hi = 64 (input rows per image)
};

// NSP = 2: the split-bf16 mode (dtype bf16x6's weight gradients, opload.h): fp32 dpre, the im2col
// vectors and the dpre rows staged as hi / lo bf16 planes, three MFMAs per fragment pair
template <int CI, int NSP = 1>
__global__ __launch_bounds__(256) void wgrad_smallc_kernel(SCArgs a) {
  constexpr int MP = 16 * CI;             // im2col length
  constexpr int NPL = (MP + 31) / 32;     // 32-column planes
  constexpr int XROW = SC_WI * CI;        // floats of one input row
  constexpr int XQ = SC_WR * XROW / 4;    // float4 items of the chunk's input rows
  constexpr int XI = (XQ + 255) / 256;    // per thread
  constexpr int DI = SC_CP * 4 / 256;     // dpre items per thread (4 per pixel, 8 elements each)
  static_assert(XROW % 4 == 0, "input rows are float4 multiples");
  // LDS: x window (fp32) | im2col planes (bf16) x NSP | dpre rows (bf16) x NSP; reused for the wave reduction
  extern __shared__ __attribute__((aligned(16))) char wsc_lds[];
  float* xw = (float*)wsc_lds;                                          // [SC_WR][SC_WC][CI]
  __bf16* ap = (__bf16*)(wsc_lds + SC_WR * SC_WC * CI * 4);              // [NSP][NPL][SC_CP][32]
  __bf16* dr = (__bf16*)(wsc_lds + SC_WR * SC_WC * CI * 4 + NSP * NPL * SC_CP * 64);  // [NSP][SC_CP][32]
  constexpr int APL = NPL * SC_CP * 32;   // bf16 elements of one split plane of ap
  constexpr int DPL = SC_CP * 32;         // ... of dr
  static_assert((SC_WR * SC_WC * CI * 4) % 16 == 0, "16-byte aligned planes");

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int grp = lane >> 4, i16 = lane & 15, q = i16 >> 2, p4 = i16 & 3;
  const int split = blockIdx.x, n0 = blockIdx.y * 32, group = blockIdx.z;
  const int cbeg = (int)((long long)a.nchunk * split / a.nsplit);
  const int cend = (int)((long long)a.nchunk * (split + 1) / a.nsplit);
  const float* X = a.X + group * a.x_gs;
  const __bf16* D = (const __bf16*)a.D + group * a.d_gs;
  const float* Df = (const float*)a.D + group * a.d_gs;
  constexpr int PER_IMG = SC_WO * SC_WO;

  // zero columns of the window and the im2col columns past MP: written once
  for (int i = tid; i < SC_WR * 2 * CI; i += 256) {
    const int r = i / (2 * CI), e = i - r * 2 * CI;
    const int col = e < CI ? 0 : SC_WC - 1;
    xw[(r * SC_WC + col) * CI + (e % CI)] = 0.f;
  }
  if (MP % 32) {
#pragma unroll
    for (int p = 0; p < NSP; ++p)
#pragma unroll
      for (int m = MP; m < NPL * 32; m += 8)
        *(sc_bf16x8*)&ap[p * APL + ((m >> 5) * SC_CP + tid) * 32 + (m & 31)] = sc_bf16x8{};
  }

  f32x4 xv[XI], dv[DI][NSP];
  auto load_chunk = [&](int c) {
    const int r0 = c * SC_CP;
    const int img = r0 / PER_IMG, oy0 = (r0 - img * PER_IMG) / SC_WO;
    const int iy0 = 2 * oy0 - 1;
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int it = tid + 256 * i;
      xv[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (it < XQ) {
        const int wr = it / (XROW / 4), j = it - wr * (XROW / 4);
        const int iy = iy0 + wr;
        if (iy >= 0 && iy < a.Hi) xv[i] = *(const f32x4*)(X + ((long long)img * a.Hi + iy) * XROW + j * 4);
      }
    }
#pragma unroll
    for (int i = 0; i < DI; ++i) {
      const int it = tid + 256 * i;
      const int k = it >> 2, sl = it & 3;
      const long long o = (long long)(r0 + k) * a.ldd + n0 + sl * 8;
      if constexpr (NSP == 1) {
        dv[i][0] = *(const f32x4*)(D + o);
      } else {  // 8 fp32 in the two registers, split at the LDS store
        dv[i][0] = *(const f32x4*)(Df + o);
        dv[i][1] = *(const f32x4*)(Df + o + 4);
      }
    }
  };

  // fragment read bases (bytes): pixel lk of a K step, column quad ch (wgrad_halo2.hip's layout)
  const int lk = 8 * (grp >> 1) + q;
  const int ch = 16 * (grp & 1) + 4 * p4;
  const int abyte = (lk * 32 + ch) * 2;
  const int dbyte = (lk * 32 + 4 * (grp & 1) * 4 + p4 * 4) * 2;

  f32x16 acc[NPL];
#pragma unroll
  for (int pl = 0; pl < NPL; ++pl)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[pl][r] = 0.f;

  if (cbeg < cend) load_chunk(cbeg);
  for (int c = cbeg; c < cend; ++c) {
    __syncthreads();  // the previous chunk's readers are done
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int it = tid + 256 * i;
      if (it < XQ) {
        const int wr = it / (XROW / 4), j = it - wr * (XROW / 4);
        float* dst = &xw[(wr * SC_WC + 1) * CI + j * 4];
#pragma unroll
        for (int e = 0; e < 4; ++e) dst[e] = xv[i][e];
      }
    }
#pragma unroll
    for (int i = 0; i < DI; ++i) {
      const int it = tid + 256 * i;
      const int o = (it >> 2) * 32 + (it & 3) * 8;
      if constexpr (NSP == 1) {
        *(f32x4*)&dr[o] = dv[i][0];
      } else {
        ol_bf16x8 pl[NSP];
        split8<NSP>(dv[i][0], dv[i][1], pl);
#pragma unroll
        for (int p = 0; p < NSP; ++p) *(ol_bf16x8*)&dr[p * DPL + o] = pl[p];
      }
    }
    __syncthreads();
    // im2col of pixel tid: m = (ky*4 + kx)*CI + ci
    {
      const int oyl = tid / SC_WO, ox = tid - oyl * SC_WO;
      float v[MP];
#pragma unroll
      for (int ky = 0; ky < 4; ++ky)
#pragma unroll
        for (int kx = 0; kx < 4; ++kx)
#pragma unroll
          for (int ci = 0; ci < CI; ++ci) v[(ky * 4 + kx) * CI + ci] = xw[((2 * oyl + ky) * SC_WC + 2 * ox + kx) * CI + ci];
#pragma unroll
      for (int m = 0; m < MP; m += 8) {
        const int o = ((m >> 5) * SC_CP + tid) * 32 + (m & 31);
        if constexpr (NSP == 1) {
          const sc_f32x8 w8 = {v[m], v[m + 1], v[m + 2], v[m + 3], v[m + 4], v[m + 5], v[m + 6], v[m + 7]};
          *(sc_bf16x8*)&ap[o] = __builtin_convertvector(w8, sc_bf16x8);
        } else {
          ol_bf16x8 pl[NSP];
          split8<NSP>(f32x4{v[m], v[m + 1], v[m + 2], v[m + 3]}, f32x4{v[m + 4], v[m + 5], v[m + 6], v[m + 7]}, pl);
#pragma unroll
          for (int p = 0; p < NSP; ++p) *(ol_bf16x8*)&ap[p * APL + o] = pl[p];
        }
      }
    }
    __syncthreads();
    if (c + 1 < cend) load_chunk(c + 1);
    const char* A = (const char*)ap;
    const char* Db = (const char*)dr;
#pragma unroll
    for (int j = 0; j < SC_CP / 16 / 4; ++j) {
      const int k0 = (j * 4 + wave) * 16;
      ol_bf16x8 bf[NSP];
#pragma unroll
      for (int p = 0; p < NSP; ++p)
        bf[p] = sc_join(sc_tr16(Db + p * DPL * 2 + dbyte + k0 * 64), sc_tr16(Db + p * DPL * 2 + dbyte + (k0 + 4) * 64));
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl) {
        ol_bf16x8 af[NSP];
#pragma unroll
        for (int p = 0; p < NSP; ++p) {
          const char* Ap = A + p * APL * 2 + pl * SC_CP * 64;
          af[p] = sc_join(sc_tr16(Ap + abyte + k0 * 64), sc_tr16(Ap + abyte + (k0 + 4) * 64));
        }
        acc[pl] = mfma_split<NSP>(af, bf, acc[pl]);
      }
    }
  }

  // four waves' accumulators, summed in wave order through LDS
  __syncthreads();
  float* red = (float*)ap;  // [3][NPL][16][64] floats <= the im2col planes
  static_assert(3 * NPL * 16 * 64 * 4 <= NPL * SC_CP * 32 * 2, "reduction fits the planes");
  if (wave > 0) {
#pragma unroll
    for (int pl = 0; pl < NPL; ++pl)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[(((wave - 1) * NPL + pl) * 16 + r) * 64 + lane] = acc[pl][r];
  }
  __syncthreads();
  if (wave > 0) return;
  float* out = a.part + group * a.p_gs + (long long)split * MP * a.N;
#pragma unroll
  for (int pl = 0; pl < NPL; ++pl)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float s = acc[pl][r];
#pragma unroll
      for (int w = 0; w < 3; ++w) s += red[((w * NPL + pl) * 16 + r) * 64 + lane];
      const int m = pl * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
      if (m < MP) out[(long long)m * a.N + n0 + l32] = s;
    }
}

}  // namespace

int wgrad_smallc_disabled() {
  static const int v = svae_knob("SVAE_NO_WSC", 0) == 1;
  return v;
}

// eligible: 4x4 stride 2 pad 1 gather from 64x64 to 32x32 row space, <= 4 contiguous fp32 gathered
// channels (conv input / the output conv-T's packed gradient), bf16 row operand with N % 32 == 0
int wgrad_smallc_ok(const WgArgs& w) {
  const ConvGeom& g = w.g;
  if (wgrad_smallc_disabled()) return 0;
  if (g.mode != GM_CONV || g.ksz != 4 || g.stride != 2 || g.pad != 1 || w.ntap != 16) return 0;
  if (g.Ho != SC_WO || g.Wo != SC_WO || g.Hi != 2 * SC_WO || g.Wi != 2 * SC_WO) return 0;
  if (w.M < 1 || w.M > 4 || w.ldg != w.M || w.g_bf16) return 0;
  if (w.nsp > 1 ? w.d_bf16 != 0 : !w.d_bf16) return 0;  // bf16 dpre, or fp32 dpre for the split planes
  if (w.N % 32 || w.ldd % 8) return 0;
  return w.rows % SC_CP == 0 && w.rows % (SC_WO * SC_WO) == 0;
}

template <int CI, int NSP>
size_t wsc_lds_bytes() {
  constexpr int NPL = (16 * CI + 31) / 32;
  return (size_t)SC_WR * SC_WC * CI * 4 + NSP * ((size_t)NPL * SC_CP * 64 + (size_t)SC_CP * 64);
}
template <int CI, int NSP>
void wsc_launch1(const SCArgs& a, dim3 grid, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)wgrad_smallc_kernel<CI, NSP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)wsc_lds_bytes<CI, NSP>());
    attr = true;
  }
  const size_t lds = wsc_lds_bytes<CI, NSP>();
  hipLaunchKernelGGL((wgrad_smallc_kernel<CI, NSP>), grid, dim3(256), lds, s, a);
}
template <int CI>
void wsc_launch(const SCArgs& a, int nsp, dim3 grid, hipStream_t s) {
  if (nsp > 1) wsc_launch1<CI, 2>(a, grid, s);
  else wsc_launch1<CI, 1>(a, grid, s);
}

// partials [split][16][M][N] of an eligible layer into part (group stride nsplit*16*M*N), ~512
// blocks with >= 2 chunks per split and the slab within cap; returns the split count (0: not
// eligible).  The caller reduces them (wgrad_reduce), e.g. routing rows to several tensors.
int wgrad_smallc_part(const WgArgs& w, int groups, float* part, long long cap, hipStream_t s) {
  if (!wgrad_smallc_ok(w)) return 0;
  SCArgs a;
  a.X = w.G; a.x_gs = w.g_gs;
  a.D = w.D; a.d_gs = w.d_gs; a.ldd = w.ldd;
  a.N = w.N;
  a.Hi = 2 * SC_WO;
  a.nchunk = w.rows / SC_CP;
  const long long per = 16LL * w.M * w.N;
  const long long tiles = (long long)(w.N / 32) * groups;
  long long ns = (512 + tiles - 1) / tiles;
  ns = std::min<long long>(ns, std::max(1, a.nchunk / 2));
  ns = std::min<long long>(ns, std::max<long long>(1, cap / (per * groups)));
  a.nsplit = (int)std::max<long long>(1, ns);
  a.part = part;
  a.p_gs = (long long)a.nsplit * per;
  dim3 grid(a.nsplit, w.N / 32, groups);
  switch (w.M) {
    case 1: wsc_launch<1>(a, w.nsp, grid, s); break;
    case 2: wsc_launch<2>(a, w.nsp, grid, s); break;
    case 3: wsc_launch<3>(a, w.nsp, grid, s); break;
    default: wsc_launch<4>(a, w.nsp, grid, s); break;
  }
  return a.nsplit;
}

// dW (TF layout [16][M][N], group stride w_gs) of an eligible layer through the slab
int wgrad_smallc(const WgArgs& w, int groups, float* slab, long long slab_cap, float* dW, long long w_gs,
                 hipStream_t s) {
  const int ns = wgrad_smallc_part(w, groups, slab, slab_cap, s);
  if (!ns) return 0;
  wgrad_reduce(slab, (long long)ns * 16 * w.M * w.N, ns, 16, w.M, w.N, dW, w_gs, w.M, nullptr, 0, 0, groups, s);
  return 1;
}
