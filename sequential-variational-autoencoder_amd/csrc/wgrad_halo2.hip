// Halo weight-GEMM, stride 1, compile-time geometry (bf16 MFMA, gfx950 transposed LDS reads).
//
//   dW[tap][m][n] = sum_p G[src(p, tap)][m] * D[p][n],   src = (y - 1 + ky, x - 1 + kx)
//
// the weight gradient of every stride-1 4x4 conv / conv-T layer (conv2d_bn_lrelu
// abstract_network.py:17-24 with stride 1; conv2d_t_bn_relu :36-43).  It replaces
// gemm_bf16.hip's wgrad_halo_kernel<32,1> for those layers: SQ counters of that kernel
// (profiles/r02_wgrad_sq_before.txt) showed ~17 VALU instructions per MFMA, almost all of it
// the per-K-step pixel -> window decode done at run time.
//
// Here the image width WO and the chunk size CP are template parameters, so for each K step
// (16 pixels) the window offset of every transposed LDS read is a compile-time constant plus a
// lane-dependent base computed once: the inner loop is LDS reads + MFMAs only.
//
// Block = KYR x WN x WK waves (8):
//   KYR kernel rows (ky) per block -> 4*KYR taps (the block's tap group),
//   WN  32-column D subtiles       -> block tile 32 (G channels) x 32*WN (D channels),
//   WK  K-interleaved wave sets    -> summed through LDS once at the end.
// Per chunk of CP pixels (whole image rows, or whole images when WO*WO < CP) the block stages
// the G window (rows +3 halo, cols +3) and the D rows once, bf16, double-buffered in LDS with
// ONE barrier per chunk; chunk c+1 is loaded into registers while chunk c computes.
// Window pitch 64 B (32 G channels) and the D row XOR swizzle (WN = 2) keep the
// ds_read_b64_tr_b16 reads conflict-free (same layouts as gemm_bf16.hip's halo weight-GEMM).
#include "common.h"
#include "knobs.h"
#include "kernels.h"
#include "opload.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef short v8i16 __attribute__((ext_vector_type(8)));

namespace {

__device__ __forceinline__ v4i16 tr16(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)(p));
}
__device__ __forceinline__ bf16x8 join(v4i16 lo, v4i16 hi) {
  v8i16 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// S: the gather stride (1: stride-1 conv / conv-T; 2: stride-2 conv, and stride-2 conv-T with dY
// as the gathered operand), input width HI = S * WO; GP: window pitch in bf16 (64 B at stride 1,
// 96 B at stride 2, where consecutive pixels of a K step sit two window pixels apart)
template <int WO, int CP, int S = 1>
struct Geo2 {
  static constexpr int HI = S * WO;
  static constexpr int GP = S == 1 ? 32 : 48;
  static constexpr int PER_IMG = WO * WO;
  static constexpr int IMG = CP <= PER_IMG ? 1 : CP / PER_IMG;   // images per chunk
  static constexpr int R = CP <= PER_IMG ? CP / WO : WO;         // image rows per chunk (per image)
  static constexpr int PR = S * (R - 1) + 4, PC = S * (WO - 1) + 4;  // window rows / cols per image
  static constexpr int NPIX = IMG * PR * PC;
  static constexpr int KSTEPS = CP / 16;
  // window position of chunk pixel k (k = il*PER_IMG' + ry*WO + rx within the chunk)
  static constexpr int wpos(int k) {
    return ((k / (R * WO)) * PR + S * ((k % (R * WO)) / WO)) * PC + S * (k % WO);
  }
};

}  // namespace

struct WH2Args {
  const float* G; long long g_gs; int ldg;
  const float* D; long long d_gs; int ldd;
  float* part; long long p_gs;   // [split][16][M][N] partials (or dW itself when nsplit == 1)
  int M, N, nsplit, nchunk;      // nchunk: chunks per group
  int g_bf16, d_bf16;            // G / D stored as bf16 (opload.h)
  int nsp;                       // 2: split-bf16 planes (fp32 G / D)
};

// NSP = 2: split-bf16 operands (dtype bf16x6's weight gradients, opload.h): the fp32 G window and D
// rows are staged as hi / lo bf16 planes (plane p of the stage at p * BUF) and every fragment pair
// runs the three plane products hi*hi + hi*lo + lo*hi
template <int WO, int CP, int KYR, int WN, int WK, bool DB, int OPB, int NSW, int PF, int S = 1, int NSP = 1>
__global__ __launch_bounds__(64 * KYR * WN * WK) void wgrad_halo2_kernel(WH2Args a) {
  static_assert(NSP == 1 || (OPB == 0 && !DB), "split planes: fp32 operands, one stage");
  using GE = Geo2<WO, CP, S>;
  constexpr int GP = GE::GP, HI = GE::HI;
  constexpr int NT = 64 * KYR * WN * WK;
  constexpr int DN = 32 * WN * NSW;               // D columns per block (NSW 32-column subtiles per wave)
  constexpr int GI = (GE::NPIX * 8 + NT - 1) / NT;  // window items (4 channels) per thread
  constexpr int DI = (CP * DN / 4 + NT - 1) / NT;   // D items per thread
  constexpr int GWB = GE::NPIX * GP;                // bf16 elements of one window buffer
  constexpr int BUF = GWB + CP * DN;                // one stage (window + D rows)
  static_assert((CP % WO) == 0 || (CP % GE::PER_IMG) == 0, "chunks are whole rows or whole images");
  static_assert(GE::KSTEPS % WK == 0, "K steps split evenly over the wave sets");
  static_assert(WO >= 8 && (WO & (WO - 1)) == 0, "power-of-two width >= 8");
  extern __shared__ __attribute__((aligned(16))) __bf16 wsm[];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int grp = lane >> 4, i16 = lane & 15, q = i16 >> 2, p4 = i16 & 3;
  const int kyw = wave % KYR, wn = (wave / KYR) % WN, wk = wave / (KYR * WN);

  const BlockXYZ blk = xcd_block();
  constexpr int NTG = 4 / KYR;                      // tap groups
  const int m0 = blk.x * 32, n0 = blk.y * DN;
  const int tg = blk.z % NTG;
  const int zs = blk.z / NTG;
  const int split = zs % a.nsplit, group = zs / a.nsplit;
  const int ky = tg * KYR + kyw;
  const long long gg0 = group * a.g_gs, dd0 = group * a.d_gs;  // element offsets (fp32 or bf16)
  constexpr bool gbf = (OPB & 1) != 0, dbf = (OPB & 2) != 0;  // G / D stored as bf16
  const int cbeg = (int)((long long)a.nchunk * split / a.nsplit);
  const int cend = (int)((long long)a.nchunk * (split + 1) / a.nsplit);

  // ---- chunk-invariant staging geometry ----
  int wrel[GI], wpr[GI];
#pragma unroll
  for (int i = 0; i < GI; ++i) {
    const int it = tid + NT * i;
    wrel[i] = 0;
    wpr[i] = -1;  // no item
    if (it < GE::NPIX * 8) {
      const int pix = it >> 3, part = it & 7;
      const int il = pix / (GE::PR * GE::PC);
      const int r2 = pix - il * GE::PR * GE::PC;
      const int pr = r2 / GE::PC, pc = r2 - pr * GE::PC;
      const int ix = pc - 1;
      wrel[i] = ((il * HI + pr) * HI + ix) * a.ldg + m0 + part * 4;
      wpr[i] = (ix >= 0 && ix < HI) ? pr : -2;  // -2: column outside the image (zero)
    }
  }

  // ---- lane-dependent LDS read bases (byte offsets within a stage) ----
  const int lk = 8 * (grp >> 1) + q;                       // this lane's pixel within a K step
  const int ch = 16 * (grp & 1) + 4 * p4;                  // this lane's G channel quad
  const int wlane = S * ((lk / WO) * GE::PC + (lk % WO));  // its window offset (additive, no carry)
  const int ga = ((wlane + ky * GE::PC) * GP + ch) * 2;    // + (wpos(k0) + kx) * GP * 2
  int da[NSW];                                              // + k0 * DN * 2
#pragma unroll
  for (int sn = 0; sn < NSW; ++sn) {
    const int slot = (wn * NSW + sn) * 8 + 4 * (grp & 1) + p4;
    const int sw = DN == 64 ? (slot ^ (((lk >> 1) & 1) << 3)) : slot;
    da[sn] = (GWB + lk * DN + sw * 4) * 2;
  }

  f32x16 acc[4][NSW];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int sn = 0; sn < NSW; ++sn)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][sn][r] = 0.f;

  // PF register sets: chunk c + PF is loaded while chunk c computes (PF = 2: two chunks of
  // compute to cover a load's latency instead of one)
  f32x4 gvs[PF][GI], dvs[PF][DI];
  auto load_chunk = [&](int c, f32x4 (&gv)[GI], f32x4 (&dv)[DI]) {
    const int row0 = c * CP;
    const int img0 = row0 / GE::PER_IMG;
    const int ry0 = (row0 - img0 * GE::PER_IMG) / WO;
    const long long gbase = ((long long)img0 * HI + S * ry0 - 1) * HI * a.ldg;
#pragma unroll
    for (int i = 0; i < GI; ++i) {
      gv[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int iy = S * ry0 - 1 + wpr[i];
      if (wpr[i] >= 0 && iy >= 0 && iy < HI) gv[i] = ld4_raw(a.G, gg0 + gbase + wrel[i], gbf);
    }
    const long long dc = dd0 + (long long)row0 * a.ldd + n0;
#pragma unroll
    for (int i = 0; i < DI; ++i) {
      const int it = tid + NT * i;
      if (it < CP * DN / 4) {
        const int k = it / (DN / 4), sl = it - k * (DN / 4);
        dv[i] = ld4_raw(a.D, dc + (long long)k * a.ldd + sl * 4, dbf);
      }
    }
  };
  // one bf16 plane (NSP = 1), or the hi / lo planes of the fp32 values (NSP = 2)
  auto put4 = [&](__bf16* st, int o, f32x4 v, bool bfs) {
    if constexpr (NSP == 1) {
      *(bf16x4*)&st[o] = raw4_bf(v, bfs);
    } else {
      ol_bf16x4 pl[NSP];
      split4<NSP>(v, pl);
#pragma unroll
      for (int p = 0; p < NSP; ++p) *(bf16x4*)&st[p * BUF + o] = pl[p];
    }
  };
  auto store_chunk = [&](__bf16* st, const f32x4 (&gv)[GI], const f32x4 (&dv)[DI]) {
#pragma unroll
    for (int i = 0; i < GI; ++i) {
      if (wpr[i] == -1) continue;
      const int it = tid + NT * i;
      put4(st, (it >> 3) * GP + (it & 7) * 4, gv[i], gbf);
    }
#pragma unroll
    for (int i = 0; i < DI; ++i) {
      const int it = tid + NT * i;
      if (it < CP * DN / 4) {
        const int k = it / (DN / 4), sl = it - k * (DN / 4);
        const int s2 = DN == 64 ? (sl ^ (((k >> 1) & 1) << 3)) : sl;
        put4(st, GWB + k * DN + s2 * 4, dv[i], dbf);
      }
    }
  };

  auto chunk_body = [&](int c, f32x4 (&gv)[GI], f32x4 (&dv)[DI]) {
    __bf16* st = DB ? wsm + ((c - cbeg) & 1) * BUF : wsm;  // DB: one barrier per chunk
    store_chunk(st, gv, dv);
    __syncthreads();
    if (c + PF < cend) load_chunk(c + PF, gv, dv);
    const char* sb = (const char*)st;
    // K steps kk = j*WK + wk: the wave set's offset wpos(16*wk) lives in gw / dw (additive for
    // every instantiated geometry), the rest is a compile-time constant of the unrolled j
    const int gw = ga + GE::wpos(16 * wk) * GP * 2;
#pragma unroll
    for (int j = 0; j < GE::KSTEPS / WK; ++j) {
      const int k0 = j * WK * 16;
      bf16x8 bfr[NSW][NSP];
#pragma unroll
      for (int sn = 0; sn < NSW; ++sn) {
        const int dw = da[sn] + 16 * wk * DN * 2;
#pragma unroll
        for (int p = 0; p < NSP; ++p)
          bfr[sn][p] = join(tr16((const __bf16*)(sb + p * BUF * 2 + dw + (k0 * DN) * 2)),
                            tr16((const __bf16*)(sb + p * BUF * 2 + dw + ((k0 + 4) * DN) * 2)));
      }
      const int w0 = GE::wpos(k0), w1 = GE::wpos(k0 + 4);
#pragma unroll
      for (int kx = 0; kx < 4; ++kx) {
        bf16x8 af[NSP];
#pragma unroll
        for (int p = 0; p < NSP; ++p)
          af[p] = join(tr16((const __bf16*)(sb + p * BUF * 2 + gw + (w0 + kx) * GP * 2)),
                       tr16((const __bf16*)(sb + p * BUF * 2 + gw + (w1 + kx) * GP * 2)));
#pragma unroll
        for (int sn = 0; sn < NSW; ++sn)  // every transposed A fragment feeds NSW MFMAs
          acc[kx][sn] = mfma_split<NSP>(af, bfr[sn], acc[kx][sn]);
      }
    }
    if constexpr (!DB) __syncthreads();  // single stage: the next store waits for every reader
  };
#pragma unroll
  for (int i = 0; i < PF; ++i)
    if (cbeg + i < cend) load_chunk(cbeg + i, gvs[i], dvs[i]);
  for (int c = cbeg; c < cend; c += PF) {
#pragma unroll
    for (int i = 0; i < PF; ++i)
      if (c + i < cend) chunk_body(c + i, gvs[i], dvs[i]);
  }

  // ---- K-interleaved wave sets: sum through LDS (fixed order: deterministic) ----
  if constexpr (WK > 1) {
    __syncthreads();
    float* red = (float*)wsm;  // [WK-1][KYR*WN][4][16][64]
    const int wl = wave % (KYR * WN);
    if (wk > 0) {
#pragma unroll
      for (int kx = 0; kx < 4; ++kx)
#pragma unroll
        for (int r = 0; r < 16; ++r) red[((((wk - 1) * KYR * WN + wl) * 4 + kx) * 16 + r) * 64 + lane] = acc[kx][0][r];
    }
    __syncthreads();
    if (wk > 0) return;
#pragma unroll
    for (int j = 1; j < WK; ++j)
#pragma unroll
      for (int kx = 0; kx < 4; ++kx)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[kx][0][r] += red[((((j - 1) * KYR * WN + wl) * 4 + kx) * 16 + r) * 64 + lane];
  }

  // ---- partial dW[tap][m][n] of this split (the gradient itself when nsplit == 1) ----
  float* out = a.part + group * a.p_gs + (long long)split * 16 * a.M * a.N;
#pragma unroll
  for (int sn = 0; sn < NSW; ++sn) {
    const int n = n0 + (wn * NSW + sn) * 32 + l32;
#pragma unroll
    for (int kx = 0; kx < 4; ++kx) {
      const int tap = ky * 4 + kx;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        out[((long long)tap * a.M + m) * a.N + n] = acc[kx][sn][r];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// planner / launcher
// ---------------------------------------------------------------------------
namespace {

template <int WO, int CP, int KYR, int WN, int WK, bool DB, int NSW, int S, int NSP = 1>
size_t wh2_lds() {
  using GE = Geo2<WO, CP, S>;
  const size_t stage = NSP * ((size_t)GE::NPIX * GE::GP + (size_t)CP * 32 * WN * NSW) * 2;
  const size_t red = WK > 1 ? (size_t)(WK - 1) * KYR * WN * 4 * 16 * 64 * 4 : 0;
  return std::max((DB ? 2 : 1) * stage, red);
}

template <int WO, int CP, int KYR, int WN, int WK, bool DB, int OPB, int NSW, int PF, int S, int NSP = 1>
void wh2_launch_op(const WH2Args& a, int groups, hipStream_t s) {
  const size_t lds = wh2_lds<WO, CP, KYR, WN, WK, DB, NSW, S, NSP>();
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)wgrad_halo2_kernel<WO, CP, KYR, WN, WK, DB, OPB, NSW, PF, S, NSP>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  dim3 grid(a.M / 32, a.N / (32 * WN * NSW), (4 / KYR) * a.nsplit * groups);
  hipLaunchKernelGGL((wgrad_halo2_kernel<WO, CP, KYR, WN, WK, DB, OPB, NSW, PF, S, NSP>), grid,
                     dim3(64 * KYR * WN * WK), lds, s, a);
}
// operand storage (G fp32/bf16 x D fp32/bf16) as a compile-time parameter: no branches in the loads
int env_int(const char* name, int dflt);
template <int WO, int CP, int KYR, int WN, int WK, bool DB, int OPB, int NSW, int S>
void wh2_launch_pf(const WH2Args& a, int groups, hipStream_t s) {
  static const int pf = env_int("SVAE_WH2_PF", 2);  // register prefetch depth in chunks (1 or 2)
  if (pf == 1) wh2_launch_op<WO, CP, KYR, WN, WK, DB, OPB, NSW, 1, S>(a, groups, s);
  else wh2_launch_op<WO, CP, KYR, WN, WK, DB, OPB, NSW, 2, S>(a, groups, s);
}
template <int WO, int CP, int KYR, int WN, int WK, bool DB, int NSW = 1, int S = 1>
void wh2_launch(const WH2Args& a, int groups, hipStream_t s) {
  if (a.nsp > 1) {  // split-bf16 planes (fp32 operands): one chunk of register prefetch
    wh2_launch_op<WO, CP, KYR, WN, WK, false, 0, NSW, 1, S, 2>(a, groups, s);
    return;
  }
  switch ((a.g_bf16 ? 1 : 0) | (a.d_bf16 ? 2 : 0)) {
    case 0: wh2_launch_pf<WO, CP, KYR, WN, WK, DB, 0, NSW, S>(a, groups, s); break;
    case 1: wh2_launch_pf<WO, CP, KYR, WN, WK, DB, 1, NSW, S>(a, groups, s); break;
    case 2: wh2_launch_pf<WO, CP, KYR, WN, WK, DB, 2, NSW, S>(a, groups, s); break;
    default: wh2_launch_pf<WO, CP, KYR, WN, WK, DB, 3, NSW, S>(a, groups, s); break;
  }
}

int env_int(const char* name, int dflt) { return svae_knob(name, dflt); }

}  // namespace

int wgrad_halo2_enabled() {
  static int v = -1;
  if (v < 0) v = env_int("SVAE_NO_WH2", 0) ? 0 : 1;
  return v;
}

// Config per layer: WN = 2 where N >= 64 (one staged G window feeds 64 D columns), else the
// 32-column tile with two K-interleaved wave sets; KYR = 4 (all 16 taps per block; the 8-tap
// variant and the double-buffered stage were measured slower in round 2 and are not built).
// Split count: ~target blocks over the machine (SVAE_WH2_TARGET, default 64: in the step the kernel
// shares the GPU with the main stream, and every halving of the splits halves the partial-slab writes
// and the reduce's reads; 128 -> 64 measured within noise, profiles/r03_ab2.txt), >= minch chunks per
// split (SVAE_WH2_MINCH, default 4), slab within capacity.
// stride 2 (SVAE_WH2_S2=0 keeps those layers on gemm_bf16.hip's generic halo weight-GEMM): 64-pixel
// chunks (the window is ~4x the chunk's pixels), row-space widths 8 and 16
static int wh2_cp(int WO, int S) { return S == 2 ? 64 : (WO == 32 ? 128 : 256); }
static int wh2_s2_enabled() {
  static const int v = env_int("SVAE_WH2_S2", 1);
  return v;
}

int wgrad_halo2_ok(const WgArgs& w) {
  const ConvGeom& g = w.g;
  if (!wgrad_halo2_enabled()) return 0;
  if (g.mode != GM_CONV || g.ksz != 4 || w.ntap != 16 || g.pad != 1) return 0;
  if (g.stride != 1 && !(g.stride == 2 && wh2_s2_enabled())) return 0;
  if (g.Ho != g.Wo || g.Hi != g.stride * g.Ho || g.Wi != g.stride * g.Wo) return 0;
  const int WO = g.Wo;
  if (g.stride == 1 ? (WO != 8 && WO != 16 && WO != 32) : (WO != 8 && WO != 16)) return 0;
  if (w.M % 32 || w.N % 32 || w.ldg % 4 || w.ldd % 4) return 0;
  return w.rows % wh2_cp(WO, g.stride) == 0;
}

int wgrad_halo2(const WgArgs& w, int groups, float* slab, long long slab_cap, float* dW, long long w_gs,
                hipStream_t s, hipEvent_t after, int target_blocks) {
  if (!wgrad_halo2_ok(w)) return 0;
  const int WO = w.g.Wo;
  const int S = w.g.stride;
  // split mode (NSP = 2, fp32 operands): 128-pixel chunks for the 8- and 16-wide layers halve the
  // staging registers (256 VGPRs + spills at 256-pixel chunks; SVAE_WH2_SPLIT_CP=256 restores them)
  static const int split_cp = env_int("SVAE_WH2_SPLIT_CP", 128);
  const bool sp128 = w.nsp > 1 && S == 1 && WO <= 16 && split_cp == 128 && w.rows % 128 == 0;
  const int cp = sp128 ? 128 : wh2_cp(WO, S);
  // split mode: 128 (its weight-GEMMs are 3x the MFMA work, so more splits spread the side stream: parity
  // mode +1.9 %, profiles/r04_knobs_ab.txt); bf16: 96 (+0.6 %, profiles/r04_knobs2_ab.txt).  SVAE_WH2_TARGET
  // overrides both
  static const int target_env = env_int("SVAE_WH2_TARGET", 0);
  const int target = target_env > 0 ? target_env : target_blocks > 0 ? target_blocks : (w.nsp > 1 ? 128 : 96);
  static const int minch = env_int("SVAE_WH2_MINCH", 4);
  // SVAE_WH2_NSW=2: a 64-column block as 4 waves of two 32-column subtiles (each transposed A
  // fragment feeds two MFMAs) instead of 8 waves of one
  static const int nsw = env_int("SVAE_WH2_NSW", 1);
  const int wn = (w.N % 64 == 0) ? 2 : 1;
  const int kyr = 4;
  WH2Args a;
  a.G = w.G; a.g_gs = w.g_gs; a.ldg = w.ldg;
  a.D = w.D; a.d_gs = w.d_gs; a.ldd = w.ldd;
  a.g_bf16 = w.g_bf16; a.d_bf16 = w.d_bf16;
  a.nsp = w.nsp > 1 ? 2 : 1;
  if (a.nsp > 1 && (a.g_bf16 || a.d_bf16)) return 0;  // split planes come from fp32 operands
  a.M = w.M; a.N = w.N;
  a.nchunk = w.rows / cp;
  const long long tiles = (long long)(w.M / 32) * (w.N / (32 * wn)) * (4 / kyr) * groups;
  long long ns = (target + tiles - 1) / tiles;
  ns = std::min<long long>(ns, std::max(1, a.nchunk / minch));
  const long long per = 16LL * w.M * w.N;
  ns = std::min<long long>(ns, std::max<long long>(1, slab_cap / (per * groups)));
  a.nsplit = (int)std::max<long long>(1, ns);
  if (a.nsplit == 1) {
    a.part = dW;
    a.p_gs = w_gs;
  } else {
    a.part = slab;
    a.p_gs = (long long)a.nsplit * per;
  }
#define WH2(WOV, CPV, KY, WNV, WKV) wh2_launch<WOV, CPV, KY, WNV, WKV, false>(a, groups, s)
#define WH2_WO(WOV, CPV)                                                            \
  if (wn == 2 && nsw == 2) { wh2_launch<WOV, CPV, 4, 1, 1, false, 2>(a, groups, s); } \
  else if (wn == 2) { WH2(WOV, CPV, 4, 2, 1); }                                     \
  else { WH2(WOV, CPV, 4, 1, 2); }
  if (sp128) {  // split planes, 128-pixel chunks
    if (WO == 16) {
      if (wn == 2) wh2_launch_op<16, 128, 4, 2, 1, false, 0, 1, 1, 1, 2>(a, groups, s);
      else wh2_launch_op<16, 128, 4, 1, 2, false, 0, 1, 1, 1, 2>(a, groups, s);
    } else {
      if (wn == 2) wh2_launch_op<8, 128, 4, 2, 1, false, 0, 1, 1, 1, 2>(a, groups, s);
      else wh2_launch_op<8, 128, 4, 1, 2, false, 0, 1, 1, 1, 2>(a, groups, s);
    }
  } else if (S == 2) {  // 64-pixel chunks: WN = 2 where N >= 64, else two K-interleaved wave sets
    if (WO == 16) {
      if (wn == 2) wh2_launch<16, 64, 4, 2, 1, false, 1, 2>(a, groups, s);
      else wh2_launch<16, 64, 4, 1, 2, false, 1, 2>(a, groups, s);
    } else {
      if (wn == 2) wh2_launch<8, 64, 4, 2, 1, false, 1, 2>(a, groups, s);
      else wh2_launch<8, 64, 4, 1, 2, false, 1, 2>(a, groups, s);
    }
  }
  else if (WO == 32) { WH2_WO(32, 128) }
  else if (WO == 16) { WH2_WO(16, 256) }
  else { WH2_WO(8, 256) }
#undef WH2_WO
#undef WH2
  if (after) hipEventRecord(after, s);
  if (a.nsplit > 1) wgrad_reduce(slab, a.p_gs, a.nsplit, 16, w.M, w.N, dW, w_gs, w.M, nullptr, 0, 0, groups, s);
  return 1;
}
