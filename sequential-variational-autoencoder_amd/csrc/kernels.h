// Host-side launch API of the Sequential-VAE HIP kernels (internal to libsvae_hip.so).
#pragma once
#include "common.h"

// Backward-BN reductions fused into the epilogue of the GEMM that produces dy (bf16 kernels):
// with dz = dy * act'(y), the epilogue emits per-row-block partials [rb][2C] = (sum dz,
// sum dz*xhat) over columns [0, C) of its final output (after accumulate) into FwdArgs::stats,
// exactly what bn_bwd_reduce would add (fixed-point accumulators, common.h stat_put).  pre == nullptr: off.
struct BwStat {
  const float* pre; int ldp; long long pre_gs;
  const float* y; int ldy; long long y_gs;      // shortcut layers: act' from the stored output
  const float* mean; const float* invstd; long long ms_gs;
  const float* beta; long long beta_gs;
  int act, C;
  int pre_bf16;                                 // pre is stored as bf16 (common.h pf_ld)
  int y_bf16;                                   // y is stored as bf16 (only its sign is used: act')
};

// Consumer-side BN(+act) of the A operand (the wave-split halo gather only): A holds the producing
// layer's pre-BN output and the gather stages a = act(bn_y(pre)) -- the expression of bn_apply, from
// the same fixed-point accumulators finalised the same way, so bitwise the applied tensor.  The block
// at tile (0, 0) of each group stores mean / invstd for the backward.
struct AinBN {
  const u64* acc; long long acc_gs, sh; int nsh;  // the producer's statistics accumulators (acc == nullptr: off)
  long long rows;                                  // rows the statistics cover
  const float* beta; long long beta_gs;
  float* mean; float* invstd; long long ms_gs;
  int act; float eps;
  int fin;                                         // mean / invstd already finalised (BnFin): read them
};

// gather-GEMM  C[p][n] (+)= act(bias + sum_{tap,k} A[src(p,tap)][k] * B[tap][k|n][n|k])
struct FwdArgs {
  const float* A; long long a_gs; int lda;
  const float* B; long long b_gs; int ldb; long long b_tap; int b_nk;
  const void* Bh;                         // bf16 NK weights (bf16 kernels only)
  float* C; long long c_gs; int ldc;
  u64* stats; long long s_gs;             // per-column fixed-point (sum,sum^2) accumulators [4*N] (common.h stat_put)
  long long s_sh; int s_nsh;              // accumulator shards: row-block rb adds into shard rb & (s_nsh-1)
  const float* bias; long long bias_gs;
  int N, Cin;
  ConvGeom g;
  int act, accumulate;
  int rows;     // rows (output pixels) per parity class
  int nclass;   // 4 for stride-2 conv-transpose, else 1
  int mtiles;   // filled by the launcher
  // split-K (bf16 path): fp32 partial slabs [ksplit][rows_total][N] + reduce/stats pass
  float* part; long long part_cap; int ksplit; int rows_total;
  BwStat bw;    // bf16 kernels: backward-BN partials instead of forward stats (bw.pre != nullptr)
  int a_bf16;   // bf16 kernels: A is stored as bf16 (element offsets / strides unchanged; opload.h)
  // split-bf16 mode (dtype = bf16x6, opload.h split8): A and B as nsp bf16 planes each (1 = plain
  // bf16); B plane p at Bh + p * b_plane elements.  Only kernels that implement it accept nsp > 1
  int nsp; long long b_plane;
  // split mode: B also holds two scaled fp16 planes (w * 2^H16_WS, opload.h) at planes 3 and 4; the
  // wave-split halo gather then runs the three-product fp16 form (halo_kw NS = 2)
  int h16;
  // the fp16 planes' per-tensor exponent (common.h h16_pair): group g's at wexp[g * wexp_gs]; nullptr: H16_WS
  const int* wexp; long long wexp_gs;
  AinBN ain;    // consumer-side BN of A (halo_kw only)
  // forward BN producers (bf16 mode): store C as bf16, the statistics taken from the rounded values;
  // only with stats, no bias / act / accumulate / bw (igemm_c_bf16_ok)
  int c_bf16;
  BnFin fin;    // last-arriver BN finalisation (common.h; halo_kw only: igemm_fin_ok)
};

// weight-GEMM  part[split][tap][m][n] = sum_{p in split} G[src(p,tap)][m] * D[p][n]
struct WgArgs {
  const float* G; long long g_gs; int ldg;
  const float* D; long long d_gs; int ldd;
  float* part; long long p_gs;
  int M, N;
  ConvGeom g;   // mode CONV or DENSE; row space = D's pixels, gathered space = G's pixels
  int rows, chunk, nsplit, ntap;
  int g_bf16, d_bf16;  // bf16 kernels: G / D stored as bf16 (opload.h)
  int nsp;             // split-bf16 planes per operand (1 = plain bf16; 2 = the 3-product fp32-class mode)
};

// weight gradient of the 64x64 -> 32x32 stride-2 4x4 layers with <= 4 image channels (wgrad_smallc.hip):
// eligibility, and the launch (splits through slab, reduced into dW); returns 0 if not eligible
int wgrad_smallc_ok(const WgArgs& w);
int wgrad_smallc(const WgArgs& w, int groups, float* slab, long long slab_cap, float* dW, long long w_gs, hipStream_t s);
int wgrad_smallc_part(const WgArgs& w, int groups, float* part, long long cap, hipStream_t s);
int igemm_fwd_bm(const FwdArgs& a);
// image-space stride-2 4x4 convs with Cin <= 4 (smallc.hip): eligibility, stats row-blocks
// (smallc_bm() output pixels each) and launch; bf = the bf16 model (B = a.Bh, operands rounded)
bool smallc_ok(const FwdArgs& a, bool bf);
int smallc_nrb(const FwdArgs& a);
int smallc_bm();
bool smallc_disabled();  // SVAE_NO_SMALLC=1
void conv_smallc(const FwdArgs& a, int groups, bool bf, hipStream_t s);
// stride-2 4x4 conv-T gathers with N <= 16 output channels (smallc.hip, bf16 operands)
bool smalln_ok(const FwdArgs& a);
void convt_smalln(const FwdArgs& a, int groups, hipStream_t s);
// bf16-MFMA variants (dtype=1): A fp32 -> bf16 in staging, B = a.Bh bf16 [tap][n][k] (ldb = k pitch)
// returns the number of stats row-blocks written to a.stats (plan: same value without launching)
// Kernel-instance ids of the bf16 GEMMs (one per template instantiation = one rocprof kernel
// name); used by the launch probe (svae_probe_*) that times every launch of one instance.
enum KernelId {
  KID_NONE = 0,
  KID_IGEMM_BF16_256x32 = 2, KID_IGEMM_BF16_256x32_SC = 3,
  KID_IGEMM_BF16_128x64 = 4, KID_IGEMM_BF16_128x64_SC = 5,
  KID_IGEMM_BF16_128x128 = 6, KID_IGEMM_BF16_128x128_SC = 7,
  KID_IGEMM_BF16_64x128 = 8, KID_IGEMM_BF16_64x128_SC = 9,
  KID_WGRAD_BF16_128x32 = 10, KID_WGRAD_BF16_128x32_SCALAR = 11,
  KID_WGRAD_BF16_128x64 = 12, KID_WGRAD_BF16_128x64_SCALAR = 13,
  KID_WGRAD_BF16_128x128 = 14, KID_WGRAD_BF16_128x128_SCALAR = 15,
  KID_HALO_256x32 = 16, KID_HALO_128x32 = 17, KID_HALO_128x64 = 18, KID_HALO_64x64 = 19,
  KID_HALO_128x128 = 20, KID_HALO_64x128 = 21,
  KID_WHALO_32_S1 = 22, KID_WHALO_32_S2 = 23, KID_WHALO_64_S1 = 24, KID_WHALO_64_S2 = 25,
  KID_WHALO2_S1 = 26,  // wgrad_halo2_kernel<...> (all instances: stride-1 halo weight-GEMM, wgrad_halo2.hip)
  KID_HALO_KW = 27,    // igemm_halo_kw_kernel<...> (all instances: small-image gather, K over waves, halo_kw.hip)
  KID_WHALO2_S2 = 28, // wgrad_halo2_kernel<..., S = 2> (stride-2 instances, separate from KID_WHALO_32_S2)
  KID_HALO_X3 = 29,    // gather_x3_kernel<...> (all instances: the split mode's fp16-plane gather, halo_x3.hip)
  KID_COUNT = 30
};
const char* kernel_name(int kid);
int igemm_bf16_kid(const FwdArgs& a);
int wgrad_bf16_kid(const WgArgs& a);
// `after` (optional) is recorded on s right after the GEMM kernel, before any split-K reduce
int igemm_bf16(FwdArgs a, int groups, hipStream_t s, hipEvent_t after = nullptr);
// path: 0 = per-tap gather kernel, 1 = halo-tile kernel (returns -1 if the shape does not
// qualify), 2 = automatic (halo when it qualifies, unless SVAE_NO_HALO=1)
int igemm_bf16_path(FwdArgs a, int groups, int path, hipStream_t s, hipEvent_t after = nullptr);
int igemm_bf16_plan(const FwdArgs& a, int groups, int* ksplit);
// small-image halo gather-GEMM with K split over the block's waves (halo_kw.hip), used where the
// tiled halo kernel would split K over the grid: stats row-blocks (0 = shape not eligible) / launch
// the split mode's fp16-plane wave-split gather (halo_x3.hip): stats row-blocks (0: not eligible) / launch (-1)
int halo_x3_plan(const FwdArgs& a, int groups);
int halo_x3(const FwdArgs& a, int groups, hipStream_t s);
int halo_kw_plan(const FwdArgs& a, int groups);
// the split-bf16 (nsp = 3) gather-GEMMs: does a launch of this shape have a split kernel (halo_kw,
// dense_kw)?  Shapes without one run the fp32 kernels (igemm_fwd) in that mode.
bool igemm_split_ok(const FwdArgs& a, int groups);
// a BN-statistics launch (a.stats set) whose kernel can store C as bf16 (FwdArgs::c_bf16)
bool igemm_c_bf16_ok(const FwdArgs& a, int groups);
// a BN-statistics launch that runs on halo_kw, whose epilogue implements FwdArgs::fin
bool igemm_fin_ok(const FwdArgs& a, int groups);
int halo_kw(const FwdArgs& a, int groups, hipStream_t s);
void wgrad_bf16(WgArgs a, int groups, hipStream_t s, hipEvent_t after = nullptr);  // taps merged into M (part [split][tap*M+m][n])
int wgrad_bf16_tiles(const WgArgs& a);
// halo weight-GEMM (csrc/gemm_bf16.hip): plan (0 = shape does not qualify) and launch.  The caller
// chooses a.nsplit over pl.h.nchunk chunks and points a.part / a.p_gs at the slab or at dW.
struct WHaloArgs {
  WgArgs w;
  int CP, lgWo, lgImgPix;  // chunk pixels, log2(Wo), log2(pixels per image within a chunk)
  int R, PR, PC, npix;      // image rows per chunk (per image), window rows/cols per image, window pixels
  int nchunk;               // chunks per group
  int ch_per_img;           // chunks per image (0 when a chunk spans several images)
  int img_per_ch;           // images per chunk (1 when chunks split an image)
};
struct WHaloPlanOut {
  WHaloArgs h;
  int bn;
  size_t lds;
  int tiles;
};
int wgrad_halo_plan(const WgArgs& a, int groups, WHaloPlanOut* out);
int wgrad_halo_enabled();
// stride-1 halo weight-GEMM with compile-time geometry (wgrad_halo2.hip): eligibility, and the
// launch (kernel + slab reduce when split); `after` is recorded right after the kernel
int wgrad_halo2_enabled();
int wgrad_halo2_ok(const WgArgs& w);
int wgrad_halo2(const WgArgs& w, int groups, float* slab, long long slab_cap, float* dW, long long w_gs,
                hipStream_t s, hipEvent_t after = nullptr, int target_blocks = 0);  // 0: the default split target
void wgrad_halo(const WHaloPlanOut& pl, const WgArgs& a, int groups, hipStream_t s, hipEvent_t after = nullptr);
// bf16 weight shadows: wn = bf16(w) for [0,n); wt = per-tap transposes listed in tiles/offs.
// nsp > 1 (split mode): plane p (at p * plane elements) holds the p-th bf16 term of opload.h split8
// wtab: the split mode's fp16-plane exponent per 64-float block (nullptr: H16_WS)
void shadow_weights(const float* w, void* wn, void* wt, long long n, const void* tiles, int ntiles, const void* offs,
                    int nsp, long long plane, hipStream_t s, const int* wtab = nullptr);
// per-tap transposed bf16 shadow of the ntiles tiles starting at `tiles` only
void shadow_t_tiles(const float* w, void* wt, const void* tiles, int ntiles, const void* offs, int nsp, long long plane,
                    hipStream_t s, const int* wtab = nullptr);
// The per-tensor exponents of the fp16 weight planes (common.h h16_wexp).  info: per GEMM weight tensor
// {offset, elements, R, Cc} (R x Cc per tap; taps = elements / (R Cc)); wtab: one exponent per 64-float
// block; ovf: the overflow flag the Adam kernels raise.
// refresh: every tensor's exponent from its max |w| (one block per tensor; clears ovf), before a full
// shadow_weights pass.  fixup: one block; when ovf is set, re-derives every exponent and rewrites the fp16
// planes of both shadows (N at wn, per-tap transposes at wt), then clears ovf -- otherwise returns at once
void wexp_refresh(const float* w, const long long* info, int ntensor, int* wtab, int* ovf, hipStream_t s);
void wexp_fixup(const float* w, const long long* info, int ntensor, int* wtab, int* ovf, void* wn, void* wt,
                long long plane, hipStream_t s);
void igemm_fwd(FwdArgs a, int groups, hipStream_t s);
void wgrad(WgArgs a, int groups, hipStream_t s);
void wgrad_reduce(const float* part, long long p_gs, int nsplit, int ntap, int M, int N, float* out0,
                  long long o0_gs, int msplit, float* out1, long long o1_gs, int accumulate, int groups,
                  hipStream_t s);

// ---- BatchNorm (training mode, beta only, eps 1e-3: abstract_network.py:22) ----
// Statistics arrive as fixed-point column accumulators acc[group][4*C] (common.h stat_put),
// added by the producing GEMM epilogue (or bn_bwd_reduce); the apply kernels finalise them.
// out = act((pre - mean)*invstd + beta [+ res]).  acc != nullptr: mean/invstd are computed from
// acc (count rows, eps) and written to mean/invstd for the backward; acc == nullptr: read them.
// Accumulators: acc[shard][group][4*C], shard stride sh words, nsh shards.
int bn_acc_shards(long long rowblocks, int cap = 16);
void bn_apply(const float* pre, int ldp, long long pre_gs, long long rows, int C, const u64* acc, long long acc_gs,
              long long sh, int nsh, float eps, float* mean, float* invstd, long long ms_gs, const float* beta, long long beta_gs,
              const float* res, int ldr, long long res_gs, int act, float* out, int ldo, long long out_gs, int groups,
              hipStream_t s, int out_bf16 = 0,   // out_bf16: write the activation as bf16 (RNE)
              int pre_bf16 = 0);                 // pre_bf16: pre is stored as bf16
// sums of dz and dz*xhat, dz = dy*act'(y)   -> added into acc[group][4*C]
// the layer's statistics finalised once (forward: mean / invstd; backward, ab != NULL: [a | b] per group and dbeta)
void bn_finalize(const u64* acc, long long acc_gs, long long sh, int nsh, long long rows, int C, float eps, float* mean,
                 float* invstd, long long ms_gs, float* ab, float* dbeta, long long dbeta_gs, int groups, hipStream_t s);
void bn_bwd_reduce(const float* dy, int lddy, long long dy_gs, const float* y, int ldy, long long y_gs,
                   const float* pre, int ldp, long long pre_gs, long long rows, int C, const float* mean,
                   const float* invstd, long long ms_gs, const float* beta, long long beta_gs, int act, u64* acc,
                   long long acc_gs, long long sh, int nsh, int groups, hipStream_t s, int pre_bf16 = 0,
                   int y_bf16 = 0);
int bn_bwd_rowblocks(long long rows);
// dpre = invstd*(dz - a - xhat*b), a = sum(dz)/n, b = sum(dz*xhat)/n from acc; dbeta = sum(dz);
// optional dres (+)= dz
void bn_bwd_apply(const float* dy, int lddy, long long dy_gs, const float* y, int ldy, long long y_gs,
                  const float* pre, int ldp, long long pre_gs, long long rows, int C, const float* mean,
                  const float* invstd, long long ms_gs, const float* beta, long long beta_gs, const u64* acc,
                  long long acc_gs, long long sh, int nsh, float* dbeta, long long dbeta_gs, int act, float* dpre, int lddp,
                  long long dpre_gs, float* dres, int ldres, long long dres_gs, int res_acc, int groups,
                  hipStream_t s, int dpre_bf16 = 0,  // dpre_bf16: write dpre as bf16 (RNE)
                  int pre_bf16 = 0,
                  const float* ab = nullptr,   // a, b finalised by the producer (BnFin mode 1): [group][2C]
                  int y_bf16 = 0);             // y stored as bf16 (act' needs its sign only)

// ---- split_latent FC(K=Dl) + BN over batch + lrelu, fused (sequential_vae.py:1801-1806) ----
// out[n][j] written at out + n*o_n + (j / F)*ldo + (j % F)
void splitfc_fwd(const float* z, int ldz, int zoff, int B, int K, const float* W, const float* beta, int J,
                 float* mean, float* invstd, float* out, long long o_n, int F, int ldo, hipStream_t s,
                 int out_bf16 = 0);  // out_bf16: the concat buffer is stored as bf16 (offsets in bf16 elements)
// one level for up to SFC_MAXT chain steps (grid.y = step; z_t at z + t * z_ts): per-step weights, beta,
// statistics and output (o_n per step: the top concat's row pitch differs at t = 0)
#define SFC_MAXT 16
struct SfcSteps {
  const float* W[SFC_MAXT];
  const float* beta[SFC_MAXT];
  float* mean[SFC_MAXT];
  float* invstd[SFC_MAXT];
  float* out[SFC_MAXT];
  long long o_n[SFC_MAXT];
};
void splitfc_fwd_steps(const float* z, long long z_ts, int ldz, int zoff, int B, int K, int J, int F, int ldo,
                       int out_bf16, const SfcSteps& a, int nt, hipStream_t s);
// writes dW [K][J], dbeta [J] and dz_part [splitfc_blocks(J)][B][K]
void splitfc_bwd(const float* z, int ldz, int zoff, int B, int K, const float* W, const float* beta, int J,
                 const float* mean, const float* invstd, const float* dout, long long o_n, int F, int ldo, float* dW,
                 float* dbeta, float* dz_part, hipStream_t s);
// dz[n][zoff+d] += sum over blocks of dz_part
void splitfc_dz_reduce(const float* dz_part, int nblk, int B, int K, float* dz, int ldz, int zoff, hipStream_t s);
int splitfc_blocks(int J);

// ---- recognition heads: [mean|std] = ladder @ [Wm|Ws] (sequential_vae.py:1592-1594,1607-1609) ----
int heads_splits(int K);
// part[split][n][coff+o] (mean) and part[split][n][pcols/2+coff+o] (std)
void heads_fwd(const float* X, long long x_gs, int B, int K, const float* Wm, const float* Ws, long long w_gs, int D,
               float* part, long long part_gs, int pcols, int coff, int groups, hipStream_t s);
struct LatentLvls {
  const float* bm[8];
  const float* bs[8];
  int off[8];
  int dim[8];
  int L;
};
// mu_raw = sum part + bm, sig = sigmoid(sum part + bs), z = clip(mu) + sig*eps, kl_img per image
void latent_fwd(const float* part, long long part_gs, int nsplit, int B, int Dz, const LatentLvls& lv,
                long long bias_gs, float clipv, float prior, int uniform, const float* eps, long long eps_gs, float* mu,
                float* sig, float* z, long long ms_gs, float* kl_img, long long kl_gs, int groups, hipStream_t s);
// dhead[n][0:Dz] = d mu_raw, dhead[n][Dz:2Dz] = d sig_pre; kl_coef (device) = reg*c_first/B
void latent_bwd(const float* mu, const float* sig, const float* eps, const float* dz, long long gs, long long eps_gs,
                int B, int Dz, const float* kl_coef, long long kc_gs, float prior, int uniform, float clipv, float* dhead,
                long long dh_gs, int groups, hipStream_t s);
// dX (+)= dhead_l @ [Wm|Ws]^T ; dW = X^T dhead_l ; db = sum_n dhead_l   (w_gs: group stride of W/dW/db)
void heads_bwd(const float* X, long long x_gs, float* dX, long long dx_gs, int B, int K, const float* Wm,
               const float* Ws, long long w_gs, int D, const float* dhead, long long dh_gs, int dcols, int coff,
               float* dWm, float* dWs, float* dbm, float* dbs, int accumulate, int groups, hipStream_t s);

// ---- small-N gather conv (N <= 4: output conv-T 32->3(+1), encoder layer-0 dgrad) ----
// C[p][o] (+)= bias + sum_tap sum_k A[src(p,tap)][k] * W(tap,o,k); W0 [tap][n0][K], W1 [tap][n1][K]
void gconv_smalln(const float* A, int lda, int K, const float* W0, int n0, const float* W1, int n1, long long w_tap,
                  long long w1_tap, const float* bias0, const float* bias1, ConvGeom g, long long rows_total,
                  float* C, int ldc, int accumulate, hipStream_t s);

// ---- output layer + highway + reconstruction (sequential_vae.py:1720-1729, :1146) ----
int output_blocks_per_img(int HW);
// packed output / ratio conv-T weights and bias of up to PACK_MAXT chain steps (misc.hip)
#define PACK_MAXT 16
struct PackOutArgs {
  const float* P;                       // flat fp32 parameters
  long long owout[PACK_MAXT], obout[PACK_MAXT];
  long long owratio[PACK_MAXT], obratio[PACK_MAXT];  // -1: no ratio layer (step 0)
  float* wpack[PACK_MAXT];
  __bf16* wpack_h[PACK_MAXT];           // nullptr in fp32 mode
  int C, F1;
  int nsp;                              // bf16 planes (3 in the split mode, 16 (C+1) F1 apart)
};
void pack_out(const PackOutArgs& a, int nt, hipStream_t s);
void output_fwd(const float* a, int B, int HW, int C, const float* xprev, const float* target, float lo, float hi,
                float minh, float maxh, float* xhat, float* rec_part, int nblk, hipStream_t s);
void output_bwd(const float* a, int B, int HW, int C, const float* xprev, const float* xhat, const float* target,
                float lo, float hi, float minh, float maxh, float rec_coef, const float* dxhat_in, float* da,
                float* dxprev, hipStream_t s);
// per-step loss reduction: stats_out[0]=mean recon, [1]=mean kl; rec_img_out[b]
void loss_reduce(const float* rec_part, int nblk, const float* kl_img, int B, int HWC, float* stats_out,
                 float* rec_img_out, hipStream_t s);

// ---- optimizer: clip(+-c) + TF Adam (sequential_vae.py:1267-1276) ----
// clip + TF Adam on n elements; wn != nullptr: also the bf16 copy of the updated weights (nsp planes
// of the split mode at wn + p * plane)
// wtab / ovf (split mode): the fp16 planes' exponent per 64-float block of the parameter buffer (element i of
// this range is element wbase + i there) and the overflow flag
void adam_step(float* w, const float* g, float* m, float* v, void* wn, long long n, float lr_t, float b1, float b2,
               float eps, float clipv, int nsp, long long plane, hipStream_t s, const int* wtab = nullptr,
               long long wbase = 0, int* ovf = nullptr);

// ---- weight sharing (homogeneous chain): virtual per-step copies <-> public tensors ----
// Pv[v + i] = P[p + i] for every segment {v, p, size} of seg[nseg][3]
void share_broadcast(const float* P, float* Pv, const long long* seg, int nseg, hipStream_t s);
// G[p + i] = sum_{k < n} Gv[cp[first + k] + i]  (fixed order) for every {p, size, first, n} of tab[ntab][4]
void share_gather(const float* Gv, float* G, const long long* tab, const long long* cp, int ntab, hipStream_t s);

// ---- misc ----
// dst[0..n) = vals[0..n) (n <= 64), values passed by value in the kernel arguments
void set_small(float* dst, const float* vals, int n, hipStream_t s);
// dense (FC) bf16 GEMM with K over the block's waves (dense_kw.hip)
bool dense_kw_ok(const FwdArgs& a, int groups);
int dense_kw_nrb(const FwdArgs& a);
int dense_kw_ks(const FwdArgs& a);
int dense_kw_rpb(const FwdArgs& a);                    // rows per splitk_reduce block                     // grid K splits (> 1: raw slabs for splitk_reduce)
int dense_kw(const FwdArgs& a, int ks, hipStream_t s);  // returns ks
void bf16_to_f32(const void* src, float* dst, long long n, hipStream_t s);  // debug copies of bf16 activations
void fill_f32(float* p, long long n, float v, hipStream_t s);
void philox_normal(float* out, long long n, unsigned long long seed, unsigned long long offset, hipStream_t s);
// column sums of X [rows][C<=4] -> out0[0..n0), out1[0..C-n0)   (part: scratch >= 1024 floats)
void colsum_small(const float* X, int ld, long long rows, int C, float* part, float* out0, int n0, float* out1,
                  hipStream_t s);

// ---- chain variants (chain.hip): chain noise, predicted-stddev network + NLL, improvement loss ----
// stddev network layers: 4x4 stride-1 TF-SAME conv, <= 8 channels, fp32 direct convolution.
// in_sig: the input is sigmoid(in) (layer 0 reads the output conv-T pre-activation, ld = C+1).
int sd_pixel_blocks(long long P);
int sd_wgrad_blocks(int B, int H);
void sd_conv_fwd(const float* in, int ldi, int in_sig, int Ci, const float* W, int Co, int H, int Wd, long long P,
                 float* pre, double* part, hipStream_t s);
// mode 0: mean / invstd of the (sum, sum^2) partials; mode 1: sums[2c..2c+1] (and dbeta[c] = sum)
void sd_stat_fin(const double* part, int nblk, int Co, long long n, float eps, int mode, float* mean, float* invstd,
                 float* sums, float* dbeta, hipStream_t s);
void sd_bn_apply(const float* pre, int Co, long long P, const float* mean, const float* invstd, const float* beta,
                 float* act, hipStream_t s);
void sd_bn_bwd_reduce(const float* dact, const float* pre, int Co, long long P, const float* mean, const float* invstd,
                      const float* beta, double* part, hipStream_t s);
void sd_bn_bwd_apply(const float* dact, const float* pre, int Co, long long P, const float* mean, const float* invstd,
                     const float* beta, const float* sums, float* dpre, hipStream_t s);
// mode 0: din = dgrad; mode 1: da[q*ldd+ci] += dgrad * s(1-s), s = sigmoid(src[q*lds+ci])
void sd_conv_dgrad(const float* dpre, int Co, const float* W, int Ci, int H, int Wd, long long P, float* din, int ldd,
                   const float* src, int lds, int mode, hipStream_t s);
// dW [4,4,Ci,Co] (part: scratch of sd_wgrad_blocks(B,H) * 16*Ci*Co floats)
void sd_conv_wgrad(const float* in, int ldi, int in_sig, int Ci, const float* dpre, int Co, int B, int H, int Wd,
                   float* part, float* dW, hipStream_t s);
void sd_head_fwd(const float* act, int Ci, const float* W5, const float* b5, float smax, const float* mle,
                 const float* target, const float* noise, float reg, int B, int C, int HW, float* sd, float* sample,
                 float* rec_part, int nblk, hipStream_t s);
void sd_head_bwd(const float* act, int Ci, const float* W5, const float* b5, float smax, const float* mle,
                 const float* target, const float* noise, float reg, float nll_coef, const float* dsample, int C,
                 long long P, float* dmle, float* dact, float* part, float* dW5, float* db5, hipStream_t s);
// sample = mle + scale * noise
void chain_noise(const float* mle, const float* noise, float scale, long long n, float* sample, hipStream_t s);
// improvement-loss seed: out = dxin + 2 coef ((x - xp) - (xn - x)) (null xp / xn / dxin: term absent)
void imp_seed(const float* dxin, const float* xp, const float* x, const float* xn, float coef, long long n, float* out,
              hipStream_t s);
// out[b] = ||a_b - b_b||^2 per image
void sqdiff_img(const float* a, const float* b, int B, long long per_img, float* out, hipStream_t s);
