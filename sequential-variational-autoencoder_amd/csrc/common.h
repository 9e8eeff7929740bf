// Shared device/host definitions for the Sequential-VAE HIP engine (gfx950 / CDNA4).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// The split mode's scaled fp16 weight planes (opload.h split8_h16 / mfma_h16): planes 3 and 4 of the
// bf16 weight shadows hold h0 = fp16(w * 2^e), h1 = fp16(w * 2^e - h0) with a per-tensor exponent e
// (the engine's exponent table, one entry per 64-float block of the parameter buffer: every tensor
// starts on a 64-float boundary).  e puts the tensor's max |w| in [2^H16_WTOP, 2^(H16_WTOP + 1)): 22-23
// significant bits for every weight down to 2^-(H16_WTOP + 3) of that maximum, and 2^(15 - H16_WTOP)x of
// headroom below fp16's largest finite value for the weights to grow before the planes are re-made
// (svae_* Adam flags a weight past 2^15 in its tensor's units; the next forward re-derives the exponent
// and the planes of every tensor before any GEMM reads them).  H16_WS: the exponent of shadows made
// without a table (operator-level test entry points, the knob-only packed output weights).
#define H16_WS 10
#define H16_WTOP 10
#define H16_WOVF 32768.f
#define H16_PLANE 3
__device__ __forceinline__ void h16_pair(float w, int e, _Float16& h0, _Float16& h1) {
  const float s = w * __uint_as_float((unsigned)(e + 127) << 23);  // (exact power of two; |e| <= 126)
  h0 = (_Float16)s;
  h1 = (_Float16)(s - (float)h0);
}
// An exponent-table entry: the exponent in the low 16 bits (signed); bit 16 set where the tensor's three bf16
// planes are read too (split mode: only the small-N conv-T of the image-channel convs' input gradients reads
// them; every other GEMM there takes the fp16 pair, so the shadow and Adam kernels skip the bf16 planes of
// the rest -- 6 bytes per weight and layout)
#define WTAB_BF16 (1 << 16)
__host__ __device__ __forceinline__ int wtab_exp(int v) { return (int)(short)(v & 0xffff); }
__host__ __device__ __forceinline__ bool wtab_bf16(int v) { return (v & WTAB_BF16) != 0; }

// the exponent for a tensor whose max |w| is wmax (0 or non-finite: H16_WS)
__host__ __device__ __forceinline__ int h16_wexp(float wmax) {
  if (!(wmax > 0.f) || !(wmax < 3.0e38f)) return H16_WS;
  int ex = 0;
  frexpf(wmax, &ex);  // wmax = f * 2^ex, f in [0.5, 1): max * 2^(H16_WTOP + 1 - ex) in [2^H16_WTOP, 2^(H16_WTOP + 1))
  const int e = H16_WTOP + 1 - ex;
  return e < -100 ? -100 : (e > 100 ? 100 : e);
}

#define SVAE_WAVE 64

enum SvaeAct { ACT_NONE = 0, ACT_RELU = 1, ACT_LRELU = 2, ACT_SIGMOID = 3 };

// Gather modes of the implicit-GEMM kernels (see DESIGN.md "conv as gather-GEMM").
//  DENSE : row p reads A[p]                      (fully connected layers)
//  CONV  : iy = oy*s - pad + ky                   (TF SAME conv2d, conv-T dgrad)
//  CONVT : oy + pad = iy*s + ky                   (TF SAME conv2d_transpose, conv dgrad);
//          stride 2 is split into 4 output-parity classes with 2x2 taps each.
enum GatherMode { GM_DENSE = 0, GM_CONV = 1, GM_CONVT = 2 };

// Division by a launch-constant d via multiply-shift (exact for 0 <= n < 2^31):
// q = (n * m) >> s with s = 31 + ceil(log2 d), m = ceil(2^s / d).
struct FastDiv {
  unsigned long long m;
  int s;
  int d;
};
static inline FastDiv make_fastdiv(int d) {
  FastDiv f;
  if (d < 1) d = 1;  // dense (FC) launches carry no spatial dims
  int l = 0;
  while ((1LL << l) < d) ++l;
  f.s = 31 + l;
  f.m = (((unsigned long long)1 << f.s) + (unsigned long long)d - 1) / (unsigned long long)d;
  f.d = d;
  return f;
}
__device__ __forceinline__ int fdiv(int n, const FastDiv& f) {
  return (int)(((unsigned long long)(unsigned)n * f.m) >> f.s);
}

struct ConvGeom {
  int mode;
  int nimg;
  int Hi, Wi;   // spatial dims of the gathered operand
  int Ho, Wo;   // spatial dims of the row space (output pixels)
  int stride, pad, ksz;
  FastDiv dHW, dW;  // row-space divisors Ho*Wo and Wo (filled by the weight-GEMM launchers)
};

__device__ __forceinline__ float lrelu_f(float x) { return fmaxf(fminf(0.1f * x, 0.f), x); }
__device__ __forceinline__ float sigmoid_f(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ float act_f(float x, int act) {
  if (act == ACT_RELU) return fmaxf(x, 0.f);
  if (act == ACT_LRELU) return lrelu_f(x);
  if (act == ACT_SIGMOID) return sigmoid_f(x);
  return x;
}
// derivative of relu/lrelu expressed through the activation OUTPUT y (y>0 <=> pre>0);
// TF tie rules: relu'(0)=0, lrelu'(0)=0.1 (abstract_network.py:8-10).
__device__ __forceinline__ float dact_from_y(float y, int act) {
  if (act == ACT_RELU) return y > 0.f ? 1.f : 0.f;
  if (act == ACT_LRELU) return y > 0.f ? 1.f : 0.1f;
  return 1.f;
}

// XCD-aware block order (cdna_hip_programming.md T1, bijective form): workgroups are dealt
// round-robin over the 8 XCDs, so linear id b runs on XCD-group b % 8.  Remap so that each
// XCD-group owns a contiguous range of logical tiles (x fastest, then y, then z): neighbouring
// tiles, which share operand panels, then share one L2.  Speed only, never correctness.
struct BlockXYZ {
  int x, y, z;
};
__device__ __forceinline__ BlockXYZ xcd_block() {
  const int X = gridDim.x, Y = gridDim.y;
  const int nwg = X * Y * gridDim.z;
  const int orig = blockIdx.x + X * (blockIdx.y + Y * blockIdx.z);
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  const int id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  BlockXYZ b;
  b.x = id % X;
  b.y = (id / X) % Y;
  b.z = id / (X * Y);
  return b;
}

// BN output before the activation, (x - mean) * invstd + beta as one explicit fma: the forward
// apply, the backward kernels and the fused GEMM epilogues all evaluate exactly this, so the
// act'(y) sign recomputed in the backward is bitwise the forward's (TF tie rules at kinks)
__device__ __forceinline__ float bn_y1(float x, float m, float is, float b) { return fmaf(x - m, is, b); }

// the fused backward-BN epilogue term for one element of the final dy (see BwStat)
__device__ __forceinline__ void bw_term(float v, float pre, float m, float is, float b, const float* y, int act,
                                        float& sd, float& sx) {
  const float yv = y ? *y : bn_y1(pre, m, is, b);
  const float dz = v * dact_from_y(yv, act);
  sd += dz;
  sx += dz * ((pre - m) * is);
}

// the same with y already loaded (has_y) or recomputed from pre
__device__ __forceinline__ void bw_term_v(float v, float pre, float m, float is, float b, bool has_y, float y, int act,
                                          float& sd, float& sx) {
  const float yv = has_y ? y : bn_y1(pre, m, is, b);
  const float dz = v * dact_from_y(yv, act);
  sd += dz;
  sx += dz * ((pre - m) * is);
}

// ---- deterministic BN statistics ----
// Every producer block adds its fp32 partial (sum, sum^2) of a column into a per-column
// fixed-point accumulator with integer atomics.  Integer adds commute, so the total does not
// depend on block order (bit-deterministic), and no finalize pass over per-block partials is
// needed: the consumer reads the C totals directly.  Value v is held as v * 2^48 split into two
// int64 words, hi = floor(v * 2^16) and lo = frac(v * 2^16) * 2^32 (resolution 2^-48 ~ 3.6e-15
// absolute; |v| < 2^47 / blocks).  Layout per group: acc[4c + {0,1}] = sum, acc[4c + {2,3}] = sum^2.
// Same-line atomics serialise, so producers spread over nsh (power of 2) shards by row-block
// (shard = rb & (nsh-1), shard stride sh words); the consumer adds the shards as integers.
typedef unsigned long long u64;

// Output stores of the main-stream kernels.  SVAE_WT=1 builds store them write-through (sc1): the
// kernel then leaves no dirty L2 lines for its end-of-kernel release to write back before the next
// dependent launch may start (MI355X_MICROARCH.md, "boundary": + dirty bytes / 6 TB/s per boundary).
#ifndef SVAE_WT
#define SVAE_WT 0
#endif
typedef int i32x4_st __attribute__((ext_vector_type(4)));
// SVAE_WT bits: 1 = the 16-byte stores (st_out16), 2 = the 8-byte ones (st_out8), 4 = the 4-byte ones
// (st_out): a 16-byte write-through store costs what a plain one does, an 8-byte one 2.7x and a
// 4-byte one ~6x per byte (MI355X_MICROARCH.md, stores of each flavour)
__device__ __forceinline__ void st_out(float* p, float v) {
#if SVAE_WT & 4
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
  *p = v;
#endif
}
__device__ __forceinline__ void st_out8(void* p, u64 v) {
#if SVAE_WT & 2
  __hip_atomic_store((u64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
  *(u64*)p = v;
#endif
}
// 16-byte store at element offset `off` of a wave-uniform base (buffer descriptor from the base)
__device__ __forceinline__ void st_out16(float* base, long long off, f32x4 v) {
#if SVAE_WT & 1
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4_st, v), r, (int)(off * 4), 0, 16);
#else
  *(f32x4*)(base + off) = v;
#endif
}
// Pre-BN conv outputs stored as bf16 (bf16 mode, DESIGN §5 "bf16 pre"): the producing epilogue rounds
// the fp32 sum (RNE) before it takes the BN statistics and stores 2 bytes; every reader widens.  Offsets
// and strides stay in elements of the storage type (a bf16 tensor's group g starts g * gs bf16 elements in)
typedef __bf16 pf_bf16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float bf_rnd(float v) { return (float)(__bf16)v; }
__device__ __forceinline__ const float* pf_at(const float* p, long long off, bool bf) {
  return bf ? (const float*)((const __bf16*)p + off) : p + off;
}
__device__ __forceinline__ float pf_ld(const float* p, long long i, bool bf) {
  return bf ? (float)((const __bf16*)p)[i] : p[i];
}
__device__ __forceinline__ f32x4 pf_ld4(const float* p, long long i, bool bf) {  // i % 4 == 0
  if (bf) return __builtin_convertvector(*(const pf_bf16x4*)((const __bf16*)p + i), f32x4);
  return *(const f32x4*)(p + i);
}
__device__ __forceinline__ void fx_add(u64* p, float v) {
  const double d = (double)v * 65536.0;  // exact
  const double fl = floor(d);
  atomicAdd(p, (u64)(long long)fl);
  atomicAdd(p + 1, (u64)((d - fl) * 4294967296.0));
}
__device__ __forceinline__ double fx_get(const u64* p) {
  return (double)(long long)p[0] * (1.0 / 65536.0) + (double)p[1] * (1.0 / 281474976710656.0);
}
__device__ __forceinline__ void stat_put(u64* acc, int c, float s, float q) {
  fx_add(acc + 4 * c, s);
  fx_add(acc + 4 * c + 2, q);
}

// Last-arriver finalisation of forward BN statistics (FwdArgs::fin): after a producer block has added its
// column partials (stat_put), it counts itself in on the group's arrival counter; the block that arrives
// last -- every other block's atomics are then complete -- sums the accumulator shards of all C columns as
// integers and writes mean / invstd with bn_apply's own fp64 expression (bitwise what bn_apply would
// compute), so the apply pass reads two floats per channel instead of gathering nsh x 4 words per channel
// in every block (that gather, served from the memory side since the atomics bypass the XCD L2s, cost
// 2.5 % of the bf16 step and 7 % of the bf16x6 step: SVAE_DBG_SKIP=16 probe)
struct BnFin {
  u64* cnt;            // arrival counters [group] (zeroed with the accumulators once per pass); nullptr: off
  int nblk;            // producer blocks (tiles) per group: set by the launcher
  const u64* acc; long long acc_gs, sh; int nsh;
  int C;
  long long rows; float eps;
  float* mean; float* invstd; long long ms_gs;  // mode 1: a = mean(dz) into mean, b = mean(dz * xhat) into invstd
  int mode;            // 0: forward (mean, invstd); 1: backward sums (a, b, and dbeta = sum dz)
  float* dbeta; long long dbeta_gs;
};
// Ordering without agent-scope fences: those write back the whole XCD L2 on gfx950 (buffer_wbl2), per block
// -- 2.3x the step.  The statistics and the counter are device-scope atomics, performed where every XCD
// sees them; a thread waits for its own statistics atomics to be acknowledged (s_waitcnt) before the
// block counts itself in, and the last block reads the accumulators with device-scope atomic loads.
__device__ __forceinline__ void bn_fin_arrive(const BnFin& f, int group, int* flag) {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0);  // this thread's stat_put atomics are performed
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __syncthreads();
  if (threadIdx.x == 0) {
    const u64 prev = __hip_atomic_fetch_add(f.cnt + group, 1ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = prev == (u64)(f.nblk - 1) ? 1 : 0;
  }
  __syncthreads();
  const int last = *flag;
  __syncthreads();  // (flag may live in a region the caller reuses)
  if (!last) return;
  const u64* acc = f.acc + group * f.acc_gs;
  for (int c = threadIdx.x; c < f.C; c += blockDim.x) {
    u64 t[4] = {0, 0, 0, 0};
    for (int k = 0; k < f.nsh; ++k)
#pragma unroll
      for (int w = 0; w < 4; ++w)
        t[w] += __hip_atomic_load(acc + k * f.sh + 4LL * c + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const double cnt = (double)f.rows;
    if (f.mode == 1) {  // bn_bwd_apply's expressions
      const double sd = fx_get(t), sx = fx_get(t + 2);
      f.mean[group * f.ms_gs + c] = (float)(sd / cnt);
      f.invstd[group * f.ms_gs + c] = (float)(sx / cnt);
      if (f.dbeta) f.dbeta[group * f.dbeta_gs + c] = (float)sd;
      continue;
    }
    const double md = fx_get(t) / cnt;
    double var = fx_get(t + 2) / cnt - md * md;
    if (var < 0.0) var = 0.0;
    f.mean[group * f.ms_gs + c] = (float)md;
    f.invstd[group * f.ms_gs + c] = (float)(1.0 / sqrt(var + (double)f.eps));
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
