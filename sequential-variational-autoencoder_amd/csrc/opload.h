// Operand loads of the bf16-MFMA GEMM kernels from fp32 OR bf16 tensors.
//
// In bf16 mode the BN-backward outputs (the gradients at the BN inputs, "dpre") are stored as
// bf16: their only consumers are the input-gradient and weight-gradient GEMMs, which round their
// operands to bf16 while staging them into LDS anyway, so storing them rounded (RNE, the same
// conversion) changes no result bit and halves the bytes written and re-read.
//
// The kernels keep their fp32 register staging and defer the conversion to the LDS store (so the
// load latency stays hidden behind the MFMAs); for a bf16 source the same registers carry the
// raw bf16 bits and the store passes them through.  `bf` is uniform per launch.
#pragma once
#include "common.h"

typedef __bf16 ol_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 ol_bf16x4 __attribute__((ext_vector_type(4)));
typedef float ol_f32x8 __attribute__((ext_vector_type(8)));
typedef float ol_f32x2 __attribute__((ext_vector_type(2)));

// 8 consecutive elements at element offset `off`: fp32 -> (lo, hi); bf16 -> lo holds the 16 bytes
__device__ __forceinline__ void ld8_raw(const void* base, long long off, bool bf, f32x4& lo, f32x4& hi) {
  if (bf) {
    lo = *(const f32x4*)((const __bf16*)base + off);
  } else {
    const float* p = (const float*)base + off;
    lo = *(const f32x4*)p;
    hi = *(const f32x4*)(p + 4);
  }
}
__device__ __forceinline__ ol_bf16x8 raw8_bf(f32x4 lo, f32x4 hi, bool bf) {
  if (bf) return __builtin_bit_cast(ol_bf16x8, lo);
  const ol_f32x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_convertvector(v, ol_bf16x8);
}
// 4 consecutive elements: fp32 -> v; bf16 -> the 8 bytes in v[0], v[1]
__device__ __forceinline__ f32x4 ld4_raw(const void* base, long long off, bool bf) {
  if (bf) {
    const ol_f32x2 t = *(const ol_f32x2*)((const __bf16*)base + off);
    return f32x4{t[0], t[1], 0.f, 0.f};
  }
  return *(const f32x4*)((const float*)base + off);
}
__device__ __forceinline__ ol_bf16x4 raw4_bf(f32x4 v, bool bf) {
  if (bf) {
    const ol_f32x2 t = {v[0], v[1]};
    return __builtin_bit_cast(ol_bf16x4, t);
  }
  return __builtin_convertvector(v, ol_bf16x4);
}
// element e of a raw 4-vector as fp32 (exact for a bf16 source)
__device__ __forceinline__ float raw4_elem(f32x4 v, int e, bool bf) {
  if (!bf) return v[e];
  const unsigned u = __float_as_uint(v[e >> 1]);
  return __uint_as_float((e & 1) ? (u & 0xFFFF0000u) : (u << 16));
}
__device__ __forceinline__ float ld1(const void* base, long long off, bool bf) {
  return bf ? (float)((const __bf16*)base)[off] : ((const float*)base)[off];
}

// ---- split-bf16 operands (dtype = bf16x6: the fp32-accurate mode on bf16 MFMA) ----
// x = p0 + p1 + p2 + r with p0 = bf16(x), p1 = bf16(x - p0), p2 = bf16(x - p0 - p1) (RNE each; every
// residual is exact in fp32), |r| <= 2^-27 |x| roughly.  A product a*b is then summed from the
// plane products down to order 2^-18 |ab|:
//   NS = 2:  a0 b0 + a0 b1 + a1 b0                         (3 MFMAs, ~2^-17 relative per product)
//   NS = 3:  a0 b0 + a0 b1 + a1 b0 + a0 b2 + a2 b0 + a1 b1  (6 MFMAs, below fp32 rounding)
// with fp32 accumulation, so a split GEMM is an fp32 GEMM to within fp32 summation error.
// In value pairs: one v_cvt_pk_bf16_f32 rounds a pair, the pair widens back with a shift and a mask, and the
// residuals are packed fp32 subtractions (v_pk_add_f32): 38 VALU per 8 values at NS = 3 where the
// vector form compiled to 62 (a single-value conversion and a shift per element to widen).  The same
// roundings and exact residuals: bitwise the same planes.
typedef __bf16 ol_bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned int ol_u32x4 __attribute__((ext_vector_type(4)));
template <int NS>
__device__ __forceinline__ void split8(f32x4 lo, f32x4 hi, ol_bf16x8 (&p)[NS]) {
  ol_f32x2 v[4] = {{lo[0], lo[1]}, {lo[2], lo[3]}, {hi[0], hi[1]}, {hi[2], hi[3]}};
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    ol_u32x4 w;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const unsigned b = __builtin_bit_cast(unsigned, __builtin_convertvector(v[j], ol_bf16x2));
      w[j] = b;
      if (s + 1 < NS) {
        const ol_f32x2 r = {__uint_as_float(b << 16), __uint_as_float(b & 0xffff0000u)};
        v[j] = v[j] - r;
      }
    }
    p[s] = __builtin_bit_cast(ol_bf16x8, w);
  }
}
template <int NS>
__device__ __forceinline__ void split4(f32x4 x, ol_bf16x4 (&p)[NS]) {
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    p[s] = __builtin_convertvector(x, ol_bf16x4);
    if (s + 1 < NS) x = x - __builtin_convertvector(p[s], f32x4);
  }
}
template <int NS>
__device__ __forceinline__ f32x16 mfma_split(const ol_bf16x8 (&a)[NS], const ol_bf16x8 (&b)[NS], f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
  if constexpr (NS >= 2) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
  }
  if constexpr (NS >= 3) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
  }
  return acc;
}

// ---- scaled fp16 hi/lo operands (the split mode's gathers, halo_kw NS = 2) ----
// x' = x * 2^s (exact), h0 = fp16(x'), h1 = fp16(x' - h0) (the residual is exact in fp32): 22-23 bits of
// x for |x'| >= 2^-3, an absolute error <= 2^-25 * 2^-s below (subnormal h1).  A product is summed as
// a0 b0 + a0 b1 + a1 b0 (3 fp16 MFMAs: each fp16 x fp16 product is exact in fp32; the dropped a1 b1 is
// <= 2^-22 |ab|), fp32 accumulation.  Activations take a block-wide running exponent per window chunk
// (max |x| * 2^s in [2^14, 2^15)), weights the fixed H16_WS below.  CPU emulation of the whole CelebA
// T=8 step: x_hat_t error vs float64 below the fp32 twin's at every t.
typedef _Float16 ol_f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 ol_f16x4 __attribute__((ext_vector_type(4)));
// (x * 2^s as a multiply by the exact power of two -- packed v_pk_mul_f32, correctly rounded like ldexp;
// h16_exp keeps s within the normal exponent range)
__device__ __forceinline__ void split8_h16(f32x4 lo, f32x4 hi, int s, ol_bf16x8 (&p)[2]) {
  const float sc = __uint_as_float((unsigned)(s + 127) << 23);
  ol_f32x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  v *= sc;
  const ol_f16x8 h0 = __builtin_convertvector(v, ol_f16x8);
  v = v - __builtin_convertvector(h0, ol_f32x8);
  const ol_f16x8 h1 = __builtin_convertvector(v, ol_f16x8);
  p[0] = __builtin_bit_cast(ol_bf16x8, h0);
  p[1] = __builtin_bit_cast(ol_bf16x8, h1);
}
__device__ __forceinline__ void split4_h16(f32x4 x, int s, ol_f16x4 (&p)[2]) {
  const f32x4 v = {__builtin_ldexpf(x[0], s), __builtin_ldexpf(x[1], s), __builtin_ldexpf(x[2], s),
                   __builtin_ldexpf(x[3], s)};
  p[0] = __builtin_convertvector(v, ol_f16x4);
  p[1] = __builtin_convertvector(v - __builtin_convertvector(p[0], f32x4), ol_f16x4);
}
__device__ __forceinline__ f32x16 mfma_h16(const ol_bf16x8 (&a)[2], const ol_bf16x8 (&b)[2], f32x16 acc) {
  const ol_f16x8 a0 = __builtin_bit_cast(ol_f16x8, a[0]), a1 = __builtin_bit_cast(ol_f16x8, a[1]);
  const ol_f16x8 b0 = __builtin_bit_cast(ol_f16x8, b[0]), b1 = __builtin_bit_cast(ol_f16x8, b[1]);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b0, acc, 0, 0, 0);
  return acc;
}
// exponent s with max * 2^s in [2^14, 2^15) for a non-negative finite max (0: s = 0)
__device__ __forceinline__ int h16_exp(float mx) {
  const int e = (int)((__float_as_uint(mx) >> 23) & 0xff);
  const int s = mx > 0.f ? 14 - (e - 127) : 0;
  return s < 126 ? s : 126;  // (a maximum below 2^-112: the planes then sit below the top binade)
}
