// Shared device helpers for the gfx950 (CDNA4) kernels of the VGGT hot path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/vggt_mi355x.h"

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef uint16_t bf16_t;  // raw bf16 bits in global memory

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

// Round-to-nearest-even fp32 -> bf16 (finite inputs; NaN stays NaN via the
// hardware convert path the compiler emits for __bf16 casts).
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}
__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
__device__ __forceinline__ float round_bf(float f) { return bf2f(f2bf(f)); }

// pack two floats into a dword of 2 bf16 (lo, hi)
// (one v_cvt_pk_bf16_f32: the two scalar conversions + shift + or of the plain
// form cost four VALU, e.g. 192 extra per 256x256 GEMM tile epilogue per wave)
__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  typedef __bf16 b16x2_t __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){lo, hi}, b16x2_t));
}

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f)); }

// GELU(x) = x * Phi(x) through a branch-free erfc (Chebyshev fit, fractional
// error < 1.2e-7 over the whole real line, i.e. ~1 fp32 ulp): one rcp, one
// exp2 and ten FMAs, no divergence.  Used where the result is rounded to
// bf16 (the GEMM fc1 epilogue), where it matches the libm erf form up to
// rare round-to-nearest ties.
__device__ __forceinline__ float gelu_fast(float x) {
  const float z = fabsf(x) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, z, 1.0f));
  float p = 0.17087277f;
  p = fmaf(p, t, -0.82215223f);
  p = fmaf(p, t, 1.48851587f);
  p = fmaf(p, t, -1.13520398f);
  p = fmaf(p, t, 0.27886807f);
  p = fmaf(p, t, -0.18628806f);
  p = fmaf(p, t, 0.09678418f);
  p = fmaf(p, t, 0.37409196f);
  p = fmaf(p, t, 1.00002368f);
  p = fmaf(p, t, -1.26551223f);
  const float e = t * __builtin_amdgcn_exp2f(fmaf(-z, z, p) * 1.4426950408889634f);  // erfc(z)
  return x * (x >= 0.f ? fmaf(-0.5f, e, 1.0f) : 0.5f * e);
}

// Two GELUs at once: the polynomial, the final products and the select run as
// packed fp32 (v_pk_fma_f32 / v_pk_mul_f32: two lanes of work per
// instruction); only rcp and exp2 stay scalar.  Same formula and error as
// gelu_fast.  For pure-VALU epilogues (no MFMA in flight on the wave).
typedef __attribute__((ext_vector_type(2))) float f32x2;
__device__ __forceinline__ f32x2 gelu_fast2(f32x2 x) {
  const f32x2 z = f32x2{fabsf(x[0]), fabsf(x[1])} * 0.70710678118654752440f;
  const f32x2 d = z * 0.5f + 1.0f;
  const f32x2 t = f32x2{__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
  f32x2 p = f32x2{0.17087277f, 0.17087277f};
  p = p * t + -0.82215223f;
  p = p * t + 1.48851587f;
  p = p * t + -1.13520398f;
  p = p * t + 0.27886807f;
  p = p * t + -0.18628806f;
  p = p * t + 0.09678418f;
  p = p * t + 0.37409196f;
  p = p * t + 1.00002368f;
  p = p * t + -1.26551223f;
  const f32x2 arg = (p - z * z) * 1.4426950408889634f;
  const f32x2 e = t * f32x2{__builtin_amdgcn_exp2f(arg[0]), __builtin_amdgcn_exp2f(arg[1])};  // erfc(z)
  const f32x2 h = e * 0.5f;
  const f32x2 phi = f32x2{x[0] >= 0.f ? 1.0f - h[0] : h[0], x[1] >= 0.f ? 1.0f - h[1] : h[1]};
  return x * phi;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// XCD-aware bijective remap of a linear block id (cdna_hip_programming.md §5
// "XCD swizzle must be bijective"): consecutive logical tiles land on the
// same XCD (blocks b and b+8 share one), so tiles that share an operand panel
// hit the same L2.
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

#define HIP_LAUNCH_CHECK()                         \
  do {                                             \
    hipError_t e_ = hipGetLastError();             \
    if (e_ != hipSuccess) return VGGT_ERR_HIP;     \
  } while (0)
