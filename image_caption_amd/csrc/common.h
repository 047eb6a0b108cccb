// Shared device helpers for the gfx950 (CDNA4) captioning kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;  // bf16 storage (raw bits)
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

#define GLOBAL_AS __attribute__((address_space(1)))
#define LDS_AS __attribute__((address_space(3)))

__device__ __forceinline__ float bf2f(bf16_t u) { return __uint_as_float(((uint32_t)u) << 16); }

__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 h = (__bf16)f;  // v_cvt_pk_bf16_f32: round-to-nearest-even, NaN stays NaN
  return __builtin_bit_cast(bf16_t, h);
}

// hi/lo split: hi = bf16(v), lo = bf16(v - hi).  hi + lo carries ~16 mantissa bits.
__device__ __forceinline__ void split_bf(float v, bf16_t& hi, bf16_t& lo) {
  hi = f2bf(v);
  lo = f2bf(v - bf2f(hi));
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// GELU(v) = v/2 (1 + erf(v / sqrt 2)) with erfc from the Chebyshev fit of Numerical Recipes §6.2
// (fractional error < 1.2e-7 everywhere): one rcp, one exp, 10 FMA, no branches - well inside the
// bf16x2 planes' 2^-17 the value is stored with.  ocml's erff costs several times that in the
// epilogue of the MLP GEMM.
__device__ __forceinline__ float gelu_erf_fast(float v) {
  const float z = fabsf(v) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(1.f + 0.5f * z);
  float y = 0.17087277f;
  y = fmaf(y, t, -0.82215223f);
  y = fmaf(y, t, 1.48851587f);
  y = fmaf(y, t, -1.13520398f);
  y = fmaf(y, t, 0.27886807f);
  y = fmaf(y, t, -0.18628806f);
  y = fmaf(y, t, 0.09678418f);
  y = fmaf(y, t, 0.37409196f);
  y = fmaf(y, t, 1.00002368f);
  y = fmaf(y, t, -1.26551223f);
  const float erfc_z = t * __expf(fmaf(-z, z, y));
  return 0.5f * v * (v >= 0.f ? 2.f - erfc_z : erfc_z);
}

