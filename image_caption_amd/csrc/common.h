// Shared device helpers for the gfx950 (CDNA4) captioning kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <utility>

typedef uint16_t bf16_t;  // bf16 storage (raw bits)
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));

#define GLOBAL_AS __attribute__((address_space(1)))
#define LDS_AS __attribute__((address_space(3)))

// LDS DMA of 16 B per lane (global_load_lds_dwordx4: lane l's 16 bytes land at M0 + 16 l) issued from inline asm.
// hipcc's waitcnt pass books the builtin's LDS write on the LGKM counter too, so behind an in-flight builtin DMA every
// use of an LDS read waits lgkmcnt(0) - the whole fragment-read pipeline drained before each MFMA group (the
// persistent fp16 GEMM's k-loop had twelve per k-step).  Issued here the DMA is invisible to that pass: the reads keep
// counted waits.  Only for kernels whose own inline-asm `s_waitcnt vmcnt` waits order the DMA before its data is read
// (a compiler-generated fence would not wait for it); extra VMEM operations the compiler does not count only make its
// own vmcnt waits conservative (in-order retirement).  M0 is saved and restored inside the statement.
__device__ __forceinline__ void lds_dma16(const void* gsrc, __attribute__((address_space(3))) void* ldst) {
  const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)ldst);
  uint32_t save;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(save)
               : "v"(gsrc), "s"(l));
}

// The same DMA as a buffer load: source = the resource's base + voff (per lane) + soff (wave-uniform SGPR).  The
// per-lane address is one 32-bit VGPR, so a stage's pieces share it and differ by soff (hipBLASLt's form), and a lane
// whose voff is at or past the resource's byte count (num_records; soff is not part of the range check) reads zeros.
typedef int32_t i32x4r __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4r buf_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)(uintptr_t)base;
  return (i32x4r){(int32_t)(uint32_t)a, (int32_t)(uint32_t)(a >> 32), (int32_t)bytes, 0x00020000};  // gfx9 raw buffer
}
__device__ __forceinline__ void lds_dma_buf16(i32x4r rsrc, uint32_t voff, uint32_t soff,
                                              __attribute__((address_space(3))) void* ldst) {
  const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)ldst);
  const uint32_t so = __builtin_amdgcn_readfirstlane(soff);  // (uniform by contract; the asm needs an SGPR)
  uint32_t save;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(save)
               : "v"(voff), "s"(rsrc), "s"(l), "s"(so));
}

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

// Two values at once: v_cvt_pk_bf16_f32 rounds both (RNE) into one dword (element 0 in the low half);
// hi/lo as split_bf, both planes packed.  Half the conversions and none of the shift/or packing of
// two split_bf calls.
__device__ __forceinline__ uint32_t pack_bf2(f32x2 v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2v));
}
__device__ __forceinline__ void split_bf2(f32x2 v, uint32_t& hi, uint32_t& lo) {
  hi = pack_bf2(v);
  const f32x2 hf = {__uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
  lo = pack_bf2(v - hf);
}

// Cross-row lane exchange without the LDS crossbar (gfx950 v_permlane16_swap / v_permlane32_swap, VALU): with both
// operands the same value, the swap leaves lane l holding {v of its row pair's even row, v of the odd row} (16-swap)
// or {v of rows 0-1, v of rows 2-3} (32-swap), whichever row l is in - so max / sum over the pair is the xor-16 / xor-32
// reduction and the other element is the partner.  (__shfl_xor compiles to ds_bpermute: an LDS round trip each.)
__device__ __forceinline__ uint32_t xor16_partner(uint32_t v) {
  const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  return (threadIdx.x & 16) ? p[0] : p[1];
}
__device__ __forceinline__ float rows4_max(float v) {  // max over lanes l, l ^ 16, l ^ 32, l ^ 48
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(q[0]), __uint_as_float(q[1]));
}
__device__ __forceinline__ float rows4_sum(float v) {  // sum over lanes l, l ^ 16, l ^ 32, l ^ 48 (same order in all four)
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}

// Lane exchanges inside a 16-lane row through DPP (a VALU operand modifier, no LDS round trip): CTRL 0xB1 / 0x4E =
// quad_perm [1,0,3,2] / [2,3,0,1] (xor 1 / xor 2), 0x141 = half-row mirror (the other quad of the lane's 8), 0x140 =
// row mirror (the other 8 of the row).  Applied in that order to a symmetric operation (+, max), every lane of the
// row ends with the same bits.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true);
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  return v + dpp_f<0x140>(v);
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  return fmaxf(v, dpp_f<0x140>(v));
}
// whole-wave reductions: the row reduction, then the rows (every lane the same bits)
__device__ __forceinline__ float wave_max(float v) { return rows4_max(row16_max(v)); }
__device__ __forceinline__ float wave_sum(float v) { return rows4_sum(row16_sum(v)); }
// (value, index) argmax over the wave, ties to the lower index: the same total order in every pairing, so every lane
// ends with the exact winner (DPP inside rows, permlane swaps across them)
__device__ __forceinline__ void argmax_take(float& bv, int& bi, float ov, int oi) {
  if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
}
__device__ __forceinline__ void wave_argmax(float& bv, int& bi) {
  argmax_take(bv, bi, dpp_f<0xB1>(bv), dpp_i<0xB1>(bi));
  argmax_take(bv, bi, dpp_f<0x4E>(bv), dpp_i<0x4E>(bi));
  argmax_take(bv, bi, dpp_f<0x141>(bv), dpp_i<0x141>(bi));
  argmax_take(bv, bi, dpp_f<0x140>(bv), dpp_i<0x140>(bi));
  const auto pv = __builtin_amdgcn_permlane16_swap(__float_as_uint(bv), __float_as_uint(bv), false, false);
  const auto pi = __builtin_amdgcn_permlane16_swap((uint32_t)bi, (uint32_t)bi, false, false);
  argmax_take(bv, bi, __uint_as_float(pv[0]), (int)pi[0]);
  argmax_take(bv, bi, __uint_as_float(pv[1]), (int)pi[1]);
  const auto qv = __builtin_amdgcn_permlane32_swap(__float_as_uint(bv), __float_as_uint(bv), false, false);
  const auto qi = __builtin_amdgcn_permlane32_swap((uint32_t)bi, (uint32_t)bi, false, false);
  argmax_take(bv, bi, __uint_as_float(qv[0]), (int)qi[0]);
  argmax_take(bv, bi, __uint_as_float(qv[1]), (int)qi[1]);
}
// value of `v` in lane `src` (a wave-uniform lane index) for every lane
__device__ __forceinline__ float lane_bcast(float v, int src) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), src));
}

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// fp16 single-plane operands (ICAP_PREC_F16 encoder): the same 16-bit storage type carries fp16 bits;
// mma<F16> picks the MFMA, cvt16<F16> / pack16x4<F16> the conversion (both round to nearest even).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));
template <bool F16>
__device__ __forceinline__ f32x4 mma(bf16x8 a, bf16x8 b, f32x4 c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                  0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bf16_t f2h(float f) { return __builtin_bit_cast(bf16_t, (_Float16)f); }
__device__ __forceinline__ float h2f(bf16_t u) { return (float)__builtin_bit_cast(_Float16, u); }
// fp16 hi/lo split (the Grid trunk's residual stream in ICAP_PREC_F16): hi = fp16(v), lo = fp16(v - hi), ~22 bits
__device__ __forceinline__ void split_h(float v, bf16_t& hi, bf16_t& lo) {
  const _Float16 h = (_Float16)v;
  hi = __builtin_bit_cast(bf16_t, h);
  lo = f2h(v - (float)h);
}
template <bool F16>
__device__ __forceinline__ bf16_t cvt16(float f) {
  if constexpr (F16) return f2h(f);
  else return f2bf(f);
}
// fp16 range guard (ICAP_PREC_F16): a packed pair holds an infinity or NaN (exponent field all ones), i.e. a value
// that overflowed 65504 on conversion or was already non-finite
__device__ __forceinline__ bool f16_pair_nonfinite(uint32_t u) {
  return (u & 0x7c00u) == 0x7c00u || (u & 0x7c000000u) == 0x7c000000u;
}
// set bit 0 of the handle's sticky status word (one vector atomic from one lane; never the scalar path)
__device__ __forceinline__ void range_flag_set(unsigned* flag) {
  __hip_atomic_fetch_or(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <bool F16>
__device__ __forceinline__ u32x2 pack16x4(f32x4 v) {
  if constexpr (F16) {
    const f16x2v a = {(_Float16)v[0], (_Float16)v[1]}, b = {(_Float16)v[2], (_Float16)v[3]};
    return (u32x2){__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b)};
  } else {
    return (u32x2){pack_bf2((f32x2){v[0], v[1]}), pack_bf2((f32x2){v[2], v[3]})};
  }
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
// gelu_erf_fast on two values with packed FMAs (v_pk_fma_f32 / v_pk_mul_f32: the ten-term chain
// issues five instructions per value pair instead of ten); the same operations, so the same results.
__device__ __forceinline__ f32x2 gelu_erf_fast2(f32x2 v) {
  const f32x2 z = __builtin_elementwise_abs(v) * 0.70710678118654752f;
  const f32x2 den = __builtin_elementwise_fma(z, (f32x2)0.5f, (f32x2)1.f);
  const f32x2 t = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
  f32x2 y = 0.17087277f;
  y = __builtin_elementwise_fma(y, t, (f32x2)-0.82215223f);
  y = __builtin_elementwise_fma(y, t, (f32x2)1.48851587f);
  y = __builtin_elementwise_fma(y, t, (f32x2)-1.13520398f);
  y = __builtin_elementwise_fma(y, t, (f32x2)0.27886807f);
  y = __builtin_elementwise_fma(y, t, (f32x2)-0.18628806f);
  y = __builtin_elementwise_fma(y, t, (f32x2)0.09678418f);
  y = __builtin_elementwise_fma(y, t, (f32x2)0.37409196f);
  y = __builtin_elementwise_fma(y, t, (f32x2)1.00002368f);
  y = __builtin_elementwise_fma(y, t, (f32x2)-1.26551223f);
  const f32x2 ex = __builtin_elementwise_fma(-z, z, y);
  const f32x2 erfc_z = t * (f32x2){__expf(ex.x), __expf(ex.y)};
  const f32x2 r = {v.x >= 0.f ? 2.f - erfc_z.x : erfc_z.x, v.y >= 0.f ? 2.f - erfc_z.y : erfc_z.y};
  return 0.5f * v * r;
}
// gelu_erf_fast on eight values (two column groups of an MFMA tile): every step is four independent packed FMAs,
// so the ten-term chain issues without the nop a dependent v_pk_fma_f32 needs behind its producer (the f32x2 form
// ran each pair's chain alone: ~500 s_nop in the MLP-1 epilogue).  The same operations per value, so the same results.
typedef float f32x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x8 gelu_erf_fast8(f32x8 v) {
  const f32x8 z = __builtin_elementwise_abs(v) * 0.70710678118654752f;
  const f32x8 den = __builtin_elementwise_fma(z, (f32x8)0.5f, (f32x8)1.f);
  f32x8 t;
#pragma unroll
  for (int e = 0; e < 8; ++e) t[e] = __builtin_amdgcn_rcpf(den[e]);
  f32x8 y = 0.17087277f;
  y = __builtin_elementwise_fma(y, t, (f32x8)-0.82215223f);
  y = __builtin_elementwise_fma(y, t, (f32x8)1.48851587f);
  y = __builtin_elementwise_fma(y, t, (f32x8)-1.13520398f);
  y = __builtin_elementwise_fma(y, t, (f32x8)0.27886807f);
  y = __builtin_elementwise_fma(y, t, (f32x8)-0.18628806f);
  y = __builtin_elementwise_fma(y, t, (f32x8)0.09678418f);
  y = __builtin_elementwise_fma(y, t, (f32x8)0.37409196f);
  y = __builtin_elementwise_fma(y, t, (f32x8)1.00002368f);
  y = __builtin_elementwise_fma(y, t, (f32x8)-1.26551223f);
  const f32x8 ex = __builtin_elementwise_fma(-z, z, y);
  f32x8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float erfc_z = t[e] * __expf(ex[e]);
    r[e] = v[e] >= 0.f ? 2.f - erfc_z : erfc_z;
  }
  return 0.5f * v * r;
}

// GELU for fp16 outputs (the f16 encoder's MLP-1 epilogue): erfc(z) from Abramowitz & Stegun 7.1.26 (five coefficients,
// |error| <= 1.5e-7 absolute in erf) - one rcp, one exp2, five FMA per value instead of ten: the result differs from
// the exact GELU by at most 4.2e-7 (fp32 evaluation over [-12, 12]), i.e. at most one fp16 ulp after the store's
// rounding (2.8 % of values), against the fp16 plane's own 2^-11 relative rounding.  (The bf16x2 paths keep the
// 1.2e-7-relative form above: their planes carry 16 significand bits.)
__device__ __forceinline__ float gelu_erf_as(float v) {  // the same operations on one value (bitwise equal)
  const float z = fabsf(v) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(z, 0.3275911f, 1.f));
  float y = 1.061405429f;
  y = fmaf(y, t, -1.453152027f);
  y = fmaf(y, t, 1.421413741f);
  y = fmaf(y, t, -0.284496736f);
  y = fmaf(y, t, 0.254829592f);
  y *= t;
  const float erfc_z = y * __builtin_amdgcn_exp2f((z * z) * -1.44269504088896341f);
  return 0.5f * v * (v >= 0.f ? 2.f - erfc_z : erfc_z);
}
__device__ __forceinline__ f32x8 gelu_erf_as8(f32x8 v) {
  const f32x8 z = __builtin_elementwise_abs(v) * 0.70710678118654752f;
  const f32x8 den = __builtin_elementwise_fma(z, (f32x8)0.3275911f, (f32x8)1.f);
  f32x8 t;
#pragma unroll
  for (int e = 0; e < 8; ++e) t[e] = __builtin_amdgcn_rcpf(den[e]);
  f32x8 y = 1.061405429f;
  y = __builtin_elementwise_fma(y, t, (f32x8)-1.453152027f);
  y = __builtin_elementwise_fma(y, t, (f32x8)1.421413741f);
  y = __builtin_elementwise_fma(y, t, (f32x8)-0.284496736f);
  y = __builtin_elementwise_fma(y, t, (f32x8)0.254829592f);
  y *= t;
  const f32x8 ex = (z * z) * -1.44269504088896341f;  // -z^2 in log2 units
  f32x8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float erfc_z = y[e] * __builtin_amdgcn_exp2f(ex[e]);
    r[e] = v[e] >= 0.f ? 2.f - erfc_z : erfc_z;
  }
  return 0.5f * v * r;
}

// int8 two-slice quantisation (the operand form of gemm_i8_kernel): 16-bit fixed point relative to
// the row maximum, q = rint(v / s) in [-32639, 32639], v1 = (q + 128) >> 8 in [-127, 127],
// v2 = q - 256 v1 in [-128, 127]; four consecutive values -> one 32-bit word per slice.  Row image
// [K/64][2][64]: the two slices of a 64-deep k block share one 128-B line, so each GEMM stage row
// is one full-line request.
__device__ __forceinline__ void q2_pack4(const float* y, float inv, uint32_t& hi, uint32_t& lo) {
  hi = lo = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int qv = __float2int_rn(fminf(fmaxf(y[k] * inv, -32639.f), 32639.f));
    const int v1 = (qv + 128) >> 8, v2 = qv - (v1 << 8);
    hi |= (uint32_t)(v1 & 0xff) << (8 * k);
    lo |= (uint32_t)(v2 & 0xff) << (8 * k);
  }
}

// ---- counter-based dropout masks (train-mode sampling and the training pass) ----
// keep(seed, site, layer, row, pos, idx) = h >= thr with h a 32-bit hash of the six integers and
// thr = round(p 2^32); kept elements are scaled by 1 / (1 - p) (torch.nn.Dropout).  The mask of an
// element depends only on its (image row, query position, index) - not on the decode step - so the
// KV-cached sampler and the teacher-forced training pass draw the same masks; oracle/dropout.py is the
// numpy restatement.  Sites: 0 positional-encoding output, 1 self-attention probabilities (idx = head
// * 128 + key), 2 self-attention output, 3 cross-attention probabilities (idx = head * 256 + memory
// token), 4 cross-attention output, 5 feed-forward hidden, 6 feed-forward output; layer 0..15.
__host__ __device__ inline uint32_t icap_mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__host__ __device__ inline uint32_t icap_drop_hash(uint32_t seed, uint32_t site, uint32_t layer, uint32_t row,
                                                   uint32_t pos, uint32_t idx) {
  uint32_t h = icap_mix32(idx * 0x9E3779B1u + 0x7F4A7C15u);
  h = icap_mix32(h ^ (pos * 0x85EBCA77u + 0xC2B2AE3Du));
  h = icap_mix32(h ^ (row * 0x27D4EB2Fu + 0x165667B1u));
  h = icap_mix32(h ^ ((site * 16u + layer) * 0x94D049BBu + 0x2545F491u));
  return icap_mix32(h ^ seed);
}

