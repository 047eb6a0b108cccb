// bf16 MFMA GEMM for gfx950: C = epi(A · W^T + bias (+ addend)) with fp32 accumulation.
//
// Every nn.Linear / 1x1-conv / patch-conv of the captioning hot path lands here
// (SURVEY.md §2.1 K1, K4-K6, K8-K10, K14, K15).  A is an activation given as one or two bf16
// planes ("split": hi = bf16(v), lo = bf16(v - hi)); the K loop simply runs over both planes
// against the same W columns, so A·W = A_hi·W + A_lo·W carries ~16 mantissa bits of the fp32
// activation at 2x the MFMA work.  W is bf16 [N][K] (the nn.Linear layout, K contiguous), so
// both operands are K-contiguous and load as 16-byte rows.
//
// Tiling: BM x BN block tile, BK = 64, 4 waves (256 threads) each owning WM x WN, built from
// v_mfma_f32_16x16x32_bf16.  Tiles are staged HBM -> LDS with global_load_lds_dwordx4 into a
// double buffer; the LDS image is lane-linear (one 1 KiB wave-instruction = 8 rows of 128 B) and
// the XOR swizzle chunk' = chunk ^ (row & 7) is applied on the SOURCE address and on the
// ds_read_b128, which makes the 16-lane row-fragment reads bank-conflict free.
#include "gemm_kern.h"

namespace {

// F16: fp16 operands (A planes, W) and fp16 output / residual planes (the ICAP_PREC_F16 Grid trunk)
template <int BM, int BN, int WM, int WN, int CONV = 0, bool F16 = false>
__global__ __launch_bounds__(256) void gemm_bf16_kernel(GemmArgs p) {
  constexpr int WAVES_N = BN / WN;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int IA = BM / 32, IB = BN / 32;  // 1 KiB staging instructions per wave per tile
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int bz = blockIdx.z;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int M = p.M, K = p.K;
  const bf16_t* __restrict__ A = p.A + (long)bz * p.a_batch;
  const bf16_t* __restrict__ W = p.W + (long)bz * p.w_batch;
  const int nk = p.nsplit * K / BK;

  long a_off[IA], b_off[IB];
  ConvRow cr[CONV ? IA : 1];
#pragma unroll
  for (int i = 0; i < IA; ++i) {
    int idx = (wave * IA + i) * 64 + lane, row = idx >> 3, cs = idx & 7;
    int gr = min(m0 + row, M - 1);
    if (CONV) {
      cr[i] = conv_row(p, gr);
      a_off[i] = (cs ^ (row & 7)) << 3;  // k offset of the lane's chunk
    } else {
      a_off[i] = (long)gr * p.lda + ((cs ^ (row & 7)) << 3);
    }
  }
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    int idx = (wave * IB + i) * 64 + lane, row = idx >> 3, cs = idx & 7;
    int gr = min(n0 + row, p.N - 1);
    b_off[i] = (long)gr * p.ldw + ((cs ^ (row & 7)) << 3);
  }

  auto stage = [&](int kt, int buf) {
    const int kg = kt * BK, plane = kg / K, kin = kg - plane * K;
    const bf16_t* Ab = A + plane * p.a_lo + kin;
    const bf16_t* Wb = W + kin;
    char* sa = smem + buf * STAGE;
    char* sb = sa + A_BYTES;
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const bf16_t* src = CONV ? conv_src<CONV>(p, A + plane * p.a_lo, cr[CONV ? i : 0], kin + (int)a_off[i])
                               : Ab + a_off[i];
      __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)src, (LDS_AS void*)(sa + (wave * IA + i) * 1024), 16,
                                       0, 0);
    }
#pragma unroll
    for (int i = 0; i < IB; ++i)
      __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)(Wb + b_off[i]),
                                       (LDS_AS void*)(sb + (wave * IB + i) * 1024), 16, 0, 0);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) stage(kt + 1, (kt + 1) & 1);
    const char* sa = smem + (kt & 1) * STAGE;
    const char* sb = sa + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + fq;
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + i * 16 + fr;
        af[i] = *(const bf16x8*)(sa + row * 128 + ((chunk ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WN + j * 16 + fr;
        bfr[j] = *(const bf16x8*)(sb + row * 128 + ((chunk ^ (row & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mma<F16>(af[i], bfr[j], acc[i][j]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: C/D layout of 16x16 MFMA: col = lane & 15, row = 4*(lane >> 4) + r
  const float* bias = p.bias ? p.bias + (long)bz * p.bias_batch : nullptr;
  bool bad = false;  // F16: a stored value that is not finite in fp16 (range guard)
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn * WN + j * 16 + fr;
    const float bv = bias ? bias[col] : 0.f;
    const float sv = p.scale ? p.scale[col] : 1.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * WM + i * 16 + fq * 4 + r;
        if (row >= M) continue;
        float v = acc[i][j][r] * sv + bv;
        if (p.addend) v += p.addend[(long)((row % p.add_group) + p.add_off) * p.add_ld + col];
        if (p.res) {
          const long ro = (long)row * p.res_ld + col;
          if constexpr (F16) v += h2f(p.res[ro]) + (p.res_planes == 2 ? h2f(p.res[ro + p.res_lo]) : 0.f);
          else v += bf2f(p.res[ro]) + bf2f(p.res[ro + p.res_lo]);
        }
        if (p.epi == EPI_GELU) v = 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
        else if (p.epi == EPI_RELU) v = fmaxf(v, 0.f);
        const long orow = p.rm_group ? (long)(row / p.rm_group) * p.rm_stride + p.rm_off + row % p.rm_group
                                     : (long)row;
        const long o = p.hm_n ? (((long)(row / p.hm_n) * (p.N / 64) + col / 64) * p.hm_n + row % p.hm_n) * 64 + col % 64
                              : (long)bz * p.c_batch + orow * p.ldc + col;
        if (p.out == OUT_F32) {
          ((float*)p.C)[o] = v;
        } else if (p.out == OUT_F32_RESID) {
          ((float*)p.C)[o] += v;
        } else if (p.out == OUT_BF16) {
          ((bf16_t*)p.C)[o] = f2bf(v);
        } else {
          bf16_t hi, lo;
          if constexpr (F16) {
            split_h(v, hi, lo);
            bad |= (hi & 0x7c00) == 0x7c00;
          } else {
            split_bf(v, hi, lo);
          }
          ((bf16_t*)p.C)[o] = hi;
          if (p.c_planes == 2) ((bf16_t*)p.C)[o + p.c_lo] = lo;
        }
      }
    }
  }
  if (F16 && p.range_flag && __any(bad) && lane == 0) range_flag_set(p.range_flag);
}

template <int BM, int BN, int WM, int WN>
hipError_t run(const GemmArgs& g, hipStream_t s) {
  constexpr int lds = 2 * (BM + BN) * BK * 2;
  if constexpr (lds > 65536) {
    static bool attr = false;
    if (!attr) {
      for (const void* f : {(const void*)gemm_bf16_kernel<BM, BN, WM, WN>, (const void*)gemm_bf16_kernel<BM, BN, WM, WN, 1>,
                            (const void*)gemm_bf16_kernel<BM, BN, WM, WN, 2>, (const void*)gemm_bf16_kernel<BM, BN, WM, WN, 0, true>,
                            (const void*)gemm_bf16_kernel<BM, BN, WM, WN, 1, true>,
                            (const void*)gemm_bf16_kernel<BM, BN, WM, WN, 2, true>}) {
        const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return e;
      }
      attr = true;
    }
  }
  dim3 grid(g.N / BN, (g.M + BM - 1) / BM, g.batch);
  if (grid.y > 65535) return hipErrorInvalidValue;
  if (g.f16) {
    if (g.cv == 1) hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, WM, WN, 1, true>), grid, dim3(256), lds, s, g);
    else if (g.cv == 2) hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, WM, WN, 2, true>), grid, dim3(256), lds, s, g);
    else hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, WM, WN, 0, true>), grid, dim3(256), lds, s, g);
  } else if (g.cv == 1) hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, WM, WN, 1>), grid, dim3(256), lds, s, g);
  else if (g.cv == 2) hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, WM, WN, 2>), grid, dim3(256), lds, s, g);
  else hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, WM, WN>), grid, dim3(256), lds, s, g);
  return hipGetLastError();
}

// ICAP_F16H (compile-time form, round 6): the ViT encoder's persistent GEMMs on gemm_f16h_kernel (one wave per SIMD,
// half-step register double buffering - gemm_kern.h) instead of gemm_f16p_kernel
#ifndef ICAP_F16H
#define ICAP_F16H 0
#endif
#if ICAP_F16H  // (a product build without the form compiles none of its kernels)
#include "gemm_variants.h"
// the f16h form's 32-bit offsets: A / W stage pieces (rows up to a whole tile past M) and the epilogue's byte range
bool f16h_ok(const GemmArgs& g) {
  const bool res = g.out == OUT_F32_RESID;
  const long cbytes = (!res && g.hm_n) ? (long)g.M * g.N * 2 : (long)g.M * g.ldc * (res ? 4 : 2);
  // ICAP_F16H 2: the long-K residual GEMMs only (ViT MLP-2, K = 3072: 272-273 against 278-281 us on two boxes,
  // profiles/r06/f16h_spread_ab.txt; the other shapes within +-3 %)
  if (ICAP_F16H == 2 && !(res && g.K >= 2048)) return false;
  return g.bias && (!g.hm_n || g.hm_n >= 16) && cbytes < (1L << 32) && (long)(g.M + 256) * g.lda * 2 < (1L << 32) &&
         (long)g.N * g.ldw * 2 < (1L << 32);
}

hipError_t launch_f16h(const GemmArgs& g, hipStream_t s, int blocks) {
  static bool attrs = false;
  if (!attrs) {
    hipError_t e = hipSuccess;
    for (const void* f : {(const void*)gemm_f16h_kernel<1, 0>, (const void*)gemm_f16h_kernel<1, 1>,
                          (const void*)gemm_f16h_kernel<1, 2>})
      if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, f16h_lds(256));
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void*)gemm_f16h_kernel<2, 0, 224>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              f16h_lds(224));
    if (e != hipSuccess) return e;
    attrs = true;
  }
  if (g.out == OUT_F32_RESID) {
    const int tiles = (g.N / 256) * ((g.M + 223) / 224);
    hipLaunchKernelGGL((gemm_f16h_kernel<2, 0, 224>), dim3(std::min(tiles, blocks)), dim3(256), f16h_lds(224), s, g);
  } else {
    const int tiles = (g.N / 256) * ((g.M + 255) / 256);
    const dim3 grid(std::min(tiles, blocks));
    if (g.hm_n) hipLaunchKernelGGL((gemm_f16h_kernel<1, 2>), grid, dim3(256), f16h_lds(256), s, g);
    else if (g.epi == EPI_GELU) hipLaunchKernelGGL((gemm_f16h_kernel<1, 1>), grid, dim3(256), f16h_lds(256), s, g);
    else hipLaunchKernelGGL((gemm_f16h_kernel<1, 0>), grid, dim3(256), f16h_lds(256), s, g);
  }
  return hipGetLastError();
}
#endif

}  // namespace

bool gemm_f16_persistent(const GemmArgs& g) {
  // tools: ICAP_F16_GEMM 6 = persistent for every fp16 GEMM, 7 = gemm_f16r_kernel; ICAP_F16_PRES 0 = the residual GEMMs in the
  // two-block form (out-proj 131 / MLP-2 340 us against 124 / 314 persistent, encoder 15.7 -> 15.0 ms/step)
  static const int form = icap_knob("ICAP_F16_GEMM", 0), pres = icap_knob("ICAP_F16_PRES", 1);
  const bool common = g.f16 && (form == 0 || form == 6 || form == 7) && !g.addend && !g.rm_group && !g.res && !g.scale && !g.cv &&
                      g.batch == 1 && g.nsplit == 1 && g.N % 256 == 0 && g.M >= 256 && g.K >= 128 && g.K % 64 == 0;
  if (!common) return false;
  if (g.out == OUT_SPLIT) return g.c_planes == 1 && (g.epi == EPI_NONE || g.epi == EPI_GELU);
  return pres && g.out == OUT_F32_RESID && g.epi == EPI_NONE;
}

int gemm_tile_class(const GemmArgs& g) {
  static const int force = icap_knob("ICAP_CONV_CLASS", 0);  // trunk convolutions (GEMMs with a BN scale)
  if (force && g.scale) {
    if (force == 256 && g.N % 256 == 0 && g.batch == 1) return PROF_GEMM_256;
    if (force == 128 && g.N % 128 == 0) return PROF_GEMM_128;
    if (force == 64) return PROF_GEMM_64;
  }
  // 256 x 256 tiles whenever N allows and there are >= 96 of them (trunk sweep, profiles/r01
  // v6_trunk_class_sweep.txt: even 98-196 tiles beat 4x as many 128 x 128 tiles); 128 x 128 only for
  // N >= 256 (at N = 128 the 64 x 64 kernel is faster)
  // the ViT's fp16 forms live in launch_gemm_256; the fp16 trunk convolutions (with a BN scale) pick as bf16 does
  if (g.f16 && !g.scale) return gemm_f16_persistent(g) ? PROF_GEMM_F16P : PROF_GEMM_256;
  const long huge_tiles = (long)((g.M + 255) / 256) * (g.N / 256) * g.batch;
  if (g.N % 256 == 0 && g.batch == 1 && huge_tiles >= 96) return PROF_GEMM_256;
  const long big_tiles = (long)((g.M + 127) / 128) * (g.N / 128) * g.batch;
  return (g.N % 128 == 0 && g.N >= 256 && big_tiles >= 512) ? PROF_GEMM_128 : PROF_GEMM_64;
}

bool gemm_narrow_ok(const GemmArgs& g);
hipError_t launch_gemm_narrow(const GemmArgs& g, hipStream_t s, int form);

// Profile class of a launch = the kernel family that runs it: the fp16 trunk's narrow convolutions run on the
// 256-family k-loop (launch_gemm_narrow) although their tile class is the 64 x 64 one
int gemm_prof_class(const GemmArgs& g) {
  const int cls = gemm_tile_class(g);
  return cls == PROF_GEMM_64 && gemm_narrow_ok(g) && icap_knob("ICAP_GEMM_NARROW", 1) ? PROF_GEMM_256 : cls;
}

hipError_t launch_gemm(const GemmArgs& g, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0 || g.K <= 0) return hipErrorInvalidValue;
  if (g.hm_n && (g.out != OUT_SPLIT || g.N % 64 || g.batch != 1 || g.rm_group || g.M % g.hm_n)) return hipErrorInvalidValue;
  if (g.K % BK != 0 || g.N % 64 != 0 || (g.nsplit != 1 && g.nsplit != 2)) return hipErrorInvalidValue;
  if (g.cv && (g.batch != 1 || !g.cv_zero || (g.cv == 1 && g.cv_cshift < 6) || g.cv_OHW <= 0 || g.cv_OW <= 0))
    return hipErrorInvalidValue;
  const int cls = gemm_tile_class(g);
  if (cls == PROF_GEMM_256 || cls == PROF_GEMM_F16P) return launch_gemm_256(g, s);
  if (cls == PROF_GEMM_128) return run<128, 128, 64, 64>(g, s);
  // the fp16 trunk's N = 64 / 128 convolutions on the 256-family k-loop (launch_gemm_narrow); ICAP_GEMM_NARROW (tools):
  // 0 = the 64 x 64 kernel below, 2-4 = the other measured tile forms
  static const int narrow = icap_knob("ICAP_GEMM_NARROW", 1);
  if (narrow && gemm_narrow_ok(g)) return launch_gemm_narrow(g, s, narrow);
  return run<64, 64, 32, 32>(g, s);
}

// ---------------------------------------------------------------------------------------------
// Wave-tile GEMM for the decode step (M = batch rows, small).  No LDS and no barriers: every
// wave owns a (16 TM) x (16 TN) output tile and streams its A and W fragments (both K-contiguous
// 16-byte rows) straight into registers, D k-steps of 32 per chunk, ping-ponging two register
// chunks so the next chunk's loads are in flight while the current one feeds the MFMAs
// (cdna_hip_programming.md §5 table, "GEMV / M <= 16" row, extended to a 2-D wave tile).
// Split-K over blockIdx.z writes fp32 partial slabs that the consumer (LayerNorm / attention)
// sums, so no atomics and bitwise-reproducible results.
namespace {

template <int TM, int TN, int WN, int D>
__global__ __launch_bounds__(256) void gemm_wave_kernel(WaveGemmArgs p) {
  constexpr int WM = 4 / WN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wn = wave % WN, wm = wave / WN;
  const int n0 = (blockIdx.x * WN + wn) * TN * 16;
  const int m0 = (blockIdx.y * WM + wm) * TM * 16;
  const int batch = blockIdx.z / p.ksplit, split = blockIdx.z % p.ksplit;
  if (n0 >= p.N || m0 >= p.M) return;  // wave-uniform
  const int fr = lane & 15, fq = lane >> 4;
  const bf16_t* A = p.A + (long)batch * p.a_batch;
  const bf16_t* W = p.W + (long)batch * p.w_batch;
  long arow[TM], wrow[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) arow[i] = (long)min(m0 + i * 16 + fr, p.M - 1) * p.lda + fq * 8;
#pragma unroll
  for (int j = 0; j < TN; ++j) wrow[j] = (long)min(n0 + j * 16 + fr, p.N - 1) * p.ldw + fq * 8;
  const int ks_total = p.nsplit * p.K / 32, per = ks_total / p.ksplit;
  const int kbeg = split * per, nchunks = per / D;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  bf16x8 xa[D][TM], xb[D][TN], ya[D][TM], yb[D][TN];

  auto load = [&](bf16x8 (&ra)[D][TM], bf16x8 (&rb)[D][TN], int ks0) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int kg = (ks0 + d) * 32, plane = kg / p.K, kin = kg - plane * p.K;
      const bf16_t* Ab = A + plane * p.a_lo + kin;
#pragma unroll
      for (int i = 0; i < TM; ++i) ra[d][i] = *(const bf16x8*)(Ab + arow[i]);
#pragma unroll
      for (int j = 0; j < TN; ++j) rb[d][j] = *(const bf16x8*)(W + kin + wrow[j]);
    }
  };
  auto compute = [&](bf16x8 (&ra)[D][TM], bf16x8 (&rb)[D][TN]) {
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(ra[d][i], rb[d][j], acc[i][j]);
  };

  load(xa, xb, kbeg);
  for (int c = 0; c < nchunks; c += 2) {
    if (c + 1 < nchunks) load(ya, yb, kbeg + (c + 1) * D);
    compute(xa, xb);
    if (c + 1 >= nchunks) break;
    if (c + 2 < nchunks) load(xa, xb, kbeg + (c + 2) * D);
    compute(ya, yb);
  }

  const float* bias = (p.bias && p.ksplit == 1) ? p.bias + (long)batch * p.bias_batch : nullptr;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + j * 16 + fr;
    if (col >= p.N) continue;
    const float bv = bias ? bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + i * 16 + fq * 4 + r;
        if (row >= p.M) continue;
        float v = acc[i][j][r] + bv;
        const long o = (long)batch * p.c_batch + (long)row * p.ldc + col;
        if (p.out == OUT_PARTIAL) {
          ((float*)p.C)[(long)split * p.part_stride + o] = v;
          continue;
        }
        if (p.epi == EPI_GELU) v = 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
        else if (p.epi == EPI_RELU) v = fmaxf(v, 0.f);
        if (p.out == OUT_F32) {
          ((float*)p.C)[o] = v;
        } else if (p.out == OUT_F32_RESID) {
          ((float*)p.C)[o] += v;
        } else if (p.out == OUT_BF16) {
          ((bf16_t*)p.C)[o] = f2bf(v);
        } else {
          bf16_t hi, lo;
          split_bf(v, hi, lo);
          ((bf16_t*)p.C)[o] = hi;
          if (p.c_planes == 2) ((bf16_t*)p.C)[o + p.c_lo] = lo;
        }
      }
    }
  }
}

template <int TM, int TN, int WN>
hipError_t run_wave(const WaveGemmArgs& g, hipStream_t s, int D) {
  constexpr int WM = 4 / WN;
  dim3 grid((g.N + WN * TN * 16 - 1) / (WN * TN * 16), (g.M + WM * TM * 16 - 1) / (WM * TM * 16),
            g.batch * g.ksplit);
  if (D == 4)
    hipLaunchKernelGGL((gemm_wave_kernel<TM, TN, WN, 4>), grid, dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL((gemm_wave_kernel<TM, TN, WN, 2>), grid, dim3(256), 0, s, g);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_gemm_wave(const WaveGemmArgs& g, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0 || g.K <= 0 || g.ksplit < 1 || g.N % 16) return hipErrorInvalidValue;
  if (g.K % 32 || (g.nsplit != 1 && g.nsplit != 2)) return hipErrorInvalidValue;
  const int steps = g.nsplit * g.K / 32;
  if (steps % g.ksplit) return hipErrorInvalidValue;
  const int per = steps / g.ksplit;
  const int D = per % 4 == 0 ? 4 : (per % 2 == 0 ? 2 : 0);
  if (D == 0) return hipErrorInvalidValue;
  if (g.out == OUT_PARTIAL && g.part_stride <= 0) return hipErrorInvalidValue;
  if (g.N % 4) return hipErrorInvalidValue;  // 4 consecutive output columns per lane
  switch (g.tile) {
    case WAVE_2x2: return run_wave<2, 2, 4>(g, s, D);
    case WAVE_1x2: return run_wave<1, 2, 4>(g, s, D);
    case WAVE_1x1: return run_wave<1, 1, 4>(g, s, D);
    case WAVE_2x1: return run_wave<2, 1, 4>(g, s, D);
    default: return hipErrorInvalidValue;
  }
}

// ---------------------------------------------------------------------------------------------
// Decode-step GEMM, "load everything first": one 4-wave block owns a 32 x 32 output tile over a
// K' range of at most 1024 (split-K covers longer K).  All of the tile's A and W bytes for that
// range (<= 128 KiB) are requested at kernel start with global_load_lds_dwordx4 - no VGPRs held,
// every request in flight at once - followed by ONE vmcnt(0) + barrier; then each wave runs the
// MFMA chain of one 16 x 16 quadrant from LDS.  For M = batch = 256 this turns a chain of
// dependent memory round trips into a single one (the wave-register kernel above paid one per
// 4-k-step chunk: 8-21 us per GEMM in profiles/r01).
// LDS image per 32-wide k-step: [A 32 rows x 64 B][W 32 rows x 64 B]; a 1 KiB DMA instruction
// covers 16 rows x 64 B (lane l -> row l >> 2, 16-byte chunk l & 3).
namespace {

constexpr int DEC_MAX_KSTEPS = 16;  // per split: 16 k-steps x 32 = K 512 -> (ns + 1) x 32 KiB of LDS
constexpr int DEC_RED_BYTES = 16 * 64 * 16;  // cross-wave reduction: 16 waves x 64 lanes x f32x4

// 16 waves: wave w computes output quadrant (w & 3) over the k-steps ks == (w >> 2) mod 4, so every
// wave has loads to issue (LDS-DMA ingest scales with the number of issuing waves: ~6 GB/s each)
// and the 4 partial quadrants are summed through LDS before the epilogue.  Per k-step the LDS holds
// ns activation-plane slices and ONE weight slice (shared by the planes), each 32 rows x 64 B with
// 16-B chunk c of row r stored at c ^ ((r >> 2) & 3) (conflict-free 16-lane fragment reads).
template <int NWV>
__global__ __launch_bounds__(NWV * 64) void gemm_dec_kernel(WaveGemmArgs p) {
  constexpr int KGRPS = NWV / 4;  // k-step groups (waves per output quadrant)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 32, m0 = blockIdx.y * 32;
  const int batch = blockIdx.z / p.ksplit, split = blockIdx.z % p.ksplit;
  const bf16_t* A = p.A + (long)batch * p.a_batch;
  const bf16_t* W = p.W + (long)batch * p.w_batch;
  const bf16_t* Wl = p.W_lo ? p.W_lo + (long)batch * p.w_batch : nullptr;
  // operands per k-step: ns activation planes, W, and (hi/lo weights) W_lo
  const int ns = p.nsplit, nops = ns + 1 + (Wl ? 1 : 0), step_bytes = nops * 2048;
  const int nks = p.K / 32 / p.ksplit, kbeg = split * nks;

  // staging: instruction q in [0, 2 * nops * nks): k-step q / (2 nops), operand, row half
  const int lrow = lane >> 2, lchunk = (lane & 3) ^ ((lrow >> 2) & 3);
  const int nq = 2 * nops * nks;
  for (int q = wave; q < nq; q += NWV) {
    const int ks = q / (2 * nops), rem = q - ks * 2 * nops, opnd = rem >> 1, half = rem & 1;
    const int kg = (kbeg + ks) * 32 + lchunk * 8;
    const int r = half * 16 + lrow;
    const bf16_t* src = opnd < ns    ? A + opnd * p.a_lo + (long)min(m0 + r, p.M - 1) * p.lda + kg
                        : opnd == ns ? W + (long)min(n0 + r, p.N - 1) * p.ldw + kg
                                     : Wl + (long)min(n0 + r, p.N - 1) * p.ldw + kg;
    __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)src,
                                     (LDS_AS void*)(smem + ks * step_bytes + opnd * 2048 + half * 1024), 16, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int quad = wave & 3, kgrp = wave >> 2;  // kgrp < KGRPS
  const int qm = quad >> 1, qn = quad & 1;
  const int fr = lane & 15, fq = lane >> 4;
  const int sw = (fq ^ ((fr >> 2) & 3)) * 16;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const char* pa = smem + (qm * 16 + fr) * 64 + sw;
  const char* pb = smem + ns * 2048 + (qn * 16 + fr) * 64 + sw;
  // W as the first operand: lane holds output row m = fr, four consecutive columns n = 4 fq + r
  for (int ks = kgrp; ks < nks; ks += KGRPS) {
    const bf16x8 b = *(const bf16x8*)(pb + ks * step_bytes);
    const bf16x8 a = *(const bf16x8*)(pa + ks * step_bytes);
    acc = mfma16(b, a, acc);
    if (ns == 2) {
      const bf16x8 al = *(const bf16x8*)(pa + 2048 + ks * step_bytes);
      acc = mfma16(b, al, acc);
    }
    if (Wl) acc = mfma16(*(const bf16x8*)(pb + 2048 + ks * step_bytes), a, acc);  // W_lo . X_hi
  }
  if (KGRPS > 1) {
    __syncthreads();  // staging area is reused for the reduction
    f32x4* red = (f32x4*)smem;
    if (kgrp) red[(kgrp * 4 + quad) * 64 + lane] = acc;
    __syncthreads();
    if (kgrp == 0) {
#pragma unroll
      for (int g = 1; g < KGRPS; ++g) acc += red[(g * 4 + quad) * 64 + lane];
    }
  }

  const int row = m0 + qm * 16 + fr;
  const int col = n0 + qn * 16 + 4 * fq;
  if (KGRPS > 1 && kgrp) return;
  if (row >= p.M || col >= p.N) return;
  f32x4 v = acc;
  if (p.bias && p.ksplit == 1) v += *(const f32x4*)(p.bias + (long)batch * p.bias_batch + col);
  if (p.epi == EPI_GELU) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = gelu_erf_fast(v[r]);
  } else if (p.epi == EPI_RELU) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
  }
  const long o = (long)batch * p.c_batch + (long)row * p.ldc + col;
  if (p.out == OUT_PARTIAL) {
    *(f32x4*)((float*)p.C + (long)split * p.part_stride + o) = v;
  } else if (p.out == OUT_F32) {
    *(f32x4*)((float*)p.C + o) = v;
  } else if (p.out == OUT_F32_RESID) {
    *(f32x4*)((float*)p.C + o) += v;
  } else {
    bf16_t h[4], l[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) split_bf(v[r], h[r], l[r]);
    bf16_t* C = (bf16_t*)p.C;
    *(u32x2*)(C + o) = (u32x2){(uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16)};
    if (p.out == OUT_SPLIT && p.c_planes == 2)
      *(u32x2*)(C + o + p.c_lo) = (u32x2){(uint32_t)l[0] | ((uint32_t)l[1] << 16), (uint32_t)l[2] | ((uint32_t)l[3] << 16)};
  }
}

}  // namespace

hipError_t launch_gemm_dec(const WaveGemmArgs& g, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0 || g.K <= 0 || g.ksplit < 1 || g.N % 16) return hipErrorInvalidValue;
  if (g.K % 32 || (g.nsplit != 1 && g.nsplit != 2)) return hipErrorInvalidValue;
  const int steps = g.K / 32;
  if (steps % g.ksplit || steps / g.ksplit > DEC_MAX_KSTEPS) return hipErrorInvalidValue;
  if (g.out == OUT_PARTIAL && g.part_stride <= 0) return hipErrorInvalidValue;
  if (g.N % 4) return hipErrorInvalidValue;  // 4 consecutive output columns per lane
  static bool attr = false;
  if (!attr) {
    for (const void* f : {(const void*)gemm_dec_kernel<4>, (const void*)gemm_dec_kernel<16>}) {
      const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, DEC_MAX_KSTEPS * 4 * 2048);
      if (e != hipSuccess) return e;
    }
    attr = true;
  }
  // few k-steps per block: 4 waves (one per quadrant, no reduction, up to 8 blocks per CU);
  // otherwise 16 waves so that enough waves issue the LDS-DMA of the larger slice
  const int nks = steps / g.ksplit, nops = g.nsplit + 1 + (g.W_lo ? 1 : 0);
  dim3 grid((g.N + 31) / 32, (g.M + 31) / 32, g.batch * g.ksplit);
  if (nks <= 4) {
    hipLaunchKernelGGL(gemm_dec_kernel<4>, grid, dim3(256), nks * nops * 2048, s, g);
  } else {
    const int lds = std::max(nks * nops * 2048, DEC_RED_BYTES);
    hipLaunchKernelGGL(gemm_dec_kernel<16>, grid, dim3(1024), lds, s, g);
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Chained per-head GEMMs (launch_chain_dec): block = (128 output columns, 32 rows, head).
// Everything it needs is DMA'd to LDS up front (X 32 x 512 planes, W1_h 64 x 512, W2 chunk
// 128 x 64: 152 KiB for bf16x2) by all 16 waves, one wait.  Phase 1: Y (32 x 64) over K = 512,
// 8 output tiles x 2 k-groups, reduced through LDS, + b1, split into bf16 planes written back to
// LDS in the MFMA operand layout.  Phase 2: O (32 x 128) = Y W2^T, one 16 x 16 tile per wave.
// Layouts as gemm_dec_kernel: per k-step rows of 64 B, chunk c of row r at c ^ ((r >> 2) & 3).
namespace {

__global__ __launch_bounds__(1024) void chain_dec_kernel(ChainArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 128, m0 = blockIdx.y * 32, h = blockIdx.z;
  const int ns = p.nsplit;
  // LDS map (bytes): X [16 ks][ns][32 rows][64 B] | W1 [16 ks][64 rows][64 B] | W2 [2 ks][128][64 B]
  const int XS = ns * 2048;  // X bytes per k-step
  char* sx = smem;
  char* sw1 = smem + 16 * XS;
  char* sw2 = sw1 + 16 * 4096;
  const bf16_t* X = p.X + (long)h * p.x_hstride;
  const bf16_t* W1 = p.W1 + (long)h * 64 * 512;
  const bf16_t* W2 = p.W2 + (long)h * p.w2_hstride;
  const int lrow = lane >> 2, lchunk = (lane & 3) ^ ((lrow >> 2) & 3);
  // DMA: X 16 ks x ns x 2 halves, W1 16 ks x 4 quarters, W2 2 ks x 8 eighths (1 KiB each)
  const int nx = 16 * ns * 2, nw1 = 64, nq = nx + nw1 + 16;
  for (int q = wave; q < nq; q += 16) {
    const bf16_t* src;
    char* dst;
    if (q < nx) {
      const int ks = q / (2 * ns), rem = q - ks * 2 * ns, pl = rem >> 1, half = rem & 1;
      const int r = half * 16 + lrow;
      src = X + pl * p.x_lo + (long)min(m0 + r, p.M - 1) * p.ldx + ks * 32 + lchunk * 8;
      dst = sx + ks * XS + pl * 2048 + half * 1024;
    } else if (q < nx + nw1) {
      const int i = q - nx, ks = i >> 2, qu = i & 3;
      src = W1 + (long)(qu * 16 + lrow) * 512 + ks * 32 + lchunk * 8;
      dst = sw1 + ks * 4096 + qu * 1024;
    } else {
      const int i = q - nx - nw1, ks = i >> 3, e = i & 7;
      src = W2 + (long)(n0 + e * 16 + lrow) * p.ldw2 + ks * 32 + lchunk * 8;
      dst = sw2 + ks * 8192 + e * 1024;
    }
    __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)src, (LDS_AS void*)dst, 16, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int fr = lane & 15, fq = lane >> 4;
  const int sw = (fq ^ ((fr >> 2) & 3)) * 16;
  // phase 1: wave -> tile (tm = t >> 2: rows, tn = t & 3: Y columns) and k-group kg (ks parity)
  const int t1 = wave & 7, kg = wave >> 3, tm = t1 >> 2, tn = t1 & 3;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int ks = kg; ks < 16; ks += 2) {
    const bf16x8 b = *(const bf16x8*)(sw1 + ks * 4096 + (tn * 16 + fr) * 64 + sw);
    const char* xa = sx + ks * XS + (tm * 16 + fr) * 64 + sw;
    acc = mfma16(b, *(const bf16x8*)xa, acc);  // lane: row fr, Y columns 4 fq + r
    if (ns == 2) acc = mfma16(b, *(const bf16x8*)(xa + 2048), acc);
  }
  __syncthreads();  // X / W1 no longer read: reuse the X area
  f32x4* red = (f32x4*)smem;
  if (kg) red[t1 * 64 + lane] = acc;
  __syncthreads();
  char* sy = smem + 8 * 1024 * 2;  // Y planes [2 ks][ns][32 rows][64 B], after the reduction area
  if (!kg) {
    acc += red[t1 * 64 + lane];
    const int col = tn * 16 + 4 * fq;  // Y column within the head (0..63)
    acc += *(const f32x4*)(p.b1 + h * 64 + col);
    bf16_t hv[4], lv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) split_bf(acc[r], hv[r], lv[r]);
    const int m = tm * 16 + fr, ks = col >> 5, c = (col & 31) >> 3;
    char* dst = sy + ks * XS + m * 64 + ((c ^ ((m >> 2) & 3)) << 4) + (col & 7) * 2;
    *(u32x2*)dst = (u32x2){(uint32_t)hv[0] | ((uint32_t)hv[1] << 16), (uint32_t)hv[2] | ((uint32_t)hv[3] << 16)};
    if (ns == 2)
      *(u32x2*)(dst + 2048) =
          (u32x2){(uint32_t)lv[0] | ((uint32_t)lv[1] << 16), (uint32_t)lv[2] | ((uint32_t)lv[3] << 16)};
  }
  __syncthreads();
  // phase 2: wave -> output tile (rows tm2 = wave >> 3, columns tn2 = wave & 7), K = 64
  const int tm2 = wave >> 3, tn2 = wave & 7;
  f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const bf16x8 b = *(const bf16x8*)(sw2 + ks * 8192 + (tn2 * 16 + fr) * 64 + sw);
    const char* ya = sy + ks * XS + (tm2 * 16 + fr) * 64 + sw;
    o = mfma16(b, *(const bf16x8*)ya, o);
    if (ns == 2) o = mfma16(b, *(const bf16x8*)(ya + 2048), o);
  }
  const int row = m0 + tm2 * 16 + fr;
  if (row >= p.M) return;
  const int col = n0 + tn2 * 16 + 4 * fq;
  if (p.out == OUT_PARTIAL) {
    *(f32x4*)((float*)p.C + (long)h * p.part_stride + (long)row * p.ldc + col) = o;
  } else {
    bf16_t hv[4], lv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) split_bf(o[r], hv[r], lv[r]);
    bf16_t* dst = (bf16_t*)p.C + (long)row * p.ldc + (long)h * p.c_hstride + col;
    *(u32x2*)dst = (u32x2){(uint32_t)hv[0] | ((uint32_t)hv[1] << 16), (uint32_t)hv[2] | ((uint32_t)hv[3] << 16)};
    if (ns == 2)
      *(u32x2*)(dst + p.c_lo) =
          (u32x2){(uint32_t)lv[0] | ((uint32_t)lv[1] << 16), (uint32_t)lv[2] | ((uint32_t)lv[3] << 16)};
  }
}

}  // namespace

hipError_t launch_chain_dec(const ChainArgs& a, hipStream_t s) {
  if (a.M <= 0 || a.N2 % 128 || a.H <= 0 || (a.nsplit != 1 && a.nsplit != 2)) return hipErrorInvalidValue;
  if (a.out != OUT_PARTIAL && a.out != OUT_SPLIT) return hipErrorInvalidValue;
  const int lds = 16 * a.nsplit * 2048 + 16 * 4096 + 2 * 8192;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)chain_dec_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             16 * 2 * 2048 + 16 * 4096 + 2 * 8192);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL(chain_dec_kernel, dim3(a.N2 / 128, (a.M + 31) / 32, a.H), dim3(1024), lds, s, a);
  return hipGetLastError();
}

hipError_t launch_gemm_256_(const GemmArgs& g, hipStream_t s);
hipError_t launch_gemm_256(const GemmArgs& g0, hipStream_t s) {
  // ICAP_GEMM_GROUP: tile raster of the bf16 encoder GEMM (0 = row-band major)
  static const int group = std::max(0, icap_knob("ICAP_GEMM_GROUP", 0));
  GemmArgs g = g0;
  if (!g.raster_group) g.raster_group = group;
  return launch_gemm_256_(g, s);
}

// Product forms of the 256-wide encoder GEMM.  The measured-and-rejected forms (8-phase template, staging-only
// ablations, 64-row and 64-deep two-block forms, tail split, ping-pong fp16 k-loop, ...) live in gemm_tools.hip,
// which only the tools build compiles; launch_gemm_256_tools takes the launch when one of its knobs asks for it.
namespace {

// The bf16 / bf16x2 encoder and trunk GEMMs, and (F16) the ICAP_PREC_F16 Grid trunk's convolutions on fp16 planes.
// EPC: the convolution epilogue (GemmArgs::scale set), compiled into its own kernels.
template <bool F16, bool EPC>
hipError_t run_256(const GemmArgs& g, hipStream_t s) {
  static bool attr = false;
  constexpr int lds2 = 3 * 3 * 256 * 32 * 2, lds1 = 4 * 2 * 256 * 32 * 2;
  if (!attr) {
    hipError_t e = hipSuccess;
    for (const void* f : {(const void*)gemm_256_kernel<2, 16, 0, 0, 256, 0, 32, 0, F16, EPC>,
                          (const void*)gemm_256_kernel<2, 16, 0, 1, 256, 0, 32, 0, F16, EPC>})
      if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds2);
    for (const void* f : {(const void*)gemm_256_kernel<1, 16, 0, 0, 256, 0, 32, 0, F16, EPC>,
                          (const void*)gemm_256_kernel<1, 16, 0, 1, 256, 0, 32, 0, F16, EPC>})
      if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds1);
    if (e != hipSuccess) return e;
    attr = true;
  }
  if (g.cv && g.cv != 1) return hipErrorInvalidValue;
  if (g.split_slots) return hipErrorNotSupported;  // the tail split is a tools-build form
  // 128 x 256 tiles, 2-stage ring, 2 blocks per CU for K >= 128: ViT 42.9 -> 41.8 ms/step (MLP-out's 591 tiles
  // become 1182: 4.6 instead of 2.3 rounds), trunk conv3 203 -> 177 us; at K = 64 the 3-stage 256 x 256 ring
  // stays ahead (tools/halfk_sweep.sh; round 3, tools/r3_trunk_sweep.sh: still so for the fp16 trunk)
  // ICAP_GEMM_TALL_MIN_K (tools): the smallest K of the two-block form
  static const int tall_min_k = icap_knob("ICAP_GEMM_TALL_MIN_K", 128);
  // the Grid encoder tail (M = B x 49 = 12544 at B = 256, bf16x2): 64 x 256 tiles of 4 waves, three blocks per CU - its
  // 196-tile GEMMs (out-proj, FFN-2, projection) otherwise leave a quarter of the CUs idle (round 3, tools/r3_ab.sh +
  // tools/r3_tail_trace.sh: projection 87.5 -> 76 us, QKV 72 -> 64, out-proj 33 -> 29, FFN-1 87 -> 84, FFN-2 82 -> 71;
  // at the ViT's M = 50432 the 128-row form stays ahead, round 1)
  if (tall_min_k && g.K >= tall_min_k && !F16 && !g.cv && g.M <= 16384) {
    const int nwgq = (g.N / 256) * ((g.M + 63) / 64);
    constexpr int ldsq = 2 * (2 * 64 * 32 * 2 + 256 * 32 * 2), ldsq1 = 2 * (64 * 32 * 2 + 256 * 32 * 2);
    if (g.nsplit == 2) hipLaunchKernelGGL((gemm_256_kernel<2, 4, 0, 0, 64, 2, 32, 0, false, EPC>), dim3(nwgq), dim3(256), ldsq, s, g);
    else hipLaunchKernelGGL((gemm_256_kernel<1, 4, 0, 0, 64, 2, 32, 0, false, EPC>), dim3(nwgq), dim3(256), ldsq1, s, g);
    return hipGetLastError();
  }
  if (tall_min_k && g.K >= tall_min_k) {
    const int nwgh = (g.N / 256) * ((g.M + 127) / 128);
    constexpr int ldsh = 2 * (2 * 128 * 32 * 2 + 256 * 32 * 2), ldsh1 = 2 * (128 * 32 * 2 + 256 * 32 * 2);
    if (g.nsplit == 2) {
      if (g.cv) hipLaunchKernelGGL((gemm_256_kernel<2, 8, 0, 1, 128, 2, 32, 0, F16, EPC>), dim3(nwgh), dim3(512), ldsh, s, g);
      else hipLaunchKernelGGL((gemm_256_kernel<2, 8, 0, 0, 128, 2, 32, 0, F16, EPC>), dim3(nwgh), dim3(512), ldsh, s, g);
    } else {
      if (g.cv) hipLaunchKernelGGL((gemm_256_kernel<1, 8, 0, 1, 128, 2, 32, 0, F16, EPC>), dim3(nwgh), dim3(512), ldsh1, s, g);
      else hipLaunchKernelGGL((gemm_256_kernel<1, 8, 0, 0, 128, 2, 32, 0, F16, EPC>), dim3(nwgh), dim3(512), ldsh1, s, g);
    }
    return hipGetLastError();
  }
  // K < 128: 256 x 256 tiles, 16 waves, 3-stage (two planes) / 4-stage ring
  const int nwg = (g.N / 256) * ((g.M + 255) / 256);
  if (g.nsplit == 2) {
    if (g.cv) hipLaunchKernelGGL((gemm_256_kernel<2, 16, 0, 1, 256, 0, 32, 0, F16, EPC>), dim3(nwg), dim3(1024), lds2, s, g);
    else hipLaunchKernelGGL((gemm_256_kernel<2, 16, 0, 0, 256, 0, 32, 0, F16, EPC>), dim3(nwg), dim3(1024), lds2, s, g);
  } else {
    if (g.cv) hipLaunchKernelGGL((gemm_256_kernel<1, 16, 0, 1, 256, 0, 32, 0, F16, EPC>), dim3(nwg), dim3(1024), lds1, s, g);
    else hipLaunchKernelGGL((gemm_256_kernel<1, 16, 0, 0, 256, 0, 32, 0, F16, EPC>), dim3(nwg), dim3(1024), lds1, s, g);
  }
  return hipGetLastError();
}

}  // namespace

// Narrow trunk convolutions (N = 64 / 128: the Grid trunk's layer1-2 conv1 / conv2 on fp16 planes): the 256-family
// k-loop with 64-deep stages on BM x BN block tiles of 64-column wave tiles, NST-stage ring.
namespace {

template <int BM, int BN, int NST, int CONV, bool EPC>
hipError_t run_narrow_(const GemmArgs& g, hipStream_t s) {
  constexpr int lds = NST * (BM * 64 * 2 + BN * 64 * 2);
  static bool attr = false;
  if (!attr && lds > 65536) {
    const hipError_t e = hipFuncSetAttribute((const void*)gemm_256_kernel<1, 8, 0, CONV, BM, NST, 64, 0, true, EPC, BN>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int nwg = (g.N / BN) * ((g.M + BM - 1) / BM);
  static const int pre = icap_knob("ICAP_CONV_PRE", 1);
  GemmArgs ga = g;
  ga.no_pre = !pre;
  hipLaunchKernelGGL((gemm_256_kernel<1, 8, 0, CONV, BM, NST, 64, 0, true, EPC, BN>), dim3(nwg), dim3(512), lds, s, ga);
  return hipGetLastError();
}

template <int BM, int BN, int NST>
hipError_t run_narrow(const GemmArgs& g, hipStream_t s) {
  const bool epc = g.out == OUT_SPLIT && g.bias && (g.epi == EPI_NONE || g.epi == EPI_RELU);
  if (g.cv == 2) return epc ? run_narrow_<BM, BN, NST, 2, true>(g, s) : run_narrow_<BM, BN, NST, 2, false>(g, s);
  if (g.cv == 1) return epc ? run_narrow_<BM, BN, NST, 1, true>(g, s) : run_narrow_<BM, BN, NST, 1, false>(g, s);
  return epc ? run_narrow_<BM, BN, NST, 0, true>(g, s) : run_narrow_<BM, BN, NST, 0, false>(g, s);
}

}  // namespace

// The fp16 trunk's narrow convolutions: the stem (N = 64 on the bordered NHWC4 image) and layer1-2's conv1 / conv2.
bool gemm_narrow_ok(const GemmArgs& g) {
  return g.f16 && g.scale && (g.N == 64 || g.N == 128) && g.K % 64 == 0 && g.batch == 1 && g.nsplit == 1 &&
         !g.addend && !g.rm_group && !g.hm_n && !g.split_slots;
}

// form 1 (default; round 3, tools/r3_narrow.sh, per launch at B = 256 against the 64 x 64 kernel): N = 64 on 256 x 64
// tiles (l1c1 162 -> 114 us, l1c2 197 -> 114), N = 128 on 128 x 128 tiles (l2c1 177 -> 102, l2c2 168 -> 97), 2-stage
// rings, two blocks per CU.  Tools forms: 2 = 128-row tiles for N = 64 too (3-stage; l1c2 137), 3 = 256 x 64 with a
// 3-stage ring (l1c2 155), 4 = 256-row tiles for N = 128 (l2c1 108, l2c2 116).
// The fp16 trunk's N % 256 == 0 convolutions on 64 x 256 tiles of the 64-deep k-loop (2-stage ring, 80 KiB: two blocks
// per CU) instead of the 128 x 256 / 256 x 256 forms, where the epilogue's HBM traffic or the tile count rules: the
// residual conv3 (l1c3 349 -> 288 us, l2c3 172 -> 161, l3c3 178 -> 154, l4c3 108 -> 93), two-plane outputs (l3ds 165 ->
// 134), K < 128 (l1ds 201 -> 183) and launches of fewer 128-row tiles than CUs (l4c2 121 -> 87); the compute-heavy rest
// stays (l3c2 82 -> 88, l2ds 141 -> 152 on 64-row tiles).  Round 3, tools/r3_c3.sh.  ICAP_GEMM_C3 (tools): 0 = off,
// 1 = 64 x 256 for the residual convolutions only, 2 = 128 x 256 2-stage, 3 = 64 x 256 3-stage, +10 = every one.
bool gemm_c3_form(const GemmArgs& g, int cus, int* form) {
  static const int knob = icap_knob("ICAP_GEMM_C3", -1);
  if (!knob || !g.f16 || !g.scale || g.N % 256 || g.K % 64 || g.batch != 1 || g.nsplit != 1 || g.cv == 2 ||
      g.addend || g.rm_group || g.hm_n || g.split_slots)
    return false;
  const long tiles128 = (long)(g.N / 256) * ((g.M + 127) / 128);
  // (layer3 conv1 - K = 1024, 392 tiles of 128 rows - measured slower on these tiles: 62 -> 68 us, tools/r3_c3b.sh)
  const bool pick = knob < 0 ? (g.res || g.c_planes == 2 || g.K < 128 || tiles128 < cus) : (knob >= 10 || g.res);
  *form = knob < 0 ? 1 : knob % 10;
  return pick;
}

hipError_t launch_gemm_c3(const GemmArgs& g, hipStream_t s, int form) {
  return form == 2 ? run_narrow<128, 256, 2>(g, s) : form == 3 ? run_narrow<64, 256, 3>(g, s) : run_narrow<64, 256, 2>(g, s);
}

hipError_t launch_gemm_narrow(const GemmArgs& g, hipStream_t s, int form) {
  if (g.N == 128) return form == 4 ? run_narrow<256, 128, 2>(g, s) : run_narrow<128, 128, 2>(g, s);
  if (form == 2) return run_narrow<128, 64, 3>(g, s);
  if (form == 3) return run_narrow<256, 64, 3>(g, s);
  return run_narrow<256, 64, 2>(g, s);
}

hipError_t launch_gemm_256_(const GemmArgs& g, hipStream_t s) {
  if (g.M <= 0 || g.N % 256 || g.K % 32 || g.batch != 1 || (g.nsplit != 1 && g.nsplit != 2))
    return hipErrorInvalidValue;
  const long last_row = g.rm_group ? (long)((g.M - 1) / g.rm_group) * g.rm_stride + g.rm_off + g.rm_group : g.M;
  if (last_row * g.ldc >= (1L << 31)) return hipErrorInvalidValue;  // epilogue uses 32-bit row offsets
  // f16 without a BN scale: the ViT encoder's single-plane GEMMs; with one: the Grid trunk's convolutions
  const bool vit16 = g.f16 && !g.scale;
  if (vit16 && (g.nsplit != 1 || g.cv || g.res || (g.out == OUT_SPLIT && g.c_planes != 1) || g.K < 128))
    return hipErrorInvalidValue;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      return hipErrorInvalidValue;
    hipError_t e = hipSuccess;
    for (const void* f : {(const void*)gemm_f16p_kernel<1>, (const void*)gemm_f16p_kernel<2>})
      if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, F16P_LDS_SO);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void*)gemm_f16p_kernel<2, 0, 224>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              2 * (224 * 128 + 256 * 128) + 2048);
    if (e != hipSuccess) {
      cus = 0;
      return e;
    }
  }
#ifdef ICAP_TOOLS
  if (!g.f16 || vit16) {
    hipError_t e = hipSuccess;
    if (launch_gemm_256_tools(g, s, cus, &e)) return e;
  }
#endif
  if (vit16) {  // fp16 single plane (ICAP_PREC_F16 encoder)
    if (gemm_f16_persistent(g)) {
      // store-only epilogues with whole 256-row bands (the ViT QKV and MLP-1 GEMMs): the persistent counted-seam
      // form (QKV 305 -> 265 us, MLP-1 423 -> 342 us at B = 256, tools/f16_forms_r2.sh); the residual GEMMs on
      // 224-row tiles (678 tiles = 2.65 per CU at N = 768 instead of 591 = 2.3)
      const int blocks = g.max_grid > 0 ? std::min(g.max_grid, cus) : cus;
#if ICAP_F16H
      if (f16h_ok(g)) return launch_f16h(g, s, blocks);
#endif
      if (g.out == OUT_F32_RESID) {
        const int tiles224 = (g.N / 256) * ((g.M + 223) / 224);
        hipLaunchKernelGGL((gemm_f16p_kernel<2, 0, 224>), dim3(std::min(tiles224, blocks)), dim3(512),
                           2 * (224 * 128 + 256 * 128) + 2048, s, g);
      } else {
        const int tiles = (g.N / 256) * ((g.M + 255) / 256);
        hipLaunchKernelGGL(gemm_f16p_kernel<1>, dim3(std::min(tiles, blocks)), dim3(512), F16P_LDS_SO, s, g);
      }
      return hipGetLastError();
    }
    // the remaining fp16 GEMMs (patch embedding, projection): 128 x 256 tiles, 2-stage ring, 2 blocks per CU
    const int nwgh = (g.N / 256) * ((g.M + 127) / 128);
    constexpr int ldsh1 = 2 * (128 * 32 * 2 + 256 * 32 * 2);
    hipLaunchKernelGGL((gemm_256_kernel<1, 8, 0, 0, 128, 2, 32, 0, true>), dim3(nwgh), dim3(512), ldsh1, s, g);
    return hipGetLastError();
  }
  // the fp16 trunk's 1x1 convolutions with K <= 256 and N >= 128 (the residual conv3, the layer1-2 downsamples):
  // W-stationary persistent blocks (conv_rmw.hip; round 3, tools/r3_rmw.sh: l1c3 290 -> 168 us, l2c3 163 -> 100, l3c3
  // 158 -> 99, l1ds 188 -> 162, l2ds 154 -> 128; Grid 9819-9935 -> 10829-10891 captions/s).  ICAP_CONV_RMW (tools):
  // 0 = the 64 x 256 tiles below, 1 = the residual convolutions only
  static const int rmw = icap_knob("ICAP_CONV_RMW", 2);
  if (rmw && conv_rmw_ok(g) && (g.res || rmw == 2)) return launch_conv_rmw(g, s, cus);
  int c3 = 0;
  if (gemm_c3_form(g, cus, &c3)) return launch_gemm_c3(g, s, c3);
  if (g.scale && !g.addend && !g.rm_group && !g.hm_n && g.out == OUT_SPLIT && g.bias &&
      (g.epi == EPI_NONE || g.epi == EPI_RELU))  // the trunk convolutions' epilogue form
    return g.f16 ? run_256<true, true>(g, s) : run_256<false, true>(g, s);
  return g.f16 ? run_256<true, false>(g, s) : run_256<false, false>(g, s);
}

// ---------------------------------------------------------------------------------------------
// int8 two-slice encoder GEMM for the LayerNorm-fed projections (ViT QKV, MLP-1, final projection
// in ICAP_PREC_I8X2).  Both operands are 16-bit fixed point under a per-row scale, held as two int8
// slices: v = s (256 v1 + v2), v1 in [-127, 127], v2 in [-128, 127] (the activation slices come from
// layernorm_i8_kernel, the weight slices from pack_i8_rows_kernel).  The product is
//   A.W^T = s_a s_w (65536 A1.W1 + 256 (A1.W2 + A2.W1) + A2.W2)
// with the last term (<= 2^-16 of the first, below the representation's own rounding) dropped, so
// three v_mfma_i32_16x16x64_i8 per 64-deep k-step and 16x16 tile; int32 accumulation is exact
// (|A1.W1| <= K 127^2 < 2^31 for K < 133k).  Against the bf16x2 form (A as hi/lo bf16 planes, W
// bf16: 6 staged bytes per k per row pair, two bf16 MFMAs per 32-deep k-step) this stages 4 bytes per k
// and does 3/4 of the MFMA cycles (the i8 16x16x64 MFMA takes the cycles of bf16 16x16x32).
// Operand row images are [K/64][2][64]: a 64-deep stage of one row is ONE full 128-B line holding
// both slices (half the L2 requests of 64-B row segments).
// Block tile 128 x 256 (8 waves as 2 x 4, each 64 x 64 = 4 x 4 MFMA tiles with a high and a mid int32
// accumulator set: 128 accumulator registers, so one block per CU), stages of two operand tiles
// (A: 128 rows, W: 256 rows, 128 B each; 16-B chunk c of row r at c ^ ((r >> 1) & 7)) in a 3-stage LDS ring
// (144 KiB) filled by global_load_lds, counted vmcnt + raw barrier, XCD remap.  The same LDS byte
// positions feed the A and B operands, so the k labelling inside the MFMA does not matter.
namespace {

typedef int i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ i32x4 mfma_i8(i32x4 a, i32x4 b, i32x4 c) {
  return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
}

// BNT = 128: 128 x 128 tiles of 4 waves (2 x 2), a 2-stage 64 KiB ring and two blocks per CU, so one
// block's epilogue overlaps the other's k-loop (ICAP_I8_TILE=128).
// KSC = 1: A carries one scale per (row, 128-deep k block) (a_kscale[M][K/128]: the block-scaled GELU
// output of MLP-1, whose producer tiles do not own whole rows).  The int32 accumulators then run over
// the two k-steps of a block only and are folded into fp32 accumulators at its end,
// acc += 256 s_a[row][kb] (256 hi + mid) - 256 hi + mid is exact in int32 for a 128-deep block
// (|.| <= 128 (256 127^2 + 2 127 128) < 2^30) - before the column scale s_w in the epilogue.
template <int NSTAGE, int NOMFMA = 0, int BNT = 256, int KSC = 0>
__global__ __launch_bounds__(BNT * 2, BNT == 256 ? 1 : 2) void gemm_i8_kernel(GemmArgs p) {
  static_assert(!KSC || NSTAGE == 2, "block scales are loaded one k-step ahead under the ring's vmcnt(0)");
  constexpr int NW = BNT / 32, BM = 128, BN = BNT, WM = 64, WN = 64, TM = WM / 16, TN = WN / 16;
  constexpr int OPB = BM * 128, OPBW = BN * 128;  // bytes per A / W tile per stage (both slices)
  constexpr int STAGE = OPB + OPBW;               // 48 KiB
  constexpr int IPW = OPB / 1024 / NW, IPWW = OPBW / 1024 / NW;
  constexpr int PER_STAGE = IPW + IPWW;           // DMA instructions per wave per stage
  static_assert(IPW >= 1 && IPWW >= 1, "tile / wave shape");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / (NW / 2), wn = wave % (NW / 2);
  const int nbn = p.N / BN, nbm = (p.M + BM - 1) / BM, nwg = nbn * nbm;
  const int orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  int bm, bn;
  if (p.raster_group > 0) {  // groups of raster_group row bands, column tiles outermost inside a group
    const int G = p.raster_group, grp = wg / (G * nbn), gm = min(G, nbm - grp * G), idx = wg - grp * G * nbn;
    bn = idx / gm;
    bm = grp * G + (idx - bn * gm);
  } else {
    bm = wg / nbn;
    bn = wg - bm * nbn;
  }
  const int m0 = bm * BM, n0 = bn * BN;
  const int M = p.M, nk = p.K / 64;
  const long ld = 2L * p.K;  // row image bytes

  // one DMA instruction = 8 rows x 128 B; lane -> row lane >> 3, LDS chunk lane & 7 holding source
  // chunk (lane & 7) ^ (row & 7) (instruction bases are multiples of 8 rows)
  // LDS chunk c of row r holds source chunk c ^ ((r >> 1) & 7): a ds_read_b128 pass (16 rows at 128-B
  // stride, one logical chunk) then covers all 64 banks - with c ^ (r & 7) rows r and r + 8 shared
  // banks (PMC: 6.1 M conflict cycles against 9.9 M LDS-active per launch).  Instruction q covers rows
  // 8q..8q+7, so (r >> 1) & 7 = 4 (q & 1) + (lane >> 4); IPW and IPWW are even, so q & 1 = i & 1.
  static_assert(IPW % 2 == 0 && IPWW % 2 == 0, "swizzle parity");
  const int sch[2] = {((lane & 7) ^ (lane >> 4)) * 16, ((lane & 7) ^ (4 + (lane >> 4))) * 16};
  const char* a_src[IPW];
#pragma unroll
  for (int i = 0; i < IPW; ++i)
    a_src[i] = (const char*)p.A + (long)min(m0 + (wave * IPW + i) * 8 + (lane >> 3), M - 1) * ld + sch[i & 1];
  const char* b_src = (const char*)p.W + (long)(n0 + wave * IPWW * 8 + (lane >> 3)) * ld;
  const long b_step = 8 * ld;
  auto stage = [&](int kt, int buf) {
    const int kin = kt * 128;
    char* s0 = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < IPW; ++i)
      __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)(a_src[i] + kin),
                                       (LDS_AS void*)(s0 + (wave * IPW + i) * 1024), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < IPWW; ++i)
      __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)(b_src + i * b_step + sch[i & 1] + kin),
                                       (LDS_AS void*)(s0 + OPB + (wave * IPWW + i) * 1024), 16, 0, 0);
  };

  i32x4 ah[TM][TN], am[TM][TN];
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      ah[i][j] = am[i][j] = (i32x4){0, 0, 0, 0};
      if (KSC) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }

  const int fr = lane & 15, fq = lane >> 4;
  // KSC: this lane's A rows (one per MFMA row tile) and their block scales for the current k-step
  const float* ksrc[TM];
  float skc[TM];
  if (KSC) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      ksrc[i] = p.a_kscale + (long)min(m0 + wm * WM + i * 16 + fr, M - 1) * (nk >> 1);
      skc[i] = ksrc[i][0];
    }
  }
  const int f1 = fr * 128 + ((fq ^ ((fr >> 1) & 7)) << 4), f2 = fr * 128 + (((4 + fq) ^ ((fr >> 1) & 7)) << 4);
#pragma unroll
  for (int s = 0; s < NSTAGE - 1; ++s)
    if (s < nk) stage(s, s);
  for (int kt = 0; kt < nk; ++kt) {
    const int younger = min(NSTAGE - 2, nk - 1 - kt);
    // lgkmcnt(0): this wave's LDS reads of the slot refilled below are complete before the barrier
    if (younger >= 2) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * PER_STAGE) : "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PER_STAGE) : "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + NSTAGE - 1 < nk) stage(kt + NSTAGE - 1, (kt + NSTAGE - 1) % NSTAGE);
    float skn[TM];
    if (KSC) {  // next k-step's block scales (complete at the next iteration's vmcnt(0))
#pragma unroll
      for (int i = 0; i < TM; ++i) skn[i] = ksrc[i][min((kt >> 1) + 1, (nk >> 1) - 1)];
    }
    const char* s0 = smem + (kt % NSTAGE) * STAGE;
    i32x4 w1[TN], w2[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      w1[j] = *(const i32x4*)(s0 + OPB + (wn * WN + j * 16) * 128 + f1);
      w2[j] = *(const i32x4*)(s0 + OPB + (wn * WN + j * 16) * 128 + f2);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const i32x4 a1 = *(const i32x4*)(s0 + (wm * WM + i * 16) * 128 + f1);
      const i32x4 a2 = *(const i32x4*)(s0 + (wm * WM + i * 16) * 128 + f2);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if (NOMFMA) {  // measurement variant (ICAP_I8_NOMFMA): staging + fragment reads only
          asm volatile("" ::"v"(a1), "v"(a2), "v"(w1[j]), "v"(w2[j]));
          continue;
        }
        if (KSC) {
          const i32x4 z = {0, 0, 0, 0};
          const bool first = !(kt & 1);
          ah[i][j] = mfma_i8(w1[j], a1, first ? z : ah[i][j]);
          am[i][j] = mfma_i8(w2[j], a1, first ? z : am[i][j]);
          am[i][j] = mfma_i8(w1[j], a2, am[i][j]);
          if (!first) {
            const float s8 = skc[i] * 256.f;
            const i32x4 t = (ah[i][j] << 8) + am[i][j];
            const f32x4 tf = {(float)t[0], (float)t[1], (float)t[2], (float)t[3]};
            acc[i][j] = __builtin_elementwise_fma(tf, (f32x4)s8, acc[i][j]);
          }
          continue;
        }
        ah[i][j] = mfma_i8(w1[j], a1, ah[i][j]);  // D = W.A^T, as the bf16 kernel
        am[i][j] = mfma_i8(w2[j], a1, am[i][j]);
        am[i][j] = mfma_i8(w1[j], a2, am[i][j]);
      }
    }
    if (KSC && (kt & 1)) {
#pragma unroll
      for (int i = 0; i < TM; ++i) skc[i] = skn[i];
    }
  }

  const int mb = m0 + wm * WM, nb = n0 + wn * WN;
  if (NOMFMA == 2) return;  // measurement: staging only, no epilogue
  f32x4 ws[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) ws[j] = *(const f32x4*)(p.w_scale + nb + j * 16 + 4 * fq);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const float sa = KSC ? 1.f : p.a_scale[min(mb + i * 16 + fr, M - 1)];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        acc[i][j][e] = KSC ? acc[i][j][e] * ws[j][e]
                           : fmaf((float)ah[i][j][e], 65536.f, (float)am[i][j][e] * 256.f) * (sa * ws[j][e]);
  }
  if (BNT == 128 && p.out == OUT_I8K) {
    // Block-scaled int8 two-slice output: a tile's 128 columns of a row are one 128-deep k block of the
    // consumer; the block maximum is a 16-value lane max, two xor shuffles over the 4 lanes (fq) holding
    // the row in a wave, and the max of the two wave columns through LDS.  The tile's row image
    // (2 x 128 B = 256 contiguous bytes of the [M][N/64][2][64] output row) is assembled in LDS, then
    // stored as full 16-B chunks.
    constexpr int PITCH8 = BN * 2 + 16;  // 272 B: rows fr of a 4-B column group hit distinct banks
    static_assert(BM * PITCH8 + 2 * BM * 4 <= NSTAGE * STAGE, "epilogue tile exceeds the ring");
    float* wmax = (float*)(smem + BM * PITCH8);  // [2 wave columns][BM rows]
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if (p.bias) acc[i][j] += *(const f32x4*)(p.bias + nb + j * 16 + 4 * fq);
        if (p.epi == EPI_GELU) {
          const f32x2 g0 = gelu_erf_fast2(acc[i][j].xy), g1 = gelu_erf_fast2(acc[i][j].zw);
          acc[i][j] = (f32x4){g0.x, g0.y, g1.x, g1.y};
        } else if (p.epi == EPI_RELU) {
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][j][e] = fmaxf(acc[i][j][e], 0.f);
        }
      }
    __syncthreads();  // every wave is past its last ring read
    const int nkb = p.N / 128;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      float mx = 0.f;
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) mx = fmaxf(mx, fabsf(acc[i][j][e]));
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      if (fq == 0) wmax[wn * BM + wm * WM + i * 16 + fr] = mx;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm * WM + i * 16 + fr;
      const float mx = fmaxf(wmax[row], wmax[BM + row]);
      const float inv = mx > 0.f ? 32639.f / mx : 0.f;
      if (wn == 0 && fq == 0 && m0 + row < M) p.c_kscale[(long)(m0 + row) * nkb + n0 / 128] = mx / 32639.f;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const float y[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        uint32_t hi, lo;
        q2_pack4(y, inv, hi, lo);
        char* d = smem + row * PITCH8 + wn * 128 + j * 16 + 4 * fq;
        *(uint32_t*)d = hi;
        *(uint32_t*)(d + 64) = lo;
      }
    }
    __syncthreads();
    char* C8 = (char*)p.C + (long)n0 * 2;
#pragma unroll 4
    for (int c = tid; c < BM * (BN * 2 / 16); c += NW * 64) {
      const int row = c / (BN * 2 / 16), ch = c % (BN * 2 / 16), m = m0 + row;
      if (m >= M) continue;
      *(u32x4*)(C8 + (long)m * 2 * p.N + ch * 16) = *(const u32x4*)(smem + row * PITCH8 + ch * 16);
    }
    return;
  }
  if (p.out == OUT_SPLIT && p.c_planes == 2 && !p.rm_group && !p.addend) {
    // Split-plane output staged through LDS: the MFMA layout gives each lane 4 columns of one row
    // (32-B row segments per wave store); transposed through LDS every lane stores 16 B and a wave
    // covers whole 512-B rows (full 128-B lines; one head block = one line in the head-major form).
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if (p.bias) {
          const f32x4 bv = *(const f32x4*)(p.bias + nb + j * 16 + 4 * fq);
          acc[i][j] += bv;
        }
        if (p.epi == EPI_GELU) {  // packed: the epilogue VALU is what the MLP-1 launch spends most on
          const f32x2 g0 = gelu_erf_fast2(acc[i][j].xy), g1 = gelu_erf_fast2(acc[i][j].zw);
          acc[i][j] = (f32x4){g0.x, g0.y, g1.x, g1.y};
        } else if (p.epi == EPI_RELU) {
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[i][j][e] = fmaxf(acc[i][j][e], 0.f);
        }
      }
    // 528-B rows (BN = 256): 16 rows of one column hit distinct banks.  The whole tile when it fits
    // the ring (BN = 256), else in row halves of one wave row each (BN = 128: 2 x 64 KiB > 64 KiB).
    constexpr int PITCH = BN * 2 + 16, NH = 2 * BM * PITCH <= NSTAGE * STAGE ? 1 : 2, HR = BM / NH;
    constexpr int PLANE = HR * PITCH;
    static_assert(2 * PLANE <= NSTAGE * STAGE, "epilogue tile exceeds the ring");
    bf16_t* C = (bf16_t*)p.C;
#pragma unroll
    for (int hf = 0; hf < NH; ++hf) {
    __syncthreads();  // every wave is past its last ring read / the previous half's reads
    if (NH == 1 || wm == hf) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        uint32_t h0, l0, h1, l1;
        split_bf2(acc[i][j].xy, h0, l0);
        split_bf2(acc[i][j].zw, h1, l1);
        char* d = smem + ((NH == 1 ? wm * WM : 0) + i * 16 + fr) * PITCH + (wn * WN + j * 16 + 4 * fq) * 2;
        *(u32x2*)d = (u32x2){h0, h1};
        *(u32x2*)(d + PLANE) = (u32x2){l0, l1};
      }
    }
    __syncthreads();
#pragma unroll 4
    for (int c = tid; c < HR * (BN / 8); c += NW * 64) {
      const int row = c / (BN / 8), ch = c % (BN / 8), m = m0 + hf * HR + row;
      if (m >= M) continue;
      const int col = n0 + ch * 8;
      const long o = p.hm_n ? (((long)(m / p.hm_n) * (p.N / 64) + col / 64) * p.hm_n + m % p.hm_n) * 64 + col % 64
                            : (long)m * p.ldc + col;
      const u32x4 vh = *(const u32x4*)(smem + row * PITCH + ch * 16);
      const u32x4 vl = *(const u32x4*)(smem + PLANE + row * PITCH + ch * 16);
      if (p.nt_store) {  // streamed past the caches: keeps the operands resident in L2 / MALL
        __builtin_nontemporal_store(vh, (u32x4*)(C + o));
        __builtin_nontemporal_store(vl, (u32x4*)(C + o + p.c_lo));
      } else {
        *(u32x4*)(C + o) = vh;
        *(u32x4*)(C + o + p.c_lo) = vl;
      }
    }
    }
    return;
  }
  GemmArgs pe = p;
  pe.scale = nullptr;
  pe.res = nullptr;
  epilogue_256<TM, TN>(pe, acc, mb, nb, fr, fq);
}

}  // namespace

hipError_t launch_gemm_i8(const GemmArgs& g, hipStream_t s) {
  const bool blocks = g.a_kscale || g.out == OUT_I8K;  // block-scaled forms: 128 x 128 tiles only
#ifndef ICAP_TOOLS
  if (blocks) return hipErrorNotSupported;  // measured and rejected: tools build only
#endif
  if (g.M <= 0 || (blocks ? g.N % 128 : g.N % 256) || g.K % (g.a_kscale ? 128 : 64) || g.batch != 1 || !(g.a_scale || g.a_kscale) ||
      !g.w_scale || g.cv || g.scale || g.res)
    return hipErrorInvalidValue;
  if (g.out == OUT_I8K && (!g.c_kscale || g.hm_n || g.rm_group || g.addend)) return hipErrorInvalidValue;
  if (g.hm_n && (g.out != OUT_SPLIT || g.N % 64 || g.rm_group || g.M % g.hm_n)) return hipErrorInvalidValue;
  const long last_row = g.rm_group ? (long)((g.M - 1) / g.rm_group) * g.rm_stride + g.rm_off + g.rm_group : g.M;
  if (last_row * g.ldc >= (1L << 31)) return hipErrorInvalidValue;  // epilogue uses 32-bit row offsets
  constexpr int NST = 3, lds = NST * (128 * 128 + 256 * 128);
  static bool attr = false;
  if (!attr) {
    for (const void* f : {(const void*)gemm_i8_kernel<NST>
#ifdef ICAP_TOOLS
                          , (const void*)gemm_i8_kernel<NST, 1>, (const void*)gemm_i8_kernel<NST, 2>
#endif
         }) {
      hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
      if (e != hipSuccess) return e;
    }
    attr = true;
  }
  static const int nomfma = icap_knob("ICAP_I8_NOMFMA", 0);  // staging-only measurement variants (wrong results)
  const int nwg = (g.N / 256) * ((g.M + 127) / 128);
  // ICAP_I8_GROUP: tile raster (0 = row-band major; 16: qkv 373 -> 338 us, mlp0 525 -> 459)
  static const int group = std::max(0, icap_knob("ICAP_I8_GROUP", 16));
  static const int nt = icap_knob("ICAP_I8_NT_STORE", 0);
  GemmArgs gg = g;
  gg.raster_group = group;
  gg.nt_store = nt;
  // ICAP_I8_TILE: 128 (default) = 128 x 128 tiles, two blocks per CU; 256 = 128 x 256 tiles, one
  // block per CU.  Headline bench 6531 -> 6563 captions/s (QKV 370 -> 367 us, MLP-1 540 -> 500 us);
  // a persistent 128 x 256 form (ring prefetch across tile seams, stores drained under the next
  // tile's k-steps) measured 6548 and a 4-wave one-wave-per-SIMD form with fragment prefetch was
  // slower still (QKV 491 us): every form lands near 365 us for QKV (profiles/r01/v17_i8_forms.txt).
  static const int tile = icap_knob("ICAP_I8_TILE", 128);
  if ((tile == 128 && g.N % 128 == 0) || blocks) {
    constexpr int lds128 = 2 * (128 * 128 + 128 * 128);
    static bool attr128 = false;
    if (!attr128) {
      for (const void* f : {(const void*)gemm_i8_kernel<2, 0, 128>
#ifdef ICAP_TOOLS
                            , (const void*)gemm_i8_kernel<2, 1, 128>, (const void*)gemm_i8_kernel<2, 0, 128, 1>
#endif
           }) {
        const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds128);
        if (e != hipSuccess) return e;
      }
      attr128 = true;
    }
    const int nwg128 = (g.N / 128) * ((g.M + 127) / 128);
#ifdef ICAP_TOOLS
    if (g.a_kscale) hipLaunchKernelGGL((gemm_i8_kernel<2, 0, 128, 1>), dim3(nwg128), dim3(256), lds128, s, gg);
    else if (nomfma) hipLaunchKernelGGL((gemm_i8_kernel<2, 1, 128>), dim3(nwg128), dim3(256), lds128, s, gg);
    else
#endif
      hipLaunchKernelGGL((gemm_i8_kernel<2, 0, 128>), dim3(nwg128), dim3(256), lds128, s, gg);
    return hipGetLastError();
  }
#ifdef ICAP_TOOLS
  if (nomfma == 2) hipLaunchKernelGGL((gemm_i8_kernel<NST, 2>), dim3(nwg), dim3(512), lds, s, gg);
  else if (nomfma) hipLaunchKernelGGL((gemm_i8_kernel<NST, 1>), dim3(nwg), dim3(512), lds, s, gg);
  else
#endif
    hipLaunchKernelGGL((gemm_i8_kernel<NST>), dim3(nwg), dim3(512), lds, s, gg);
  return hipGetLastError();
}
