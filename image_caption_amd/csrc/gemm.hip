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
#include "common.h"
#include "kernels.h"

namespace {

constexpr int BK = 64;

template <int BM, int BN, int WM, int WN>
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
#pragma unroll
  for (int i = 0; i < IA; ++i) {
    int idx = (wave * IA + i) * 64 + lane, row = idx >> 3, cs = idx & 7;
    int gr = min(m0 + row, M - 1);
    a_off[i] = (long)gr * p.lda + ((cs ^ (row & 7)) << 3);
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
    for (int i = 0; i < IA; ++i)
      __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)(Ab + a_off[i]),
                                       (LDS_AS void*)(sa + (wave * IA + i) * 1024), 16, 0, 0);
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
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: C/D layout of 16x16 MFMA: col = lane & 15, row = 4*(lane >> 4) + r
  const float* bias = p.bias ? p.bias + (long)bz * p.bias_batch : nullptr;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn * WN + j * 16 + fr;
    const float bv = bias ? bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * WM + i * 16 + fq * 4 + r;
        if (row >= M) continue;
        float v = acc[i][j][r] + bv;
        if (p.addend) v += p.addend[(long)((row % p.add_group) + p.add_off) * p.add_ld + col];
        if (p.epi == EPI_GELU) v = 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
        else if (p.epi == EPI_RELU) v = fmaxf(v, 0.f);
        const long orow = p.rm_group ? (long)(row / p.rm_group) * p.rm_stride + p.rm_off + row % p.rm_group
                                     : (long)row;
        const long o = (long)bz * p.c_batch + orow * p.ldc + col;
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

template <int BM, int BN, int WM, int WN>
hipError_t run(const GemmArgs& g, hipStream_t s) {
  constexpr int lds = 2 * (BM + BN) * BK * 2;
  dim3 grid(g.N / BN, (g.M + BM - 1) / BM, g.batch);
  hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, WM, WN>), grid, dim3(256), lds, s, g);
  return hipGetLastError();
}

}  // namespace

int gemm_tile_class(const GemmArgs& g) {
  const long huge_tiles = (long)((g.M + 255) / 256) * (g.N / 256) * g.batch;
  if (g.N % 256 == 0 && g.batch == 1 && huge_tiles >= 256) return PROF_GEMM_256;
  const long big_tiles = (long)((g.M + 127) / 128) * (g.N / 128) * g.batch;
  return (g.N % 128 == 0 && big_tiles >= 512) ? PROF_GEMM_128 : PROF_GEMM_64;
}

hipError_t launch_gemm(const GemmArgs& g, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0 || g.K <= 0) return hipErrorInvalidValue;
  if (g.K % BK != 0 || g.N % 64 != 0 || (g.nsplit != 1 && g.nsplit != 2)) return hipErrorInvalidValue;
  const int cls = gemm_tile_class(g);
  if (cls == PROF_GEMM_256) return launch_gemm_256(g, s);
  if (cls == PROF_GEMM_128) return run<128, 128, 64, 64>(g, s);
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

constexpr int DEC_MAX_KSTEPS = 32;  // 32 k-steps x 32 = K' 1024 -> 128 KiB of LDS

__global__ __launch_bounds__(256) void gemm_dec_kernel(WaveGemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 32, m0 = blockIdx.y * 32;
  const int batch = blockIdx.z / p.ksplit, split = blockIdx.z % p.ksplit;
  const bf16_t* A = p.A + (long)batch * p.a_batch;
  const bf16_t* W = p.W + (long)batch * p.w_batch;
  const int ks_total = p.nsplit * p.K / 32, nks = ks_total / p.ksplit, kbeg = split * nks;

  // staging: instruction q in [0, 4 * nks): k-step q >> 2, operand (q >> 1) & 1, row half q & 1
  const int lrow = lane >> 2, lchunk = lane & 3;
  for (int q = wave; q < 4 * nks; q += 4) {
    const int ks = q >> 2, opnd = (q >> 1) & 1, half = q & 1;
    const int kg = (kbeg + ks) * 32 + lchunk * 8;
    const int r = half * 16 + lrow;
    const bf16_t* src;
    if (opnd == 0) {
      const int plane = kg / p.K, kin = kg - plane * p.K;
      src = A + plane * p.a_lo + (long)min(m0 + r, p.M - 1) * p.lda + kin;
    } else {
      src = W + (long)min(n0 + r, p.N - 1) * p.ldw + (kg % p.K);
    }
    __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)src,
                                     (LDS_AS void*)(smem + ks * 4096 + opnd * 2048 + half * 1024), 16, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int qm = wave >> 1, qn = wave & 1;  // this wave's 16 x 16 quadrant
  const int fr = lane & 15, fq = lane >> 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const char* pa = smem + (qm * 16 + fr) * 64 + fq * 16;
  const char* pb = smem + 2048 + (qn * 16 + fr) * 64 + fq * 16;
  for (int ks = 0; ks < nks; ++ks) {
    const bf16x8 a = *(const bf16x8*)(pa + ks * 4096);
    const bf16x8 b = *(const bf16x8*)(pb + ks * 4096);
    acc = mfma16(a, b, acc);
  }

  const int col = n0 + qn * 16 + fr;
  if (col >= p.N) return;
  const float bv = (p.bias && p.ksplit == 1) ? p.bias[(long)batch * p.bias_batch + col] : 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = m0 + qm * 16 + fq * 4 + r;
    if (row >= p.M) continue;
    float v = acc[r] + bv;
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

}  // namespace

hipError_t launch_gemm_dec(const WaveGemmArgs& g, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0 || g.K <= 0 || g.ksplit < 1 || g.N % 16) return hipErrorInvalidValue;
  if (g.K % 32 || (g.nsplit != 1 && g.nsplit != 2)) return hipErrorInvalidValue;
  const int steps = g.nsplit * g.K / 32;
  if (steps % g.ksplit || steps / g.ksplit > DEC_MAX_KSTEPS) return hipErrorInvalidValue;
  if (g.out == OUT_PARTIAL && g.part_stride <= 0) return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute((const void*)gemm_dec_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             DEC_MAX_KSTEPS * 4096);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int lds = steps / g.ksplit * 4096;
  dim3 grid((g.N + 31) / 32, (g.M + 31) / 32, g.batch * g.ksplit);
  hipLaunchKernelGGL(gemm_dec_kernel, grid, dim3(256), lds, s, g);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Encoder GEMM, 256 x 256 block tile, 8 waves (2 x 4, each 128 x 64 = 8 x 4 MFMA 16x16 tiles).
// A stage holds the k-slice (32 deep) of EVERY activation plane plus the W slice, so the hi and lo
// planes share one staged W tile (175 FLOP of MFMA work per staged byte in bf16x2 mode, vs 128 when
// W is re-staged per plane).  Stages go HBM/L2 -> LDS by global_load_lds into a 3-stage (bf16x2,
// 3 x 48 KiB) or 4-stage (bf16, 4 x 32 KiB) ring; a COUNTED vmcnt before each raw s_barrier keeps
// the younger stages in flight across barriers (__syncthreads would drain them).  PMC on the
// 2-stage 64-deep predecessor (profiles/r01): MFMA busy 31 %, waves parked 50 %, LDS bank conflicts
// 0, staged bytes arriving at ~22-25 GB/s per CU - the stream is latency-bound on bytes in flight.  Blocks are remapped so each XCD owns a contiguous run of logical
// tiles (bijective form of cdna_hip_programming.md §5 "XCD swizzle"): the tiles of one row band
// share their A rows in that XCD's L2.
namespace {

template <int NS>
__global__ __launch_bounds__(512) void gemm_256_kernel(GemmArgs p) {
  constexpr int BM = 256, BN = 256, WM = 128, WN = 64, TM = WM / 16, TN = WN / 16;
  constexpr int KS = 32;                            // k per stage (one MFMA k-step)
  constexpr int OPB = BM * KS * 2;                  // 16 KiB per operand tile per stage
  constexpr int STAGE = (NS + 1) * OPB;             // A planes + W share one stage
  constexpr int NSTAGE = NS == 2 ? 3 : 4;           // 144 / 128 KiB of LDS
  constexpr int IPW = OPB / 1024 / 8;               // 1 KiB DMA instructions per wave per operand (2)
  constexpr int PER_STAGE = IPW * (NS + 1);         // DMA instructions per wave per stage
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  // XCD-aware bijective remap of the linear block id
  const int nbn = p.N / BN, nbm = (p.M + BM - 1) / BM, nwg = nbn * nbm;
  const int orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int bm = wg / nbn, bn = wg - bm * nbn;
  const int m0 = bm * BM, n0 = bn * BN;
  const int M = p.M, K = p.K;
  const int nk = K / KS;

  // Stage image: per operand tile, rows of 64 B (32 bf16 of k); one DMA instruction = 16 rows.
  // 16-byte chunk c of row r lives at chunk c ^ sw(r), sw(r) = ((r >> 3) & 1) << 1, which makes
  // the ds_read_b128 fragment reads (16 rows x one chunk per lane group) bank-conflict free.
  const int srow = wave * IPW * 16 + (lane >> 2);
  const int schunk = (lane & 3) ^ (((srow >> 3) & 1) << 1);
  const bf16_t* a_base = p.A + (long)min(m0 + srow, M - 1) * p.lda + schunk * 8;
  const bf16_t* b_base = p.W + (long)min(n0 + srow, p.N - 1) * p.ldw + schunk * 8;
  const long a_step = 16 * p.lda, b_step = 16 * p.ldw;
  const bool a_tail = m0 + BM > M;
  auto stage = [&](int kt, int buf) {
    const int kin = kt * KS;
    char* s0 = smem + buf * STAGE;
#pragma unroll
    for (int pl = 0; pl < NS; ++pl) {
      const bf16_t* Ab = a_base + pl * p.a_lo + kin;
#pragma unroll
      for (int i = 0; i < IPW; ++i) {
        const bf16_t* src = Ab + i * a_step;
        if (a_tail && m0 + srow + i * 16 >= M) src = Ab + (long)(M - 1 - m0 - srow) * p.lda;
        __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)src,
                                         (LDS_AS void*)(s0 + pl * OPB + (wave * IPW + i) * 1024), 16, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < IPW; ++i)
      __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)(b_base + kin + i * b_step),
                                       (LDS_AS void*)(s0 + NS * OPB + (wave * IPW + i) * 1024), 16, 0, 0);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  const int foff = fr * 64 + ((fq ^ (((fr >> 3) & 1) << 1)) << 4);
#pragma unroll
  for (int s = 0; s < NSTAGE - 1; ++s)
    if (s < nk) stage(s, s);
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt must have landed for every wave: leave the younger prefetched stages in flight
    const int younger = min(NSTAGE - 2, nk - 1 - kt);
    if (younger >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER_STAGE) : "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_STAGE) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // refill the buffer read in iteration kt-1 (every wave has passed this barrier)
    if (kt + NSTAGE - 1 < nk) stage(kt + NSTAGE - 1, (kt + NSTAGE - 1) % NSTAGE);
    const char* s0 = smem + (kt % NSTAGE) * STAGE;
    bf16x8 bfr[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) bfr[j] = *(const bf16x8*)(s0 + NS * OPB + (wn * WN + j * 16) * 64 + foff);
#pragma unroll
    for (int pl = 0; pl < NS; ++pl)
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const bf16x8 af = *(const bf16x8*)(s0 + pl * OPB + (wm * WM + i * 16) * 64 + foff);
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(bfr[j], af, acc[i][j]);  // D = W·A^T
      }
  }

  // epilogue.  The MFMA computed the transposed tile (W as the A operand), so lane l holds
  // output row m = i*16 + (l & 15) and FOUR consecutive output columns n = j*16 + 4*(l >> 4) + r:
  // every store is a 16-byte (fp32) or 8-byte (bf16 plane) vector.
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * WN + j * 16 + 4 * fq;
    const f32x4 bv = p.bias ? *(const f32x4*)(p.bias + n) : (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wm * WM + i * 16 + fr;
      f32x4 v = acc[i][j] + bv;
      if (p.addend) {
        const int row = min(m, M - 1);
        v += *(const f32x4*)(p.addend + (long)((row % p.add_group) + p.add_off) * p.add_ld + n);
      }
      if (p.epi == EPI_GELU) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = 0.5f * v[r] * (1.f + erff(v[r] * 0.70710678118654752f));
      } else if (p.epi == EPI_RELU) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
      }
      acc[i][j] = v;
    }
  }
  auto out_index = [&](int i, int j, long& o) -> bool {
    const int m = m0 + wm * WM + i * 16 + fr;
    const long orow = p.rm_group ? (long)(m / p.rm_group) * p.rm_stride + p.rm_off + m % p.rm_group : (long)m;
    o = orow * p.ldc + n0 + wn * WN + j * 16 + 4 * fq;
    return m < M;
  };
  if (p.out == OUT_F32 || p.out == OUT_F32_RESID) {
    float* C = (float*)p.C;
    const bool add = p.out == OUT_F32_RESID;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        long o;
        if (out_index(i, j, o)) *(f32x4*)(C + o) = add ? *(const f32x4*)(C + o) + acc[i][j] : acc[i][j];
      }
  } else {
    bf16_t* C = (bf16_t*)p.C;
    const bool lo_plane = p.out == OUT_SPLIT && p.c_planes == 2;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        long o;
        if (out_index(i, j, o)) {
          bf16_t h[4], l[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) split_bf(acc[i][j][r], h[r], l[r]);
          *(u32x2*)(C + o) = (u32x2){(uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16)};
          if (lo_plane)
            *(u32x2*)(C + o + p.c_lo) =
                (u32x2){(uint32_t)l[0] | ((uint32_t)l[1] << 16), (uint32_t)l[2] | ((uint32_t)l[3] << 16)};
        }
      }
  }
}

}  // namespace

hipError_t launch_gemm_256(const GemmArgs& g, hipStream_t s) {
  if (g.M <= 0 || g.N % 256 || g.K % 32 || g.batch != 1 || (g.nsplit != 1 && g.nsplit != 2))
    return hipErrorInvalidValue;
  constexpr int lds2 = 3 * 3 * 256 * 32 * 2, lds1 = 4 * 2 * 256 * 32 * 2;
  static bool attr = false;
  if (!attr) {
    hipError_t e =
        hipFuncSetAttribute((const void*)gemm_256_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, lds2);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void*)gemm_256_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, lds1);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int nwg = (g.N / 256) * ((g.M + 255) / 256);
  if (g.nsplit == 2)
    hipLaunchKernelGGL(gemm_256_kernel<2>, dim3(nwg), dim3(512), lds2, s, g);
  else
    hipLaunchKernelGGL(gemm_256_kernel<1>, dim3(nwg), dim3(512), lds1, s, g);
  return hipGetLastError();
}
