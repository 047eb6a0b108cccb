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
  const long big_tiles = (long)((g.M + 127) / 128) * (g.N / 128) * g.batch;
  return (g.N % 128 == 0 && big_tiles >= 512) ? PROF_GEMM_128 : PROF_GEMM_64;
}

hipError_t launch_gemm(const GemmArgs& g, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0 || g.K <= 0) return hipErrorInvalidValue;
  if (g.K % BK != 0 || g.N % 64 != 0 || (g.nsplit != 1 && g.nsplit != 2)) return hipErrorInvalidValue;
  if (gemm_tile_class(g) == PROF_GEMM_128) return run<128, 128, 64, 64>(g, s);
  return run<64, 64, 32, 32>(g, s);
}
