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

// Implicit-GEMM convolution rows (GemmArgs::cv): a staging lane's output pixel, fixed for the K loop.
struct ConvRow {
  int pb, oy, ox;  // input pixel index of the window origin (stride applied), its y and x
};
__device__ __forceinline__ ConvRow conv_row(const GemmArgs& p, int gr) {
  const int b = gr / p.cv_OHW, rem = gr - b * p.cv_OHW, oh = rem / p.cv_OW, ow = rem - oh * p.cv_OW;
  const int oy = oh * p.cv_stride, ox = ow * p.cv_stride;
  return {(b * p.cv_H + oy) * p.cv_W + ox, oy, ox};
}
// Source of the 16-byte chunk at k (8 consecutive k, one tap) of row r; base = A + plane offset.
template <int CONV>
__device__ __forceinline__ const bf16_t* conv_src(const GemmArgs& p, const bf16_t* base, const ConvRow& r, int k) {
  if (CONV == 2)  // stem: kernel row kh = k / 32 of the bordered NHWC4 image, 8 pixels x 4 channels
    return base + (long)(r.pb + (k >> 5) * p.cv_W) * 4 + (k & 31);
  const int tap = k >> p.cv_cshift, c = k & ((1 << p.cv_cshift) - 1);
  const int kh = (tap * 11) >> 5, kw = tap - 3 * kh;  // tap / 3, tap % 3 for tap < 9
  const int iy = r.oy + kh - 1, ix = r.ox + kw - 1;
  const bool ok = (unsigned)iy < (unsigned)p.cv_H && (unsigned)ix < (unsigned)p.cv_W;
  const bf16_t* src = base + ((long)(r.pb + (kh - 1) * p.cv_W + kw - 1) << p.cv_cshift) + c;
  return ok ? src : p.cv_zero;
}

template <int BM, int BN, int WM, int WN, int CONV = 0>
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
          v += bf2f(p.res[ro]) + bf2f(p.res[ro + p.res_lo]);
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
  if (grid.y > 65535) return hipErrorInvalidValue;
  if (g.cv == 1) hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, WM, WN, 1>), grid, dim3(256), lds, s, g);
  else if (g.cv == 2) hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, WM, WN, 2>), grid, dim3(256), lds, s, g);
  else hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, WM, WN>), grid, dim3(256), lds, s, g);
  return hipGetLastError();
}

}  // namespace

bool gemm_f16_persistent(const GemmArgs& g) {
  // tools: ICAP_F16_GEMM 6 = persistent for every fp16 GEMM; ICAP_F16_PRES 0 = the residual GEMMs in the
  // two-block form (out-proj 131 / MLP-2 340 us against 124 / 314 persistent, encoder 15.7 -> 15.0 ms/step)
  static const int form = icap_knob("ICAP_F16_GEMM", 0), pres = icap_knob("ICAP_F16_PRES", 1);
  const bool common = g.f16 && (form == 0 || form == 6) && !g.addend && !g.rm_group && !g.res && !g.scale && !g.cv &&
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
  if (g.f16) return gemm_f16_persistent(g) ? PROF_GEMM_F16P : PROF_GEMM_256;  // the fp16 forms live in launch_gemm_256
  const long huge_tiles = (long)((g.M + 255) / 256) * (g.N / 256) * g.batch;
  if (g.N % 256 == 0 && g.batch == 1 && huge_tiles >= 96) return PROF_GEMM_256;
  const long big_tiles = (long)((g.M + 127) / 128) * (g.N / 128) * g.batch;
  return (g.N % 128 == 0 && g.N >= 256 && big_tiles >= 512) ? PROF_GEMM_128 : PROF_GEMM_64;
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

// ---------------------------------------------------------------------------------------------
// Epilogue of the 256 x 256 encoder GEMMs.  The MFMA computed the transposed tile (W as the A
// operand), so lane l holds output row m = mb + i*16 + (l & 15) and FOUR consecutive columns
// n = nb + j*16 + 4*(l >> 4) + r: every store is a 16-byte (fp32) or 8-byte (bf16 plane) vector.
// Every runtime condition is hoisted out of the element loops and the loads are issued in batches
// (4 bias vectors; 8 residual vectors per column group), so a block waits a handful of memory
// latencies instead of one per element (a per-element "load or not" branch makes hipcc wait
// vmcnt(0) after each load).  Rows >= M load from row M - 1 and are not stored.
namespace {

template <int TM, int TN, bool F16 = false>
__device__ __forceinline__ void epilogue_256(const GemmArgs& p, f32x4 (&acc)[TM][TN], int mb, int nb, int fr,
                                             int fq) {
  const int M = p.M;
  if (p.scale) {
    f32x4 sv[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) sv[j] = *(const f32x4*)(p.scale + nb + j * 16 + 4 * fq);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] *= sv[j];
  }
  if (p.bias) {
    f32x4 bv[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) bv[j] = *(const f32x4*)(p.bias + nb + j * 16 + 4 * fq);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] += bv[j];
  }
  if (p.addend) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      f32x4 ad[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = min(mb + i * 16 + fr, M - 1);
        ad[i] = *(const f32x4*)(p.addend + (long)((row % p.add_group) + p.add_off) * p.add_ld + nb + j * 16 + 4 * fq);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[i][j] += ad[i];
    }
  }
  if (p.res) {  // residual from bf16 planes (hi + lo), 4 consecutive columns = 8 B per plane
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      u32x2 rh[TM], rl[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const long ro = (long)min(mb + i * 16 + fr, M - 1) * p.res_ld + nb + j * 16 + 4 * fq;
        rh[i] = *(const u32x2*)(p.res + ro);
        rl[i] = *(const u32x2*)(p.res + ro + p.res_lo);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t wh = rh[i][r >> 1] >> ((r & 1) * 16), wl = rl[i][r >> 1] >> ((r & 1) * 16);
          acc[i][j][r] += bf2f((bf16_t)(wh & 0xffff)) + bf2f((bf16_t)(wl & 0xffff));
        }
    }
  }
  if (p.epi == EPI_GELU) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = gelu_erf_fast(acc[i][j][r]);
  } else if (p.epi == EPI_RELU) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = fmaxf(acc[i][j][r], 0.f);
  }
  int orow[TM];  // element offset of the row (launch_gemm_256 guarantees < 2^31); -1: row >= M
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = mb + i * 16 + fr;
    const int mc = min(m, M - 1);
    if (p.hm_n)  // head-major: this wave's 64 columns [nb, nb + 64) are one head block
      orow[i] = (int)((((long)(mc / p.hm_n) * (p.N / 64) + nb / 64) * p.hm_n + mc % p.hm_n) * 64 - nb);
    else
      orow[i] = (int)((p.rm_group ? (long)(mc / p.rm_group) * p.rm_stride + p.rm_off + mc % p.rm_group : (long)mc) *
                      p.ldc);
    if (m >= M) orow[i] = -1 - orow[i];
  }

  if (p.out == OUT_F32) {
    float* C = (float*)p.C;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        if (orow[i] >= 0) *(f32x4*)(C + orow[i] + nb + j * 16 + 4 * fq) = acc[i][j];
  } else if (p.out == OUT_F32_RESID) {
    float* C = (float*)p.C;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i0 = 0; i0 < TM; i0 += 4) {
        f32x4 c[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ro = orow[i0 + i] < 0 ? -1 - orow[i0 + i] : orow[i0 + i];
          c[i] = *(const f32x4*)(C + ro + nb + j * 16 + 4 * fq);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (orow[i0 + i] >= 0) *(f32x4*)(C + orow[i0 + i] + nb + j * 16 + 4 * fq) = c[i] + acc[i0 + i][j];
      }
  } else if (F16) {  // one fp16 plane
    bf16_t* C = (bf16_t*)p.C;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        if (orow[i] >= 0) *(u32x2*)(C + orow[i] + nb + j * 16 + 4 * fq) = pack16x4<true>(acc[i][j]);
  } else {
    bf16_t* C = (bf16_t*)p.C;
    const bool lo_plane = p.out == OUT_SPLIT && p.c_planes == 2;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if (orow[i] < 0) continue;
        const long o = orow[i] + nb + j * 16 + 4 * fq;
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

}  // namespace

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

// BMT = 128 with NW = 8 and NST = 2: the same 64 x 64 wave tiles in a 128 x 256 block tile with a
// 2-stage ring (64 KiB of LDS), so two blocks share a CU and one's epilogue overlaps the other's
// k-loop (the output-heavy, short-K trunk GEMMs).
// KSD = 64: 64-deep stages (two MFMA k-steps): every operand row segment is a full 128-B line
// (8 rows x 128 B per DMA instruction, chunk c of row r at c ^ (r & 7)) and half the barriers.
// TS = 1: tail split (GemmArgs::split_ws): each XCD owns a contiguous range of c tiles (the XCD remap);
// with S = split_slots block slots per XCD the last c % S tiles (a partial final round, c > S) run as
// two blocks each, one per K half.  Both halves leave their fp32 partial tile with agent-scope stores,
// wait for them to complete and take a ticket; the second adds the other's partial (a + b: the same
// bits whichever finished first) and runs the epilogue.
template <int NS, int NW, int NOMFMA = 0, int CONV = 0, int BMT = 256, int NST = 0, int KSD = 32, int TS = 0,
          bool F16 = false>
__global__ __launch_bounds__(NW * 64, (BMT == 128 && KSD == 32) ? 4 : (BMT == 64 ? 3 : 1)) void gemm_256_kernel(
    GemmArgs p) {
  constexpr int WGM = NW / 4;                       // wave grid WGM x 4
  constexpr int BM = BMT, BN = 256, WM = BM / WGM, WN = 64, TM = WM / 16, TN = WN / 16;
  constexpr int KS = KSD;                           // k per stage (one or two MFMA k-steps)
  constexpr int RPI = KS == 64 ? 8 : 16;            // rows per 1 KiB DMA instruction
  constexpr int OPB = BM * KS * 2;                  // A bytes per plane per stage (16 KiB at BM 256)
  constexpr int OPBW = BN * KS * 2;                 // W bytes per stage (16 KiB)
  constexpr int STAGE = NS * OPB + OPBW;            // A planes + W share one stage
  constexpr int NSTAGE = NST ? NST : (NS == 2 ? 3 : 4);  // 144 / 128 KiB of LDS at BM 256
  constexpr int IPW = OPB / 1024 / NW;              // 1 KiB DMA instructions per wave per A plane
  constexpr int IPWW = OPBW / 1024 / NW;            // ... for W
  static_assert(IPW >= 1 && IPWW >= 1 && WM % 16 == 0, "tile / wave shape");
  constexpr int PER_STAGE = IPW * NS + IPWW;        // DMA instructions per wave per stage
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  // XCD-aware bijective remap of the linear block id
  const int nbn = p.N / BN, nbm = (p.M + BM - 1) / BM, nwg = nbn * nbm;
  const int orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int xbase = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  int wg = xbase + (orig >> 3);
  const int M = p.M, K = p.K;
  const int nk = K / KS;
  int kbeg = 0, kend = nk, part = -1, slot = 0;
  if (TS) {  // (the launch has 8 x max(c + tail) blocks; the XCD's surplus exits)
    const int S = p.split_slots, li = orig >> 3, cx = q + (xcd < r);
    const int tq1 = q + 1 > S ? (q + 1) % S : 0, tq = q > S ? q % S : 0, tail = xcd < r ? tq1 : tq;
    if (li >= cx + tail) return;
    if (li >= cx - tail) {
      const int v = li - (cx - tail);
      wg = xbase + cx - tail + (v >> 1);
      part = v & 1;
      slot = (xcd < r ? xcd * tq1 : r * tq1 + (xcd - r) * tq) + (v >> 1);
      kbeg = part ? nk / 2 : 0;
      kend = part ? nk : nk / 2;
    }
  }
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

  // Stage image: per operand tile, rows of 64 B (32 bf16 of k); one DMA instruction = 16 rows.
  // 16-byte chunk c of row r lives at chunk c ^ sw(r), sw(r) = ((r >> 3) & 1) << 1, which makes
  // the ds_read_b128 fragment reads (16 rows x one chunk per lane group) bank-conflict free.
  const int srow = KS == 64 ? wave * IPW * 8 + (lane >> 3) : wave * IPW * 16 + (lane >> 2);
  const int srow_w = KS == 64 ? wave * IPWW * 8 + (lane >> 3) : wave * IPWW * 16 + (lane >> 2);
  // (the swizzle depends on row bits that are equal for srow and srow_w: instruction bases are
  // multiples of RPI)
  const int schunk = KS == 64 ? (lane & 7) ^ (srow & 7) : (lane & 3) ^ (((srow >> 3) & 1) << 1);
  const bf16_t* a_base = p.A + (long)min(m0 + srow, M - 1) * p.lda + schunk * 8;
  const bf16_t* b_base = p.W + (long)min(n0 + srow_w, p.N - 1) * p.ldw + schunk * 8;
  const long a_step = RPI * p.lda, b_step = RPI * p.ldw;
  const bool a_tail = m0 + BM > M;
  ConvRow cr[CONV ? IPW : 1];
  if (CONV)
#pragma unroll
    for (int i = 0; i < IPW; ++i) cr[i] = conv_row(p, min(m0 + srow + i * RPI, M - 1));
  auto stage = [&](int kt, int buf) {
    const int kin = kt * KS;
    char* s0 = smem + buf * STAGE;
    if (NOMFMA == 3) {  // measurement: same bytes per stage as full 128-B lines (A as [M][2K], W as row pairs)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = (wave * 2 + i) * 8 + (lane >> 3);
        const bf16_t* src = p.A + (long)min(m0 + row, M - 1) * 2 * p.lda + kt * 64 + (lane & 7) * 8;
        __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)src, (LDS_AS void*)(s0 + (wave * 2 + i) * 1024), 16,
                                         0, 0);
      }
      const int pair = wave * 8 + (lane >> 3);
      const bf16_t* wsrc = p.W + (long)((n0 >> 1) + pair) * 2 * p.ldw + kt * 64 + (lane & 7) * 8;
      __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)wsrc, (LDS_AS void*)(s0 + 2 * OPB + wave * 1024), 16,
                                       0, 0);
      return;
    }
#pragma unroll
    for (int pl = 0; pl < NS; ++pl) {
      const bf16_t* Ab = a_base + pl * p.a_lo + kin;
#pragma unroll
      for (int i = 0; i < IPW; ++i) {
        const bf16_t* src = Ab + i * a_step;
        if (CONV) src = conv_src<CONV>(p, p.A + pl * p.a_lo, cr[CONV ? i : 0], kin + schunk * 8);
        else if (a_tail && m0 + srow + i * RPI >= M) src = Ab + (long)(M - 1 - m0 - srow) * p.lda;
        __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)src,
                                         (LDS_AS void*)(s0 + pl * OPB + (wave * IPW + i) * 1024), 16, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < IPWW; ++i)
      __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)(b_base + kin + i * b_step),
                                       (LDS_AS void*)(s0 + NS * OPB + (wave * IPWW + i) * 1024), 16, 0, 0);
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
    if (kbeg + s < kend) stage(kbeg + s, s);
  for (int kt = kbeg; kt < kend; ++kt) {
    // stage kt must have landed for every wave: leave the younger prefetched stages in flight
    const int younger = min(NSTAGE - 2, kend - 1 - kt);
    // lgkmcnt(0): this wave's LDS reads of the previous step must be done before the barrier that
    // lets other waves' DMA overwrite that buffer (a 2-stage ring refills it one step later)
    if (younger >= 2) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * PER_STAGE) : "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PER_STAGE) : "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // refill the buffer read in iteration kt-1 (every wave has passed this barrier)
    if (kt + NSTAGE - 1 < kend) stage(kt + NSTAGE - 1, (kt - kbeg + NSTAGE - 1) % NSTAGE);
    const char* s0 = smem + ((kt - kbeg) % NSTAGE) * STAGE;
    if (NOMFMA >= 2) continue;
    if constexpr (KS == 64) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int fo = fr * 128 + (((ks * 4 + fq) ^ (fr & 7)) << 4);
        bf16x8 bfr[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = *(const bf16x8*)(s0 + NS * OPB + (wn * WN + j * 16) * 128 + fo);
#pragma unroll
        for (int pl = 0; pl < NS; ++pl)
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const bf16x8 af = *(const bf16x8*)(s0 + pl * OPB + (wm * WM + i * 16) * 128 + fo);
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = mma<F16>(bfr[j], af, acc[i][j]);
          }
      }
    } else {
      bf16x8 bfr[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = *(const bf16x8*)(s0 + NS * OPB + (wn * WN + j * 16) * 64 + foff);
#pragma unroll
      for (int pl = 0; pl < NS; ++pl)
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const bf16x8 af = *(const bf16x8*)(s0 + pl * OPB + (wm * WM + i * 16) * 64 + foff);
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            if (NOMFMA) {  // measurement variant: staging pipeline only (keeps the fragment reads live)
              asm volatile("" ::"v"(af), "v"(bfr[j]));
            } else {
              acc[i][j] = mma<F16>(bfr[j], af, acc[i][j]);  // D = W·A^T
            }
          }
        }
    }
  }

  if (TS && part >= 0) {
    constexpr int NT = NW * 64, NE = TM * TN * 4;
    float* mine = p.split_ws + ((long)slot * 2 + part) * NE * NT;
    const float* other = p.split_ws + ((long)slot * 2 + (part ^ 1)) * NE * NT;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          __hip_atomic_store(mine + ((i * TN + j) * 4 + e) * NT + tid, acc[i][j][e], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's partial is complete
    __syncthreads();                                   // ... every thread's (and every ring read)
    if (tid == 0) *(int*)smem = __hip_atomic_fetch_add(p.split_cnt + slot, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (*(volatile int*)smem == 0) return;  // the other half finishes the tile
    if (tid == 0) __hip_atomic_store(p.split_cnt + slot, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc[i][j][e] += __hip_atomic_load(other + ((i * TN + j) * 4 + e) * NT + tid, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
  }
  epilogue_256<TM, TN, F16>(p, acc, m0 + wm * WM, n0 + wn * WN, fr, fq);
}

// ---------------------------------------------------------------------------------------------
// Persistent fp16 encoder GEMM (ICAP_PREC_F16): 256 x 256 tiles, 8 waves (2 x 4, wave tile 128 x 64),
// 64-deep stages (every operand row segment one full 128-B line, chunk c of row r at c ^ (r & 7)) in a
// 2-stage LDS ring (128 KiB, one block per CU), and one block per CU that walks its XCD's tiles.  Why
// persistent: at M = 50432 a k-step of this tile takes as long as hipBLASLt's (K sweep at N = 2304,
// tools/f16_ksweep.sh: 188.6 vs 177 us per 768 of K), but every tile of a one-block-per-CU launch pays its
// dispatch, the first stage's full memory latency and its epilogue with nothing overlapping them - 92 us
// of the 281 us QKV GEMM (hipBLASLt: 19).  Here the (tile, k-step) sequence of a block is ONE stream of
// stages: the last k-step of a tile already DMAs the next tile's first stage, whose latency then hides
// behind that k-step's MFMAs and the epilogue.  Tiles: the XCD-bijective remap of gemm_256_kernel gives
// XCD x a contiguous range of logical tiles (row-band major), its blocks take every nbx-th of them, so the
// tiles in flight on one XCD share their A row bands in its L2.
// SO (store-only epilogues: bias (+ GELU) -> one fp16 plane, optionally head-major; K >= 128; a ragged last
// row band stores only its rows < M and hands the next tile the uncounted vmcnt(0) wait):
// the epilogue's stores must not hold the next tile's k-loop.  VMEM operations retire in issue order (the
// compiler's own s_waitcnt model on gfx950 counts loads and stores in one in-order counter), so the k-loop
// waits with counts that leave the previous tile's stores in flight: at a tile seam the next tile's stages
// 0 AND 1 are issued before the epilogue (its bias was loaded before stage 0, behind the previous tile's
// MFMAs), k-step 0 waits vmcnt(8 + 32) (stage 0 done; stage 1 and the 32 stores per wave may pend),
// k-step 1 vmcnt(32); the stores then drain behind two k-steps of MFMAs.
// MODE 2 (RES: out = OUT_F32_RESID, C += acc + bias, K >= 128): the residual GEMMs (ViT out-proj,
// MLP-2).  The epilogue reads the fp32 residual in two halves of 16 loads per lane (registers: acc + 64); the
// next tile's stage 0 is in flight behind the last k-step, its stage 1 is issued after the epilogue's stores
// (the residual loads' waits would otherwise wait for it), and k-step 0 needs no vmcnt wait: the residual loads
// retired after stage 0 (in order).
// ABL (tools build only): 1 = no k-loop DMA, 2 = no MFMA - timing ablations (tools/f16_ablate.sh); 3 = the
// compiler's own fragment-read order, 4 = the read pipeline per k-half, 5 = the stage DMA before the first reads,
// 6 = reads 3 groups ahead instead of 2 (within box noise, tools/f16x3_check.sh), 7 = s_setprio(1) around each
// MFMA group (no gain, tools/f16_pf.sh), 8 = 8-byte SO stores.
// BMT: tile rows, 256 or (RES) 224 - wave tiles 112 x 64, the A stage 224 rows (wave 7 DMAs W rows only): at
// N = 768 the 256-row tiles are 591 = 2.3 per CU (3 rounds, the last 30 % full), 224-row tiles 678 = 2.65 per CU
// (3 rounds of 7/8 the work).
template <int MODE, int ABL = 0, int BMT = 256>
__global__ __launch_bounds__(512, 1) void gemm_f16p_kernel(GemmArgs p) {
  constexpr bool SO = MODE == 1, RES = MODE == 2;
  // fragment reads: ABL 0 = one pipeline over the k-step's 16 A fragments, each read XD MFMA groups ahead (the
  // second k-half's W fragments with the read XD ahead of its first group); 4 = per k-half (PF = 2);
  // 3 and the ablations = the compiler's order (reads 2, waits for both, runs 8).  Per ViT layer 1039 -> 1013
  // (per k-half) -> 997 us (tools/f16_pf.sh)
  constexpr int PF = ABL == 4 ? 2 : 0;
  constexpr bool XK = ABL == 0 || ABL >= 5, XK_LATE = ABL == 0 || ABL >= 6;
  constexpr int XD = ABL == 6 ? 3 : 2;  // XK read distance in MFMA groups (tools: 6 = 3 - within noise of 2)
  constexpr bool XPRIO = ABL == 7;      // tools: s_setprio(1) around each MFMA group
  static_assert(BMT == 256 || (RES && BMT == 224), "224-row tiles only for the residual form (no counted waits)");
  constexpr int BM = BMT, BN = 256, KS = 64, NW = 8, WM = BM / 2, WN = 64, TM = WM / 16, TN = 4;
  constexpr int OPA = BM * KS * 2, OPB = BN * KS * 2, STAGE = OPA + OPB;  // A 32 (28) KiB + W 32 KiB
  constexpr int IPW = OPB / 1024 / NW;                // 4 DMA instructions per wave per operand
  constexpr int PER_STAGE = 2 * IPW;                  // 8 per wave per stage
  // SO stores per wave per tile: WIDE = 16 B per lane (two 4-column groups of a row joined across the lane pair
  // fq ^ 1: 16 stores), else 8 B (32 stores; tools ABL 8)
  constexpr bool WIDE = ABL != 8;
  constexpr int NSTORE = WIDE ? TM * TN / 2 : TM * TN;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int nbn = p.N / BN, nbm = (p.M + BM - 1) / BM, nwg = nbn * nbm;
  const int xcd = blockIdx.x & 7, q = nwg >> 3, r = nwg & 7;
  const int xbase = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q, xcnt = q + (xcd < r);
  const int nbx = ((int)gridDim.x - xcd + 7) >> 3, lb = blockIdx.x >> 3;  // blocks on this XCD, rank among them
  if (lb >= xcnt) return;
  const int M = p.M, nk = p.K / KS;
  const int srow = wave * IPW * 8 + (lane >> 3), schunk = (lane & 7) ^ (srow & 7);
  const int fr = lane & 15, fq = lane >> 4;

  auto stage = [&](int t, int kt, int buf) {  // tile t (logical), k-step kt -> ring buffer buf
    const int bm = t / nbn, bn = t - bm * nbn, m0 = bm * BM, n0 = bn * BN;
    char* s0 = smem + buf * STAGE;
    const bf16_t* Ab = p.A + kt * KS + schunk * 8;
    const bf16_t* Wb = p.W + (long)(n0 + srow) * p.ldw + kt * KS + schunk * 8;
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      if (BM < 256 && (wave * IPW + i) * 8 >= BM) break;  // (wave-uniform) rows past the tile's A image
      const int row = min(m0 + srow + i * 8, M - 1);
      __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)(Ab + (long)row * p.lda),
                                       (LDS_AS void*)(s0 + (wave * IPW + i) * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < IPW; ++i)
      __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)(Wb + (long)i * 8 * p.ldw),
                                       (LDS_AS void*)(s0 + OPA + (wave * IPW + i) * 1024), 16, 0, 0);
  };
  // SO: the tile's 256 bias values go to LDS slot (tile count & 1) by one DMA instruction of wave 0, issued
  // before the tile's first stage (so the counted waits below never count it) - no registers held across
  // the k-loop (the kernel is at the 256-register limit of two waves per SIMD)
  float* sbias = (float*)(smem + 2 * STAGE);
  auto load_bias = [&](int t, int slot) {
    if (wave == 0 && p.bias) {
      const int n0 = (t - (t / nbn) * nbn) * BN;
      __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)(p.bias + n0 + lane * 4),
                                       (LDS_AS void*)(sbias + slot * 256), 16, 0, 0);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  int t = xbase + lb, step = 0, tcount = 0;
  if (SO || RES) load_bias(t, 0);
  stage(t, 0, 0);
  bool seam = false;  // this tile's stages 0 and 1 were issued before the previous tile's epilogue stores
  bool range_bad = false;  // SO: some stored fp16 value is not finite (p.range_flag set once, after the last tile)
  for (;;) {
    const int tn = t + nbx < xbase + xcnt ? t + nbx : -1;  // this block's next tile
    for (int kt = 0; kt < nk; ++kt, ++step) {
      // lgkmcnt(0): this wave's reads of the buffer about to be refilled are done before the barrier
      if (SO && seam && kt == 0) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PER_STAGE + NSTORE) : "memory");
      else if (SO && seam && kt == 1) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NSTORE) : "memory");
      else if (RES && seam && kt == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      int st_t = -1, st_kt = 0;  // the stage this k-step DMAs into the other buffer (-1: none)
      if ((SO || RES) && seam && kt == 0) {
        // stage 1 of this tile is already in flight
      } else if (kt + 1 < nk) {
        st_t = t, st_kt = kt + 1;
      } else if (tn >= 0) {  // the next tile's bias, then its first stage, behind this k-step's MFMAs
        if (SO || RES) load_bias(tn, (tcount + 1) & 1);
        st_t = tn;
      }
      if (ABL == 1) st_t = -1;
      // XK (default): the k-step's first fragment reads go out before the stage's 8 DMA instructions, whose
      // issue then covers their latency (ABL 5: DMA first)
      if (!XK_LATE && st_t >= 0) stage(st_t, st_kt, (step + 1) & 1);
      const char* s0 = smem + (step & 1) * STAGE;
      if constexpr (XK) {
        const int fo0 = fr * 128 + ((fq ^ (fr & 7)) << 4), fo1 = fr * 128 + (((4 + fq) ^ (fr & 7)) << 4);
        bf16x8 b2[2][TN], a2[2 * TM];
#pragma unroll
        for (int j = 0; j < TN; ++j) b2[0][j] = *(const bf16x8*)(s0 + OPA + (wn * WN + j * 16) * 128 + fo0);
#pragma unroll
        for (int g = 0; g < XD; ++g) a2[g] = *(const bf16x8*)(s0 + (wm * WM + g * 16) * 128 + fo0);
        if constexpr (XK_LATE) {
          __builtin_amdgcn_sched_barrier(0);
          if (st_t >= 0) stage(st_t, st_kt, (step + 1) & 1);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int g = 0; g < 2 * TM; ++g) {
          const int nx = g + XD;
          if (nx == TM) {
#pragma unroll
            for (int j = 0; j < TN; ++j) b2[1][j] = *(const bf16x8*)(s0 + OPA + (wn * WN + j * 16) * 128 + fo1);
          }
          if (nx < 2 * TM) a2[nx] = *(const bf16x8*)(s0 + (wm * WM + (nx % TM) * 16) * 128 + (nx < TM ? fo0 : fo1));
          __builtin_amdgcn_sched_barrier(0);
          if (XPRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[g % TM][j] = mma<true>(b2[g / TM][j], a2[g], acc[g % TM][j]);
          if (XPRIO) __builtin_amdgcn_s_setprio(0);
          __builtin_amdgcn_sched_barrier(0);
        }
        continue;
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int fo = fr * 128 + (((ks * 4 + fq) ^ (fr & 7)) << 4);
        bf16x8 bfr[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = *(const bf16x8*)(s0 + OPA + (wn * WN + j * 16) * 128 + fo);
        if constexpr (PF > 0) {
          bf16x8 a[TM];
#pragma unroll
          for (int i = 0; i < PF; ++i) a[i] = *(const bf16x8*)(s0 + (wm * WM + i * 16) * 128 + fo);
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            if (i + PF < TM) a[i + PF] = *(const bf16x8*)(s0 + (wm * WM + (i + PF) * 16) * 128 + fo);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = mma<true>(bfr[j], a[i], acc[i][j]);
            __builtin_amdgcn_sched_barrier(0);
          }
          continue;
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const bf16x8 af = *(const bf16x8*)(s0 + (wm * WM + i * 16) * 128 + fo);
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            if (ABL == 2) asm volatile("" ::"v"(bfr[j]), "v"(af));  // (PF = 0 for the ablations)
            else acc[i][j] = mma<true>(bfr[j], af, acc[i][j]);
          }
        }
      }
    }
    const int bm = t / nbn, bn = t - bm * nbn, mb = bm * BM + wm * WM, nb = bn * BN + wn * WN;
    if constexpr (SO) {
      if (tn >= 0) {  // every wave is done reading the last stage's buffer: stage 1 of the next tile into it
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (ABL != 1) stage(tn, 1, (step + 1) & 1);  // step = the next tile's k-step 0 here; its k-step 1 reads (step + 1) & 1
      }
      const bool tail = bm * BM + BM > M;  // the last row band of a ragged M: rows >= M are not stored
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = min(mb + i * 16 + fr, M - 1);
        const long orow = p.hm_n ? (((long)(m / p.hm_n) * (p.N / 64) + nb / 64) * p.hm_n + m % p.hm_n) * 64 - nb
                                 : (long)m * p.ldc;
        bf16_t* C = (bf16_t*)p.C + orow + 4 * fq;
        const bool ok = !tail || mb + i * 16 + fr < M;
        u32x2 pk[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          f32x4 v = acc[i][j];
          if (p.bias) v += *(const f32x4*)(sbias + (tcount & 1) * 256 + wn * WN + j * 16 + 4 * fq);
          if (p.epi == EPI_GELU) {
            const f32x2 lo = gelu_erf_fast2((f32x2){v[0], v[1]}), hi = gelu_erf_fast2((f32x2){v[2], v[3]});
            v = (f32x4){lo[0], lo[1], hi[0], hi[1]};
          }
          pk[j] = pack16x4<true>(v);
          if (ok && (f16_pair_nonfinite(pk[j][0]) || f16_pair_nonfinite(pk[j][1]))) range_bad = true;
          if (!WIDE && ok) *(u32x2*)(C + nb + j * 16) = pk[j];
        }
        if constexpr (WIDE) {
          // lanes fq (even) and fq + 1 hold columns 4 fq .. 4 fq + 7 of tiles j and j + 1: the even lane keeps
          // tile j's 8 columns, the odd lane tile j + 1's (the partner is 16 lanes away, same row)
          const bool odd = fq & 1;
#pragma unroll
          for (int j = 0; j < TN; j += 2) {
            const u32x2 snd = odd ? pk[j] : pk[j + 1];
            const u32x2 rcv = {(uint32_t)__shfl_xor((int)snd[0], 16, 64), (uint32_t)__shfl_xor((int)snd[1], 16, 64)};
            const u32x4 w = odd ? (u32x4){rcv[0], rcv[1], pk[j + 1][0], pk[j + 1][1]}
                                : (u32x4){pk[j][0], pk[j][1], rcv[0], rcv[1]};
            if (ok) *(u32x4*)(C + nb + (odd ? (j + 1) * 16 - 4 : j * 16)) = w;
          }
        }
      }
      // the counted waits of the next tile assume all NSTORE stores per wave were issued: not after a ragged tile
      // (its next tile waits vmcnt(0) and re-issues its stage 1 - the same bytes into the same buffer)
      seam = !tail;
    } else if constexpr (RES) {
      float* Cb = (float*)p.C + nb + 4 * fq;
      const float* bl = sbias + (tcount & 1) * 256 + wn * WN + 4 * fq;
      const bool tail = bm * BM + BM > M;  // ragged last row band: rows >= M neither read nor stored
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {  // row tiles [4 h2, min(TM, 4 h2 + 4))
        f32x4 rv[4][TN];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            if (h2 * 4 + i < TM)
              rv[i][j] = *(const f32x4*)(Cb + (long)min(mb + (h2 * 4 + i) * 16 + fr, M - 1) * p.ldc + j * 16);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (h2 * 4 + i >= TM) break;
          const int m = mb + (h2 * 4 + i) * 16 + fr;
          if (tail && m >= M) continue;
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            f32x4 a = acc[h2 * 4 + i][j];
            if (p.bias) a += *(const f32x4*)(bl + j * 16);
            *(f32x4*)(Cb + (long)m * p.ldc + j * 16) = rv[i][j] + a;
          }
        }
      }
      if (tn >= 0) {  // stage 1 of the next tile into the last stage's buffer, after the stores
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (ABL != 1) stage(tn, 1, (step + 1) & 1);
      }
      // k-step 0 of the next tile skips its vmcnt wait because the residual loads retired after its stage 0;
      // every lane loads (rows clamped), so that holds for ragged tiles too
      seam = true;
    } else {
      epilogue_256<TM, TN, true>(p, acc, mb, nb, fr, fq);
    }
    if (tn < 0) break;
    t = tn;
    ++tcount;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  // after the tile loop: no counted wait follows, so this store cannot disturb the seams' vmcnt arithmetic
  if (SO && p.range_flag && __any(range_bad) && lane == 0) range_flag_set(p.range_flag);
}

#ifdef ICAP_TOOLS
// ---------------------------------------------------------------------------------------------
// Persistent fp16 encoder GEMM, ping-pong form (gemm_f16q_kernel): the tile walk, tiles, modes (SO / RES)
// and epilogues of gemm_f16p_kernel, with a k-loop in which the two waves of each SIMD alternate between
// LDS reads and MFMAs.  gemm_f16p_kernel runs both waves of a SIMD in the same state (read 2 A fragments,
// wait, 8 MFMAs): its LDS latency is exposed at ~44 % MFMA issue.  Here waves 0-3 (rows 0-127 of the tile)
// lead and waves 4-7 (rows 128-255) trail by ONE barrier, and every phase is
//     R: [odd phase: counted vmcnt] [2 LDS-DMA instructions] [epilogue part] ds_read of the phase's operands
//     -- s_barrier --  M: 16 MFMA (setprio 1)  -- s_barrier --
// so a SIMD's leading wave issues its MFMAs while its trailing wave reads, and the other way round.
// Phases of a 64-deep k-step (rh = 64-row half of the wave tile, h = 32-deep k-half):
//     (rh0, h0): A 4 + W 4 reads; (rh1, h0): A 4; (rh1, h1): A 4 + W 4; (rh0, h1): A 4
// so every LDS byte is read once per wave and the h0 half of a k-step is free after its second phase.
// LDS: a ring of 4 k-half slots (A [256][32] + W [256][32] fp16, 64-B rows, 32 KiB each; 16-B chunk c of
// row r at c ^ (-(r >> 2) & 3), conflict-free for the ds_read_b128 lane groups of MI355X_MICROARCH.md) plus
// two 1 KiB bias slots.  Half v (the block's halves in (tile, k) order) is read in phases 2v, 2v + 1.
// Global phase q: the leading group's R(q) lies between barriers 2q - 1 and 2q, the trailing group's between
// 2q and 2q + 1, and every wave's reads of phase q are consumed by its MFMAs before barrier 2q + 2.  So
//   * half v's A rows are DMA'd in R(2v - 5), its W rows in R(2v - 4): after barrier 4v - 12, by which every
//     read of half v - 4 (same slot) is done;
//   * R(2v - 1) waits vmcnt(4) (half v + 1's 4 instructions may pend) before barrier 4v - 2 / 4v - 1, and
//     half v is first read in R(2v), after barrier 4v - 1 / 4v.
// A tile's epilogue is split over the next tile's first two R segments (rows rh0 before the MFMAs that
// overwrite acc[0..3], rh1 before acc[4..7]), so one group's stores overlap the other's MFMAs; their 16 + 16
// stores per wave stay in flight: the following odd waits count 20, then 36 (VMEM retires in issue order;
// a wait may count fewer operations than were issued after its target, never more - so extra operations
// such as the RES residual loads or wave 0's bias DMA only make it conservative).  A ragged last row band
// skips stores, so its successors count 4.  RES issues each half's residual loads before the segment's DMA
// instructions (the compiler's wait for them then leaves the fresh DMA in flight).
// Measured (tools/f16q_check.sh, tools build, ICAP_F16_PP=1): correct - all GPU tests pass with it - but slower
// than gemm_f16p_kernel: QKV 258 -> 305 us, MLP-1 356 -> 457, MLP-2 324 -> 402, encoder 15.2 -> 17.8 ms/step.
// The k-loop is not held by LDS latency: gemm_f16p_kernel's timing ablations (tools/f16_ablate.sh) put its DMA
// alone and its LDS reads + MFMAs alone at ~200 us each for QKV, and here the 64-B k-half rows double the
// cache-line requests of every DMA instruction.  Kept in the tools build only.
template <int MODE>
__global__ __launch_bounds__(512, 1) void gemm_f16q_kernel(GemmArgs p) {
  constexpr bool SO = MODE == 1, RES = MODE == 2;
  static_assert(SO || RES, "store-only or residual epilogue");
  constexpr int BM = 256, BN = 256, WM = 128, WN = 64, TN = 4;
  constexpr int SLOT = 32768, OPH = 16384;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int nbn = p.N / BN, nbm = (p.M + BM - 1) / BM, nwg = nbn * nbm;
  const int xcd = blockIdx.x & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int xbase = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8, xcnt = q8 + (xcd < r8);
  const int nbx = ((int)gridDim.x - xcd + 7) >> 3, lb = blockIdx.x >> 3;
  if (lb >= xcnt) return;
  const int M = p.M, hpt = p.K / 32;            // k-halves per tile (even, >= 4)
  const int ntl = (xcnt - lb + nbx - 1) / nbx;  // tiles xbase + lb + j nbx, j < ntl
  const int nh = ntl * hpt;
  const int fr = lane & 15, fq = lane >> 4;
  const int schunk = (lane & 3) ^ ((4 - (lane >> 4)) & 3);  // DMA lane: row lane >> 2 of a 16-row block
  const int fsw = (fq ^ ((4 - (fr >> 2)) & 3)) << 4;         // fragment lane: row fr of a 16-row tile
  float* sbias = (float*)(smem + 4 * SLOT);

  auto tile_of = [&](int j) { return xbase + lb + j * nbx; };
  auto stage = [&](int v, int part) {  // half v, part 0 = its A rows, 1 = its W rows: 2 instructions per wave
    const int j = v / hpt, hh = v - j * hpt, t = tile_of(j);
    const int bm = t / nbn, bn = t - bm * nbn;
    char* dst = smem + (v & 3) * SLOT + part * OPH + wave * 2048;
    const int r0 = wave * 32 + (lane >> 2);
    if (part == 0) {
      const bf16_t* src = p.A + hh * 32 + schunk * 8;
#pragma unroll
      for (int i = 0; i < 2; ++i)
        __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)(src + (long)min(bm * BM + r0 + i * 16, M - 1) * p.lda),
                                         (LDS_AS void*)(dst + i * 1024), 16, 0, 0);
    } else {
      const bf16_t* src = p.W + (long)(bn * BN + r0) * p.ldw + hh * 32 + schunk * 8;
#pragma unroll
      for (int i = 0; i < 2; ++i)
        __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)(src + (long)i * 16 * p.ldw),
                                         (LDS_AS void*)(dst + i * 1024), 16, 0, 0);
    }
  };
  auto load_bias = [&](int j) {  // tile j's 256 bias values -> bias slot j & 1 (wave 0, one DMA instruction)
    if (wave == 0 && p.bias) {
      const int t = tile_of(j), n0 = (t - (t / nbn) * nbn) * BN;
      __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)(p.bias + n0 + lane * 4),
                                       (LDS_AS void*)(sbias + (j & 1) * 256), 16, 0, 0);
    }
  };

  f32x4 acc[8][TN];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  f32x4 rv[4][TN];  // RES: one row half of the residual
  // tile je's rows of half rh: RES loads (issued before the segment's DMA), then bias (+ GELU) and stores
  auto epi_load = [&](int je, int rh) {
    if constexpr (RES) {
      const int t = tile_of(je), bm = t / nbn, bn = t - bm * nbn;
      const int mb = bm * BM + wm * WM, nb = bn * BN + wn * WN;
      const float* Cb = (const float*)p.C + nb + 4 * fq;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          rv[i][j] = *(const f32x4*)(Cb + (long)min(mb + (rh * 4 + i) * 16 + fr, M - 1) * p.ldc + j * 16);
    }
  };
  auto epi_store = [&](int je, int rh) {
    const int t = tile_of(je), bm = t / nbn, bn = t - bm * nbn;
    const int mb = bm * BM + wm * WM, nb = bn * BN + wn * WN;
    const bool tail = bm * BM + BM > M;
    const float* bl = sbias + (je & 1) * 256 + wn * WN + 4 * fq;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ii = rh * 4 + i, mr = mb + ii * 16 + fr;
      if constexpr (SO) {
        const int m = min(mr, M - 1);
        const long orow = p.hm_n ? (((long)(m / p.hm_n) * (p.N / 64) + nb / 64) * p.hm_n + m % p.hm_n) * 64 - nb
                                 : (long)m * p.ldc;
        bf16_t* C = (bf16_t*)p.C + orow + 4 * fq;
        const bool ok = !tail || mr < M;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          f32x4 v = acc[ii][j];
          if (p.bias) v += *(const f32x4*)(bl + j * 16);
          if (p.epi == EPI_GELU) {
            const f32x2 lo = gelu_erf_fast2((f32x2){v[0], v[1]}), hi = gelu_erf_fast2((f32x2){v[2], v[3]});
            v = (f32x4){lo[0], lo[1], hi[0], hi[1]};
          }
          if (ok) *(u32x2*)(C + nb + j * 16) = pack16x4<true>(v);
        }
      } else {
        float* Cb = (float*)p.C + nb + 4 * fq;
        if (!tail || mr < M) {
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            f32x4 a = acc[ii][j];
            if (p.bias) a += *(const f32x4*)(bl + j * 16);
            *(f32x4*)(Cb + (long)mr * p.ldc + j * 16) = rv[i][j] + a;
          }
        }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[ii][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
    return tail;
  };

  // prologue: halves 0 and 1 and half 2's A rows in flight, half 0 retired
  load_bias(0);
  stage(0, 0);
  stage(0, 1);
  stage(1, 0);
  stage(1, 1);
  stage(2, 0);
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (wm) __builtin_amdgcn_s_barrier();  // the trailing group runs one barrier behind
  asm volatile("" ::: "memory");

  bf16x8 af[4], bfr[4];
  const int nsteps = nh >> 1, kspt = hpt >> 1;  // 64-deep k-steps: in total, per tile
  int ec = 0;        // odd-phase waits left that count the previous tile's epilogue stores (20, then 36)
  int je = -1;       // tile whose epilogue runs in this k-step's first two R segments (-1: none)
  int kt = 0, j = 0;  // k-step within tile j
  for (int s = 0; s < nsteps; ++s) {
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const int q = 4 * s + ph, h = ph >> 1, rh = (ph == 1 || ph == 2) ? 1 : 0;
      // ---- R segment
      if (ph & 1) {
        if ((q + 3) / 2 < nh) {  // half (q + 1) / 2 retired; half (q + 3) / 2 (+ epilogue stores) may pend
          if (ec == 2) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
          else if (ec == 1) asm volatile("s_waitcnt vmcnt(36)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (ec) --ec;
      }
      if (ph <= 1 && je >= 0) epi_load(je, ph);
      __builtin_amdgcn_sched_barrier(0);
      if (ph & 1) {
        const int vs = (q + 5) / 2;
        if (vs < nh) {
          if (vs % hpt == 0) load_bias(vs / hpt);
          stage(vs, 0);
        }
      } else {
        const int vs = (q + 4) / 2;
        if (vs < nh) stage(vs, 1);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (ph <= 1 && je >= 0) {
        const bool tail = epi_store(je, ph);
        if (ph == 0) ec = tail ? 0 : 2;
        else je = -1;
      }
      const char* sb = smem + ((2 * s + h) & 3) * SLOT;
      if (ph == 0 || ph == 2) {
#pragma unroll
        for (int jj = 0; jj < TN; ++jj) bfr[jj] = *(const bf16x8*)(sb + OPH + (wn * WN + jj * 16 + fr) * 64 + fsw);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *(const bf16x8*)(sb + (wm * WM + rh * 64 + i * 16 + fr) * 64 + fsw);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      // ---- M segment
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < TN; ++jj) acc[rh * 4 + i][jj] = mma<true>(bfr[jj], af[i], acc[rh * 4 + i][jj]);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
    if (++kt == kspt) {  // tile j done: its epilogue runs in the next k-step's first two R segments
      kt = 0;
      je = j++;
    }
  }
  // the last tile: the leading group matches the trailing group's extra barrier first
  if (!wm) __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  epi_load(je, 0);
  epi_store(je, 0);
  epi_load(je, 1);
  epi_store(je, 1);
}

#endif  // ICAP_TOOLS

}  // namespace

// ---------------------------------------------------------------------------------------------
// Encoder GEMM, 8-phase schedule (cdna_hip_programming.md "The 256^2 8-phase template").
// 256 x 256 block tile, BK = 64, 8 waves as 2 (M) x 4 (N), wave tile 128 x 64 = 8 x 4 MFMA tiles,
// computed as four 64 x 32 quadrants, one per phase:
//   phase: ds_read the quadrant's register subtile -> issue ONE half-tile of LDS-DMA prefetch ->
//          [last phase of a K-tile: counted vmcnt] -> s_barrier -> lgkmcnt(0) -> setprio(1),
//          16 MFMA, setprio(0) -> s_barrier
// LDS (128 KiB): 2 K-tile buffers x {A, W} x 2 k-halves x 256 rows x 64 B; 16-B chunk c of row r at
// c ^ (((r >> 3) & 1) << 1) (pre-swizzled on the DMA source, conflict-free 16-row fragment reads).
// Half-tiles (16 KiB, 2 DMA instructions per wave) are the operand rows of ONE quadrant, loaded in
// the order of their last read in a K-tile (A qm=0 @ phase 0, W qn=1 @ 1, A qm=1 @ 2, W qn=0 @ 3): load j
// (= 4 t + x) is issued in phase j - 7, one phase after the lgkmcnt(0)+barrier that retired the
// previous reads of its buffer, and every K-tile is retired by a vmcnt(6) (3 half-tiles left in
// flight) in the last phase of the K-tile before it.  bf16x2: the activation planes are further
// K-tiles (K' = nsplit K; the W k-tile is re-staged per plane from L2).
namespace {

template <bool ROW128, bool F16 = false>
__global__ __launch_bounds__(512) void gemm_8ph_kernel(GemmArgs p) {
  constexpr int BM = 256, BK = 64, KH = 16384, BUF = 65536;  // k-half region, buffer bytes
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int nbn = p.N / BM, nbm = (p.M + BM - 1) / BM, nwg = nbn * nbm;
  const int orig = blockIdx.x, xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int bm = wg / nbn, bn = wg - bm * nbn;
  const int m0 = bm * BM, n0 = bn * BM;
  const int M = p.M, K = p.K;
  const int ktp = K / BK, nk = p.nsplit * ktp, nloads = 4 * nk;

  // DMA geometry: a half-tile is the part of the K-tile ONE phase's quadrant reads, so its last
  // read falls in one phase: A half q = rows {64 q .. 64 q + 63} of both wave rows (wr = 0, 1),
  // W half q = rows {64 wc + 32 q .. + 31} of all four wave columns.  Wave w DMAs 16 of those rows
  // per k-half (one 1 KiB instruction each); the LDS image stays row-major [k-half][256 rows][64 B].
  // ROW128: LDS image [256 rows][128 B] per operand (both k-halves in one row), one DMA instruction
  // = 8 rows x a full 128-B line, chunk c of row r at c ^ ((r >> 1) & 7); otherwise [k-half][rows][64 B]
  // with 16 rows x 64 B per instruction, chunk c at c ^ (((r >> 3) & 1) << 1).
  const int lchunk = (lane & 3) ^ ((((lane >> 2) >> 3) & 1) << 1);  // 64-B rows: row bit 3 == (lane >> 2) bit 3
  const int a_row0 = (wave >> 2) * 128 + (wave & 3) * 16;          // + 64 q
  const int w_row0 = (wave >> 1) * 64 + (wave & 1) * 16;            // + 32 q
  auto issue = [&](int j) {  // half-tile load j -> K-tile j / 4, half x = j % 4 (A q0, W q1, A q1, W q0)
    const int t = j >> 2, x = j & 3;
    const bool isA = !(x & 1);
    const int q = (x == 1 || x == 2) ? 1 : 0;
    const int plane = t / ktp, k0 = (t - plane * ktp) * BK;
    const int rbase = isA ? a_row0 + 64 * q : w_row0 + 32 * q;  // this wave's 16 rows
    char* dst = smem + (t & 1) * BUF + (isA ? 0 : 2 * KH) + rbase * (ROW128 ? 128 : 64);
    if (ROW128) {
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const int row = rbase + g * 8 + (lane >> 3);                 // rbase is 16-aligned
        const int c128 = (lane & 7) ^ ((row >> 1) & 7);
        const bf16_t* src = isA ? p.A + plane * p.a_lo + (long)min(m0 + row, M - 1) * p.lda + k0 + c128 * 8
                                : p.W + (long)(n0 + row) * p.ldw + k0 + c128 * 8;
        __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)src, (LDS_AS void*)(dst + g * 1024), 16, 0, 0);
      }
    } else {
      const int row = rbase + (lane >> 2);
      const bf16_t* src = isA ? p.A + plane * p.a_lo + (long)min(m0 + row, M - 1) * p.lda + k0 + lchunk * 8
                              : p.W + (long)(n0 + row) * p.ldw + k0 + lchunk * 8;
      __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)src, (LDS_AS void*)dst, 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const GLOBAL_AS void*)(src + 32), (LDS_AS void*)(dst + KH), 16, 0, 0);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  bf16x8 ra[4][2], rb[2][2];  // register subtiles: A [m-tile][k-half], W [n-tile][k-half]

  const int fr = lane & 15, fq = lane >> 4;
  // fragment (row r = 16-aligned base + fr, k-chunk kh * 4 + fq) byte offsets within an operand image
  const int fsw = (fq ^ (((fr >> 3) & 1) << 1)) << 4;  // row bit 3 == fr bit 3 (tile rows are 16-aligned)
  auto foff = [&](int rbase, int kh) -> int {
    if (ROW128) return (rbase + fr) * 128 + (((kh * 4 + fq) ^ ((fr >> 1) & 7)) << 4);
    return kh * KH + (rbase + fr) * 64 + fsw;
  };
  auto read_a = [&](const char* buf, int qm) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) ra[i][kh] = *(const bf16x8*)(buf + foff(wr * 128 + qm * 64 + i * 16, kh));
  };
  auto read_b = [&](const char* buf, int qn) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) rb[j][kh] = *(const bf16x8*)(buf + 2 * KH + foff(wc * 64 + qn * 32 + j * 16, kh));
  };
  auto mfma_q = [&](int qm, int qn) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[qm * 4 + i][qn * 2 + j] = mma<F16>(rb[j][kh], ra[i][kh], acc[qm * 4 + i][qn * 2 + j]);
    __builtin_amdgcn_s_setprio(0);
  };

  // prologue: loads 0..6 in flight, K-tile 0 retired
  for (int j = 0; j < 7 && j < nloads; ++j) issue(j);
  if (nloads > 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  for (int t = 0; t < nk; ++t) {
    const char* buf = smem + (t & 1) * BUF;
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const int qm = ph >> 1, qn = (ph == 1 || ph == 2) ? 1 : 0;
      if (ph == 0) {
        read_b(buf, 0);
        __builtin_amdgcn_sched_barrier(0);
        read_a(buf, 0);
      } else if (ph == 2) {
        read_a(buf, 1);
      } else {
        read_b(buf, qn);
      }
      const int j = 4 * t + ph + 7;
      if (j < nloads) issue(j);
      if (ph == 3) {
        // retire K-tile t + 1: loads beyond 4t + 7 that are already issued may stay in flight
        const int ahead = min(nloads, 4 * t + 11) - (4 * t + 8);
        if (ahead >= 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else if (ahead == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else if (ahead == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      mfma_q(qm, qn);
      __builtin_amdgcn_s_barrier();
    }
  }

  epilogue_256<8, 4, F16>(p, acc, m0 + wr * 128, n0 + wc * 64, fr, fq);
}

}  // namespace

hipError_t launch_gemm_256_(const GemmArgs& g, hipStream_t s);
hipError_t launch_gemm_256(const GemmArgs& g0, hipStream_t s) {
  // ICAP_GEMM_GROUP: tile raster of the bf16 encoder GEMM (0 = row-band major)
  static const int group = std::max(0, icap_knob("ICAP_GEMM_GROUP", 0));
  GemmArgs g = g0;
  if (!g.raster_group) g.raster_group = group;
  return launch_gemm_256_(g, s);
}
hipError_t launch_gemm_256_(const GemmArgs& g, hipStream_t s) {
  if (g.M <= 0 || g.N % 256 || g.K % 32 || g.batch != 1 || (g.nsplit != 1 && g.nsplit != 2))
    return hipErrorInvalidValue;
  const long last_row = g.rm_group ? (long)((g.M - 1) / g.rm_group) * g.rm_stride + g.rm_off + g.rm_group : g.M;
  if (last_row * g.ldc >= (1L << 31)) return hipErrorInvalidValue;  // epilogue uses 32-bit row offsets
  constexpr int lds2 = 3 * 3 * 256 * 32 * 2, lds1 = 4 * 2 * 256 * 32 * 2;
  static int nw = 0;
  if (!nw) {
    nw = icap_knob("ICAP_GEMM256_WAVES", 16);  // experiment knob: 8, 16, or 1/2 = 8-phase kernel
    if (nw != 8 && nw != 16 && nw != 1 && nw != 2 && nw != 160 && nw != 161 && nw != 162) nw = 16;
    hipError_t e = hipSuccess;
#ifdef ICAP_TOOLS
    for (const void* f : {(const void*)gemm_8ph_kernel<false>, (const void*)gemm_8ph_kernel<true>})
      if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 131072) != hipSuccess)
        return hipErrorInvalidValue;
    for (const void* f : {(const void*)gemm_256_kernel<2, 16, 1>, (const void*)gemm_256_kernel<2, 16, 2>,
                          (const void*)gemm_256_kernel<2, 16, 3>})
      if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds2);
#endif
    for (const void* f : {(const void*)gemm_256_kernel<2, 8>, (const void*)gemm_256_kernel<2, 16>,
                          (const void*)gemm_256_kernel<2, 16, 0, 1>})
      if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds2);
    for (const void* f : {(const void*)gemm_256_kernel<1, 8>, (const void*)gemm_256_kernel<1, 16>,
                          (const void*)gemm_256_kernel<1, 16, 0, 1>})
      if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds1);
    if (e != hipSuccess) return e;
  }
  // 128 x 256 tiles, 2-stage ring, 2 blocks per CU for K >= ICAP_GEMM_TALL_MIN_K (default 128; 0 = off):
  // ViT 42.9 -> 41.8 ms/step (MLP-out's 591 tiles become 1182: 4.6 instead of 2.3 rounds), trunk
  // conv3 203 -> 177 us; at K = 64 the 3-stage 256 x 256 ring stays ahead (tools/halfk_sweep.sh)
  static const int tall_min_k = icap_knob("ICAP_GEMM_TALL_MIN_K", 128);
  // ICAP_GEMM_TALL_BM: 128 (default) or 64 (64 x 256 tiles, 4 waves, 3 blocks per CU)
  static const int tall_bm = icap_knob("ICAP_GEMM_TALL_BM", 128) == 64 ? 64 : 128;
  if (g.f16) {  // fp16 single plane (ICAP_PREC_F16 encoder)
    if (g.nsplit != 1 || g.cv || g.res || g.scale || (g.out == OUT_SPLIT && g.c_planes != 1) || g.K < 128)
      return hipErrorInvalidValue;
    // ICAP_F16_GEMM: 0 = 128 x 256 tiles, 2-stage ring, 2 blocks per CU; 1 / 2 = 256 x 256 8-phase (64-B / 128-B LDS rows)
    static const int form = icap_knob("ICAP_F16_GEMM", 0);
    if ((form == 1 || form == 2) && g.K % 64 == 0) {
      static bool attr8 = false;
      if (!attr8) {
        for (const void* f : {(const void*)gemm_8ph_kernel<false, true>, (const void*)gemm_8ph_kernel<true, true>})
          if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 131072) != hipSuccess)
            return hipErrorInvalidValue;
        attr8 = true;
      }
      const int nwg8 = (g.N / 256) * ((g.M + 255) / 256);
      if (form == 2) hipLaunchKernelGGL((gemm_8ph_kernel<true, true>), dim3(nwg8), dim3(512), 131072, s, g);
      else hipLaunchKernelGGL((gemm_8ph_kernel<false, true>), dim3(nwg8), dim3(512), 131072, s, g);
      return hipGetLastError();
    }
    // store-only epilogues with whole 256-row bands (the ViT QKV and MLP-1 GEMMs): the persistent counted-seam
    // form by default (QKV 305 -> 265 us, MLP-1 423 -> 342 us at B = 256, tools/f16_forms_r2.sh); form 6 (tools)
    // also runs the residual GEMMs persistent (slower: the residual epilogue's loads serialise the seam)
    const bool so = gemm_f16_persistent(g);
    if ((form == 6 && g.K % 64 == 0) || so) {
      static int cus = 0;
      if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
          return hipErrorInvalidValue;
        for (const void* f : {(const void*)gemm_f16p_kernel<0>, (const void*)gemm_f16p_kernel<1>,
                              (const void*)gemm_f16p_kernel<2>, (const void*)gemm_f16p_kernel<2, 0, 224>})
          if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * 64 * 1024 + 2048) != hipSuccess)
            return hipErrorInvalidValue;
#ifdef ICAP_TOOLS
        for (const void* f : {(const void*)gemm_f16q_kernel<1>, (const void*)gemm_f16q_kernel<2>})
          if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 4 * 32 * 1024 + 2048) != hipSuccess)
            return hipErrorInvalidValue;
#endif
      }
      const int tiles = (g.N / 256) * ((g.M + 255) / 256);
      const dim3 grid(std::min(tiles, cus));
#ifdef ICAP_TOOLS
      // ICAP_F16P_ABL (tools): gemm_f16p_kernel without its k-loop DMA (1) or without its MFMAs (2) - wrong
      // results, timing only (tools/f16_ablate.sh); 3 / 4 / 5: the compiler's fragment-read order / the read pipeline per k-half / the stage's DMA
      // before the first fragment reads
      static const int abl = icap_knob("ICAP_F16P_ABL", 0);
      if (so && abl >= 1 && abl <= 8) {
        static bool attr = false;
        if (!attr) {
          for (const void* f : {(const void*)gemm_f16p_kernel<1, 1>, (const void*)gemm_f16p_kernel<2, 1>,
                                (const void*)gemm_f16p_kernel<1, 2>, (const void*)gemm_f16p_kernel<2, 2>,
                                (const void*)gemm_f16p_kernel<1, 3>, (const void*)gemm_f16p_kernel<2, 3, 224>,
                                (const void*)gemm_f16p_kernel<1, 4>, (const void*)gemm_f16p_kernel<2, 4, 224>,
                                (const void*)gemm_f16p_kernel<1, 5>, (const void*)gemm_f16p_kernel<2, 5, 224>,
                                (const void*)gemm_f16p_kernel<1, 6>, (const void*)gemm_f16p_kernel<2, 6, 224>,
                                (const void*)gemm_f16p_kernel<1, 7>, (const void*)gemm_f16p_kernel<2, 7, 224>,
                                (const void*)gemm_f16p_kernel<1, 8>})
            if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 2 * 64 * 1024 + 2048) != hipSuccess)
              return hipErrorInvalidValue;
          attr = true;
        }
        const bool res = g.out == OUT_F32_RESID;
        if (abl == 1 && res) hipLaunchKernelGGL((gemm_f16p_kernel<2, 1>), grid, dim3(512), 2 * 64 * 1024 + 2048, s, g);
        else if (abl == 1) hipLaunchKernelGGL((gemm_f16p_kernel<1, 1>), grid, dim3(512), 2 * 64 * 1024 + 2048, s, g);
        else if (abl == 2 && res) hipLaunchKernelGGL((gemm_f16p_kernel<2, 2>), grid, dim3(512), 2 * 64 * 1024 + 2048, s, g);
        else if (abl == 2) hipLaunchKernelGGL((gemm_f16p_kernel<1, 2>), grid, dim3(512), 2 * 64 * 1024 + 2048, s, g);
        else if (res && abl == 3)
          hipLaunchKernelGGL((gemm_f16p_kernel<2, 3, 224>), dim3(std::min((g.N / 256) * ((g.M + 223) / 224), cus)),
                             dim3(512), 2 * (224 * 128 + 256 * 128) + 2048, s, g);
        else if (res && abl == 4)
          hipLaunchKernelGGL((gemm_f16p_kernel<2, 4, 224>), dim3(std::min((g.N / 256) * ((g.M + 223) / 224), cus)),
                             dim3(512), 2 * (224 * 128 + 256 * 128) + 2048, s, g);
        else if (res && abl == 5)
          hipLaunchKernelGGL((gemm_f16p_kernel<2, 5, 224>), dim3(std::min((g.N / 256) * ((g.M + 223) / 224), cus)),
                             dim3(512), 2 * (224 * 128 + 256 * 128) + 2048, s, g);
        else if (res && abl == 6)
          hipLaunchKernelGGL((gemm_f16p_kernel<2, 6, 224>), dim3(std::min((g.N / 256) * ((g.M + 223) / 224), cus)),
                             dim3(512), 2 * (224 * 128 + 256 * 128) + 2048, s, g);
        else if (res && abl == 7)
          hipLaunchKernelGGL((gemm_f16p_kernel<2, 7, 224>), dim3(std::min((g.N / 256) * ((g.M + 223) / 224), cus)),
                             dim3(512), 2 * (224 * 128 + 256 * 128) + 2048, s, g);
        else if (res)  // (8: the SO store width; the residual form as built)
          hipLaunchKernelGGL((gemm_f16p_kernel<2, 0, 224>), dim3(std::min((g.N / 256) * ((g.M + 223) / 224), cus)),
                             dim3(512), 2 * (224 * 128 + 256 * 128) + 2048, s, g);
        else if (abl == 3) hipLaunchKernelGGL((gemm_f16p_kernel<1, 3>), grid, dim3(512), 2 * 64 * 1024 + 2048, s, g);
        else if (abl == 4) hipLaunchKernelGGL((gemm_f16p_kernel<1, 4>), grid, dim3(512), 2 * 64 * 1024 + 2048, s, g);
        else if (abl == 5) hipLaunchKernelGGL((gemm_f16p_kernel<1, 5>), grid, dim3(512), 2 * 64 * 1024 + 2048, s, g);
        else if (abl == 6) hipLaunchKernelGGL((gemm_f16p_kernel<1, 6>), grid, dim3(512), 2 * 64 * 1024 + 2048, s, g);
        else if (abl == 7) hipLaunchKernelGGL((gemm_f16p_kernel<1, 7>), grid, dim3(512), 2 * 64 * 1024 + 2048, s, g);
        else hipLaunchKernelGGL((gemm_f16p_kernel<1, 8>), grid, dim3(512), 2 * 64 * 1024 + 2048, s, g);
        return hipGetLastError();
      }
      // ICAP_F16_PP=1 (tools): the ping-pong k-loop (gemm_f16q_kernel; slower)
      static const int pp = icap_knob("ICAP_F16_PP", 0);
      if (so && pp) {
        if (g.out == OUT_F32_RESID)
          hipLaunchKernelGGL(gemm_f16q_kernel<2>, grid, dim3(512), 4 * 32 * 1024 + 2048, s, g);
        else
          hipLaunchKernelGGL(gemm_f16q_kernel<1>, grid, dim3(512), 4 * 32 * 1024 + 2048, s, g);
        return hipGetLastError();
      }
#endif
      // residual GEMMs: 224-row tiles (ICAP_F16_RES_BM=256 in the tools build: the 256-row form)
      static const int res_bm = icap_knob("ICAP_F16_RES_BM", 224);
      if (so && g.out == OUT_F32_RESID && res_bm == 224) {
        const int tiles224 = (g.N / 256) * ((g.M + 223) / 224);
        hipLaunchKernelGGL((gemm_f16p_kernel<2, 0, 224>), dim3(std::min(tiles224, cus)), dim3(512),
                           2 * (224 * 128 + 256 * 128) + 2048, s, g);
        return hipGetLastError();
      }
      if (so && g.out == OUT_F32_RESID)
        hipLaunchKernelGGL(gemm_f16p_kernel<2>, grid, dim3(512), 2 * 64 * 1024 + 2048, s, g);
      else if (so)
        hipLaunchKernelGGL(gemm_f16p_kernel<1>, grid, dim3(512), 2 * 64 * 1024 + 2048, s, g);
      else
        hipLaunchKernelGGL(gemm_f16p_kernel<0>, grid, dim3(512), 2 * 64 * 1024, s, g);
      return hipGetLastError();
    }
#ifdef ICAP_TOOLS
    // 3 / 4: 128 x 256 tiles with 64-deep (full-line) stages, 2 / 3 stages (96 / 144 KiB, one block per CU);
    // 5: 256 x 256 tiles, 64-deep stages, 2 stages (128 KiB)
    if (form >= 3 && form <= 5 && g.K % 64 == 0) {
      static bool attr = false;
      if (!attr) {
        if (hipFuncSetAttribute((const void*)gemm_256_kernel<1, 8, 0, 0, 128, 2, 64, 0, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 2 * 48 * 1024) != hipSuccess ||
            hipFuncSetAttribute((const void*)gemm_256_kernel<1, 8, 0, 0, 128, 3, 64, 0, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 3 * 48 * 1024) != hipSuccess ||
            hipFuncSetAttribute((const void*)gemm_256_kernel<1, 8, 0, 0, 256, 2, 64, 0, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 2 * 64 * 1024) != hipSuccess)
          return hipErrorInvalidValue;
        attr = true;
      }
      if (form == 5)
        hipLaunchKernelGGL((gemm_256_kernel<1, 8, 0, 0, 256, 2, 64, 0, true>), dim3((g.N / 256) * ((g.M + 255) / 256)),
                           dim3(512), 2 * 64 * 1024, s, g);
      else if (form == 4)
        hipLaunchKernelGGL((gemm_256_kernel<1, 8, 0, 0, 128, 3, 64, 0, true>), dim3((g.N / 256) * ((g.M + 127) / 128)),
                           dim3(512), 3 * 48 * 1024, s, g);
      else
        hipLaunchKernelGGL((gemm_256_kernel<1, 8, 0, 0, 128, 2, 64, 0, true>), dim3((g.N / 256) * ((g.M + 127) / 128)),
                           dim3(512), 2 * 48 * 1024, s, g);
      return hipGetLastError();
    }
#endif
    const int nwgh = (g.N / 256) * ((g.M + 127) / 128);
    constexpr int ldsh1 = 2 * (128 * 32 * 2 + 256 * 32 * 2);
    hipLaunchKernelGGL((gemm_256_kernel<1, 8, 0, 0, 128, 2, 32, 0, true>), dim3(nwgh), dim3(512), ldsh1, s, g);
    return hipGetLastError();
  }
  if (tall_min_k && g.K >= tall_min_k && (nw == 8 || nw == 16) && tall_bm == 64 && !g.cv) {
    const int nwgq = (g.N / 256) * ((g.M + 63) / 64);
    constexpr int ldsq = 2 * (2 * 64 * 32 * 2 + 256 * 32 * 2), ldsq1 = 2 * (64 * 32 * 2 + 256 * 32 * 2);
    if (g.nsplit == 2) hipLaunchKernelGGL((gemm_256_kernel<2, 4, 0, 0, 64, 2>), dim3(nwgq), dim3(256), ldsq, s, g);
    else hipLaunchKernelGGL((gemm_256_kernel<1, 4, 0, 0, 64, 2>), dim3(nwgq), dim3(256), ldsq1, s, g);
    return hipGetLastError();
  }
  // ICAP_GEMM_TALL_KS: 32 (default) or 64 (64-deep stages, 128 KiB, 1 block per CU)
  static const int tall_ks = icap_knob("ICAP_GEMM_TALL_KS", 32) == 64 ? 64 : 32;
  if (tall_min_k && g.K >= tall_min_k && (nw == 8 || nw == 16) && tall_ks == 64 && g.K % 64 == 0) {
    const int nwgh = (g.N / 256) * ((g.M + 127) / 128);
    constexpr int lds64 = 2 * (2 * 128 * 64 * 2 + 256 * 64 * 2), lds64_1 = 2 * (128 * 64 * 2 + 256 * 64 * 2);
    static bool attr64 = false;
    if (!attr64) {
      hipError_t e = hipSuccess;
      for (const void* f : {(const void*)gemm_256_kernel<2, 8, 0, 0, 128, 2, 64>,
                            (const void*)gemm_256_kernel<2, 8, 0, 1, 128, 2, 64>})
        if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds64);
      for (const void* f : {(const void*)gemm_256_kernel<1, 8, 0, 0, 128, 2, 64>,
                            (const void*)gemm_256_kernel<1, 8, 0, 1, 128, 2, 64>})
        if (e == hipSuccess) e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds64_1);
      if (e != hipSuccess) return e;
      attr64 = true;
    }
    if (g.cv && g.cv != 1) return hipErrorInvalidValue;
    if (g.nsplit == 2) {
      if (g.cv) hipLaunchKernelGGL((gemm_256_kernel<2, 8, 0, 1, 128, 2, 64>), dim3(nwgh), dim3(512), lds64, s, g);
      else hipLaunchKernelGGL((gemm_256_kernel<2, 8, 0, 0, 128, 2, 64>), dim3(nwgh), dim3(512), lds64, s, g);
    } else {
      if (g.cv) hipLaunchKernelGGL((gemm_256_kernel<1, 8, 0, 1, 128, 2, 64>), dim3(nwgh), dim3(512), lds64_1, s, g);
      else hipLaunchKernelGGL((gemm_256_kernel<1, 8, 0, 0, 128, 2, 64>), dim3(nwgh), dim3(512), lds64_1, s, g);
    }
    return hipGetLastError();
  }
  if (tall_min_k && g.K >= tall_min_k && (nw == 8 || nw == 16)) {
    const int nwgh = (g.N / 256) * ((g.M + 127) / 128);
    constexpr int ldsh = 2 * (2 * 128 * 32 * 2 + 256 * 32 * 2), ldsh1 = 2 * (128 * 32 * 2 + 256 * 32 * 2);
    if (g.cv && g.cv != 1) return hipErrorInvalidValue;
#ifdef ICAP_TOOLS  // tail split of the residual GEMMs: measured and rejected
    const int S = g.split_slots, q = nwgh >> 3;
    if (g.split_ws && g.split_cnt && S > 0 && !g.cv && q + 1 > S && (g.K / 32) % 2 == 0) {
      const int tq1 = (q + 1) % S, tq = q > S ? q % S : 0;
      const int per_xcd = std::max(q + 1 + tq1, q + tq);
      if (g.nsplit == 2)
        hipLaunchKernelGGL((gemm_256_kernel<2, 8, 0, 0, 128, 2, 32, 1>), dim3(8 * per_xcd), dim3(512), ldsh, s, g);
      else
        hipLaunchKernelGGL((gemm_256_kernel<1, 8, 0, 0, 128, 2, 32, 1>), dim3(8 * per_xcd), dim3(512), ldsh1, s, g);
      return hipGetLastError();
    }
#else
    if (g.split_slots) return hipErrorNotSupported;
#endif
    if (g.nsplit == 2) {
      if (g.cv) hipLaunchKernelGGL((gemm_256_kernel<2, 8, 0, 1, 128, 2>), dim3(nwgh), dim3(512), ldsh, s, g);
      else hipLaunchKernelGGL((gemm_256_kernel<2, 8, 0, 0, 128, 2>), dim3(nwgh), dim3(512), ldsh, s, g);
    } else {
      if (g.cv) hipLaunchKernelGGL((gemm_256_kernel<1, 8, 0, 1, 128, 2>), dim3(nwgh), dim3(512), ldsh1, s, g);
      else hipLaunchKernelGGL((gemm_256_kernel<1, 8, 0, 0, 128, 2>), dim3(nwgh), dim3(512), ldsh1, s, g);
    }
    return hipGetLastError();
  }
  const int nwg = (g.N / 256) * ((g.M + 255) / 256);
  const GemmArgs& g2 = g;
  if (g.cv) {  // implicit-GEMM 3x3 convolution
    if (g.cv != 1) return hipErrorInvalidValue;
    if (g.nsplit == 2) hipLaunchKernelGGL((gemm_256_kernel<2, 16, 0, 1>), dim3(nwg), dim3(1024), lds2, s, g2);
    else hipLaunchKernelGGL((gemm_256_kernel<1, 16, 0, 1>), dim3(nwg), dim3(1024), lds1, s, g2);
    return hipGetLastError();
  }
#ifdef ICAP_TOOLS  // measured-and-rejected forms: the 8-phase kernel, staging-only variants (wrong results)
  if ((nw == 1 || nw == 2) && g.K % 64 == 0) {
    if (nw == 2) hipLaunchKernelGGL(gemm_8ph_kernel<true>, dim3(nwg), dim3(512), 131072, s, g);
    else hipLaunchKernelGGL(gemm_8ph_kernel<false>, dim3(nwg), dim3(512), 131072, s, g);
    return hipGetLastError();
  }
  if ((nw == 160 || nw == 161 || nw == 162) && g.nsplit == 2) {
    if (nw == 160) hipLaunchKernelGGL((gemm_256_kernel<2, 16, 1>), dim3(nwg), dim3(1024), lds2, s, g2);
    else if (nw == 161) hipLaunchKernelGGL((gemm_256_kernel<2, 16, 2>), dim3(nwg), dim3(1024), lds2, s, g2);
    else hipLaunchKernelGGL((gemm_256_kernel<2, 16, 3>), dim3(nwg), dim3(1024), lds2, s, g2);
    return hipGetLastError();
  }
#endif
  if (g.nsplit == 2) {
    if (nw == 16) hipLaunchKernelGGL((gemm_256_kernel<2, 16>), dim3(nwg), dim3(1024), lds2, s, g2);
    else hipLaunchKernelGGL((gemm_256_kernel<2, 8>), dim3(nwg), dim3(512), lds2, s, g2);
  } else {
    if (nw == 16) hipLaunchKernelGGL((gemm_256_kernel<1, 16>), dim3(nwg), dim3(1024), lds1, s, g2);
    else hipLaunchKernelGGL((gemm_256_kernel<1, 8>), dim3(nwg), dim3(512), lds1, s, g2);
  }
  return hipGetLastError();
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
