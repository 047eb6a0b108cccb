// Device templates of the encoder GEMMs, shared by the product translation unit (gemm.hip) and the tools
// build's measurement unit (gemm_tools.hip, compiled only with -DICAP_TOOLS): the implicit-conv row helpers,
// the 256-wide epilogue, gemm_256_kernel and the persistent fp16 gemm_f16p_kernel.  Template parameters that
// select measured-and-rejected variants (NOMFMA, TS, KSD = 64, ABL) and the rejected gemm_f16r_kernel (three A
// slots) are instantiated only by gemm_tools.hip.
#pragma once
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

}  // namespace

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
          if constexpr (F16)
            acc[i][j][r] += h2f((bf16_t)(wh & 0xffff)) + h2f((bf16_t)(wl & 0xffff));
          else
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
        for (int r = 0; r < 4; ++r) acc[i][j][r] = F16 ? gelu_erf_as(acc[i][j][r]) : gelu_erf_fast(acc[i][j][r]);
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
  } else if (F16) {  // one fp16 plane, or hi / lo fp16 planes (c_planes == 2: the Grid trunk's residual stream)
    bf16_t* C = (bf16_t*)p.C;
    const bool lo_plane = p.out == OUT_SPLIT && p.c_planes == 2;
    bool bad = false;  // fp16 range guard: a stored value that is not finite in fp16
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if (orow[i] < 0) continue;
        const u32x2 hv = pack16x4<true>(acc[i][j]);
        bad |= f16_pair_nonfinite(hv[0]) || f16_pair_nonfinite(hv[1]);
        *(u32x2*)(C + orow[i] + nb + j * 16 + 4 * fq) = hv;
        if (lo_plane) {
          f32x4 lo;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const uint32_t w = hv[r >> 1] >> ((r & 1) * 16);
            lo[r] = acc[i][j][r] - h2f((bf16_t)(w & 0xffff));
          }
          *(u32x2*)(C + orow[i] + nb + j * 16 + 4 * fq + p.c_lo) = pack16x4<true>(lo);
        }
      }
    if (p.range_flag && __any(bad) && (threadIdx.x & 63) == 0) range_flag_set(p.range_flag);
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

// Epilogue of the trunk convolutions (GemmArgs::scale set: eval BatchNorm folded into scale / shift): out =
// relu?(acc * scale + shift (+ residual planes)) as split planes (bf16, or fp16 with F16), nothing else - no row
// remaps, addends or other output forms, so the accumulators plus one column group's operands are all that is live
// (the generic epilogue_256 spilled 34-38 VGPRs at the 128-register budget of two blocks per CU).
// The residual planes of a wave's conv tile, loaded whole (PRE: issued before the tile's first stage, so their latency
// overlaps the stage DMA instead of adding one more memory round trip after the k-loop).  Rows >= M load row M - 1.
template <int TM, int TN, bool F16>
__device__ __forceinline__ void conv_res_load(const GemmArgs& p, int mb, int nb, int fr, int fq, u32x2 (&rh)[TN][TM],
                                              u32x2 (&rl)[TN][TM]) {
  if (!p.res) return;
  const bool res2 = !(F16 && p.res_planes == 1);
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const long ro = (long)min(mb + i * 16 + fr, p.M - 1) * p.res_ld + nb + j * 16 + 4 * fq;
      rh[j][i] = *(const u32x2*)(p.res + ro);
      rl[j][i] = res2 ? *(const u32x2*)(p.res + ro + p.res_lo) : (u32x2){0u, 0u};
    }
}

// PRE: the residual planes come in prh / prl (conv_res_load), else they are loaded here per column-group batch.
template <int TM, int TN, bool F16, bool PRE = false>
__device__ __forceinline__ void epilogue_conv(const GemmArgs& p, f32x4 (&acc)[TM][TN], int mb, int nb, int fr, int fq,
                                              const u32x2 (*prh)[TM] = nullptr, const u32x2 (*prl)[TM] = nullptr) {
  const int M = p.M;
  const bool res = p.res != nullptr, res2 = !(F16 && p.res_planes == 1), lo_out = p.c_planes == 2;
  const bool relu = p.epi == EPI_RELU;
  constexpr int JG = TN >= 2 ? 2 : 1;  // column groups per batch of loads (one memory latency per batch; all 4: 172 VGPRs spilled)
  bf16_t* C = (bf16_t*)p.C;
  bool bad = false;  // F16: a stored value that is not finite in fp16 (range guard)
#pragma unroll
  for (int j0 = 0; j0 < TN; j0 += JG) {
    f32x4 sv[JG], bv[JG];
    u32x2 rh[JG][TM], rl[JG][TM];
#pragma unroll
    for (int jj = 0; jj < JG; ++jj) {
      const int col = nb + (j0 + jj) * 16 + 4 * fq;
      sv[jj] = *(const f32x4*)(p.scale + col);
      bv[jj] = *(const f32x4*)(p.bias + col);
    }
    if (PRE) {
#pragma unroll
      for (int jj = 0; jj < JG; ++jj)
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          rh[jj][i] = prh[j0 + jj][i];
          rl[jj][i] = prl[j0 + jj][i];
        }
    } else if (res) {  // (plane count hoisted: a per-element "load or not" select would wait after each load)
      if (res2) {
#pragma unroll
        for (int jj = 0; jj < JG; ++jj)
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const long ro = (long)min(mb + i * 16 + fr, M - 1) * p.res_ld + nb + (j0 + jj) * 16 + 4 * fq;
            rh[jj][i] = *(const u32x2*)(p.res + ro);
            rl[jj][i] = *(const u32x2*)(p.res + ro + p.res_lo);
          }
      } else {
#pragma unroll
        for (int jj = 0; jj < JG; ++jj)
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const long ro = (long)min(mb + i * 16 + fr, M - 1) * p.res_ld + nb + (j0 + jj) * 16 + 4 * fq;
            rh[jj][i] = *(const u32x2*)(p.res + ro);
            rl[jj][i] = (u32x2){0u, 0u};
          }
      }
    }
#pragma unroll
    for (int jj = 0; jj < JG; ++jj) {
      const int j = j0 + jj, col = nb + j * 16 + 4 * fq;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = mb + i * 16 + fr;
        f32x4 v = acc[i][j] * sv[jj] + bv[jj];
        if (res)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const uint32_t wh = rh[jj][i][r >> 1] >> ((r & 1) * 16), wl = rl[jj][i][r >> 1] >> ((r & 1) * 16);
            if constexpr (F16)
              v[r] += h2f((bf16_t)(wh & 0xffff)) + h2f((bf16_t)(wl & 0xffff));
            else
              v[r] += bf2f((bf16_t)(wh & 0xffff)) + bf2f((bf16_t)(wl & 0xffff));
          }
        if (relu)
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
        if (m >= M) continue;
        const long o = (long)m * p.ldc + col;
        const u32x2 hv = pack16x4<F16>(v);
        if (F16) bad |= f16_pair_nonfinite(hv[0]) || f16_pair_nonfinite(hv[1]);
        *(u32x2*)(C + o) = hv;
        if (lo_out) {
          f32x4 lo;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const bf16_t hb = (bf16_t)((hv[r >> 1] >> ((r & 1) * 16)) & 0xffff);
            lo[r] = v[r] - (F16 ? h2f(hb) : bf2f(hb));
          }
          *(u32x2*)(C + o + p.c_lo) = pack16x4<F16>(lo);
        }
      }
    }
  }
  if (F16 && p.range_flag && __any(bad) && (threadIdx.x & 63) == 0) range_flag_set(p.range_flag);
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
// EPC: the epilogue is epilogue_conv (the trunk convolutions: GemmArgs::scale set) instead of epilogue_256 - a
// compile-time choice, so each kernel holds one epilogue's registers (both in one kernel spilled 27-36 VGPRs).
// BNT: block tile columns, 256 or (narrow outputs: the trunk's layer1-2 convolutions, N = 64 / 128) 128 or 64 - the
// wave grid becomes (NW / (BNT / 64)) x (BNT / 64) of 64-column wave tiles, two blocks per CU.
template <int NS, int NW, int NOMFMA = 0, int CONV = 0, int BMT = 256, int NST = 0, int KSD = 32, int TS = 0,
          bool F16 = false, bool EPC = false, int BNT = 256>
__global__ __launch_bounds__(NW * 64, (BMT == 128 && KSD == 32) ? 4 : (BNT < 256 ? 2 : (BMT == 64 ? 3 : 1)))
void gemm_256_kernel(GemmArgs p) {
  constexpr int WGN = BNT / 64, WGM = NW / WGN;     // wave grid WGM x WGN
  constexpr int BM = BMT, BN = BNT, WM = BM / WGM, WN = 64, TM = WM / 16, TN = WN / 16;
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
  const int wm = wave / WGN, wn = wave % WGN;
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
        lds_dma16(src, (LDS_AS void*)(s0 + pl * OPB + (wave * IPW + i) * 1024));
      }
    }
#pragma unroll
    for (int i = 0; i < IPWW; ++i)
      lds_dma16(b_base + kin + i * b_step, (LDS_AS void*)(s0 + NS * OPB + (wave * IPWW + i) * 1024));
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  const int foff = fr * 64 + ((fq ^ (((fr >> 3) & 1) << 1)) << 4);
  // PRE (the 64-deep conv forms): the residual planes load before the first stage - older than every stage DMA, so
  // the counted waits below still count only stages (the first one also covers these loads)
  constexpr bool PRE = EPC && KSD == 64;
  u32x2 prh[PRE ? TN : 1][TM], prl[PRE ? TN : 1][TM];
  if constexpr (PRE)
    if (!p.no_pre) conv_res_load<TM, TN, F16>(p, m0 + wm * WM, n0 + wn * WN, fr, fq, prh, prl);
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
  if constexpr (EPC) {  // trunk convolutions
    if (PRE && !p.no_pre) epilogue_conv<TM, TN, F16, PRE>(p, acc, m0 + wm * WM, n0 + wn * WN, fr, fq, prh, prl);
    else epilogue_conv<TM, TN, F16>(p, acc, m0 + wm * WM, n0 + wn * WN, fr, fq);
  }
  else {
    epilogue_256<TM, TN, F16>(p, acc, m0 + wm * WM, n0 + wn * WN, fr, fq);
  }
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
// MFMA group (no gain, tools/f16_pf.sh), 8 = 8-byte SO stores, 9 = no LDS fragment reads (opaque registers), 10 = no
// k-loop DMA and no k-step barrier, 11 = 10 without the SO stores, 12 = 10 without the SO epilogue (timing
// ablations, round 3: tools/r3_ablate.sh).
// BMT: tile rows, 256 or (RES) 224 - wave tiles 112 x 64, the A stage 224 rows (wave 7 DMAs W rows only): at
// N = 768 the 256-row tiles are 591 = 2.3 per CU (3 rounds, the last 30 % full), 224-row tiles 678 = 2.65 per CU
// (3 rounds of 7/8 the work).
// The LDS position of 16-byte chunk c of row r in a 64-deep (128-B row) stage of the persistent fp16 GEMMs; the stage
// DMA reads chunk swz_chunk(l & 7, r) into lane l's slot, the fragment reads find chunk c at swz_chunk(c, r).
// ICAP_SWZ 0: c ^ (r & 7) - conflict-free ds_read_b128 fragment reads, but the DMA's lanes then read each 64-B half-line
// out of order and the address unit splits it (round-6 PMC: TCP accesses 2x hipBLASLt's on the same bytes, TA busy
// 1.68x); 1: c ^ (4 ((r >> 1) & 1)) - each half-line read in order by 4 consecutive lanes, 2-way read conflicts
#ifndef ICAP_SWZ
#define ICAP_SWZ 0
#endif
__device__ __forceinline__ int swz_chunk(int c, int r) { return ICAP_SWZ ? c ^ (((r >> 1) & 1) << 2) : c ^ (r & 7); }

// The LayerNorm fold of the f16 ViT encoder (GemmArgs::xh / ln_*; rows.hip launch_ln_fold_*), measured and rejected in
// round 6 (its residual epilogue's fp16 copy of x and the store-only epilogue's row affine cost
// more than the LayerNorm passes they remove); compiled into variant builds only (-DICAP_LN_FOLD=1 for gemm.hip and
// icap.cpp)
#ifndef ICAP_LN_FOLD
#define ICAP_LN_FOLD 0
#endif
// dynamic LDS of gemm_f16p_kernel<1> (and <2> at 256 rows): 2 stages of 64 KiB, then the bias slots (2 x 1 KiB), the
// LayerNorm fold's column-sum slots (2 x 1 KiB) and row (a, b) slots (2 x 2 KiB), then the stream-K ticket word
constexpr int F16P_LDS_TAIL = ICAP_LN_FOLD ? 8192 : 2048;
constexpr int f16p_lds(int BM) { return 2 * (BM * 128 + 256 * 128) + F16P_LDS_TAIL + 16; }
constexpr int F16P_LDS_SO = f16p_lds(256);

// stage pieces wave w of gemm_f16p_kernel issues per stage: its A rows (8 per piece, up to the tile's BM rows) + IPW W
constexpr int f16p_stage_pieces(int BM, int IPW, int w) {
  const int a = (BM - w * IPW * 8) / 8;
  return (a <= 0 ? 0 : a < IPW ? a : IPW) + IPW;
}
// the opening waits: vmcnt(IPW) for a wave with w IPW 8 >= BM (224-row tiles: W pieces only), else vmcnt(2 IPW)
constexpr bool f16p_waits_match(int BM, int IPW, int NW) {
  for (int w = 0; w < NW; ++w)
    if (f16p_stage_pieces(BM, IPW, w) != ((BM < 256 && w * IPW * 8 >= BM) ? IPW : 2 * IPW)) return false;
  return true;
}

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
  // the counted opening / seam waits below assume wave w issues f16p_stage_pieces(BM, IPW, w) pieces per stage (the
  // stage lambda's A loop stops at the tile's last row): PER_STAGE, or IPW (W rows only) for a wave past a 224-row
  // tile's A image (ADVICE r4 / VERDICT r5: tie each wait to the pieces the wave issues)
  static_assert(f16p_waits_match(BM, IPW, NW), "per-wave stage piece counts vs the opening waits");
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
  const int srow = wave * IPW * 8 + (lane >> 3), schunk = swz_chunk(lane & 7, srow);
  const int fr = lane & 15, fq = lane >> 4;

#ifndef ICAP_F16P_PRIO
#define ICAP_F16P_PRIO 0
#endif
  // ICAP_F16P_PRIO (compile-time form, round 5): the younger wave of each SIMD (waves 4-7) at priority 1 for the
  // whole launch (cdna_hip_programming.md T5, static form) - within noise (frac 0.2913-0.2929, same box), off
  if (ICAP_F16P_PRIO && __builtin_amdgcn_readfirstlane(tid) >= 256) __builtin_amdgcn_s_setprio(1);

#ifndef ICAP_F16P_BUF
#define ICAP_F16P_BUF 1
#endif
#ifndef ICAP_F16P_PROD
#define ICAP_F16P_PROD 0
#endif
  // ICAP_F16P_PROD (compile-time form, round 5, buffer DMA only): the stage DMA issued by waves 0-3 alone (16 pieces
  // each), so one wave per SIMD carries the DMA issue cost and the other only MFMAs; the counted seam waits then
  // differ per wave (a wave waits only for the pieces it issued; the barrier publishes them)
  constexpr bool PROD = ICAP_F16P_PROD && ICAP_F16P_BUF;
#ifndef ICAP_F16P_LB
#define ICAP_F16P_LB 1
#endif
  // ICAP_F16P_LB (compile-time form, round 5): the k-step barrier moved two MFMA groups before the end of the k-step
  // (the "late point"): there the wave waits for the next stage (vmcnt) and for its own reads of this buffer
  // (lgkmcnt), passes the barrier, issues the stage after next into this buffer and reads the next k-step's first
  // fragments, whose latency then hides behind this k-step's last two MFMA groups instead of stalling every wave at
  // the top of the next k-step.  Every tile's stages 0 and 1 are issued before its k-step 0 (prologue / seam); the
  // stage after next is issued at each late point (the next tile's stage 0 at the last-but-one k-step); the last
  // k-step of a tile has no late point (the epilogue needs every group).
  constexpr bool LB = ICAP_F16P_LB && XK && !PROD && ABL == 0;
  // ICAP_F16P_BUF (compile-time form, round 5): the stage pieces as buffer loads (32-bit per-lane row offsets in the
  // resource of A / W, the k-step in the scalar offset) instead of flat 64-bit per-lane addresses: 10 fewer VGPRs and
  // frac 0.2924-0.2931 -> 0.2941-0.2951 on one box (profiles/r05/gemm_buf_ab.txt; 0 = the flat form)
  const long bytesA = (long)M * p.lda * 2, bytesW = (long)p.N * p.ldw * 2;
  const i32x4r rsA = buf_rsrc(p.A, (uint32_t)(bytesA < 0xffffffffL ? bytesA : 0xffffffffL));
  const i32x4r rsW = buf_rsrc(p.W, (uint32_t)(bytesW < 0xffffffffL ? bytesW : 0xffffffffL));
  auto stage = [&](int t, int kt, int buf) {  // tile t (logical), k-step kt -> ring buffer buf
    const int bm = t / nbn, bn = t - bm * nbn, m0 = bm * BM, n0 = bn * BN;
    char* s0 = smem + buf * STAGE;
    if constexpr (ICAP_F16P_BUF) {
      // PROD: waves 0 .. 3 issue the pieces of waves w and w + 4 (the others issue none)
      if (PROD && wave >= 4) return;
#pragma unroll
      for (int v = 0; v < (PROD ? 2 : 1); ++v) {
        const int vw = wave + 4 * v, vrow = srow + v * 4 * IPW * 8;
#pragma unroll
        for (int i = 0; i < IPW; ++i) {
          if (BM < 256 && (vw * IPW + i) * 8 >= BM) break;
          const int row = min(m0 + vrow + i * 8, M - 1);
          lds_dma_buf16(rsA, (uint32_t)(row * p.lda + schunk * 8) * 2, (uint32_t)kt * KS * 2,
                        (LDS_AS void*)(s0 + (vw * IPW + i) * 1024));
        }
#pragma unroll
        for (int i = 0; i < IPW; ++i)
          lds_dma_buf16(rsW, (uint32_t)((n0 + vrow + i * 8) * p.ldw + schunk * 8) * 2, (uint32_t)kt * KS * 2,
                        (LDS_AS void*)(s0 + OPA + (vw * IPW + i) * 1024));
      }
      return;
    }
    const bf16_t* Ab = p.A + kt * KS + schunk * 8;
    const bf16_t* Wb = p.W + (long)(n0 + srow) * p.ldw + kt * KS + schunk * 8;
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      if (BM < 256 && (wave * IPW + i) * 8 >= BM) break;  // (wave-uniform) rows past the tile's A image
      const int row = min(m0 + srow + i * 8, M - 1);
      lds_dma16(Ab + (long)row * p.lda, (LDS_AS void*)(s0 + (wave * IPW + i) * 1024));
    }
#pragma unroll
    for (int i = 0; i < IPW; ++i) lds_dma16(Wb + (long)i * 8 * p.ldw, (LDS_AS void*)(s0 + OPA + (wave * IPW + i) * 1024));
  };
  // SO: the tile's 256 bias values go to LDS slot (tile count & 1) by one DMA instruction of wave 0, issued
  // before the tile's first stage (so the counted waits below never count it) - no registers held across
  // the k-loop (the kernel is at the 256-register limit of two waves per SIMD)
  float* sbias = (float*)(smem + 2 * STAGE);
  // LayerNorm fold (SO with p.ln_ab, kernels.h): per tile also the 256 column sums s_n (slot after the bias slots, wave
  // 1) and the tile's 256 rows' (a, b) (wave 2: rows 0-127, wave 3: 128-255) - older than the tile's stage 0 like the
  // bias, so no counted wait moves
  const bool lnf = ICAP_LN_FOLD && SO && p.ln_ab != nullptr;
  float* ssum = sbias + 2 * 256;
  float2* sab = (float2*)(sbias + 4 * 256);
  // (buffer-load DMAs: one per-lane 32-bit offset shared by the three sources, the tile's offset in an SGPR - 64-bit
  // per-lane addresses held across the k-loop spilled)
  const i32x4r rsb = buf_rsrc(p.bias, (uint32_t)p.N * 4), rss = buf_rsrc(p.ln_sum, (uint32_t)p.N * 4);
  const i32x4r rsab = buf_rsrc(p.ln_ab, (uint32_t)(M + 256) * 8);  // (padded by a tile past M: ragged bands in bounds)
  auto load_bias = [&](int t, int slot) {
    const int bm = t / nbn, n0 = (t - bm * nbn) * BN;
    if (wave == 0 && p.bias) lds_dma_buf16(rsb, (uint32_t)lane * 16, (uint32_t)n0 * 4, (LDS_AS void*)(sbias + slot * 256));
    if (lnf && wave >= 1 && wave <= 3) {
      if (wave == 1) lds_dma_buf16(rss, (uint32_t)lane * 16, (uint32_t)n0 * 4, (LDS_AS void*)(ssum + slot * 256));
      else
        lds_dma_buf16(rsab, (uint32_t)lane * 16, (uint32_t)(bm * BM + (wave - 2) * 128) * 8,
                      (LDS_AS void*)(sab + slot * 256 + (wave - 2) * 128));
    }
  };

  // Stream-K (round 6, ICAP_F16P_SK = 1 for gemm.hip and icap.cpp, variant builds; measured slower - DESIGN.md section 8:
  // with the partial exchange removed the schedule alone gains nothing on MLP-1 / MLP-2, so the last partial round of
  // whole tiles costs less than its share of tiles, and the exchange adds 20-40 us per launch; the late-barrier k-loop
  // only).  Whole tiles leave a partial last round: 2364 MLP-1
  // tiles are 9.23 per CU (10 rounds), the residual GEMMs' 678 tiles 2.65 (3 rounds).  Per XCD the xcnt tiles are
  // walked by VB virtual lanes: RP whole rounds (lane v: tiles v, v + VB, ...), then the remaining T2 = xcnt - RP VB
  // tiles (VB <= T2 < 3 VB) as one sequence of T2 nk k-steps cut into VB contiguous ranges at even k-steps - lane v
  // runs [bnd(v), bnd(v + 1)).  Every range is >= nk + 2 k-steps long, so a tile is cut at most once: its head
  // [0, k) ends one lane's range, its tail [k, nk) opens the next.  A cut tile's two units meet through the workspace
  // slot of their boundary: the first to finish stores its fp32 accumulators (device-coherent stores) and raises the
  // slot's ready word, the second adds them to its own (fp32 addition commutes: the same sums whichever comes first)
  // and runs the tile's epilogue.  The schedule depends on the shape only (VB is fixed; a grid of fewer blocks runs
  // several lanes per block), so the results do not depend on the grid (CU-masked encoder streams).
  constexpr int VB = F16P_SK_VB;
  constexpr int SKW = NW * 64 * TM * TN * 4;  // floats of one partial tile
  static_assert(SKW <= F16P_SK_SLOT, "stream-K slot size");
  const int xq = xcnt / VB, xr = xcnt - xq * VB;
  int RP = -1;  // whole rounds before the stream-K part; -1: no stream-K (every tile whole, t, t + nbx, ...)
  if (ICAP_F16P_SK && LB && (SO || RES) && p.sk_ws && p.sk_cnt && xr && nbx <= VB && (nk & 1) == 0 && nk >= 2) {
    if (xq >= 1 && xr * nk >= 2 * VB) RP = xq - 1;  // ranges of (VB + xr) nk / VB >= nk + 2 k-steps
    else if (xq >= 2) RP = xq - 2;                    // (2 VB + xr) nk / VB >= 2 nk
  }
  const bool sk = RP >= 0;
  const int sk_t0 = xbase + (sk ? RP : 0) * VB, sk_w2h = sk ? (xcnt - RP * VB) * nk / 2 : 0;
  auto bnd = [&](int v) { return 2 * (int)((uint32_t)v * (uint32_t)sk_w2h / (uint32_t)VB); };
  struct Unit {
    int t, k0, k1, v, r;  // tile (-1: none), k-steps [k0, k1), lane, whole round (r == RP: the stream-K part)
  };
  auto sk_unit = [&](int v, int pos) -> Unit {  // lane v's unit at k-step pos of the stream-K sequence
    const int u = (int)((uint32_t)pos / (uint32_t)nk), k0 = pos - u * nk;
    return Unit{sk_t0 + u, k0, min(nk, bnd(v + 1) - u * nk), v, RP};
  };
  auto first_unit = [&](int v) -> Unit { return RP > 0 ? Unit{xbase + v, 0, nk, v, 0} : sk_unit(v, bnd(v)); };
  auto next_unit = [&](const Unit& c) -> Unit {
    if (!sk) return Unit{c.t + nbx < xbase + xcnt ? c.t + nbx : -1, 0, nk, 0, 0};
    if (c.r + 1 < RP) return Unit{xbase + c.v + (c.r + 1) * VB, 0, nk, c.v, c.r + 1};
    if (c.r + 1 == RP) return sk_unit(c.v, bnd(c.v));
    const int pos = (c.t + 1 - sk_t0) * nk;  // a unit ending inside its tile ends its lane's range
    if (c.k1 == nk && pos < bnd(c.v + 1)) return Unit{c.t + 1, 0, min(nk, bnd(c.v + 1) - pos), c.v, RP};
    return c.v + nbx < VB ? first_unit(c.v + nbx) : Unit{-1, 0, nk, 0, 0};
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  Unit cu = sk ? first_unit(lb) : Unit{xbase + lb, 0, nk, 0, 0};
  int t = cu.t, step = 0, tcount = 0;
  if (SO || RES) load_bias(t, 0);
  stage(t, cu.k0, 0);
  if (LB) stage(t, cu.k0 + 1, 1);  // LB: both stages of a tile's opening in flight before its k-step 0
  bool seam = false;  // this tile's stages 0 and 1 were issued before the previous tile's epilogue stores
  bool range_bad = false;  // SO: some stored fp16 value is not finite (p.range_flag set once, after the last tile)
  // stream-K: the (ticket, ready) broadcast word in LDS after the bias / fold slots
  int* const sk_word = (int*)(smem + 2 * STAGE + F16P_LDS_TAIL);
  // a cut tile's meeting (block-uniform; every wave calls it): true = this block runs the tile's epilogue with the other
  // unit's accumulators added.  The first unit's block stores its partial and raises ready; the second waits for ready
  // (bounded: a lost partner ends the wait instead of hanging the grid) and loads the partial
#ifndef ICAP_SK_ABL
#define ICAP_SK_ABL 0
#endif
  auto sk_meet = [&](const Unit& c) -> bool {
    if (ICAP_SK_ABL == 2) return c.k0 == 0;  // timing ablation (wrong sums): no exchange, the head unit stores
    const int slot = (blockIdx.x & 7) * VB + (c.k0 > 0 ? c.v : c.v + 1);
    int* const cnt = p.sk_cnt + 2 * slot;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(p.sk_ws + (long)slot * F16P_SK_SLOT, 0, SKW * 4, 0x00020000);
    if (tid == 0) *sk_word = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const bool second = *(volatile int*)sk_word != 0;
    if (!second) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)  // device-coherent (sc1) 16-byte stores, [i TN + j][thread]
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs,
                                                 (uint32_t)((i * TN + j) * NW * 64 + tid) * 16, 0, 16);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's partial is complete
      __syncthreads();
      if (tid == 0) __hip_atomic_store(cnt + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    if (tid == 0) {
      for (int it = 0; it < (1 << 22) && __hip_atomic_load(cnt + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0; ++it)
        __builtin_amdgcn_s_sleep(1);
      __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // zero at rest for the next launch
      __hip_atomic_store(cnt + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < TM; ++i) {  // one row tile at a time (registers: the accumulators fill the file)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] += __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)((i * TN + j) * NW * 64 + tid) * 16, 0, 17));
      __builtin_amdgcn_sched_barrier(0);
    }
    return true;
  };
  for (;;) {
    const Unit un = next_unit(cu);  // this block's next unit
    const int tn = un.t;
    if constexpr (LB) {
      const int fo0 = fr * 128 + (swz_chunk(fq, fr) << 4), fo1 = fr * 128 + (swz_chunk(4 + fq, fr) << 4);
      bf16x8 b2[2][TN], a2[2 * TM];
      for (int kt = cu.k0; kt < cu.k1; ++kt, ++step) {
        const char* s0 = smem + (step & 1) * STAGE;
        if (kt == cu.k0) {  // a tile's opening: stage 0 landed (stage 1 and, after a seam, the stores may still fly)
          if (SO && seam) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PER_STAGE + NSTORE) : "memory");
          else if (RES && seam) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          // (224-row tiles: the last wave DMAs W rows only, IPW pieces per stage - stage 1 in flight is IPW, not 8)
          else if (BM < 256 && wave * IPW * 8 >= BM) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(IPW) : "memory");
          else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PER_STAGE) : "memory");
          __builtin_amdgcn_s_barrier();
#pragma unroll
          for (int j = 0; j < TN; ++j) b2[0][j] = *(const bf16x8*)(s0 + OPA + (wn * WN + j * 16) * 128 + fo0);
#pragma unroll
          for (int g = 0; g < XD; ++g) a2[g] = *(const bf16x8*)(s0 + (wm * WM + g * 16) * 128 + fo0);
        }
        const bool late = kt + 1 < cu.k1;  // the last k-step of a tile has no late point
        // a k-step entered from a late point carries its b2[0] fragments only (register budget): A fragments 0 and 1 now
        if (kt > cu.k0) {
          a2[0] = *(const bf16x8*)(s0 + (wm * WM) * 128 + fo0);
          a2[1] = *(const bf16x8*)(s0 + (wm * WM + 16) * 128 + fo0);
        }
        auto group = [&](int g) {  // reads two groups ahead, then group g's MFMAs
          const int nx = g + XD;
          if (nx == TM) {
#pragma unroll
            for (int j = 0; j < TN; ++j) b2[1][j] = *(const bf16x8*)(s0 + OPA + (wn * WN + j * 16) * 128 + fo1);
          }
          if (nx < 2 * TM) a2[nx] = *(const bf16x8*)(s0 + (wm * WM + (nx % TM) * 16) * 128 + (nx < TM ? fo0 : fo1));
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[g % TM][j] = mma<true>(b2[g / TM][j], a2[g], acc[g % TM][j]);
          __builtin_amdgcn_sched_barrier(0);
        };
#pragma unroll
        for (int g = 0; g < 2 * TM - XD; ++g) group(g);
        if (late) {
          // the late point: the next stage landed (after a seam's k-step 0 the stores may still fly; the RES seam
          // issued stage 1 after its stores), this wave's reads of this buffer retired, then the barrier
          if (SO && seam && kt == cu.k0) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NSTORE) : "memory");
          else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");
          // the next k-step's first fragments (its buffer is the other one), then the stage after next into this one
          const char* s1 = smem + ((step + 1) & 1) * STAGE;
          bf16x8 nb[TN];
#pragma unroll
          for (int j = 0; j < TN; ++j) nb[j] = *(const bf16x8*)(s1 + OPA + (wn * WN + j * 16) * 128 + fo0);
          __builtin_amdgcn_sched_barrier(0);
          if (kt + 2 < cu.k1) {
            stage(t, kt + 2, step & 1);
          } else if (tn >= 0) {  // the next unit's bias and first stage
            if (SO || RES) load_bias(tn, (tcount + 1) & 1);
            stage(tn, un.k0, step & 1);
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int g = 2 * TM - XD; g < 2 * TM; ++g) {  // this k-step's last groups (their fragments are in registers)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[g % TM][j] = mma<true>(b2[g / TM][j], a2[g], acc[g % TM][j]);
            __builtin_amdgcn_sched_barrier(0);
          }
#pragma unroll
          for (int j = 0; j < TN; ++j) b2[0][j] = nb[j];
        } else {
#pragma unroll
          for (int g = 2 * TM - XD; g < 2 * TM; ++g) group(g);
        }
      }
    } else
    for (int kt = 0; kt < nk; ++kt, ++step) {
      // lgkmcnt(0): this wave's reads of the buffer about to be refilled are done before the barrier
      if (SO && seam && kt == 0) {
        if (!PROD) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PER_STAGE + NSTORE) : "memory");
        else if (wave < 4) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * PER_STAGE + NSTORE) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NSTORE) : "memory");
      }
      else if (SO && seam && kt == 1) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NSTORE) : "memory");
      else if (RES && seam && kt == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      if (ABL < 10) __builtin_amdgcn_s_barrier();
      int st_t = -1, st_kt = 0;  // the stage this k-step DMAs into the other buffer (-1: none)
      if ((SO || RES) && seam && kt == 0) {
        // stage 1 of this tile is already in flight
      } else if (kt + 1 < nk) {
        st_t = t, st_kt = kt + 1;
      } else if (tn >= 0) {  // the next tile's bias, then its first stage, behind this k-step's MFMAs
        if (SO || RES) load_bias(tn, (tcount + 1) & 1);
        st_t = tn;
      }
      if (ABL == 1 || ABL >= 10) st_t = -1;
      // XK (default): the k-step's first fragment reads go out before the stage's 8 DMA instructions, whose
      // issue then covers their latency (ABL 5: DMA first)
      if (!XK_LATE && st_t >= 0) stage(st_t, st_kt, (step + 1) & 1);
      const char* s0 = smem + (step & 1) * STAGE;
      if constexpr (XK) {
        const int fo0 = fr * 128 + (swz_chunk(fq, fr) << 4), fo1 = fr * 128 + (swz_chunk(4 + fq, fr) << 4);
        bf16x8 b2[2][TN], a2[2 * TM];
        auto rd = [&](const char* ptr) -> bf16x8 {  // ABL 9: an opaque register instead of the LDS read
          if constexpr (ABL == 9) {
            u32x4 v = {(uint32_t)lane, 1u, 2u, (uint32_t)tid};
            asm volatile("" : "+v"(v));
            return __builtin_bit_cast(bf16x8, v);
          } else {
            return *(const bf16x8*)ptr;
          }
        };
#pragma unroll
        for (int j = 0; j < TN; ++j) b2[0][j] = rd(s0 + OPA + (wn * WN + j * 16) * 128 + fo0);
#pragma unroll
        for (int g = 0; g < XD; ++g) a2[g] = rd(s0 + (wm * WM + g * 16) * 128 + fo0);
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
            for (int j = 0; j < TN; ++j) b2[1][j] = rd(s0 + OPA + (wn * WN + j * 16) * 128 + fo1);
          }
          if (nx < 2 * TM) a2[nx] = rd(s0 + (wm * WM + (nx % TM) * 16) * 128 + (nx < TM ? fo0 : fo1));
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
        const int fo = fr * 128 + (swz_chunk(ks * 4 + fq, fr) << 4);
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
    // stream-K: a cut tile's first unit stores its partial and skips the epilogue (its waits: sk_meet ends in vmcnt(0))
    const bool epi = !sk || (cu.k0 == 0 && cu.k1 == nk) || sk_meet(cu);
    if constexpr (SO) {
      if (tn >= 0) {  // every wave is done reading the last stage's buffer: stage 1 of the next tile into it
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (ABL != 1 && ABL < 10) stage(tn, un.k0 + 1, (step + 1) & 1);  // step = the next unit's first k-step here; its second reads (step + 1) & 1
      }
      // (no epilogue stores: the next opening's seam count would not hold - plain counted waits)
      if (!epi) seam = false;
      else {
      const bool tail = bm * BM + BM > M;  // the last row band of a ragged M: rows >= M are not stored
      // straight-line per row tile (no per-element branches, so the scheduler interleaves the TN x 2 independent GELU
      // chains instead of padding each dependent packed FMA with a nop): bias in registers, head-major row offsets
      // stepped by 16 rows, the fp16 range test as an OR of exponent carries - (h & 0x7c00) + 0x400 reaches bit 15
      // exactly when h is Inf / NaN - masked by the row's store predicate
      f32x4 bj[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bj[j] = p.bias ? *(const f32x4*)(sbias + (tcount & 1) * 256 + wn * WN + j * 16 + 4 * fq) : (f32x4){0.f, 0.f, 0.f, 0.f};
      const float* sl = ssum + (tcount & 1) * 256 + wn * WN + 4 * fq;  // (the column sums: read per row tile, no registers
                                                                      // held across the epilogue)
      const bool gelu = p.epi == EPI_GELU, hm_step = p.hm_n >= 16;
      int hq = 0, hr = 0;  // (row / hm_n, row % hm_n) of row tile i's row (hm_step)
      if (hm_step) {
        hq = (mb + fr) / p.hm_n;
        hr = mb + fr - hq * p.hm_n;
      }
      uint32_t rbits = 0;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if constexpr (ABL == 12) {
#pragma unroll
          for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(acc[i][j]));
          continue;
        }
        const int mr = mb + i * 16 + fr;
        const bool ok = !tail || mr < M;
        long orow;
        if (hm_step) {
          orow = (((long)hq * (p.N / 64) + nb / 64) * p.hm_n + hr) * 64 - nb;
          hr += 16;
          if (hr >= p.hm_n) hr -= p.hm_n, ++hq;
        } else if (p.hm_n) {
          const int m = min(mr, M - 1);
          orow = (((long)(m / p.hm_n) * (p.N / 64) + nb / 64) * p.hm_n + m % p.hm_n) * 64 - nb;
        } else {
          orow = (long)min(mr, M - 1) * p.ldc;
        }
        bf16_t* C = (bf16_t*)p.C + orow + 4 * fq;
        if (lnf) {  // LN fold: acc a_r - b_r s_n (+ the bias below)
          const float2 ab = sab[(tcount & 1) * 256 + wm * WM + i * 16 + fr];
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            f32x4 sv = *(const f32x4*)(sl + j * 16);
            asm volatile("" : "+v"(sv));  // (read here, not hoisted over the epilogue)
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[i][j][e] = fmaf(acc[i][j][e], ab.x, -ab.y * sv[e]);
          }
        }
        u32x2 pk[TN];
        if (gelu) {
          static_assert(TN % 2 == 0, "GELU in column-group pairs");
#pragma unroll
          for (int j = 0; j < TN; j += 2) {
            const f32x4 v0 = acc[i][j] + bj[j], v1 = acc[i][j + 1] + bj[j + 1];
            const f32x8 g = gelu_erf_as8((f32x8){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]});
            pk[j] = pack16x4<true>((f32x4){g[0], g[1], g[2], g[3]});
            pk[j + 1] = pack16x4<true>((f32x4){g[4], g[5], g[6], g[7]});
          }
        } else {
#pragma unroll
          for (int j = 0; j < TN; ++j) pk[j] = pack16x4<true>(acc[i][j] + bj[j]);
        }
        uint32_t rb = 0;
#pragma unroll
        for (int j = 0; j < TN; ++j)
          rb |= ((pk[j][0] & 0x7c007c00u) + 0x04000400u) | ((pk[j][1] & 0x7c007c00u) + 0x04000400u);
        rbits |= ok ? rb : 0u;
        if constexpr (!WIDE) {
#pragma unroll
          for (int j = 0; j < TN; ++j)
            if (ok) *(u32x2*)(C + nb + j * 16) = pk[j];
        } else {
          // lanes fq (even) and fq + 1 hold columns 4 fq .. 4 fq + 7 of tiles j and j + 1: the even lane keeps
          // tile j's 8 columns, the odd lane tile j + 1's (the partner is 16 lanes away, same row)
          const bool odd = fq & 1;
#pragma unroll
          for (int j = 0; j < TN; j += 2) {
            const u32x2 snd = odd ? pk[j] : pk[j + 1];
            const u32x2 rcv = {xor16_partner(snd[0]), xor16_partner(snd[1])};
            const u32x4 w = odd ? (u32x4){rcv[0], rcv[1], pk[j + 1][0], pk[j + 1][1]}
                                : (u32x4){pk[j][0], pk[j][1], rcv[0], rcv[1]};
            if constexpr (ABL == 11) asm volatile("" ::"v"(w), "v"(C));
            // streaming stores (round 5): the QKV / MLP-1 outputs (232 / 310 MB) with cache policy nt | sc1 (aux 18) stream
            // past the L2 and leave it to the operands - plain nt: encoder 13.32-13.38 -> 13.12-13.24 ms on one box,
            // nt | sc1 another -0.1 ms against plain nt on another, sc1 alone +0.4 ms (profiles/r05/gemm_so_nt_ab.txt);
            // the residual epilogue's fp32 loads / stores nt: slower.  num_records = 0xffffffff: the launcher admits
            // outputs up to 2^31 elements = 4 GiB of fp16, the whole uint32 byte-offset range (a 2^31 - 1 byte count
            // silently dropped every store past 2 GiB: ViT MLP-1 from B ~ 1775 - tests/test_gpu_6_ops.py)
            else if (ok)
              __builtin_amdgcn_raw_buffer_store_b128(
                  w, __builtin_amdgcn_make_buffer_rsrc(p.C, 0, -1, 0x00020000),
                  (uint32_t)((C + nb + (odd ? (j + 1) * 16 - 4 : j * 16)) - (bf16_t*)p.C) * 2, 0, 18);
          }
        }
      }
      if (rbits & 0x80008000u) range_bad = true;
      // the counted waits of the next tile assume all NSTORE stores per wave were issued: not after a ragged tile
      // (its next tile waits vmcnt(0) and re-issues its stage 1 - the same bytes into the same buffer)
      seam = !tail;
      }
    } else if constexpr (RES) {
      float* Cb = (float*)p.C + nb + 4 * fq;
      const float* bl = sbias + (tcount & 1) * 256 + wn * WN + 4 * fq;
      const bool tail = bm * BM + BM > M;  // ragged last row band: rows >= M neither read nor stored
      // LN fold (variant builds): the residual stream as two fp16 planes, hi at xh and lo = fp16(x - hi) at xh + c_lo
      // (the same 4 bytes per element as fp32; the hi plane is the store-only GEMMs' A operand)
      const bool hl = ICAP_LN_FOLD && p.xh != nullptr;
      auto unpack4 = [](u32x2 v) -> f32x4 {
        return (f32x4){h2f((bf16_t)(v[0] & 0xffff)), h2f((bf16_t)(v[0] >> 16)), h2f((bf16_t)(v[1] & 0xffff)),
                       h2f((bf16_t)(v[1] >> 16))};
      };
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {  // row tiles [4 h2, min(TM, 4 h2 + 4))
        if (!epi) break;  // stream-K: the tile's other unit stores it
        f32x4 rv[4][TN];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            if (h2 * 4 + i < TM) {
              const long row = min(mb + (h2 * 4 + i) * 16 + fr, M - 1);
              if (hl) {
                const bf16_t* hp = p.xh + row * p.ldc + nb + j * 16 + 4 * fq;
                rv[i][j] = unpack4(*(const u32x2*)hp) + unpack4(*(const u32x2*)(hp + p.c_lo));
              } else {
                rv[i][j] = *(const f32x4*)(Cb + row * p.ldc + j * 16);
              }
            }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (h2 * 4 + i >= TM) break;
          const int m = mb + (h2 * 4 + i) * 16 + fr;
          f32x4 o[TN];
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            f32x4 a = acc[h2 * 4 + i][j];
            if (p.bias) a += *(const f32x4*)(bl + j * 16);
            o[j] = rv[i][j] + a;
          }
          if (hl) {
            // LN fold: the new row as hi / lo planes and this 64-column group's (mean, M2) - the 4 lanes fr + 16 q hold
            // the group's 64 values of row m (rows >= M: clamped loads, nothing stored)
            float sm = 0.f;
#pragma unroll
            for (int j = 0; j < TN; ++j) sm += (o[j][0] + o[j][1]) + (o[j][2] + o[j][3]);
            const float mg = rows4_sum(sm) * (1.0f / 64.0f);
            float m2 = 0.f;
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
              for (int e = 0; e < 4; ++e) m2 = fmaf(o[j][e] - mg, o[j][e] - mg, m2);
            m2 = rows4_sum(m2);
            if (!tail || m < M) {
#pragma unroll
              for (int j = 0; j < TN; ++j) {
                bf16_t* hp = p.xh + (long)m * p.ldc + nb + j * 16 + 4 * fq;
                const u32x2 hi = pack16x4<true>(o[j]);
                *(u32x2*)hp = hi;
                *(u32x2*)(hp + p.c_lo) = pack16x4<true>(o[j] - unpack4(hi));
              }
              if (fq == 0) *(float2*)(p.ln_part + 2 * ((long)(nb / 64) * M + m)) = make_float2(mg, m2);
            }
            continue;
          }
          if (tail && m >= M) continue;
#pragma unroll
          for (int j = 0; j < TN; ++j) *(f32x4*)(Cb + (long)m * p.ldc + j * 16) = o[j];
        }
      }
      if (tn >= 0) {  // stage 1 of the next tile into the last stage's buffer, after the stores
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (ABL != 1 && ABL < 10) stage(tn, un.k0 + 1, (step + 1) & 1);
      }
      // k-step 0 of the next tile skips its vmcnt wait because the residual loads retired after its stage 0;
      // every lane loads (rows clamped), so that holds for ragged tiles too
      seam = true;
    } else {
      epilogue_256<TM, TN, true>(p, acc, mb, nb, fr, fq);
    }
    if (tn < 0) break;
    t = tn;
    cu = un;
    ++tcount;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  // after the tile loop: no counted wait follows, so this store cannot disturb the seams' vmcnt arithmetic
  if (SO && p.range_flag && __any(range_bad) && lane == 0) range_flag_set(p.range_flag);
}

// ---------------------------------------------------------------------------------------------
// Persistent fp16 encoder GEMM, one wave per SIMD (round 4): the 256 x 256 tile as 4 waves (2 x 2), each a 128 x 128
// wave tile = 8 x 8 MFMA 16x16 tiles, 256 fp32 accumulators per lane in AGPRs (1 wave per SIMD owns the whole
// 512-register file).  This is the shape of hipBLASLt's own gfx950 kernel for these GEMMs
// (Custom_Cijk_Alik_Bljk_HHS_BH_MT256x256x64_MI16x16x1: 256 threads; per wave and 64-deep k-step 128 MFMA,
// 32 ds_read_b128, 16 LDS-DMA pieces and one barrier - read from its disassembly).  Against gemm_f16p_kernel (8 waves
// of 128 x 64) the CU reads 128 KiB of fragments from LDS per k-step instead of 192 KiB for the same 512 MFMAs (every
// fragment feeds 8 MFMAs), and each SIMD's matrix pipe is fed by ONE wave's stream.
// Kept from gemm_f16p_kernel: the XCD raster, 64-deep full-line stages (chunk c of row r at c ^ (r & 7)) in a 2-stage
// ring, the bias slot, the counted tile seams.  A stage is 16 DMA pieces per wave (8 A + 8 W); DI = 1 issues them one
// per 8-MFMA group, DI = 0 in one burst behind the k-step's first fragment reads.
// Register discipline (all 256 AGPRs hold accumulators, so the compiler has no room to re-assign them): the MFMAs
// update their accumulator in place from inline asm ("+a"), the k-loop is one do-while body (no peeled copies, no
// zero-trip path), the epilogue reads each accumulator through an opaque copy where it is used, and every epilogue
// load / store is a buffer operation on a 32-bit offset (rows >= M: loads return zeros, stores are dropped by the
// resource's range check), so the epilogue has no per-element branches and issues exactly NSTORE stores per tile.
// EP (store-only modes, MODE 1): 0 = + bias, 1 = + bias then GELU, 2 = + bias into head-major planes (the ViT QKV:
// [image][q|k|v x head][token][64], hm_n tokens per image; a wave tile spans two heads).  MODE 2 = residual (C += acc
// + bias, fp32).  BMT = 224 (MODE 2 only): wave tiles 112 x 128, wave 3 stages 4 A pieces.
// acc += W-fragment x A-fragment (v_mfma_f32_16x16x32_f16), the accumulator tied in place to an AGPR tuple.  A chain of
// MFMAs on one accumulator needs no wait states; the epilogue's first accumulator read is behind explicit s_nops.
__device__ __forceinline__ void mfma16_f16_acc(f32x4& acc, bf16x8 a, bf16x8 b) {
  asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
// An accumulator's value in VGPRs at this point of the epilogue.  The empty "+a" statement re-defines the accumulator in
// its AGPR here, so the AGPR -> VGPR copy cannot be hoisted above it: without it the compiler copies every accumulator
// to VGPRs right at the k-loop exit (~250 v_accvgpr_read at once, then the epilogue spills).
__device__ __forceinline__ f32x4 acc_v(f32x4& a) {
  asm volatile("" : "+a"(a));
  f32x4 v = a;
  asm volatile("" : "+v"(v));
  return v;
}

template <int MODE, int EP = 0, int DI = 1, int BMT = 256>
__global__ __launch_bounds__(256, 1) void gemm_f16w_kernel(GemmArgs p) {
  constexpr bool SO = MODE == 1, RES = MODE == 2;
  static_assert(SO || RES, "store-only or residual epilogue");
  static_assert(BMT == 256 || (RES && BMT == 224), "224-row tiles only for the residual form (no counted waits)");
  constexpr int BM = BMT, BN = 256, KS = 64, NW = 4, WM = BM / 2, WN = 128, TM = WM / 16, TN = WN / 16, XD = 2;
  constexpr int OPA = BM * KS * 2, OPB = BN * KS * 2, STAGE = OPA + OPB;
  constexpr int IPW = OPB / 1024 / NW;  // 8 DMA pieces per wave per operand
  constexpr int PER_STAGE = 2 * IPW;    // 16 per wave per stage (BM 256)
  constexpr int NSTORE = TM * TN / 2;   // SO: 16-byte stores per wave per tile
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // wave-uniform values in SGPRs (the divergence analysis cannot see that threadIdx.x >> 6 is uniform)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nbn = p.N / BN, nbm = (p.M + BM - 1) / BM, nwg = nbn * nbm;
  const int xcd = blockIdx.x & 7, q = nwg >> 3, r = nwg & 7;
  const int xbase = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q, xcnt = q + (xcd < r);
  const int nbx = ((int)gridDim.x - xcd + 7) >> 3, lb = blockIdx.x >> 3;
  if (lb >= xcnt) return;
  const int M = p.M, nk = p.K / KS;
  const int srow = wave * IPW * 8 + (lane >> 3), schunk = (lane & 7) ^ (srow & 7);
  const int fr = lane & 15, fq = lane >> 4;

  // stage pieces: one per-lane 32-bit offset per operand (A: this lane's row of the staged tile; W: fixed), the piece's
  // row step and the k-step in the wave-uniform soffset; A rows >= M read zeros (past the resource's byte count)
  const i32x4r ra = buf_rsrc(p.A, (uint32_t)((long)M * p.lda * 2)), rw = buf_rsrc(p.W, (uint32_t)((long)p.N * p.ldw * 2));
  const uint32_t vw = (uint32_t)((srow * p.ldw + schunk * 8) * 2);
  struct Src {
    uint32_t va;  // this lane's A offset (piece 0) in the staged tile
    uint32_t sw;  // W: the staged tile's first row + k-step byte offset
    uint32_t sk;  // A: k-step byte offset
  };
  auto src = [&](int t, int kt) -> Src {
    const int bm = t / nbn, bn = t - bm * nbn;
    return {(uint32_t)(((bm * BM + srow) * p.lda + schunk * 8) * 2), (uint32_t)((bn * BN) * p.ldw * 2 + kt * KS * 2),
            (uint32_t)(kt * KS * 2)};
  };
  auto piece = [&](const Src& sc, int buf, int i) {
    char* s0 = smem + buf * STAGE;
    if (i < IPW) {
      if (BM < 256 && (wave * IPW + i) * 8 >= BM) return;  // (wave-uniform) rows past the tile's A image
      lds_dma_buf16(ra, sc.va + (uint32_t)(i * 16 * p.lda), sc.sk, (LDS_AS void*)(s0 + (wave * IPW + i) * 1024));
    } else {
      const int j = i - IPW;
      lds_dma_buf16(rw, vw, sc.sw + (uint32_t)(j * 16 * p.ldw), (LDS_AS void*)(s0 + OPA + (wave * IPW + j) * 1024));
    }
  };
  auto stage = [&](int t, int kt, int buf) {
    const Src sc = src(t, kt);
#pragma unroll
    for (int i = 0; i < PER_STAGE; ++i) piece(sc, buf, i);
  };
  float* sbias = (float*)(smem + 2 * STAGE);
  auto load_bias = [&](int t, int slot) {
    if (wave == 0 && p.bias) {
      const int n0 = (t - (t / nbn) * nbn) * BN;
      lds_dma16(p.bias + n0 + lane * 4, (LDS_AS void*)(sbias + slot * 256));
    }
  };
  // epilogue buffer resources: rows >= M (ragged last band) fall past the byte count
  const long cbytes = EP == 2 ? (long)M * p.N * 2 : (long)M * p.ldc * (RES ? 4 : 2);  // (the launcher keeps it < 2^31)
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(p.C, 0, (int)cbytes, 0x00020000);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  int t = xbase + lb, step = 0, tcount = 0;
  load_bias(t, 0);
  stage(t, 0, 0);
  bool seam = false;       // this tile's stages 0 and 1 were issued before the previous tile's epilogue stores
  bool range_bad = false;  // SO: some stored fp16 value is not finite
  for (;;) {
    const int tn = t + nbx < xbase + xcnt ? t + nbx : -1;
    int kt = 0;
#pragma clang loop unroll(disable)
    do {
      if (SO && seam && kt == 0) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(PER_STAGE + NSTORE) : "memory");
      else if (SO && seam && kt == 1) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NSTORE) : "memory");
      else if (RES && seam && kt == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      int st_t = -1, st_kt = 0;
      if (seam && kt == 0) {
        // stage 1 of this tile is already in flight
      } else if (kt + 1 < nk) {
        st_t = t, st_kt = kt + 1;
      } else if (tn >= 0) {
        load_bias(tn, (tcount + 1) & 1);
        st_t = tn;
      }
      st_t = __builtin_amdgcn_readfirstlane(st_t);
      const Src sc = src(st_t >= 0 ? st_t : t, st_kt);
      const int sbuf = (step + 1) & 1;
      const char* s0 = smem + (step & 1) * STAGE;
      const int fo0 = fr * 128 + ((fq ^ (fr & 7)) << 4), fo1 = fr * 128 + (((4 + fq) ^ (fr & 7)) << 4);
      bf16x8 b2[2][TN], a2[2 * TM];
#pragma unroll
      for (int j = 0; j < TN; ++j) b2[0][j] = *(const bf16x8*)(s0 + OPA + (wn * WN + j * 16) * 128 + fo0);
#pragma unroll
      for (int g = 0; g < XD; ++g) a2[g] = *(const bf16x8*)(s0 + (wm * WM + g * 16) * 128 + fo0);
      if (!DI && st_t >= 0) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < PER_STAGE; ++i) piece(sc, sbuf, i);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int g = 0; g < 2 * TM; ++g) {
        const int nx = g + XD;
        if (nx == TM) {
#pragma unroll
          for (int j = 0; j < TN; ++j) b2[1][j] = *(const bf16x8*)(s0 + OPA + (wn * WN + j * 16) * 128 + fo1);
        }
        if (nx < 2 * TM) a2[nx] = *(const bf16x8*)(s0 + (wm * WM + (nx % TM) * 16) * 128 + (nx < TM ? fo0 : fo1));
        if (DI && st_t >= 0) {  // 16 pieces over 2 TM groups (TM 7: the last two groups take two)
          constexpr int EXTRA = PER_STAGE - 2 * TM;
          piece(sc, sbuf, g);
          if (EXTRA > 0 && g >= 2 * TM - EXTRA) piece(sc, sbuf, g + EXTRA);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < TN; ++j) mfma16_f16_acc(acc[g % TM][j], b2[g / TM][j], a2[g]);
        __builtin_amdgcn_sched_barrier(0);
      }
      ++step;
    } while (++kt < nk);
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" ::: "memory");  // XDL MFMA write -> v_accvgpr_read (<= 18 states)
    const int bm = t / nbn, bn = t - bm * nbn, mb = bm * BM + wm * WM, nb = bn * BN + wn * WN;
    const float* bl = sbias + (tcount & 1) * 256 + wn * WN + 4 * fq;  // re-read from LDS where used
    if constexpr (SO) {
      // every wave is done reading the last stage's buffer: stage 1 of the next tile into it.  Unconditional (after the
      // last tile: a re-read of this tile's stage 1 that nothing reads), so no branch separates the k-loop from the
      // epilogue - the accumulator reads then stay in the epilogue's row-tile blocks instead of all being hoisted to
      // the loop exit
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      stage(tn >= 0 ? tn : t, 1, (step + 1) & 1);
      // byte offset of (row tile i, column tile j = 0) for this lane; head-major: columns 64..127 of the wave tile are
      // the next head, hm_n * 64 elements further
      int hq = 0, hr = 0;
      if (EP == 2) {
        hq = (mb + fr) / p.hm_n;
        hr = mb + fr - hq * p.hm_n;
      }
      const uint32_t head2 = EP == 2 ? (uint32_t)(p.hm_n * 64 - 64) * 2 : 0;
      const bool odd = fq & 1;
      uint32_t rbits = 0;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        __builtin_amdgcn_sched_barrier(0);
        uint32_t orow;  // element offset of column nb in this lane's row
        if (EP == 2) {
          orow = (uint32_t)(((hq * (p.N / 64) + nb / 64) * p.hm_n + hr) * 64);
          hr += 16;
          if (hr >= p.hm_n) hr -= p.hm_n, ++hq;
        } else {
          orow = (uint32_t)((mb + i * 16 + fr) * p.ldc + nb);
        }
        const uint32_t ob = (orow + 4 * fq) * 2;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {  // the row tile in two halves of 4 column tiles (one 64-column head each)
          u32x2 pk[4];
          f32x4 av[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) av[j] = acc_v(acc[i][hh * 4 + j]) + *(const f32x4*)(bl + (hh * 4 + j) * 16);
          if (EP == 1) {
#pragma unroll
            for (int j = 0; j < 4; j += 2) {
              const f32x8 gv = gelu_erf_as8((f32x8){av[j][0], av[j][1], av[j][2], av[j][3], av[j + 1][0], av[j + 1][1],
                                                     av[j + 1][2], av[j + 1][3]});
              pk[j] = pack16x4<true>((f32x4){gv[0], gv[1], gv[2], gv[3]});
              pk[j + 1] = pack16x4<true>((f32x4){gv[4], gv[5], gv[6], gv[7]});
            }
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) pk[j] = pack16x4<true>(av[j]);
          }
#pragma unroll
          for (int j = 0; j < 4; ++j)
            rbits |= ((pk[j][0] & 0x7c007c00u) + 0x04000400u) | ((pk[j][1] & 0x7c007c00u) + 0x04000400u);
#pragma unroll
          for (int j = 0; j < 4; j += 2) {
            // lanes fq (even) and fq + 1 hold columns 4 fq .. 4 fq + 7 of tiles j and j + 1: the even lane stores tile j's
            // 8 columns, the odd lane tile j + 1's (the partner is 16 lanes away, same row)
            const u32x2 snd = odd ? pk[j] : pk[j + 1];
            const u32x2 rcv = {xor16_partner(snd[0]), xor16_partner(snd[1])};
            const u32x4 w = odd ? (u32x4){rcv[0], rcv[1], pk[j + 1][0], pk[j + 1][1]}
                                : (u32x4){pk[j][0], pk[j][1], rcv[0], rcv[1]};
            const uint32_t off = ob + (uint32_t)((odd ? (hh * 4 + j + 1) * 16 - 4 : (hh * 4 + j) * 16) * 2) + (hh ? head2 : 0);
            __builtin_amdgcn_raw_buffer_store_b128(w, rc, off, 0, 0);
          }
        }
      }
      // rows >= M (zeros + bias) are finite whenever the real rows' bias is: the OR over all rows is the guard
      if (rbits & 0x80008000u) range_bad = true;
      seam = true;
    } else {
      constexpr int RB = 4;  // row tiles per residual batch (RB x TN 16-byte loads in flight per lane)
#pragma unroll
      for (int h2 = 0; h2 < (TM + RB - 1) / RB; ++h2) {
        __builtin_amdgcn_sched_barrier(0);
        f32x4 rv[RB][TN];
#pragma unroll
        for (int i = 0; i < RB; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            if (h2 * RB + i < TM)
              rv[i][j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                       rc, (uint32_t)(((mb + (h2 * RB + i) * 16 + fr) * p.ldc + nb + j * 16 + 4 * fq) * 4),
                                                       0, 0));
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          if (h2 * RB + i >= TM) break;
          __builtin_amdgcn_sched_barrier(0);
          const uint32_t orow = (uint32_t)(((mb + (h2 * RB + i) * 16 + fr) * p.ldc + nb + 4 * fq) * 4);
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            f32x4 a = acc_v(acc[h2 * RB + i][j]);
            if (p.bias) a += *(const f32x4*)(bl + j * 16);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, rv[i][j] + a), rc, orow + j * 64, 0, 0);
          }
        }
      }
      if (tn >= 0) {  // stage 1 of the next tile into the last stage's buffer, after the stores
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        stage(tn, 1, (step + 1) & 1);
      }
      seam = true;
    }
    if (tn < 0) break;
    t = tn;
    ++tcount;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup has ended
  if (SO && p.range_flag && __any(range_bad) && lane == 0) range_flag_set(p.range_flag);
}
constexpr int f16w_lds(int bm) { return 2 * (bm * 128 + 256 * 128) + 2048; }

// ---------------------------------------------------------------------------------------------
// Persistent fp16 encoder GEMM, one wave per SIMD, half-step register double buffering (round 6).
// What hipBLASLt's gfx950 kernel for these shapes does that gemm_f16w_kernel did not (its main loop, disassembled from
// torch's bundled TensileLibrary_HH_HH_HA_Bias_..._Alik_Bljk_..._gfx950.co, kernel
// Custom_Cijk_Alik_Bljk_HHS_BH_Bias_HA_S_SAV_NTD_SK3_UserArgs_MT256x256x64_MI16x16x1):
//  * every fragment of a k-step lives in registers: the 16 fragments of the k-step's second 32-deep half are read
//    during the first half's 64 MFMAs (one ds_read_b128 per MFMA), and the next k-step's first-half fragments during
//    the second half's last MFMAs - a fragment read has a whole half-step (~1000 cycles) to land, and no MFMA waits
//    on one;
//  * so the stage buffer of k-step i is free a quarter into k-step i: after one counted lgkmcnt(0) + barrier, the
//    16 stage pieces of k-step i + 2 go into it, spread one per two MFMAs; they land ~1.75 k-steps later, when
//    k-step i + 1's last quarter waits vmcnt(pieces issued since) + barrier and reads them (2 barriers per k-step,
//    no wait at the top of a k-step).  gemm_f16w_kernel waited vmcnt(0) + barrier at the top of every k-step with
//    reads two MFMA groups ahead; gemm_f16p_kernel's 8 waves read 192 KiB of fragments per k-step against 128 here.
// Kept: the XCD-contiguous persistent raster, 64-deep full-line stages (chunk c of row r at c ^ (r & 7)), buffer-load
// stage pieces (rows >= M read zeros), in-place AGPR accumulators (mfma16_f16_acc / acc_v), f16w's epilogues.  The
// (tile, k-step) sequence of a block is one stream: the last two k-steps of a tile issue the next tile's stages 0
// and 1 (and its bias, one 512-B LDS-DMA per wave, before stage 0), and read its k-step 0 first-half fragments, so
// the epilogue runs between two tiles with nothing to wait for; its stores (NSTORE per wave, buffer stores: rows >= M
// are dropped by the range check, every lane issues every store, so the count is exact) are younger than the next
// tile's stage 1, which k-step 0 of that tile waits for with vmcnt(NSTORE + 16).
// BMT = 224 (residual form): wave tiles 112 x 128, every wave stages 7 A pieces (28 = 224 / 8) + 8 W pieces.
// EP (MODE 1): 0 = + bias, 1 = + bias then GELU, 2 = + bias into head-major planes.  MODE 2 = residual (C += acc + bias).
constexpr int f16h_lds(int bm) { return 2 * (bm * 128 + 256 * 128) + 2048; }
// f(integral_constant<int, 0>), ..., f(integral_constant<int, N - 1>) in order: a straight-line sequence whose index is a
// constant in every copy (a 128-step `#pragma unroll` loop exceeds the unroller's threshold and leaves the fragment
// arrays dynamically indexed, in scratch)
template <class F, int... Ms>
__device__ __forceinline__ void unroll_seq(F&& f, std::integer_sequence<int, Ms...>) {
  (f(std::integral_constant<int, Ms>{}), ...);
}

#ifndef ICAP_F16H_ABL
#define ICAP_F16H_ABL 0  // timing ablations (variant builds only, wrong results): 1 no k-loop DMA, 2 no k-loop fragment
#endif                   // reads, 3 no k-loop barriers, 4 no MFMAs, 5 no epilogue stores
template <int MODE, int EP = 0, int BMT = 256>
__global__ __launch_bounds__(256, 1) void gemm_f16h_kernel(GemmArgs p) {
  constexpr int ABL = ICAP_F16H_ABL;
  constexpr bool SO = MODE == 1, RES = MODE == 2;
  static_assert(SO || RES, "store-only or residual epilogue");
  static_assert(BMT == 256 || (RES && BMT == 224), "224-row tiles only for the residual form");
  constexpr int BM = BMT, BN = 256, KS = 64, WM = BM / 2, WN = 128, TM = WM / 16, TN = WN / 16;
  constexpr int OPA = BM * KS * 2, OPB = BN * KS * 2, STAGE = OPA + OPB;
  constexpr int APW = BM / 8 / 4, WPW = 8, PIECES = APW + WPW;  // stage pieces per wave (A rows, W rows)
  constexpr int NMF = 2 * TM * TN;                               // MFMAs per wave per k-step
  constexpr int NSTORE = SO ? TM * TN / 2 : TM * TN;             // epilogue stores per wave per tile
  // the k-step's event points (MFMA indices m): the second half's NR fragment reads one per two MFMAs from m = 0, the
  // buffer barrier at RB, the bias slot + PIECES stage pieces one per DSTEP MFMAs from DMA0 (spread over the rest of
  // the k-step: issued in a burst they queue at the CU's address unit and stall the wave's MFMA issue - round-6 timing
  // ablations), the stage-(i + 1) wait + barrier at LW, then the next first half's reads one per two MFMAs
  constexpr int NR = TM + TN, RB = 2 * NR, DMA0 = RB + 2, DSTEP = (NMF - 8 - DMA0) / (PIECES + 1);
  constexpr int LW = NMF - 2 * NR - 4;
  // stage (i + 2) pieces issued before LW (the bias DMA, when issued, is older than them: the wait then covers it too)
  constexpr int NB_LW = (LW - DMA0 - 1) / DSTEP < PIECES ? (LW - DMA0 - 1) / DSTEP : PIECES;
  static_assert(DSTEP >= 2 && DMA0 + PIECES * DSTEP < NMF, "stage pieces inside the k-step");
  static_assert(LW > RB && LW + 2 * NR - 2 < NMF, "next first-half reads inside the k-step");
  static_assert(NSTORE + NB_LW <= 63 || RES, "counted seam wait fits vmcnt");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nbn = p.N / BN, nbm = (p.M + BM - 1) / BM, nwg = nbn * nbm;
  const int xcd = blockIdx.x & 7, q = nwg >> 3, r = nwg & 7;
  const int xbase = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q, xcnt = q + (xcd < r);
  const int nbx = ((int)gridDim.x - xcd + 7) >> 3, lb = blockIdx.x >> 3;
  if (lb >= xcnt) return;
  const int M = p.M, nk = p.K / KS;
  const int fr = lane & 15, fq = lane >> 4;
  const int schunk = swz_chunk(lane & 7, lane >> 3);  // a piece is 8 rows x 128 B; row & 7 = lane >> 3

  // stage pieces: per-lane 32-bit offsets (A: this lane's row of the wave's first piece in the staged tile, stepped by
  // 8 rows per piece; W: fixed), the tile's W rows and the k-step in the wave-uniform soffset
  const i32x4r ra = buf_rsrc(p.A, (uint32_t)((long)M * p.lda * 2)), rw = buf_rsrc(p.W, (uint32_t)((long)p.N * p.ldw * 2));
  const uint32_t vw = (uint32_t)(((wave * WPW * 8 + (lane >> 3)) * p.ldw + schunk * 8) * 2);
  const uint32_t astep = (uint32_t)(8 * p.lda * 2), wstep = (uint32_t)(8 * p.ldw * 2);
  float* sbias = (float*)(smem + 2 * STAGE);
  // stage (tile t, k-step kt) piece i (0 .. PIECES - 1) into ring buffer buf
  auto piece = [&](int t, int kt, int buf, int i) {
    const int bm = t / nbn, bn = t - bm * nbn;
    char* s0 = smem + buf * STAGE;
    if (i < APW) {
      const uint32_t va = (uint32_t)(((bm * BM + (wave * APW + i) * 8 + (lane >> 3)) * p.lda + schunk * 8) * 2);
      lds_dma_buf16(ra, va, (uint32_t)(kt * KS * 2), (LDS_AS void*)(s0 + (wave * APW + i) * 1024));
    } else {
      const int j = i - APW;
      lds_dma_buf16(rw, vw + j * wstep, (uint32_t)(bn * BN * p.ldw * 2 + kt * KS * 2),
                    (LDS_AS void*)(s0 + OPA + (wave * WPW + j) * 1024));
    }
  };
  (void)astep;
  // the tile's bias: each wave DMAs the 128 values of its column half (lanes 0-31, 512 B) into slot `slot`
  auto load_bias = [&](int t, int slot) {
    const int n0 = (t - (t / nbn) * nbn) * BN + wn * WN;
    if (lane < 32) lds_dma16(p.bias + n0 + lane * 4, (LDS_AS void*)(sbias + slot * 256 + wn * WN));
  };
  // epilogue buffer resource: rows >= M (ragged last band) fall past the byte count (the launcher keeps it < 2^32)
  const long cbytes = EP == 2 ? (long)M * p.N * 2 : (long)M * p.ldc * (RES ? 4 : 2);
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(p.C, 0, (int)(uint32_t)cbytes, 0x00020000);
  const int fo0 = fr * 128 + (swz_chunk(fq, fr) << 4), fo1 = fr * 128 + (swz_chunk(4 + fq, fr) << 4);
  const int arow = wm * WM * 128, wrow = OPA + wn * WN * 128;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  bf16x8 fa[2][TM], fb[2][TN];  // [half][fragment]: this k-step's first-half (0) and second-half (1) fragments
  int t = xbase + lb, step = 0, tcount = 0;
  // prologue: bias, stages 0 and 1 of the first tile, then k-step 0's first-half fragments
  load_bias(t, 0);
#pragma unroll
  for (int i = 0; i < PIECES; ++i) piece(t, 0, 0, i);
  const bool two = nk > 1;
  if (two) {
#pragma unroll
    for (int i = 0; i < PIECES; ++i) piece(t, 1, 1, i);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PIECES) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int j = 0; j < TN; ++j) fb[0][j] = *(const bf16x8*)(smem + wrow + j * 16 * 128 + fo0);
#pragma unroll
  for (int i = 0; i < TM; ++i) fa[0][i] = *(const bf16x8*)(smem + arow + i * 16 * 128 + fo0);
  bool seam = false;       // SO: the previous tile's NSTORE stores are younger than this tile's stage 1
  bool range_bad = false;  // SO: some stored fp16 value is not finite
  for (;;) {
    const int tn = t + nbx < xbase + xcnt ? t + nbx : -1;
    int kt = 0;
#pragma clang loop unroll(disable)
    do {
      const char* s0 = smem + (step & 1) * STAGE;
      const char* s1 = smem + ((step + 1) & 1) * STAGE;
      // the stage this k-step issues (k-step kt + 2 of this tile, else stage kt + 2 - nk of the next tile) into s0
      // (none - the last tile's last two k-steps: a dummy re-load of this tile's last stage into the free buffer, so
      // every k-step issues PIECES pieces and the counted waits stay the same; nothing reads it)
      int st_t = t, st_kt = nk - 1;
      if (kt + 2 < nk) st_kt = kt + 2;
      else if (tn >= 0) st_t = tn, st_kt = kt + 2 - nk;
      st_t = __builtin_amdgcn_readfirstlane(st_t);
      st_kt = __builtin_amdgcn_readfirstlane(st_kt);
      const bool bias_next = st_t != t && st_kt == 0;  // the next tile's bias goes with its stage 0
      // stage kt + 1 (this tile's, or the next tile's stage 0) exists: wait for it at the late point, read its
      // first-half fragments
      const bool has_next = kt + 1 < nk || tn >= 0;
      // younger than stage kt + 1 at the late point: this k-step's PIECES pieces (+ the bias DMA before them, which the
      // wait then covers too), and (SO, k-step 0 after a seam) the NSTORE stores of the previous tile's epilogue; RES:
      // the epilogue's own waits on its residual loads retired stage 1 already (in-order counter)
      const bool after_seam = seam && kt == 0;
      unroll_seq([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        // second-half fragment reads (W first: the first second-half MFMAs need all TN of them and A 0)
        constexpr int r1 = m / 2, r0 = (m - LW) / 2;  // read slots
        if constexpr (ABL == 2 || (m & 1)) {
        } else if constexpr (r1 < TN) fb[1][r1] = *(const bf16x8*)(s0 + wrow + r1 * 16 * 128 + fo1);
        else if constexpr (r1 < TN + TM) fa[1][r1 - TN] = *(const bf16x8*)(s0 + arow + (r1 - TN) * 16 * 128 + fo1);
        if constexpr (m == RB && ABL != 3) {  // every wave's reads of this buffer are done: it takes stage kt + 2
          // (the builtin, not asm: the compiler's waitcnt pass then knows the reads landed and adds no waits of its own
          // for them - lgkmcnt saturates at 15, so it would otherwise stall on the next first-half reads)
          __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0); vmcnt / expcnt at their maxima
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");
        }
        if constexpr (ABL != 1 && m >= DMA0 && m <= DMA0 + PIECES * DSTEP && (m - DMA0) % DSTEP == 0) {
          constexpr int i = (m - DMA0) / DSTEP;  // 0: the bias (stage 0 of the next tile only), then the pieces
          if constexpr (i == 0) {
            if (bias_next) load_bias(st_t, (tcount + 1) & 1);
          } else {
            piece(st_t, st_kt, step & 1, i - 1);
          }
        }
        if constexpr (m == LW && ABL != 3) {
          if (has_next) {  // stage kt + 1 landed (this wave's pieces, then every wave's)
            if (SO && after_seam) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(SO ? NSTORE + NB_LW : 0) : "memory");
            else if (!(RES && after_seam)) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NB_LW) : "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
          }
        }
        // (unconditional: without a next stage the values are never used)
        if constexpr (ABL == 2 || m < LW || ((m - LW) & 1)) {
        } else if constexpr (r0 < TN) fb[0][r0] = *(const bf16x8*)(s1 + wrow + r0 * 16 * 128 + fo0);
        else if constexpr (r0 < TN + TM) fa[0][r0 - TN] = *(const bf16x8*)(s1 + arow + (r0 - TN) * 16 * 128 + fo0);
        __builtin_amdgcn_sched_barrier(0);
        constexpr int h = m / (TM * TN), a = (m % (TM * TN)) / TN, b = m % TN;
        if constexpr (ABL == 4) asm volatile("" ::"v"(fb[h][b]), "v"(fa[h][a]));
        else mfma16_f16_acc(acc[a][b], fb[h][b], fa[h][a]);
        __builtin_amdgcn_sched_barrier(0);
      }, std::make_integer_sequence<int, NMF>{});
      ++step;
    } while (++kt < nk);
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" ::: "memory");  // XDL MFMA write -> v_accvgpr_read (<= 18 states)
    const int bm = t / nbn, bn = t - bm * nbn, mb = bm * BM + wm * WM, nb = bn * BN + wn * WN;
    const float* bl = sbias + (tcount & 1) * 256 + wn * WN + 4 * fq;  // re-read from LDS where used
    if constexpr (SO) {
      int hq = 0, hr = 0;
      if (EP == 2) {
        hq = (mb + fr) / p.hm_n;
        hr = mb + fr - hq * p.hm_n;
      }
      const uint32_t head2 = EP == 2 ? (uint32_t)(p.hm_n * 64 - 64) * 2 : 0;
      const bool odd = fq & 1;
      uint32_t rbits = 0;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        __builtin_amdgcn_sched_barrier(0);
        uint32_t orow;  // element offset of column nb in this lane's row
        if (EP == 2) {
          orow = (uint32_t)(((hq * (p.N / 64) + nb / 64) * p.hm_n + hr) * 64);
          hr += 16;
          if (hr >= p.hm_n) hr -= p.hm_n, ++hq;
        } else {
          orow = (uint32_t)((mb + i * 16 + fr) * p.ldc + nb);
        }
        const uint32_t ob = (orow + 4 * fq) * 2;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {  // the row tile in two halves of 4 column tiles (one 64-column head each)
          u32x2 pk[4];
          f32x4 av[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) av[j] = acc_v(acc[i][hh * 4 + j]) + *(const f32x4*)(bl + (hh * 4 + j) * 16);
          if (EP == 1) {
#pragma unroll
            for (int j = 0; j < 4; j += 2) {
              const f32x8 gv = gelu_erf_as8((f32x8){av[j][0], av[j][1], av[j][2], av[j][3], av[j + 1][0], av[j + 1][1],
                                                     av[j + 1][2], av[j + 1][3]});
              pk[j] = pack16x4<true>((f32x4){gv[0], gv[1], gv[2], gv[3]});
              pk[j + 1] = pack16x4<true>((f32x4){gv[4], gv[5], gv[6], gv[7]});
            }
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) pk[j] = pack16x4<true>(av[j]);
          }
#pragma unroll
          for (int j = 0; j < 4; ++j)
            rbits |= ((pk[j][0] & 0x7c007c00u) + 0x04000400u) | ((pk[j][1] & 0x7c007c00u) + 0x04000400u);
#pragma unroll
          for (int j = 0; j < 4; j += 2) {
            // lanes fq (even) and fq + 1 hold columns 4 fq .. 4 fq + 7 of tiles j and j + 1: the even lane stores tile j's
            // 8 columns, the odd lane tile j + 1's (the partner is 16 lanes away, same row); streaming stores (nt | sc1)
            const u32x2 snd = odd ? pk[j] : pk[j + 1];
            const u32x2 rcv = {xor16_partner(snd[0]), xor16_partner(snd[1])};
            const u32x4 w = odd ? (u32x4){rcv[0], rcv[1], pk[j + 1][0], pk[j + 1][1]}
                                : (u32x4){pk[j][0], pk[j][1], rcv[0], rcv[1]};
            const uint32_t off = ob + (uint32_t)((odd ? (hh * 4 + j + 1) * 16 - 4 : (hh * 4 + j) * 16) * 2) + (hh ? head2 : 0);
            if constexpr (ABL == 5) asm volatile("" ::"v"(w), "v"(off));
            else __builtin_amdgcn_raw_buffer_store_b128(w, rc, off, 0, 18);
          }
        }
      }
      // rows >= M (zeros + bias) are finite whenever the real rows' bias is: the OR over all rows is the guard
      if (rbits & 0x80008000u) range_bad = true;
    } else {
      constexpr int RBK = 4;  // row tiles per residual batch (RBK x TN 16-byte loads in flight per lane)
#pragma unroll
      for (int h2 = 0; h2 < (TM + RBK - 1) / RBK; ++h2) {
        __builtin_amdgcn_sched_barrier(0);
        f32x4 rv[RBK][TN];
#pragma unroll
        for (int i = 0; i < RBK; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            if (h2 * RBK + i < TM)
              rv[i][j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                       rc, (uint32_t)(((mb + (h2 * RBK + i) * 16 + fr) * p.ldc + nb + j * 16 + 4 * fq) * 4),
                                                       0, 0));
#pragma unroll
        for (int i = 0; i < RBK; ++i) {
          if (h2 * RBK + i >= TM) break;
          __builtin_amdgcn_sched_barrier(0);
          const uint32_t orow = (uint32_t)(((mb + (h2 * RBK + i) * 16 + fr) * p.ldc + nb + 4 * fq) * 4);
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            f32x4 a = acc_v(acc[h2 * RBK + i][j]) + *(const f32x4*)(bl + j * 16);
            if constexpr (ABL == 5) asm volatile("" ::"v"(rv[i][j] + a), "v"(orow));
            else __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, rv[i][j] + a), rc, orow + j * 64, 0, 0);
          }
        }
      }
    }
    seam = true;
    if (tn < 0) break;
    t = tn;
    ++tcount;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may land after the workgroup has ended
  if (SO && p.range_flag && __any(range_bad) && lane == 0) range_flag_set(p.range_flag);
}

// ---------------------------------------------------------------------------------------------
// Persistent fp16 encoder GEMM with the A operand two k-steps ahead (round 3; tools build only, ICAP_F16_GEMM=7:
// correct - 104 GPU tests with it as the product form - but per ViT layer 973-991 us against 979-981 for
// gemm_f16p_kernel on the same box, tools/r3_lib_ab.sh: the k-loop is not held by the stage's DMA latency).  gemm_f16p_kernel's 2-stage ring keeps
// ONE 64 KiB stage in flight per CU, so every k-step waits out that stage's whole DMA latency (its timing ablations:
// the DMA path alone runs as long as the MFMA path alone and the two overlap poorly).  Here the 160 KiB hold three A
// slots and two W slots: the block's (tile, k-step) sequence is one stream of steps s, and step s issues W(s + 1) and
// A(s + 2) - up to 96 KiB in flight, and the A rows (row bands from HBM / MALL; W is L2-resident) get two k-steps to
// land.  Tiles, raster, fragment-read pipeline and epilogues as gemm_f16p_kernel; the bias is read from global
// memory in the epilogue (no LDS left at 256-row tiles; 1 KiB per tile, L2-resident).
// Waits at step s: W(s) and A(s) landed; younger in issue order are A(s + 1) (this wave's IPW instructions, if it
// stages A rows and A(s + 1) exists) and the previous tile's epilogue stores (NSTORE per wave) - a ragged tile (rows
// >= M not stored) leaves an uncounted number, and the next step waits for everything.  The epilogue's own loads
// (bias, RES residual) are waited for by the compiler, which retires every older DMA with them (in-order counter).
constexpr int F16R_LDS_256 = 3 * 256 * 128 + 2 * 256 * 128, F16R_LDS_224 = 3 * 224 * 128 + 2 * 256 * 128;
template <int MODE, int BMT>
__global__ __launch_bounds__(512, 1) void gemm_f16r_kernel(GemmArgs p) {
  constexpr bool SO = MODE == 1, RES = MODE == 2;
  static_assert(SO || RES, "store-only or residual epilogue");
  static_assert(BMT == 256 || BMT == 224, "tile rows");
  constexpr int BM = BMT, BN = 256, KS = 64, NW = 8, WM = BM / 2, WN = 64, TM = WM / 16, TN = 4, XD = 2;
  constexpr int OPA = BM * KS * 2, OPB = BN * KS * 2;  // bytes per A / W slot
  constexpr int IPW = OPB / 1024 / NW;                 // 4 DMA instructions per wave per W stage (A: 4 or none)
  constexpr int NSTORE = SO ? TM * TN / 2 : TM * TN;   // epilogue stores per wave (SO: 16 B per lane)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const sa = smem;            // A slots [3][BM rows][128 B]
  char* const sw = smem + 3 * OPA;  // W slots [2][256 rows][128 B]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int nbn = p.N / BN, nbm = (p.M + BM - 1) / BM, nwg = nbn * nbm;
  const int xcd = blockIdx.x & 7, q = nwg >> 3, r = nwg & 7;
  const int xbase = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q, xcnt = q + (xcd < r);
  const int nbx = ((int)gridDim.x - xcd + 7) >> 3, lb = blockIdx.x >> 3;
  if (lb >= xcnt) return;
  const int M = p.M, nk = p.K / KS, tend = xbase + xcnt;
  const int srow = wave * IPW * 8 + (lane >> 3), schunk = (lane & 7) ^ (srow & 7);
  const bool a_rows = BM == 256 || wave * IPW * 8 < BM;  // (wave-uniform) BM 224: wave 7 stages W rows only
  const int fr = lane & 15, fq = lane >> 4;

  auto stage_a = [&](int t, int kt, int slot) {
    if (!a_rows) return;
    const int m0 = (t / nbn) * BM;
    const bf16_t* Ab = p.A + kt * KS + schunk * 8;
    char* d = sa + slot * OPA + wave * IPW * 1024;
#pragma unroll
    for (int i = 0; i < IPW; ++i) lds_dma16(Ab + (long)min(m0 + srow + i * 8, M - 1) * p.lda, (LDS_AS void*)(d + i * 1024));
  };
  auto stage_w = [&](int t, int kt, int slot) {
    const int n0 = (t - (t / nbn) * nbn) * BN;
    const bf16_t* Wb = p.W + (long)(n0 + srow) * p.ldw + kt * KS + schunk * 8;
    char* d = sw + slot * OPB + wave * IPW * 1024;
#pragma unroll
    for (int i = 0; i < IPW; ++i) lds_dma16(Wb + (long)i * 8 * p.ldw, (LDS_AS void*)(d + i * 1024));
  };
  auto adv = [&](int& tt, int& kk) {  // next position of the block's step stream
    if (++kk == nk) kk = 0, tt += nbx;
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  int t = xbase + lb;
  int t1 = t, k1 = 0, t2, k2;  // positions of steps s + 1 and s + 2
  adv(t1, k1);
  t2 = t1, k2 = k1;
  adv(t2, k2);
  stage_a(t, 0, 0);
  stage_w(t, 0, 0);
  if (t1 < tend) stage_a(t1, k1, 1);
  int sA = 0, sW = 0;                    // slots of step s
  bool st_prev = false, rag_prev = false;  // the previous step ended a tile (counted stores / ragged)
  bool range_bad = false;
  for (;;) {
    for (int kt = 0; kt < nk; ++kt) {
      const bool a_pend = a_rows && t1 < tend;  // A(s + 1) in flight behind W(s)
      if (rag_prev) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      else if (a_pend && st_prev) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(IPW + NSTORE) : "memory");
      else if (a_pend) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(IPW) : "memory");
      else if (st_prev) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NSTORE) : "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      st_prev = rag_prev = false;
      const char* A0 = sa + sA * OPA;
      const char* W0 = sw + sW * OPB;
      const int fo0 = fr * 128 + ((fq ^ (fr & 7)) << 4), fo1 = fr * 128 + (((4 + fq) ^ (fr & 7)) << 4);
      bf16x8 b2[2][TN], a2[2 * TM];
#pragma unroll
      for (int j = 0; j < TN; ++j) b2[0][j] = *(const bf16x8*)(W0 + (wn * WN + j * 16) * 128 + fo0);
#pragma unroll
      for (int g = 0; g < XD; ++g) a2[g] = *(const bf16x8*)(A0 + (wm * WM + g * 16) * 128 + fo0);
      __builtin_amdgcn_sched_barrier(0);
      // every wave is past step s - 1: its W slot takes W(s + 1), its A slot A(s + 2)
      if (t1 < tend) stage_w(t1, k1, sW ^ 1);
      if (t2 < tend) stage_a(t2, k2, sA == 0 ? 2 : sA - 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int g = 0; g < 2 * TM; ++g) {
        const int nx = g + XD;
        if (nx == TM) {
#pragma unroll
          for (int j = 0; j < TN; ++j) b2[1][j] = *(const bf16x8*)(W0 + (wn * WN + j * 16) * 128 + fo1);
        }
        if (nx < 2 * TM) a2[nx] = *(const bf16x8*)(A0 + (wm * WM + (nx % TM) * 16) * 128 + (nx < TM ? fo0 : fo1));
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[g % TM][j] = mma<true>(b2[g / TM][j], a2[g], acc[g % TM][j]);
        __builtin_amdgcn_sched_barrier(0);
      }
      sA = sA == 2 ? 0 : sA + 1;
      sW ^= 1;
      t1 = t2, k1 = k2;
      adv(t2, k2);
    }
    const int bm = t / nbn, bn = t - bm * nbn, mb = bm * BM + wm * WM, nb = bn * BN + wn * WN;
    const bool tail = bm * BM + BM > M;  // ragged last row band: rows >= M neither read (RES) nor stored
    f32x4 bj[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j)
      bj[j] = p.bias ? *(const f32x4*)(p.bias + nb + j * 16 + 4 * fq) : (f32x4){0.f, 0.f, 0.f, 0.f};
    if constexpr (SO) {
      // as gemm_f16p_kernel's store-only epilogue (straight-line, head-major rows stepped, fp16 range OR)
      const bool gelu = p.epi == EPI_GELU, hm_step = p.hm_n >= 16;
      int hq = 0, hr = 0;
      if (hm_step) {
        hq = (mb + fr) / p.hm_n;
        hr = mb + fr - hq * p.hm_n;
      }
      uint32_t rbits = 0;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int mr = mb + i * 16 + fr;
        const bool ok = !tail || mr < M;
        long orow;
        if (hm_step) {
          orow = (((long)hq * (p.N / 64) + nb / 64) * p.hm_n + hr) * 64 - nb;
          hr += 16;
          if (hr >= p.hm_n) hr -= p.hm_n, ++hq;
        } else if (p.hm_n) {
          const int m = min(mr, M - 1);
          orow = (((long)(m / p.hm_n) * (p.N / 64) + nb / 64) * p.hm_n + m % p.hm_n) * 64 - nb;
        } else {
          orow = (long)min(mr, M - 1) * p.ldc;
        }
        bf16_t* C = (bf16_t*)p.C + orow + 4 * fq;
        u32x2 pk[TN];
        if (gelu) {
#pragma unroll
          for (int j = 0; j < TN; j += 2) {
            const f32x4 v0 = acc[i][j] + bj[j], v1 = acc[i][j + 1] + bj[j + 1];
            const f32x8 g = gelu_erf_as8((f32x8){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]});
            pk[j] = pack16x4<true>((f32x4){g[0], g[1], g[2], g[3]});
            pk[j + 1] = pack16x4<true>((f32x4){g[4], g[5], g[6], g[7]});
          }
        } else {
#pragma unroll
          for (int j = 0; j < TN; ++j) pk[j] = pack16x4<true>(acc[i][j] + bj[j]);
        }
        uint32_t rb = 0;
#pragma unroll
        for (int j = 0; j < TN; ++j)
          rb |= ((pk[j][0] & 0x7c007c00u) + 0x04000400u) | ((pk[j][1] & 0x7c007c00u) + 0x04000400u);
        rbits |= ok ? rb : 0u;
        const bool odd = fq & 1;
#pragma unroll
        for (int j = 0; j < TN; j += 2) {
          const u32x2 snd = odd ? pk[j] : pk[j + 1];
          const u32x2 rcv = {xor16_partner(snd[0]), xor16_partner(snd[1])};
          const u32x4 w = odd ? (u32x4){rcv[0], rcv[1], pk[j + 1][0], pk[j + 1][1]}
                              : (u32x4){pk[j][0], pk[j][1], rcv[0], rcv[1]};
          if (ok) *(u32x4*)(C + nb + (odd ? (j + 1) * 16 - 4 : j * 16)) = w;
        }
      }
      if (rbits & 0x80008000u) range_bad = true;
    } else {
      float* Cb = (float*)p.C + nb + 4 * fq;
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
          for (int j = 0; j < TN; ++j) *(f32x4*)(Cb + (long)m * p.ldc + j * 16) = rv[i][j] + (acc[h2 * 4 + i][j] + bj[j]);
        }
      }
    }
    st_prev = true;
    rag_prev = tail;
    t += nbx;
    if (t >= tend) break;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  if (SO && p.range_flag && __any(range_bad) && lane == 0) range_flag_set(p.range_flag);
}

}  // namespace
