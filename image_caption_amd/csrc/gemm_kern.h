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

// dynamic LDS of gemm_f16p_kernel<1> (and <2> at 256 rows): 2 stages of 64 KiB, then the bias slots (2 x 1 KiB)
constexpr int F16P_LDS_SO = 2 * 64 * 1024 + 2048;
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
  // (a buffer-load DMA: the per-lane 32-bit offset, the tile's offset in an SGPR)
  const i32x4r rsb = buf_rsrc(p.bias, (uint32_t)p.N * 4);
  auto load_bias = [&](int t, int slot) {
    const int n0 = (t % nbn) * BN;
    if (wave == 0 && p.bias) lds_dma_buf16(rsb, (uint32_t)lane * 16, (uint32_t)n0 * 4, (LDS_AS void*)(sbias + slot * 256));
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  int t = xbase + lb, step = 0, tcount = 0;
  if (SO || RES) load_bias(t, 0);
  stage(t, 0, 0);
  if (LB) stage(t, 1, 1);  // LB: both stages of a tile's opening in flight before its k-step 0
  bool seam = false;  // this tile's stages 0 and 1 were issued before the previous tile's epilogue stores
  bool range_bad = false;  // SO: some stored fp16 value is not finite (p.range_flag set once, after the last tile)
  for (;;) {
    const int tn = t + nbx < xbase + xcnt ? t + nbx : -1;  // this block's next tile
    if constexpr (LB) {
      const int fo0 = fr * 128 + (swz_chunk(fq, fr) << 4), fo1 = fr * 128 + (swz_chunk(4 + fq, fr) << 4);
      bf16x8 b2[2][TN], a2[2 * TM];
      for (int kt = 0; kt < nk; ++kt, ++step) {
        const char* s0 = smem + (step & 1) * STAGE;
        if (kt == 0) {  // a tile's opening: stage 0 landed (stage 1 and, after a seam, the stores may still fly)
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
        const bool late = kt + 1 < nk;  // the last k-step of a tile has no late point
        // a k-step entered from a late point carries its b2[0] fragments only (register budget): A fragments 0 and 1 now
        if (kt > 0) {
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
          if (SO && seam && kt == 0) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NSTORE) : "memory");
          else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");
          // the next k-step's first fragments (its buffer is the other one), then the stage after next into this one
          const char* s1 = smem + ((step + 1) & 1) * STAGE;
          bf16x8 nb[TN];
#pragma unroll
          for (int j = 0; j < TN; ++j) nb[j] = *(const bf16x8*)(s1 + OPA + (wn * WN + j * 16) * 128 + fo0);
          __builtin_amdgcn_sched_barrier(0);
          if (kt + 2 < nk) {
            stage(t, kt + 2, step & 1);
          } else if (tn >= 0) {  // the next tile's bias and stage 0
            if (SO || RES) load_bias(tn, (tcount + 1) & 1);
            stage(tn, 0, step & 1);
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
    if constexpr (SO) {
      if (tn >= 0) {  // every wave is done reading the last stage's buffer: stage 1 of the next tile into it
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (ABL != 1 && ABL < 10) stage(tn, 1, (step + 1) & 1);  // step = the next tile's k-step 0 here; its k-step 1 reads (step + 1) & 1
      }
      const bool tail = bm * BM + BM > M;  // the last row band of a ragged M: rows >= M are not stored
      // straight-line per row tile (no per-element branches, so the scheduler interleaves the TN x 2 independent GELU
      // chains instead of padding each dependent packed FMA with a nop): bias in registers, head-major row offsets
      // stepped by 16 rows, the fp16 range test as an OR of exponent carries - (h & 0x7c00) + 0x400 reaches bit 15
      // exactly when h is Inf / NaN - masked by the row's store predicate
      f32x4 bj[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bj[j] = p.bias ? *(const f32x4*)(sbias + (tcount & 1) * 256 + wn * WN + j * 16 + 4 * fq) : (f32x4){0.f, 0.f, 0.f, 0.f};
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
            if (h2 * 4 + i < TM) {
              const long row = min(mb + (h2 * 4 + i) * 16 + fr, M - 1);
              rv[i][j] = *(const f32x4*)(Cb + row * p.ldc + j * 16);
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
          if (tail && m >= M) continue;
#pragma unroll
          for (int j = 0; j < TN; ++j) *(f32x4*)(Cb + (long)m * p.ldc + j * 16) = o[j];
        }
      }
      if (tn >= 0) {  // stage 1 of the next tile into the last stage's buffer, after the stores
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (ABL != 1 && ABL < 10) stage(tn, 1, (step + 1) & 1);
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

}  // namespace
