// Measured-and-rejected encoder GEMM forms, compiled only into the tools build (-DICAP_TOOLS; build.py adds this
// file to the sources only then, so the product library contains none of it).  Each form is kept because DESIGN.md
// §4-5 quotes its measurement and tools/*.sh re-runs it: the ping-pong fp16 k-loop (gemm_f16q_kernel), the 8-phase
// 256^2 template (gemm_8ph_kernel), and the measurement instantiations of the product templates in gemm_kern.h
// (staging-only NOMFMA variants, 64-row / 64-deep two-block forms, tail split, fp16 ablations ABL 1-8).
#ifndef ICAP_TOOLS
#error "gemm_tools.hip belongs to the tools build only (-DICAP_TOOLS)"
#endif
#include "gemm_kern.h"
#include "gemm_variants.h"

#include <algorithm>

namespace {

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

// Tools-build dispatch of launch_gemm_256_: returns true (and the launch status in *err) when a measurement knob
// selects one of the forms above or a measurement instantiation of the product templates; false leaves the launch
// to the product forms.  Knob meanings as documented in DESIGN.md §4-5.
bool launch_gemm_256_tools(const GemmArgs& g, hipStream_t s, int cus, hipError_t* err) {
  auto done = [&]() {
    *err = hipGetLastError();
    return true;
  };
  auto attr = [&](const void* f, int bytes) {
    const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e != hipSuccess) *err = e;
    return e == hipSuccess;
  };
  constexpr int lds2 = 3 * 3 * 256 * 32 * 2, lds1 = 4 * 2 * 256 * 32 * 2;
  constexpr int LP = F16P_LDS_SO, LP224 = 2 * (224 * 128 + 256 * 128) + 2048;
  if (g.f16) {
    // ICAP_F16_GEMM: 1 / 2 = 256 x 256 8-phase (64-B / 128-B LDS rows); 3 / 4 = 128 x 256 tiles with 64-deep
    // stages, 2 / 3 stages; 5 = 256 x 256 tiles, 64-deep stages; 6 = persistent for every fp16 GEMM
    static const int form = icap_knob("ICAP_F16_GEMM", 0);
    if ((form == 1 || form == 2) && g.K % 64 == 0) {
      if (!attr((const void*)gemm_8ph_kernel<false, true>, 131072) || !attr((const void*)gemm_8ph_kernel<true, true>, 131072))
        return true;
      const int nwg8 = (g.N / 256) * ((g.M + 255) / 256);
      if (form == 2) hipLaunchKernelGGL((gemm_8ph_kernel<true, true>), dim3(nwg8), dim3(512), 131072, s, g);
      else hipLaunchKernelGGL((gemm_8ph_kernel<false, true>), dim3(nwg8), dim3(512), 131072, s, g);
      return done();
    }
    const bool so = gemm_f16_persistent(g), res = g.out == OUT_F32_RESID;
    const dim3 grid(std::min((g.N / 256) * ((g.M + 255) / 256), cus));
    if (form == 7 && so) {  // the A operand two k-steps ahead (gemm_kern.h; measured equal)
      if (res) {
        if (!attr((const void*)gemm_f16r_kernel<2, 224>, F16R_LDS_224)) return true;
        hipLaunchKernelGGL((gemm_f16r_kernel<2, 224>), dim3(std::min((g.N / 256) * ((g.M + 223) / 224), cus)), dim3(512),
                           F16R_LDS_224, s, g);
      } else {
        if (!attr((const void*)gemm_f16r_kernel<1, 256>, F16R_LDS_256)) return true;
        hipLaunchKernelGGL((gemm_f16r_kernel<1, 256>), grid, dim3(512), F16R_LDS_256, s, g);
      }
      return done();
    }
    const dim3 grid224(std::min((g.N / 256) * ((g.M + 223) / 224), cus));
    // ICAP_F16_GEMM 8 / 9 / 10: the one-wave-per-SIMD form (gemm_f16w_kernel) with the stage pieces spread over the
    // MFMA groups (8), in one burst (9), or spread with 256-row residual tiles (10)
    if ((form == 8 || form == 9 || form == 10) && so) {
#define F16W(MODE_, EP_, DI_, BM_, GRID_)                                                                 \
  {                                                                                                       \
    if (!attr((const void*)gemm_f16w_kernel<MODE_, EP_, DI_, BM_>, f16w_lds(BM_))) return true;           \
    hipLaunchKernelGGL((gemm_f16w_kernel<MODE_, EP_, DI_, BM_>), GRID_, dim3(256), f16w_lds(BM_), s, g);  \
  }
      if (!res) {
        const int ep = g.hm_n ? 2 : g.epi == EPI_GELU ? 1 : 0;
        if (form == 9) {
          if (ep == 2) F16W(1, 2, 0, 256, grid) else if (ep == 1) F16W(1, 1, 0, 256, grid) else F16W(1, 0, 0, 256, grid)
        } else {
          if (ep == 2) F16W(1, 2, 1, 256, grid) else if (ep == 1) F16W(1, 1, 1, 256, grid) else F16W(1, 0, 1, 256, grid)
        }
      } else if (form == 10) {
        F16W(2, 0, 1, 256, grid)
      } else if (form == 9) {
        F16W(2, 0, 0, 224, grid224)
      } else {
        F16W(2, 0, 1, 224, grid224)
      }
#undef F16W
      return done();
    }
    // ICAP_F16P_ABL: gemm_f16p_kernel without its k-loop DMA (1) or without its MFMAs (2) - wrong results,
    // timing only (tools/f16_ablate.sh); 3 / 4 / 5: the compiler's fragment-read order / the read pipeline per
    // k-half / the stage's DMA before the first fragment reads; 6: reads 3 groups ahead; 7: setprio; 8: 8-B stores
    static const int abl = icap_knob("ICAP_F16P_ABL", 0);
    if (so && abl >= 1 && abl <= 12) {
#define F16P_ABL(A_)                                                                                  \
  if (abl == A_) {                                                                                    \
    if (!res) {                                                                                       \
      if (!attr((const void*)gemm_f16p_kernel<1, A_>, LP)) return true;                               \
      hipLaunchKernelGGL((gemm_f16p_kernel<1, A_>), grid, dim3(512), LP, s, g);                       \
    } else if constexpr (A_ >= 3) {                                                                   \
      constexpr int AB = A_ == 8 ? 0 : A_;                                                            \
      if (!attr((const void*)gemm_f16p_kernel<2, AB, 224>, LP224)) return true;                       \
      hipLaunchKernelGGL((gemm_f16p_kernel<2, AB, 224>), grid224, dim3(512), LP224, s, g);            \
    } else {                                                                                          \
      if (!attr((const void*)gemm_f16p_kernel<2, A_>, LP)) return true;                               \
      hipLaunchKernelGGL((gemm_f16p_kernel<2, A_>), grid, dim3(512), LP, s, g);                       \
    }                                                                                                 \
    return done();                                                                                    \
  }
      F16P_ABL(1) F16P_ABL(2) F16P_ABL(3) F16P_ABL(4) F16P_ABL(5) F16P_ABL(6) F16P_ABL(7) F16P_ABL(8)
      F16P_ABL(9) F16P_ABL(10) F16P_ABL(11) F16P_ABL(12)
#undef F16P_ABL
    }
    // ICAP_F16_PP=1: the ping-pong k-loop (gemm_f16q_kernel; slower)
    static const int pp = icap_knob("ICAP_F16_PP", 0);
    if (so && pp) {
      constexpr int LQ = 4 * 32 * 1024 + 2048;
      if (res) {
        if (!attr((const void*)gemm_f16q_kernel<2>, LQ)) return true;
        hipLaunchKernelGGL(gemm_f16q_kernel<2>, grid, dim3(512), LQ, s, g);
      } else {
        if (!attr((const void*)gemm_f16q_kernel<1>, LQ)) return true;
        hipLaunchKernelGGL(gemm_f16q_kernel<1>, grid, dim3(512), LQ, s, g);
      }
      return done();
    }
    // ICAP_F16_RES_BM=256: the residual GEMMs on 256-row persistent tiles
    static const int res_bm = icap_knob("ICAP_F16_RES_BM", 224);
    if (so && res && res_bm != 224) {
      hipLaunchKernelGGL(gemm_f16p_kernel<2>, grid, dim3(512), LP, s, g);
      return done();
    }
    if (form == 6 && !so && g.K % 64 == 0) {  // the generic persistent mode (shared epilogue; spills)
      if (!attr((const void*)gemm_f16p_kernel<0>, 2 * 64 * 1024)) return true;
      hipLaunchKernelGGL(gemm_f16p_kernel<0>, grid, dim3(512), 2 * 64 * 1024, s, g);
      return done();
    }
    if (!so && form >= 3 && form <= 5 && g.K % 64 == 0) {
      if (!attr((const void*)gemm_256_kernel<1, 8, 0, 0, 128, 2, 64, 0, true>, 2 * 48 * 1024) ||
          !attr((const void*)gemm_256_kernel<1, 8, 0, 0, 128, 3, 64, 0, true>, 3 * 48 * 1024) ||
          !attr((const void*)gemm_256_kernel<1, 8, 0, 0, 256, 2, 64, 0, true>, 2 * 64 * 1024))
        return true;
      if (form == 5)
        hipLaunchKernelGGL((gemm_256_kernel<1, 8, 0, 0, 256, 2, 64, 0, true>), dim3((g.N / 256) * ((g.M + 255) / 256)),
                           dim3(512), 2 * 64 * 1024, s, g);
      else if (form == 4)
        hipLaunchKernelGGL((gemm_256_kernel<1, 8, 0, 0, 128, 3, 64, 0, true>), dim3((g.N / 256) * ((g.M + 127) / 128)),
                           dim3(512), 3 * 48 * 1024, s, g);
      else
        hipLaunchKernelGGL((gemm_256_kernel<1, 8, 0, 0, 128, 2, 64, 0, true>), dim3((g.N / 256) * ((g.M + 127) / 128)),
                           dim3(512), 2 * 48 * 1024, s, g);
      return done();
    }
    return false;
  }
  // bf16 / bf16x2.  ICAP_GEMM256_WAVES: 16 (default), 8 (the 8-wave 256 x 256 form below K = 128), 1 / 2 (the
  // 8-phase kernel), 160-162 (staging-only variants, wrong results); ICAP_GEMM_TALL_MIN_K: the smallest K of the
  // 128 x 256 two-block form (0 = off); ICAP_GEMM_TALL_BM=64: 64 x 256 tiles, 4 waves, 3 blocks per CU;
  // ICAP_GEMM_TALL_KS=64: 64-deep stages (128 KiB, one block per CU); ICAP_GEMM_TAIL (icap.cpp): tail split
  static const int nw = icap_knob("ICAP_GEMM256_WAVES", 16);
  static const int tall_min_k = icap_knob("ICAP_GEMM_TALL_MIN_K", 128);
  static const int tall_bm = icap_knob("ICAP_GEMM_TALL_BM", 128) == 64 ? 64 : 128;
  static const int tall_ks = icap_knob("ICAP_GEMM_TALL_KS", 32) == 64 ? 64 : 32;
  const bool tall = tall_min_k && g.K >= tall_min_k && nw != 1 && nw != 2 && nw < 160;
  const int nwgh = (g.N / 256) * ((g.M + 127) / 128), nwg = (g.N / 256) * ((g.M + 255) / 256);
  if (g.cv && g.cv != 1) return false;
  if (tall && tall_bm == 64 && !g.cv) {
    const int nwgq = (g.N / 256) * ((g.M + 63) / 64);
    constexpr int ldsq = 2 * (2 * 64 * 32 * 2 + 256 * 32 * 2), ldsq1 = 2 * (64 * 32 * 2 + 256 * 32 * 2);
    if (g.nsplit == 2) hipLaunchKernelGGL((gemm_256_kernel<2, 4, 0, 0, 64, 2>), dim3(nwgq), dim3(256), ldsq, s, g);
    else hipLaunchKernelGGL((gemm_256_kernel<1, 4, 0, 0, 64, 2>), dim3(nwgq), dim3(256), ldsq1, s, g);
    return done();
  }
  if (tall && tall_ks == 64 && g.K % 64 == 0) {
    constexpr int lds64 = 2 * (2 * 128 * 64 * 2 + 256 * 64 * 2), lds64_1 = 2 * (128 * 64 * 2 + 256 * 64 * 2);
    if (!attr((const void*)gemm_256_kernel<2, 8, 0, 0, 128, 2, 64>, lds64) ||
        !attr((const void*)gemm_256_kernel<2, 8, 0, 1, 128, 2, 64>, lds64) ||
        !attr((const void*)gemm_256_kernel<1, 8, 0, 0, 128, 2, 64>, lds64_1) ||
        !attr((const void*)gemm_256_kernel<1, 8, 0, 1, 128, 2, 64>, lds64_1))
      return true;
    if (g.nsplit == 2) {
      if (g.cv) hipLaunchKernelGGL((gemm_256_kernel<2, 8, 0, 1, 128, 2, 64>), dim3(nwgh), dim3(512), lds64, s, g);
      else hipLaunchKernelGGL((gemm_256_kernel<2, 8, 0, 0, 128, 2, 64>), dim3(nwgh), dim3(512), lds64, s, g);
    } else {
      if (g.cv) hipLaunchKernelGGL((gemm_256_kernel<1, 8, 0, 1, 128, 2, 64>), dim3(nwgh), dim3(512), lds64_1, s, g);
      else hipLaunchKernelGGL((gemm_256_kernel<1, 8, 0, 0, 128, 2, 64>), dim3(nwgh), dim3(512), lds64_1, s, g);
    }
    return done();
  }
  if (tall) {  // tail split of the residual GEMMs: measured and rejected
    const int S = g.split_slots, q = nwgh >> 3;
    if (g.split_ws && g.split_cnt && S > 0 && !g.cv && q + 1 > S && (g.K / 32) % 2 == 0) {
      constexpr int ldsh = 2 * (2 * 128 * 32 * 2 + 256 * 32 * 2), ldsh1 = 2 * (128 * 32 * 2 + 256 * 32 * 2);
      const int tq1 = (q + 1) % S, tq = q > S ? q % S : 0;
      const int per_xcd = std::max(q + 1 + tq1, q + tq);
      if (g.nsplit == 2)
        hipLaunchKernelGGL((gemm_256_kernel<2, 8, 0, 0, 128, 2, 32, 1>), dim3(8 * per_xcd), dim3(512), ldsh, s, g);
      else
        hipLaunchKernelGGL((gemm_256_kernel<1, 8, 0, 0, 128, 2, 32, 1>), dim3(8 * per_xcd), dim3(512), ldsh1, s, g);
      return done();
    }
    return false;
  }
  if (g.cv) return false;
  if ((nw == 1 || nw == 2) && g.K % 64 == 0) {
    if (!attr((const void*)gemm_8ph_kernel<false>, 131072) || !attr((const void*)gemm_8ph_kernel<true>, 131072))
      return true;
    if (nw == 2) hipLaunchKernelGGL(gemm_8ph_kernel<true>, dim3(nwg), dim3(512), 131072, s, g);
    else hipLaunchKernelGGL(gemm_8ph_kernel<false>, dim3(nwg), dim3(512), 131072, s, g);
    return done();
  }
  if ((nw == 160 || nw == 161 || nw == 162) && g.nsplit == 2) {
    if (!attr((const void*)gemm_256_kernel<2, 16, 1>, lds2) || !attr((const void*)gemm_256_kernel<2, 16, 2>, lds2) ||
        !attr((const void*)gemm_256_kernel<2, 16, 3>, lds2))
      return true;
    if (nw == 160) hipLaunchKernelGGL((gemm_256_kernel<2, 16, 1>), dim3(nwg), dim3(1024), lds2, s, g);
    else if (nw == 161) hipLaunchKernelGGL((gemm_256_kernel<2, 16, 2>), dim3(nwg), dim3(1024), lds2, s, g);
    else hipLaunchKernelGGL((gemm_256_kernel<2, 16, 3>), dim3(nwg), dim3(1024), lds2, s, g);
    return done();
  }
  if (nw == 8) {
    if (!attr((const void*)gemm_256_kernel<2, 8>, lds2) || !attr((const void*)gemm_256_kernel<1, 8>, lds1)) return true;
    if (g.nsplit == 2) hipLaunchKernelGGL((gemm_256_kernel<2, 8>), dim3(nwg), dim3(512), lds2, s, g);
    else hipLaunchKernelGGL((gemm_256_kernel<1, 8>), dim3(nwg), dim3(512), lds1, s, g);
    return done();
  }
  return false;
}
