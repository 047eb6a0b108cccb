// Measured-and-rejected forms of the persistent fp16 encoder GEMM (gemm_kern.h's gemm_f16p_kernel is the product,
// DESIGN.md section 4 / 8): the one-wave-per-SIMD forms gemm_f16w_kernel (round 4, tools build) and gemm_f16h_kernel
// (round 6, hipBLASLt's pipeline; variant builds -DICAP_F16H) and the 3-stage ring gemm_f16r_kernel (tools build).
// Included by gemm_tools.hip and, under ICAP_F16H only, by gemm.hip - a product build compiles none of them.
#pragma once
#include <utility>

#include "gemm_kern.h"

namespace {

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
