// W-stationary persistent 1x1 convolution for the fp16 Grid trunk's residual conv3 (GemmArgs::f16 with a BN scale and
// a residual: out = relu(acc * scale + shift + residual planes) as fp16 planes).
//
// Why: the conv3 GEMMs are short-K (64 / 128 / 256), wide-N and output-heavy - per output element they move 2-4 B of
// residual in and 2-4 B of output out against K MACs - so they are HBM streams with a small GEMM attached (layer3
// conv3 at B = 256: 436 MB for 26 GFLOP; 165 us on the 64 x 256 tiles of the 256-family kernel = 2.6 TB/s).  In that
// kernel every tile re-stages its 256-column W slice (128 KiB at K = 256) and waits a memory round trip per k-step and
// another for the residual, with two tiles per CU in flight.  Here one block per CU keeps its 128-column W slice
// resident in LDS for the whole launch and walks row tiles: each tile's A rows (the branch output, one fp16 plane) and
// residual planes are LDS-DMA'd one tile AHEAD into a 2-deep ring, so at a tile's top only the previous tile's stores
// may still be in flight (a counted vmcnt leaves them there) and the A / residual latency hides behind a tile of MFMAs
// and the epilogue.  (A first form loaded the residual into registers a tile ahead: hipcc then waited vmcnt(0) before
// the epilogue - its wait analysis cannot see across the loop - which also waited for the prefetches.)  Scale / shift
// live in registers (an epilogue load would make the in-order counter wait for the prefetches).  Blocks: XCD x (blockIdx & 7) owns row tiles x, x + 8, ...; its blocks split into ncg column groups x
// walkers, so a row tile's A is read by the ncg blocks of one XCD (one L2) and each XCD's L2 holds the whole W.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int CR_BN = 128, CR_TN = 2;

// KB = K / 64 (1, 2, 4); BM = 64 (K <= 128) or 32 (K = 256: the LDS budget).  LDS: the W image [KB][128][128 B] and two
// tile buffers, each the A image [KB][BM][128 B] and the residual image [planes][BM][256 B] (16-byte chunk c of row r at
// c ^ (r & 15): the epilogue's 8-byte reads of 16 rows x one chunk are conflict-free).  Every operand of the tile loop
// arrives by LDS-DMA, which writes no VGPR: hipcc inserts no wait for it, so the only waits are the counted ones below.
template <int KB, int BM>
__global__ __launch_bounds__(512, 1) void conv_rmw_kernel(GemmArgs p) {
  constexpr int K = 64 * KB, TM = BM / 32;
  constexpr int WIMG = CR_BN * K * 2, AIMG = BM * K * 2, RPL = BM * CR_BN * 2, BUF = AIMG + 2 * RPL;
  constexpr int IPW_W = WIMG / 1024 / 8, IPW_A = AIMG / 1024 / 8, IPW_R = RPL / 1024 / 8;
  static_assert(IPW_A >= 1 && IPW_W >= 1 && IPW_R >= 1 && TM >= 1, "tile shape");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* wimg = smem;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wm = wave >> 2, wn = wave & 3;
  const int fr = lane & 15, fq = lane >> 4;
  const int M = p.M, ncg = p.N / CR_BN, nrt = (M + BM - 1) / BM;
  const int xcd = blockIdx.x & 7, lb = blockIdx.x >> 3, nb8 = (int)gridDim.x >> 3;
  const int cg = lb % ncg, walker = lb / ncg, nwalk = nb8 / ncg;
  if (walker >= nwalk) return;
  // this block's row tiles: rt(i) = xcd + 8 (walker + nwalk i)
  auto tile_of = [&](int i) { return xcd + 8 * (walker + nwalk * i); };
  if (tile_of(0) >= nrt) return;
  const int n0 = cg * CR_BN;
  const bool has_res = p.res != nullptr, res2 = has_res && p.res_planes != 1, lo_out = p.c_planes == 2;

  // W slice: rows n0 .. n0 + 127, all of K (16 DMA instructions per 64-deep k block)
#pragma unroll
  for (int i = 0; i < IPW_W; ++i) {
    const int ins = wave * IPW_W + i, kb = ins >> 4, r = (ins & 15) * 8 + (lane >> 3);
    const bf16_t* src = p.W + (long)(n0 + r) * p.ldw + kb * 64 + (((lane & 7) ^ (r & 7)) << 3);
    lds_dma16(src, (LDS_AS void*)(wimg + ins * 1024));
  }
  // row tile rt's A rows (8 rows x 128 B per instruction) and residual rows (4 rows x 256 B) into buffer buf
  auto stage = [&](int rt, int buf) {
    char* b0 = smem + WIMG + buf * BUF;
#pragma unroll
    for (int i = 0; i < IPW_A; ++i) {
      const int ins = wave * IPW_A + i, kb = ins / (BM / 8), r = (ins % (BM / 8)) * 8 + (lane >> 3);
      const int row = min(rt * BM + r, M - 1);
      const bf16_t* src = p.A + (long)row * p.lda + kb * 64 + (((lane & 7) ^ (r & 7)) << 3);
      lds_dma16(src, (LDS_AS void*)(b0 + ins * 1024));
    }
#pragma unroll
    for (int pl = 0; pl < 2; ++pl) {
      if (!has_res || (pl == 1 && !res2)) break;
#pragma unroll
      for (int i = 0; i < IPW_R; ++i) {
        const int ins = wave * IPW_R + i, r = ins * 4 + (lane >> 4);
        const int row = min(rt * BM + r, M - 1);
        const bf16_t* src = p.res + pl * p.res_lo + (long)row * p.res_ld + n0 + (((lane & 15) ^ (r & 15)) << 3);
        lds_dma16(src, (LDS_AS void*)(b0 + AIMG + pl * RPL + ins * 1024));
      }
    }
  };
  f32x4 sv[CR_TN], bv[CR_TN];
#pragma unroll
  for (int j = 0; j < CR_TN; ++j) {
    const int col = n0 + wn * 32 + j * 16 + 4 * fq;
    sv[j] = *(const f32x4*)(p.scale + col);
    bv[j] = *(const f32x4*)(p.bias + col);
  }
  const bool relu = p.epi == EPI_RELU;
  uint32_t rbits = 0;  // fp16 range test: OR of (h & 0x7c00) + 0x400 per half (bit 15 <=> Inf / NaN)
  bf16_t* C = (bf16_t*)p.C;

  stage(tile_of(0), 0);
  for (int i = 0;; ++i) {
    const int buf = i & 1, rt = tile_of(i), rn = tile_of(i + 1);
    // this tile's stage was issued before the previous tile's stores, which may stay in flight: wait for all but them
    if (i == 0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    else if (lo_out) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * TM * CR_TN) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(TM * CR_TN) : "memory");
    __builtin_amdgcn_s_barrier();  // the stage landed for every wave; every wave is done reading the other buffer
    if (rn < nrt) stage(rn, buf ^ 1);
    const char* aimg = smem + WIMG + buf * BUF;
    const char* rimg = aimg + AIMG;
    f32x4 acc[TM][CR_TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < CR_TN; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2 * KB; ++ks) {
      const int kb = ks >> 1, c = (ks & 1) * 4 + fq;
      bf16x8 wf[CR_TN], af[TM];
#pragma unroll
      for (int j = 0; j < CR_TN; ++j) {
        const int r = wn * 32 + j * 16 + fr;
        wf[j] = *(const bf16x8*)(wimg + kb * (CR_BN * 128) + r * 128 + ((c ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const int r = wm * (BM / 2) + a * 16 + fr;
        af[a] = *(const bf16x8*)(aimg + kb * (BM * 128) + r * 128 + ((c ^ (r & 7)) << 4));
      }
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int j = 0; j < CR_TN; ++j) acc[a][j] = mma<true>(wf[j], af[a], acc[a][j]);
    }
    // epilogue: lane holds row m = mb + a * 16 + fr, columns nb + j * 16 + 4 fq .. + 3
    const int mb = rt * BM + wm * (BM / 2), nb = n0 + wn * 32;
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      const int r = wm * (BM / 2) + a * 16 + fr, m = mb + a * 16 + fr;
      u32x2 hv[CR_TN], lv[CR_TN];
#pragma unroll
      for (int j = 0; j < CR_TN; ++j) {
        const int chunk = wn * 4 + j * 2 + (fq >> 1);  // 16-byte chunk of the 256-byte residual row
        const int off = r * 256 + ((chunk ^ (r & 15)) << 4) + (fq & 1) * 8;
        const u32x2 wh = has_res ? *(const u32x2*)(rimg + off) : (u32x2){0u, 0u};
        const u32x2 wl = res2 ? *(const u32x2*)(rimg + RPL + off) : (u32x2){0u, 0u};
        f32x4 v = acc[a][j] * sv[j] + bv[j];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t h = wh[e >> 1] >> ((e & 1) * 16), l = wl[e >> 1] >> ((e & 1) * 16);
          v[e] += h2f((bf16_t)(h & 0xffff)) + h2f((bf16_t)(l & 0xffff));
        }
        if (relu)
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
        hv[j] = pack16x4<true>(v);
        f32x4 lo;
#pragma unroll
        for (int e = 0; e < 4; ++e) lo[e] = v[e] - h2f((bf16_t)((hv[j][e >> 1] >> ((e & 1) * 16)) & 0xffff));
        lv[j] = pack16x4<true>(lo);
        const uint32_t rb = ((hv[j][0] & 0x7c007c00u) + 0x04000400u) | ((hv[j][1] & 0x7c007c00u) + 0x04000400u);
        rbits |= m < M ? rb : 0u;
      }
      if (m < M) {  // (only the launch's last row tile has rows >= M, and it is the last tile of its block)
        const long o = (long)m * p.ldc + nb + 4 * fq;
#pragma unroll
        for (int j = 0; j < CR_TN; ++j) *(u32x2*)(C + o + j * 16) = hv[j];
        if (lo_out)
#pragma unroll
          for (int j = 0; j < CR_TN; ++j) *(u32x2*)(C + o + j * 16 + p.c_lo) = lv[j];
      }
    }
    if (rn >= nrt) break;
  }
  if (p.range_flag && __any((rbits & 0x80008000u) != 0) && lane == 0) range_flag_set(p.range_flag);
}

template <int KB, int BM>
hipError_t run_conv_rmw(const GemmArgs& g, hipStream_t s, int blocks) {
  constexpr int lds = CR_BN * 64 * KB * 2 + 2 * (BM * 64 * KB * 2 + 2 * BM * CR_BN * 2);
  static bool attr = false;
  if (!attr && lds > 65536) {
    const hipError_t e =
        hipFuncSetAttribute((const void*)conv_rmw_kernel<KB, BM>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL((conv_rmw_kernel<KB, BM>), dim3(blocks), dim3(512), lds, s, g);
  return hipGetLastError();
}

}  // namespace

bool conv_rmw_ok(const GemmArgs& g) {
  const int ncg = g.N / CR_BN;
  return g.f16 && g.scale && g.bias && g.out == OUT_SPLIT && (g.epi == EPI_NONE || g.epi == EPI_RELU) &&
         g.cv == 0 && g.nsplit == 1 && g.batch == 1 && !g.addend && !g.rm_group && !g.hm_n && !g.split_slots &&
         (g.K == 64 || g.K == 128 || g.K == 256) && g.ldw == g.K && g.N % CR_BN == 0 && ncg <= 32 &&
         (ncg & (ncg - 1)) == 0 && g.M > 0;
}

hipError_t launch_conv_rmw(const GemmArgs& g, hipStream_t s, int cus) {
  if (!conv_rmw_ok(g)) return hipErrorInvalidValue;
  const int ncg = g.N / CR_BN, nb8 = cus / 8 / ncg * ncg;  // blocks per XCD: a multiple of the column groups
  if (nb8 < ncg) return hipErrorInvalidValue;
  const int blocks = 8 * nb8;
  return g.K == 64 ? run_conv_rmw<1, 64>(g, s, blocks) : g.K == 128 ? run_conv_rmw<2, 64>(g, s, blocks)
                                                                     : run_conv_rmw<4, 32>(g, s, blocks);
}
